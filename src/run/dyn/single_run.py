"""Drop-in for the reference's ``src/run/dyn/single_run.py:23-29``: ``python src/run/dyn/single_run.py`` from the directory that holds
``configs/`` loads ``configs/dynamical_systems/perm_equiv_gncde_config.yaml`` and trains it on this engine (engine.trainer.Trainer -> gncde.run.Trainer).
wandb is not used (metrics are JSON lines on stdout); ``--config <yaml>`` overrides the path and the other flags
of ``python -m gncde.run`` (--epochs, --out, ...) pass through."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..",
                                "perm-equiv-graph-neural-cdes_amd"))

from gncde import run  # noqa: E402

CONFIG = "configs/dynamical_systems/perm_equiv_gncde_config.yaml"

if __name__ == "__main__":
    run.single_run(CONFIG)
