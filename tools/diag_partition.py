"""Diagnostic (GPU): is the dyn model's PID-solve gradient additive over sample partitions?  The full-batch
gradient of the summed loss must equal the sum of the gradients over any partition of the samples (what the
data-parallel trainer relies on).  Prints the relative difference per partition."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]

import torch  # noqa: E402
import yaml  # noqa: E402

from gncde import run, train  # noqa: E402


def main():
    with open(os.path.join(ROOT, "configs", "heat_grid_small.yaml")) as fh:
        cfg = yaml.safe_load(fh)
    cfg["dataset"].update(num_nodes=16, time_tick=16, batch_size=int(os.environ.get("DIAG_B", "5")))
    tr = run.Trainer(cfg, epochs=1, steps_per_interval=None)
    ds, model = tr.build()
    ts_tr, coef_tr, tcoef_tr = ds.graph_path(ds.id_train)
    y_tr = ds.true_y[:, torch.as_tensor(ds.id_train, device=ds.true_y.device)]
    prob = model.vector_field.problem_from_layout(ts_tr, coef_tr, tcoef_tr)
    opt = train.ClipAdamW(model, learning_rate=0.01)
    B = prob.B

    def grad_of(own):
        p = prob.take(own)
        x0 = ds.x0[torch.as_tensor(own, device=ds.x0.device)]
        y = y_tr[torch.as_tensor(own, device=y_tr.device)]
        spec = model._spec(p.ts, evolving_out=True)
        spec.stats_out = torch.zeros(len(own), 4, dtype=torch.int32, device=x0.device)
        opt.zero_grad()
        pred = model.predict_packed(p, x0, spec).squeeze(-1)
        sse = ((pred - y) ** 2).sum()
        sse.backward()
        return opt.flat_grad().double().cpu(), spec.stats_out[:, 0].tolist(), float(sse)

    full, steps, sse = grad_of(list(range(B)))
    print("steps per sample", steps, "sse", sse)
    parts_list = [[[i] for i in range(B)], [[0, 3], [1, 2, 4]], [[0, 1, 2], [3, 4]], [[4, 3, 2, 1, 0]]]
    for parts in parts_list:
        parts = [[i for i in p if i < B] for p in parts]
        parts = [p for p in parts if p]
        tot = torch.zeros_like(full)
        s = 0.0
        for p in parts:
            g, st, e = grad_of(p)
            tot += g
            s += e
        d = float((tot - full).abs().max() / full.abs().max())
        print(parts, f"grad rel diff {d:.3e}", f"sse {s:.6g} vs {sse:.6g}")
    # per-sample gradient: solo vs inside the full batch (drop others by a zero label weight is not possible: use
    # the singleton grads above); also the forward predictions solo vs in batch
    with torch.no_grad():
        spec = model._spec(prob.ts, evolving_out=True)
        pf = model.predict_packed(prob, ds.x0, spec)
        for i in range(B):
            p = prob.take([i])
            sp = model._spec(p.ts, evolving_out=True)
            pi = model.predict_packed(p, ds.x0[i:i + 1], sp)
            print("sample", i, "forward solo vs batch max diff", float((pi[0] - pf[i]).abs().max()))


if __name__ == "__main__":
    main()
