"""GPU, two ranks on one device (gloo carries the collective): the data-parallel training step end to end —
shard_range -> GPU solve + discrete adjoint per rank -> gradient all-reduce -> gncde_clip_adamw — equals the
single-process full-batch step (trainer.py:288-327 semantics).  The 8-GPU RCCL run is the
driver's; this exercises the same code path with a transport that shares one card."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, N, T, HID = 6, 16, 5, 16


def _problem_data():
    from oracle import gncde_oracle as O
    rng = np.random.default_rng(77)
    ts_l, co_l = [], []
    for _ in range(B):
        ts, X = O.make_graph_control(rng, N, T)
        ts_l.append(ts)
        co_l.append(O.backward_hermite_coefficients(ts, X))
    ts = np.stack(ts_l)
    coeffs = tuple(np.stack([c[q] for c in co_l]) for q in range(4))
    x0 = rng.standard_normal((B, N, 1))
    labels = np.tanh(rng.standard_normal((B, T, N)))
    return ts, coeffs, x0, labels


def _model():
    from gncde.models import GraphNeuralCDE, vector_fields as V
    vf = V.PermEquivGraphVectorField(HID, HID, HID, 2, 16, N, key=5)
    return GraphNeuralCDE({"hidden_dim": HID}, vf, "cubic", 3, solver={"method": "rk4", "steps_per_interval": 2})


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "perm-equiv-graph-neural-cdes_amd")]
    import torch.distributed as dist
    from gncde import train
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        ts, coeffs, x0, labels = _problem_data()
        a, b = train.shard_range(B, rank, world)
        model = _model().to("cuda")
        opt = train.ClipAdamW(model, learning_rate=1e-2, weight_decay=1e-4)
        for _ in range(2):
            loss, _, _ = train.make_step(opt, model.loss_terms, torch.tensor(ts[a:b]),
                                         tuple(c[a:b] for c in coeffs), torch.tensor(x0[a:b]),
                                         torch.tensor(labels[a:b]))
        out[rank, :-1] = opt.flat.cpu()
        out[rank, -1] = float(loss)
    finally:
        dist.destroy_process_group()


def test_two_rank_step_equals_full_batch():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from gncde import train
    ts, coeffs, x0, labels = _problem_data()
    model = _model().to("cuda")
    opt = train.ClipAdamW(model, learning_rate=1e-2, weight_decay=1e-4)
    for _ in range(2):
        loss, _, _ = train.make_step(opt, model.loss_terms, torch.tensor(ts), coeffs, torch.tensor(x0),
                                     torch.tensor(labels))
    ref = opt.flat.cpu()
    world = 2
    out = torch.zeros(world, ref.numel() + 1, dtype=torch.float32).share_memory_()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert torch.equal(out[0], out[1])  # replicas stay identical without a parameter broadcast
    assert torch.allclose(out[0, :-1], ref, rtol=0, atol=2e-6)  # only the reduction order differs
    assert abs(float(out[0, -1]) - float(loss)) <= 1e-5 * abs(float(loss))
