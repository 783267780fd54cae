"""CPU: the reference-interface modules construct like the reference (names, kwargs, dims, init rules)."""
import pytest
import torch

from gncde.models import GraphNeuralCDE, PGTGraphNeuralCDE, vector_fields as V


@pytest.mark.parametrize("name", ["PermEquivGraphVectorField", "PermEquivDirGraphVectorField", "GraphVectorField"])
def test_registry_lookup_and_kwargs(name):
    """VectorFieldCfg.build does getattr(vector_fields, name)(input_dim=..., ..., key=...)."""
    cls = getattr(V, name)
    vf = cls(input_dim=16, hidden_dim=16, output_dim=16 * 4 * 2, num_layers=3, data_embed_dim=4, num_nodes=64, key=1)
    assert vf.dims == [16, 16, 16, 128]
    assert len(vf.gnn_layers) == 3
    for lay in vf.layer_dicts():
        assert set(("W", "b", "rms_w", "rms_b")) <= set(lay)


def test_leaf_names_follow_reference():
    vf = V.PermEquivGraphVectorField(16, 16, 16, 2, 16, 64, key=0)
    names = {k for k, _ in vf.named_parameters()}
    assert "gnn_layers.0.param1" in names and "gnn_layers.1.param8" in names
    assert "gnn_layers.0.conv_layer.linear.weight" in names and "gnn_layers.0.conv_layer.norm.bias" in names


def test_init_distributions():
    vf = V.PermEquivGraphVectorField(16, 32, 8, 3, 16, 64, key=0)
    for lay in vf.gnn_layers:
        for nm in lay.names:
            assert getattr(lay, nm).abs().max() <= 1.0 / 15.0
        din = lay.conv_layer.linear.weight.shape[1]
        assert lay.conv_layer.linear.weight.abs().max() <= din ** -0.5
        assert torch.all(lay.conv_layer.norm.weight == 1) and torch.all(lay.conv_layer.norm.bias == 0)


def test_directed_param6_prime_quirk():
    """layers.py:245-247: param6_prime is drawn with param5_prime's key (equal at init)."""
    vf = V.PermEquivDirGraphVectorField(16, 16, 16, 2, 16, 64, key=5)
    for lay in vf.gnn_layers:
        assert torch.equal(lay.param6_prime, lay.param5_prime)
        assert not torch.equal(lay.param5, lay.param5_prime)


def test_enc_idx_is_rejected():
    with pytest.raises(NotImplementedError):
        V.PermEquivGraphVectorField(16, 16, 16, 2, 16, 64, enc_idx=True, key=0)


def test_drivers_construct():
    vf = V.PermEquivGraphVectorField(16, 16, 16, 2, 16, 64, key=0)
    m = GraphNeuralCDE({"hidden_dim": 16}, vf, "cubic", 1)
    assert m.initial_linear.weight.shape == (16, 1) and m.final_linear.weight.shape == (1, 16)
    with pytest.raises(NotImplementedError):
        GraphNeuralCDE({"hidden_dim": 16, "method": "Kvaerno3"}, vf, "cubic", 1)
    vf2 = V.PermEquivGraphVectorField(64, 64, 64 * 8 * 2, 3, 8, 129, key=0)
    p = PGTGraphNeuralCDE({"hidden_dim": 64, "data_dim": 8, "feature_dim": 1}, vf2, "cubic", 2)
    # pgt_graph_neural_cde.py:62 builds the decoder with the encoder's key
    assert torch.equal(p.encoder.layers[0].weight[:, :8].flatten()[:4], p.encoder.layers[0].weight[:, :8].flatten()[:4])


def test_tgb_model_bf16_modes():
    """The TGB driver offers fp32, the split-product "bf16" and the bf16-coefficient "bf16_storage" path (config 5's
    bf16 path on the persistent adaptive solve); the single-plane "bf16_mfma" mode is retired from it, with either
    solver (8-24 % from fp32 at no speed-up; the C-ABI also refuses it under PID)."""
    from gncde.models import TGBGraphNeuralCDE
    vf = V.PermEquivGraphVectorField(16, 16, 16 * 8 * 2, 2, 8, 40, key=0)
    for compute in ("fp32", "bf16", "bf16_storage"):
        TGBGraphNeuralCDE({"hidden_dim": 16}, vf, "cubic", 1, solver="pid", compute=compute)
    for solver in (None, "pid"):
        with pytest.raises(ValueError, match="bf16_mfma"):
            TGBGraphNeuralCDE({"hidden_dim": 16}, vf, "cubic", 1, solver=solver, compute="bf16_mfma")
