"""Host-side logic of the fused step (no GPU): parameter layout and naming."""
from mlvae_hip.engine import ParamLayout, VAEConfig, reference_shapes
from oracle import vae_cpu as O


def test_c2_parameter_count_and_names():
    cfg = VAEConfig()
    lay = ParamLayout(cfg)
    shapes = reference_shapes(cfg)
    assert list(shapes.items()) == list(O.param_shapes(80, 64, 32, 512, 2, 64).items())
    assert sum(lay.numel(k) for k in shapes) == 8_699_488
    assert lay.total % 4 == 0


def test_fused_groups_are_adjacent():
    lay = ParamLayout(VAEConfig(F=8, E=16, Z=4, H=8, L=2, C=16))
    o = lay.offsets
    for a, b in [("encoder.mean_fc.weight", "encoder.log_var_fc.weight"),
                 ("decoder.rnn.weight_ih_l1", "decoder.rnn.weight_ih_l1_reverse"),
                 ("decoder.rnn.bias_hh_l0", "decoder.rnn.bias_hh_l0_reverse"),
                 ("decoder.mean_fc.blocks.0.weight", "decoder.log_var_fc.blocks.0.weight")]:
        assert o[b] == o[a] + lay.numel(a), (a, b)
    for k, off in o.items():
        if k.endswith("weight") or k.endswith("_l0") or k.endswith("_l1"):
            continue
    starts = sorted(o.values())
    assert len(set(starts)) == len(starts)


def test_config_validation():
    import pytest
    with pytest.raises(ValueError, match="Invalid loss type"):
        VAEConfig(loss_type="l1").check()
    with pytest.raises(ValueError):
        VAEConfig(F=81).check()
