"""The Conv1d encoder variant (BASELINE.json configs[3]) on CPU: the oracle's two restatements
agree (torch conv1d in encoder_forward, the explicit shifted-sum conv1d_numpy), the parameter
layout of the fused engine matches the module (modules/conv_vae.py) and the oracle.  The
reference has no Conv1d: this variant's parity is "unpinned" -- the
oracle is torch.nn.Conv1d semantics, checked here against an independent restatement."""
import numpy as np
import torch
import torch.nn.functional as Fn

from mlvae_hip.engine import ParamLayout, VAEConfig, reference_shapes
from oracle import vae_cpu as O


def test_numpy_conv_matches_torch_conv1d():
    g = torch.Generator().manual_seed(0)
    for (B, T, Cin, Cout, K) in [(2, 37, 12, 8, 5), (1, 3, 4, 16, 7), (3, 64, 20, 4, 1), (2, 9, 6, 6, 9)]:
        x = torch.randn(B, T, Cin, generator=g, dtype=torch.float64)
        w = torch.randn(Cout, Cin, K, generator=g, dtype=torch.float64)
        b = torch.randn(Cout, generator=g, dtype=torch.float64)
        ref = Fn.conv1d(x.transpose(1, 2), w, b, padding=K // 2).transpose(1, 2)
        got = O.conv1d_numpy(x.numpy(), w.numpy(), b.numpy())
        assert np.abs(got - ref.numpy()).max() < 1e-12 * max(1.0, np.abs(ref.numpy()).max())


def test_encoder_forward_conv_variant():
    p = O.init_params(12, 16, 4, 8, 2, 16, seed=5, dtype=torch.float64, enc_conv=5)
    assert p["encoder.conv.0.blocks.0.weight"].shape == (16, 12, 5)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 30, 12, generator=g, dtype=torch.float64)
    eps = torch.randn(2, 30, 4, generator=g, dtype=torch.float64)
    out = O.encoder_forward(p, x, eps)
    lr = lambda v: np.where(v > 0, v, 0.01 * v)
    h = lr(O.conv1d_numpy(x.numpy(), p["encoder.conv.0.blocks.0.weight"].numpy(),
                          p["encoder.conv.0.blocks.0.bias"].numpy()))
    h = lr(O.conv1d_numpy(h, p["encoder.conv.0.blocks.2.weight"].numpy(),
                          p["encoder.conv.0.blocks.2.bias"].numpy()))
    mean = h @ p["encoder.mean_fc.weight"].numpy().T + p["encoder.mean_fc.bias"].numpy()
    assert np.abs(out["mean"].numpy() - mean).max() < 1e-10


def test_conv_layout_matches_module_and_oracle():
    from modules.conv_vae import ConvVAE
    cfg = VAEConfig(F=80, E=64, Z=32, H=64, L=2, C=64, enc_conv=5, prec="bf16").check()
    shapes = reference_shapes(cfg)
    assert list(shapes.items()) == list(O.param_shapes(80, 64, 32, 64, 2, 64, enc_conv=5).items())
    enc = ConvVAE([80, 64, 64], 32, kernel_size=5)
    mod = {f"encoder.{k}": tuple(v.shape) for k, v in enc.named_parameters()}
    assert mod == {k: v for k, v in shapes.items() if k.startswith("encoder.")}
    lay = ParamLayout(cfg)
    assert lay.numel("encoder.conv.0.blocks.0.weight") == 64 * 80 * 5


def test_conv_config_validation():
    import pytest
    with pytest.raises(ValueError, match="odd"):
        VAEConfig(enc_conv=4, prec="bf16").check()
    with pytest.raises(ValueError, match="bf16"):
        VAEConfig(enc_conv=5, prec="fp32").check()
