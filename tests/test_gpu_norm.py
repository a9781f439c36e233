"""InputNormalization(norm_type='global') inside the fused step (csrc/norm.hip) against the
restatement brain/features.py (SpeechBrain 0.5 semantics; parity unpinned: SpeechBrain is not in
the reference tree): several training batches with ragged lengths (incl. the 127/500 quirk) and
a zero-length filler, epochs below and at update_until_epoch (running update, then frozen), an
eval batch, and the normalised batch feeding the step exactly as the module's output would."""
import pytest
import torch

from gpu_utils import need_gpu

pytestmark = pytest.mark.gpu


def _batches(B, T, F, n, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n):
        x = torch.randn(B, T, F, generator=g) * (1 + i) + 0.5 * i
        lens = torch.linspace(0.4, 1.0, B)
        lens[1] = 127 / T
        if i == 2:
            lens[0] = 0.0          # a zero-length filler (data-parallel evaluation remainder)
        out.append((x, lens))
    return out


def test_device_normaliser_matches_module_over_epochs():
    need_gpu()
    from brain.features import InputNormalization
    from mlvae_hip.engine import VAEConfig, VAEEngine
    B, T, F = 6, 500, 80
    eng = VAEEngine(VAEConfig(F=F, E=64, Z=32, H=64, L=1, C=64, dropout=0.0, prec="fp32"))
    dev, ref = InputNormalization(update_until_epoch=3), InputNormalization(update_until_epoch=3)
    for i, (x, lens) in enumerate(_batches(B, T, F, 6, 11)):
        epoch = [1, 1, 2, 3, 3, 4][i]             # running update below update_until_epoch, then frozen
        if i == 5:
            dev.eval(), ref.eval()
        got = eng.normalise(x.cuda(), lens.cuda(), dev, epoch=epoch)
        want = ref(x, lens, epoch=epoch)
        torch.cuda.synchronize()
        assert dev.count == ref.count
        assert torch.allclose(dev.glob_mean.cpu(), ref.glob_mean, rtol=1e-5, atol=1e-6), i
        assert torch.allclose(dev.glob_std.cpu(), ref.glob_std, rtol=1e-5, atol=1e-6), i
        assert torch.allclose(got.cpu(), want, rtol=1e-5, atol=1e-5), i


def test_fused_step_with_normaliser_equals_normalised_input():
    """train_step(x, normalizer=norm) = train_step(norm(x)) on the same engine state."""
    need_gpu()
    from brain.features import InputNormalization
    from mlvae_hip.engine import VAEConfig, VAEEngine
    from oracle import vae_cpu as O
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16")
    B, T = 32, 200
    params = O.init_params(cfg.F, cfg.E, cfg.Z, cfg.H, cfg.L, cfg.C, seed=5)
    (x, lens), = _batches(B, T, cfg.F, 1, 12)
    n1, n2 = InputNormalization(), InputNormalization()
    e1 = VAEEngine(cfg, params=params, seed=9)
    e2 = VAEEngine(cfg, params=params, seed=9)
    l1 = e1.train_step(x.cuda(), lens.cuda(), normalizer=n1, epoch=0)
    xn = n2(x.cuda(), lens.cuda(), epoch=0)
    l2 = e2.train_step(xn, lens.cuda())
    torch.cuda.synchronize()
    # the step consumed the kernels' normalised batch (equal to the module's to fp32 rounding of
    # the statistics' summation order) and the module state moved the same way
    used = e1.work(B, T).x
    assert torch.allclose(used, xn, rtol=1e-5, atol=1e-5)
    assert n1.count == n2.count == 1
    assert torch.allclose(n1.glob_mean, n2.glob_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(l1.cpu(), l2.cpu(), rtol=1e-5, atol=1e-7)
