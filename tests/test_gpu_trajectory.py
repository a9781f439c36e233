"""ELBO parity along a training trajectory, and fp32-mode whole-step parity at the benchmarked sizes.

VERDICT r03: at PyTorch-default init the loss is the model-free value 0.5 (log 2 pi + E[x^2])
whatever the decoder computes, so a one-step ELBO check cannot see a decoder error.  Here the
fused engine and the CPU oracle (oracle/vae_cpu.py) each train their OWN copy of the c2 model
(F=80, enc [80,64,64], z=32, BiLSTM 2x512, dec-FC [1024,64,64,80], dropout 0.15) for 160
fit_batch steps (ref:src/models/md_model.py:77-88: forward, backward, check_gradients clip 5.0,
Adam 1e-3) over four fixed batches of low-rank, temporally smooth frames that the model can
learn: the loss leaves the 1.419 init floor and falls below 1.10.  Every step's randomness is
the engine's own (in-kernel Philox eps read back, dropout masks replayed on the host), the
oracle threads its own Adam state, and the ELBO of EVERY step is compared:

  * fp32 mode (the north-star "ELBO within 1e-4 relative" mode): <= 1e-4 at every step;
  * bf16 mode (bf16 MFMA operands, fp16 gate buffer): <= BF16_TRAJ at every step (measured,
    DESIGN.md section 2).

The per-step curves are printed (DESIGN.md section 2 records them)."""
import numpy as np
import pytest
import torch

from gpu_utils import need_gpu
from philox_np import dropout_mask
from step_parity import errors, report, run_step

pytestmark = pytest.mark.gpu

F, E, Z, H, L, C = 80, 64, 32, 512, 2, 64
B, T = 8, 100
STEPS = 160
BF16_TRAJ = 1e-2


def _batches(seed=5):
    """Four fixed batches of learnable frames: x = s A + 0.1 n with an 8-d latent s that drifts
    in time (a normalised random walk), A fixed [8, 80]; lens ragged in two of them."""
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(8, F, generator=g) / 8 ** 0.5
    out = []
    for i in range(4):
        s = torch.cumsum(torch.randn(B, T, 8, generator=g), 1) / torch.arange(1, T + 1).sqrt().view(1, T, 1)
        x = s @ A + 0.1 * torch.randn(B, T, F, generator=g)
        lens = torch.ones(B) if i % 2 == 0 else torch.linspace(0.7, 1.0, B)
        out.append((x, lens))
    return out


def _trajectory(prec):
    from mlvae_hip.engine import VAEConfig, VAEEngine
    from oracle import vae_cpu as O
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec=prec)
    params = O.init_params(F, E, Z, H, L, C, seed=7)
    eng = VAEEngine(cfg, params=params, seed=31)
    ocfg = dict(L=L, loss_type="likelihood", kld_weight=1e-3)
    ref, state = params, {}
    data = _batches()
    gpu_l, ref_l, rel = [], [], []
    for st in range(STEPS):
        x, lens = data[st % 4]
        k = eng.rng_step
        loss = eng.train_step(x.cuda(), lens.cuda())
        torch.cuda.synchronize()
        w = eng.work(B, T)
        eps = w.eps_used.detach().cpu().view(B, T, Z)
        masks = torch.stack([torch.from_numpy(dropout_mask((eng.seed * 1000003 + k * 131 + li) & ((1 << 63) - 1),
                                                           B * T * 2 * H, 0.15)).view(B, T, 2 * H)
                             for li in range(L - 1)])
        ref, rec = O.train_step(ref, state, x, lens, eps, ocfg, masks, impl="aten")
        a, b = float(loss[2].item()), float(rec["out"]["loss"].item())
        gpu_l.append(a)
        ref_l.append(b)
        rel.append(abs(a - b) / abs(b))
    eng.check_errors()
    drift = max((eng.view(kk).cpu() - v).abs().max().item() for kk, v in ref.items())
    return np.array(gpu_l), np.array(ref_l), np.array(rel), drift


@pytest.mark.parametrize("prec,bound", [("fp32", 1e-4), ("bf16", BF16_TRAJ)])
def test_elbo_trajectory_160_steps_matches_oracle(prec, bound):
    need_gpu()
    gpu_l, ref_l, rel, drift = _trajectory(prec)
    marks = [0, 1, 10, 40, 80, 120, STEPS - 1]
    print(f"\n[trajectory {prec}] " + " ".join(f"s{i}:{gpu_l[i]:.5f}/{ref_l[i]:.5f}({rel[i]:.1e})" for i in marks)
          + f" | max rel {rel.max():.2e} at step {int(rel.argmax())}, median {np.median(rel):.2e}, "
          f"min loss {ref_l.min():.4f}, final max |param - oracle| {drift:.2e}")
    assert ref_l[0] > 1.3 and ref_l[-20:].mean() < 1.10, "the model must leave the init floor"
    assert np.all(np.isfinite(gpu_l))
    assert rel.max() <= bound, (rel.max(), int(rel.argmax()))


@pytest.mark.parametrize("B_,seed", [(32, 1301), (256, 1303)])
def test_fp32_mode_whole_step_at_bench_sizes(B_, seed):
    """The fp32 parity mode at c2's B=32, T=500 and at the bench's c3_fp32 size B=256, T=500:
    the ELBO within 1e-4 relative (north star), outputs and gradients at fp32 accuracy, the Adam
    update checks of step_parity.py."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec="fp32")
    Tn = 500
    lens = torch.linspace(0.6, 1.0, B_)
    lens[3], lens[7] = 127 / 500, 254 / 500
    eng, w, rec, new_ref, params = run_step(cfg, B_, Tn, seed, lens)
    e, grads = errors(eng, w, rec, new_ref, params, B_, Tn)
    report(f"fp32 mode B={B_} T=500", e, grads)
    assert e["loss"] <= 1e-4 and e["recon_loss"] <= 1e-4 and e["kld_loss"] <= 1e-4, e
    for k in ("mu", "log_var", "mu_x", "log_var_x"):
        assert e[k] <= 1e-4, (k, e[k])
    for k, v in grads.items():
        assert v <= 1e-3, (k, v)
    assert e["update_sign"] >= 0.999 and e["update_err"] <= 1e-2, e
