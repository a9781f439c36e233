"""ELBO parity along a training trajectory, and fp32-mode whole-step parity at the benchmarked sizes.

VERDICT r03: at PyTorch-default init the loss is the model-free value 0.5 (log 2 pi + E[x^2])
whatever the decoder computes, so a one-step ELBO check cannot see a decoder error.  Here the fused
engine trains the c2 model (F=80, enc [80,64,64], z=32, BiLSTM 2x512, dec-FC [1024,64,64,80],
dropout 0.15) for 160 fit_batch steps (ref:src/models/md_model.py:77-88: forward, backward,
check_gradients clip 5.0, Adam 1e-3) over four fixed batches of low-rank, temporally smooth frames
the model can learn: the loss leaves the 1.419 init floor and falls below 1.10.  Every step's
randomness is the engine's own (in-kernel eps read back, dropout masks replayed on the host).

* Teacher-forced: before EVERY step the oracle (oracle/vae_cpu.py) is handed the engine's state
  (parameters, Adam moments, step count) and takes the same step.  The ELBO of every step -- on a
  model that has learned, so the decoder's outputs decide it -- and the Adam update are compared:
  fp32 mode (the north-star "ELBO within 1e-4 relative" mode) <= 1e-4 at every step; bf16 mode
  <= BF16_ELBO (measured).
* Free-running: the oracle trains its OWN copy from the same init for 100 steps, threading its own
  Adam state.  Two fp32 implementations that round differently drift apart through the chaotic
  training dynamics (Adam moves weights with tiny gradients by ~lr whichever way their sign falls),
  so the oracle is run a second time on the batch in reverse utterance order (the same
  mathematics, rounded differently at every step): the engine-vs-oracle ELBO gap must stay within
  1e-4 while the dynamics are still smooth (the first 20 steps) and, later, within a small factor
  of the gap between the oracle and itself -- a kernel error would show up as a gap far above
  that intrinsic sensitivity.

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
FREE_STEPS = 100
BF16_ELBO = 2e-3


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


def _engine(prec):
    from mlvae_hip.engine import VAEConfig, VAEEngine
    from oracle import vae_cpu as O
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec=prec)
    params = O.init_params(F, E, Z, H, L, C, seed=7)
    return VAEEngine(cfg, params=params, seed=31), params


def _gpu_step(eng, x, lens):
    """One engine step; returns (its ELBO, the eps it drew, the dropout masks it drew)."""
    k = eng.rng_step
    loss = eng.train_step(x.cuda(), lens.cuda())
    torch.cuda.synchronize()
    w = eng.work(B, T)
    eps = w.eps_used.detach().cpu().view(B, T, Z)
    masks = torch.stack([torch.from_numpy(dropout_mask((eng.seed * 1000003 + k * 131 + li) & ((1 << 63) - 1),
                                                       B * T * 2 * H, 0.15)).view(B, T, 2 * H)
                         for li in range(L - 1)])
    return float(loss[2].item()), eps, masks


OCFG = dict(L=L, loss_type="likelihood", kld_weight=1e-3)


@pytest.mark.parametrize("prec,bound", [("fp32", 1e-4), ("bf16", BF16_ELBO)])
def test_elbo_trajectory_teacher_forced_160_steps(prec, bound):
    need_gpu()
    from oracle import vae_cpu as O
    from step_parity import update_errors
    eng, _ = _engine(prec)
    data = _batches()
    rel, ref_l, gpu_l, signs, uerrs = [], [], [], [], []
    for st in range(STEPS):
        x, lens = data[st % 4]
        before = {k: v.detach().cpu().clone() for k, v in eng.named_parameters().items()}
        state = {"step": int(eng.step_ctr.item()),
                 "m": {k: eng.view(k, eng.exp_avg).detach().cpu().clone() for k in before},
                 "v": {k: eng.view(k, eng.exp_avg_sq).detach().cpu().clone() for k in before}}
        got, eps, masks = _gpu_step(eng, x, lens)
        new_ref, rec = O.train_step(before, state, x, lens, eps, OCFG, masks, impl="aten")
        want = float(rec["out"]["loss"].item())
        gpu_l.append(got)
        ref_l.append(want)
        rel.append(abs(got - want) / abs(want))
        if st % 20 == 0 or st == STEPS - 1:
            sg, ue, _ = update_errors(eng, rec, new_ref, before)
            signs.append(sg)
            uerrs.append(ue)
    eng.check_errors()
    rel, ref_l = np.array(rel), np.array(ref_l)
    marks = [0, 1, 10, 40, 80, 120, STEPS - 1]
    print(f"\n[teacher-forced {prec}] " + " ".join(f"s{i}:{gpu_l[i]:.5f}/{ref_l[i]:.5f}({rel[i]:.1e})" for i in marks)
          + f" | max rel {rel.max():.2e} at step {int(rel.argmax())}, median {np.median(rel):.2e}, "
          f"final-20 mean loss {ref_l[-20:].mean():.4f}; update sign min {min(signs) * 100:.2f} %, "
          f"update err max {max(uerrs):.2e}")
    assert ref_l[0] > 1.3 and ref_l[-20:].mean() < 1.10, "the model must leave the init floor"
    assert rel.max() <= bound, (rel.max(), int(rel.argmax()))
    if prec == "fp32":
        assert min(signs) >= 0.999 and max(uerrs) <= 1e-2, (signs, uerrs)
    else:
        assert min(signs) >= 0.995 and max(uerrs) <= 0.15, (signs, uerrs)


def test_elbo_trajectory_free_running_fp32_against_a_reordered_oracle():
    need_gpu()
    from oracle import vae_cpu as O
    eng, params = _engine("fp32")
    # the control: the oracle itself on the batch in reverse utterance order -- the same
    # mathematics (the utterances are independent, every sum over them is order-free in exact
    # arithmetic) summed in another order, so it rounds differently at every step, as a second
    # fp32 implementation does
    data = _batches()
    ref, st_ref, ctl, st_ctl = params, {}, params, {}
    g_l, r_l, c_l = [], [], []
    rv = torch.arange(B - 1, -1, -1)
    for st in range(FREE_STEPS):
        x, lens = data[st % 4]
        got, eps, masks = _gpu_step(eng, x, lens)
        ref, rec = O.train_step(ref, st_ref, x, lens, eps, OCFG, masks, impl="aten")
        ctl, recc = O.train_step(ctl, st_ctl, x[rv], lens[rv], eps[rv], OCFG, masks[:, rv], impl="aten")
        g_l.append(got)
        r_l.append(float(rec["out"]["loss"].item()))
        c_l.append(float(recc["out"]["loss"].item()))
    eng.check_errors()
    g_l, r_l, c_l = map(np.array, (g_l, r_l, c_l))
    gap = np.abs(g_l - r_l) / np.abs(r_l)
    ctl_gap = np.abs(c_l - r_l) / np.abs(r_l)
    print("\n[free-running fp32] step: engine-vs-oracle / reordered-oracle-vs-oracle gap  " +
          " ".join(f"s{i}:{gap[i]:.1e}/{ctl_gap[i]:.1e}" for i in (0, 10, 20, 30, 40, 60, 80, FREE_STEPS - 1)))
    assert gap[:20].max() <= 1e-4, gap[:20].max()
    # later steps: the engine stays about as close to the oracle as the oracle is to itself
    # summing in another order (a kernel error would open a gap far beyond that)
    late = slice(40, FREE_STEPS)
    assert np.median(gap[late]) <= 30 * max(np.median(ctl_gap[late]), 1e-6), \
        (np.median(gap[late]), np.median(ctl_gap[late]))


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
