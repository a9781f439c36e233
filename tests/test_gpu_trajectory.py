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
  fp32 mode <= 1e-4 at every step, and the benchmarked bf16 mode (split-bf16 encoder / heads
  forward) <= 1e-4 at every step too -- the north star's "ELBO within 1e-4 relative".
* Free-running, fp64-anchored (round 5): the engine and the fp32 oracle each train their OWN copy
  from the same init for 100 steps, and the fp64 oracle a third on the same (exactly promoted)
  inputs and randomness.  Two fp32 implementations that round differently drift apart through the
  chaotic training dynamics, so each is measured against the fp64 truth, with a pre-registered
  bound on the engine's drift relative to the fp32 oracle's (the test's docstring).
* fp32 mode at the bench sizes, three-way: engine and fp32 oracle against fp64, every output and
  gradient tensor (test_fp32_mode_whole_step_at_bench_sizes).

The per-step curves are printed (DESIGN.md section 2 records them)."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

from gpu_utils import need_gpu, norm_rel
from philox_np import dropout_mask
from step_parity import errors, report, run_step

pytestmark = pytest.mark.gpu

F, E, Z, H, L, C = 80, 64, 32, 512, 2, 64
B, T = 8, 100
STEPS = 160
FREE_STEPS = 100
# the benchmarked bf16 step holds the north star too (round 6): its ELBO error was the bf16
# rounding of the encoder's and the heads' weights (tools/elbo_budget.py), which the split-bf16
# forward removes (VAEEngine.split_fwd); measured max 7.0e-5 over the 160 steps (was 4.5e-4)
BF16_ELBO = 1e-4


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


def _p64(params):
    return OrderedDict((k, v.double()) for k, v in params.items())


def _envelope(a):
    """Running maximum: a signed ELBO difference crosses zero now and then, so the per-step |gap|
    of two independent drifts can dip to ~0 at any step; its envelope is the stable quantity."""
    return np.maximum.accumulate(np.asarray(a))


def test_elbo_trajectory_free_running_fp32_against_fp64():
    """Free-running fp32 trajectory anchored on the fp64 oracle.  The engine
    (fp32 mode) and the fp32 oracle each train their own copy for 100 steps from the same fp32
    parameters; the fp64 oracle trains a third copy on the same (exactly promoted) inputs, eps and
    dropout masks.  Both fp32 runs drift from the fp64 truth through rounding amplified by the
    training dynamics; an engine with only fp32-rounding-level error drifts no faster than the fp32
    oracle does.  Pre-registered bound (round 5, before the first run): at every step until the
    fp32 oracle itself is 1e-4 away from fp64, the envelope of the engine's ELBO gap to fp64 stays
    within 3x the envelope of the fp32 oracle's gap (floored at the fp32 epsilon: no fp32 result
    is closer to the truth than its own storage rounding).  Parameter-space distances to fp64 are
    printed alongside."""
    need_gpu()
    from oracle import vae_cpu as O
    eng, params = _engine("fp32")
    data = _batches()
    p32, s32, p64, s64 = params, {}, _p64(params), {}
    ge, go, de, do = [], [], [], []
    for st in range(FREE_STEPS):
        x, lens = data[st % 4]
        got, eps, masks = _gpu_step(eng, x, lens)
        p32, r32 = O.train_step(p32, s32, x, lens, eps, OCFG, masks, impl="aten")
        p64, r64 = O.train_step(p64, s64, x.double(), lens, eps.double(), OCFG, masks.double(), impl="aten")
        truth = float(r64["out"]["loss"].item())
        ge.append(abs(got - truth) / abs(truth))
        go.append(abs(float(r32["out"]["loss"].item()) - truth) / abs(truth))
        if st % 10 == 9 or st < 3:
            n64 = sum(v.pow(2).sum().item() for v in p64.values()) ** 0.5
            de.append((st, sum((eng.view(k).detach().cpu().double() - v).pow(2).sum().item()
                               for k, v in p64.items()) ** 0.5 / n64,
                       sum((p32[k].double() - v).pow(2).sum().item() for k, v in p64.items()) ** 0.5 / n64))
    eng.check_errors()
    ge, go = np.array(ge), np.array(go)
    env_e, env_o = _envelope(ge), _envelope(go)
    over = np.nonzero(go > 1e-4)[0]
    stop = int(over[0]) if len(over) else FREE_STEPS
    print("\n[free-running fp32 vs fp64] step: |ELBO - fp64| engine / fp32 oracle  " +
          " ".join(f"s{i}:{ge[i]:.1e}/{go[i]:.1e}" for i in (0, 1, 2, 5, 10, 20, 30, 40, 60, 80, FREE_STEPS - 1)))
    print(f"[free-running fp32 vs fp64] window: steps 0..{stop - 1} (fp32 oracle first past 1e-4 at "
          f"{stop}); envelope ratio max {np.max(env_e[:stop] / np.maximum(env_o[:stop], FP32_EPS)):.2f}")
    print("[free-running fp32 vs fp64] |theta - theta64| / |theta64| engine / fp32 oracle  " +
          " ".join(f"s{s_}:{a:.1e}/{b:.1e}" for s_, a, b in de))
    assert stop >= 10, f"the fp32 oracle left fp64 after {stop} steps: no window to compare in"
    bound = 3.0 * np.maximum(env_o[:stop], FP32_EPS)
    bad = np.nonzero(env_e[:stop] > bound)[0]
    assert len(bad) == 0, (int(bad[0]), float(env_e[bad[0]]), float(bound[bad[0]]))


FP32_EPS = 2.0 ** -23


@pytest.mark.timeout(400)
@pytest.mark.parametrize("B_,seed", [(32, 1301), (256, 1303)])
def test_fp32_mode_whole_step_at_bench_sizes(B_, seed):
    """The fp32 parity mode at c2's B=32, T=500 and at the bench's c3_fp32 size B=256, T=500,
    three ways: the engine and the fp32 oracle each against the fp64 oracle on
    the same parameters, inputs and randomness.  Pre-registered bound (round 5): for the ELBO, the
    encoder / decoder outputs and every gradient tensor, the engine's norm-relative error to fp64
    is <= 3x the fp32 oracle's (floored at the fp32 epsilon); plus the absolute bounds of the
    earlier test (ELBO 1e-4 relative -- the north star -- and the Adam update checks).

    Round 5: the B=256 gradient excess of round 4 (1e-4 to 1e-5 in both the engine and the fp32
    oracle) was LeakyReLU-derivative flips -- a heads first-layer pre-activation within rounding of
    0 whose sign fp32 gets wrong takes the 0.01 slope instead of 1, and that one entry of dP1 moves
    every gradient behind it.  The oracle has one such flip (log_var head) at this seed; the engine
    had one in the mean head while its fp32 recurrence used the hardware tanh (1 - 2/(1+e^2x),
    relatively inaccurate near 0: rnn_out 1.2e-6 from fp64).  With libm cell math in the fp32 mode
    the engine had none (tools/parity_heads_dw1.py counts them) and every row was within 4e-7
    of fp64.  A flip is a branch decision at a non-differentiable point, not an accumulated
    rounding error, and whether one occurs at a given seed changes with any rounding change
    upstream (a GEMM's summation order brought one back): so each side's gradients are now
    compared with the fp64 step that takes the same branches at its own flipped entries
    (oracle.vae_cpu._LReLUKink; the flip counts are printed), and the bounds stand as
    registered -- engine <= 3x oracle and <= 1e-6 absolute on every row."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig
    from step_parity import kink_flips, oracle_fp64
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec="fp32")
    Tn = 500
    lens = torch.linspace(0.6, 1.0, B_)
    lens[3], lens[7] = 127 / 500, 254 / 500
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    eng, w, rec, new_ref, params = run_step(cfg, B_, Tn, seed, lens)
    e, grads = errors(eng, w, rec, new_ref, params, B_, Tn)
    report(f"fp32 mode B={B_} T=500 vs fp32 oracle", e, grads)
    _, r64 = oracle_fp64(cfg, params, rec["inputs"])
    o64 = r64["out"]
    # LeakyReLU kinks: where the engine's / the fp32 oracle's heads first-layer pre-activation
    # fell on the other side of 0 than fp64's, their gradients are compared with the fp64 step
    # taking the same branch there (kink_flips; each side against its own branch choices)
    pre64 = o64["dec"]["p1_pre"]
    sg_e = (w.P1.detach().cpu() > 0).view(B_, Tn, 2 * C)
    pre32 = rec["out"]["dec"]["p1_pre"]
    sg_o = torch.cat([pre32["decoder.mean_fc"] > 0, pre32["decoder.log_var_fc"] > 0], dim=-1)
    fl_e, fl_o = kink_flips(pre64, sg_e, C), kink_flips(pre64, sg_o, C)
    cnt = lambda f: {k.split(".")[1]: int(v.sum()) for k, v in (f or {}).items()}
    print(f"[fp32 mode B={B_}] LeakyReLU-kink flips vs fp64: engine {cnt(fl_e)} fp32 oracle {cnt(fl_o)}")
    g_e = r64["grads"] if fl_e is None else oracle_fp64(cfg, params, rec["inputs"], fl_e)[1]["grads"]
    g_o = r64["grads"] if fl_o is None else oracle_fp64(cfg, params, rec["inputs"], fl_o)[1]["grads"]
    rel = lambda a, b: abs(float(a) - float(b)) / abs(float(b))
    outs = {"loss": (w.loss[2].item(), rec["out"]["loss"].item(), o64["loss"].item()),
            "kld_loss": (w.loss[0].item(), rec["out"]["kld_loss"].item(), o64["kld_loss"].item()),
            "recon_loss": (w.loss[1].item(), rec["out"]["recon_loss"].item(), o64["recon_loss"].item())}
    rows = [(k, rel(a, t), rel(b, t)) for k, (a, b, t) in outs.items()]
    tens = {"mu": (w.ML[:, :Z].reshape(B_, Tn, Z), rec["out"]["enc"]["mean"], o64["enc"]["mean"]),
            "log_var": (w.ML[:, Z:].reshape(B_, Tn, Z), rec["out"]["enc"]["log_var"], o64["enc"]["log_var"]),
            "mu_x": (w.MUX.reshape(B_, Tn, -1), rec["out"]["dec"]["mean"], o64["dec"]["mean"]),
            "log_var_x": (w.LVX.reshape(B_, Tn, -1), rec["out"]["dec"]["log_var"], o64["dec"]["log_var"])}
    rows += [(k, norm_rel(a, t), norm_rel(b, t)) for k, (a, b, t) in tens.items()]
    rows += [(k, norm_rel(g, g_e[k]), norm_rel(rec["grads"][k], g_o[k]))
             for k, g in eng.named_grads().items()]
    print(f"[fp32 mode B={B_} T=500, error vs fp64] name: engine / fp32 oracle (ratio)")
    for k, a, b in rows:
        print(f"  {k:42s} {a:.2e} / {b:.2e} ({a / max(b, FP32_EPS):.2f})")
    worst = max(rows, key=lambda r: r[1] / max(r[2], FP32_EPS))
    print(f"[fp32 mode B={B_}] worst engine/oracle ratio {worst[1] / max(worst[2], FP32_EPS):.2f} ({worst[0]})")
    for k, a, b in rows:
        assert a <= 3.0 * max(b, FP32_EPS), (k, a, b)
        assert a <= 1e-6, (k, a, b)
    assert e["loss"] <= 1e-4 and e["recon_loss"] <= 1e-4 and e["kld_loss"] <= 1e-4, e
    assert e["update_sign"] >= 0.999 and e["update_err"] <= 1e-2, e
