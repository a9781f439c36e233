"""Whole-step parity of the fused engine against the CPU oracle (oracle/vae_cpu.py), shared by
the -m gpu parity tests.

One ``VAEEngine.train_step`` runs on the GPU with its own in-kernel randomness (Philox eps in the
encoder, Philox dropout masks in the recurrence / dgrad epilogue); the eps it drew is read back
and the masks are replayed on the host (tests/philox_np.py), so the oracle sees the SAME
randomness through the SAME fused path that bench.py times.

Post-Adam check.  Adam's first step moves every weight by about lr in the direction of -sign(g),
so a max-|delta| bound cannot tell a right update from a wrong one.  Two checks that can:
  * sign agreement of the update (new - old) with the oracle's update, over the weights whose
    oracle gradient is not negligible (|g| > FLOOR x the rms of its tensor's gradient);
  * the norm-relative error of the update vector over those weights.
A step that moved every parameter the wrong way scores 0 % agreement and error 2.
"""
from collections import OrderedDict

import numpy as np
import torch

from gpu_utils import norm_rel
from oracle import vae_cpu as O
from philox_np import dropout_mask

FLOOR = 0.1   # |g| > FLOOR * rms(g of the tensor): the weights whose update direction is defined


def run_step(cfg, B, T, seed, lens, x=None):
    """One fused train step on the GPU and the oracle's step on the same inputs/randomness.
    Returns (engine, work, oracle record, oracle post-Adam params, initial params)."""
    from mlvae_hip.engine import VAEEngine
    g = torch.Generator().manual_seed(seed)
    params = O.init_params(cfg.F, cfg.E, cfg.Z, cfg.H, cfg.L, cfg.C, seed=seed, enc_conv=cfg.enc_conv)
    if x is None:
        x = torch.randn(B, T, cfg.F, generator=g)
    eng = VAEEngine(cfg, params=params, seed=seed)
    eng.train_step(x.cuda(), lens.cuda())
    torch.cuda.synchronize()
    eng.check_errors()
    w = eng.work(B, T)
    eps = w.eps_used.detach().cpu().view(B, T, cfg.Z)
    masks = None
    if cfg.dropout > 0 and cfg.L > 1:
        ms = []
        for li in range(cfg.L - 1):
            s = (eng.seed * 1000003 + 0 * 131 + li) & ((1 << 63) - 1)   # engine._drop_seed, rng_step 0
            ms.append(torch.from_numpy(dropout_mask(s, B * T * 2 * cfg.H, cfg.dropout)).view(B, T, 2 * cfg.H))
        masks = torch.stack(ms)
    new_ref, rec = O.train_step(params, {}, x, lens, eps,
                                dict(L=cfg.L, loss_type=cfg.loss_type, kld_weight=cfg.kld_weight),
                                masks, impl="aten")
    rec["inputs"] = (x, lens, eps, masks)
    return eng, w, rec, new_ref, params


def oracle_fp64(cfg, params, inputs, head_kink=None):
    """The oracle's step in fp64 on the SAME fp32-representable parameters, inputs and randomness
    (promoted exactly): the truth both the engine and the fp32 oracle are measured against.  lens
    stays fp32 -- length_to_mask's fp32 rel*T quirk is the reference's semantics, not rounding.
    head_kink: {head prefix: bool [B, T, C]} -- the heads' first-layer LeakyReLU derivative
    branch flipped there (kink_flips)."""
    x, lens, eps, masks = inputs
    p64 = OrderedDict((k, v.double()) for k, v in params.items())
    return O.train_step(p64, {}, x.double(), lens, eps.double(),
                        dict(L=cfg.L, loss_type=cfg.loss_type, kld_weight=cfg.kld_weight,
                             head_kink=head_kink),
                        None if masks is None else masks.double(), impl="aten")


HEADS = (("decoder.mean_fc", 0), ("decoder.log_var_fc", 1))


KINK_TOL = 1e-5      # a flipped entry's |pre64| / max |pre64| of its (frame, head) row
KINK_MAX = 4         # flipped entries per head per step


def kink_flips(pre64, p1_signs, C, tol=KINK_TOL, cap=KINK_MAX):
    """Where an fp32 computation of the heads' first layer landed on the other side of the
    LeakyReLU kink than fp64: {prefix: bool [B, T, C]} (None: no flip).  pre64: the fp64
    oracle's pre-activations (rec["out"]["dec"]["p1_pre"]); p1_signs: bool [B, T, 2C], the fp32
    side's pre-activation > 0 (the engine's saved post-activation P1 has the same sign).

    A flip is only absorbed into the truth (the fp64 step taking the same branch there) when it is
    a rounding-level decision: every flipped entry must lie
    within tol x the largest |pre64| of its (frame, head) row of 0, and there may be at most cap
    of them per head.  A systematic sign error in P1 -- many entries, or entries far from 0 --
    fails here instead of being rebuilt into the reference gradients."""
    out = {}
    for name, h in HEADS:
        p = pre64[name]
        f = p1_signs[..., h * C:(h + 1) * C] != (p > 0)
        n = int(f.sum())
        if n == 0:
            continue
        rowmax = p.abs().amax(dim=-1, keepdim=True).expand_as(p)
        ratio = (p.abs()[f] / rowmax[f]).max().item()
        assert n <= cap, f"{name}: {n} LeakyReLU sign flips against fp64 (at most {cap})"
        assert ratio <= tol, f"{name}: a sign flip at |pre64| = {ratio:.2e} x its row's max (>{tol:g})"
        out[name] = f
    return out or None


def run_second_step(cfg, B, T, seed, lens):
    """Two fused steps on the GPU; the oracle replays the SECOND from the engine's state after
    the first (parameters, Adam moments and step count), with step 2's eps and dropout masks.
    For paths whose first step differs (the fp8 mode's delayed scaling needs a previous amax).
    Returns (engine, work, record, oracle post-Adam params, params before step 2)."""
    from mlvae_hip.engine import VAEEngine
    g = torch.Generator().manual_seed(seed)
    params = O.init_params(cfg.F, cfg.E, cfg.Z, cfg.H, cfg.L, cfg.C, seed=seed, enc_conv=cfg.enc_conv)
    x1 = torch.randn(B, T, cfg.F, generator=g)
    x2 = torch.randn(B, T, cfg.F, generator=g)
    eng = VAEEngine(cfg, params=params, seed=seed)
    eng.train_step(x1.cuda(), lens.cuda())
    torch.cuda.synchronize()
    before = {k: v.detach().cpu().clone() for k, v in eng.named_parameters().items()}
    state = {"step": int(eng.step_ctr.item()),
             "m": {k: eng.view(k, eng.exp_avg).detach().cpu().clone() for k in before},
             "v": {k: eng.view(k, eng.exp_avg_sq).detach().cpu().clone() for k in before}}
    eng.train_step(x2.cuda(), lens.cuda())
    torch.cuda.synchronize()
    eng.check_errors()
    w = eng.work(B, T)
    eps = w.eps_used.detach().cpu().view(B, T, cfg.Z)
    masks = None
    if cfg.dropout > 0 and cfg.L > 1:
        ms = [torch.from_numpy(dropout_mask((eng.seed * 1000003 + 1 * 131 + li) & ((1 << 63) - 1),
                                            B * T * 2 * cfg.H, cfg.dropout)).view(B, T, 2 * cfg.H)
              for li in range(cfg.L - 1)]
        masks = torch.stack(ms)
    new_ref, rec = O.train_step(before, state, x2, lens, eps,
                                dict(L=cfg.L, loss_type=cfg.loss_type, kld_weight=cfg.kld_weight),
                                masks, impl="aten")
    return eng, w, rec, new_ref, before


def update_errors(eng, rec, new_ref, params):
    """(sign agreement over the defined-direction weights, norm-relative update error over them,
    max |param - oracle|)."""
    agree = tot = 0
    num = den = 0.0
    dmax = 0.0
    for k, old in params.items():
        gr = rec["grads"][k].double()
        rms = gr.pow(2).mean().sqrt().item()
        new = eng.view(k).detach().cpu().double()
        ref = new_ref[k].double()
        dmax = max(dmax, (new - ref).abs().max().item())
        if rms == 0.0:
            continue
        m = gr.abs() > FLOOR * rms
        dg = (new - old.double())[m]
        dr = (ref - old.double())[m]
        agree += int((torch.sign(dg) == torch.sign(dr)).sum().item())
        tot += int(m.sum().item())
        num += (dg - dr).pow(2).sum().item()
        den += dr.pow(2).sum().item()
    return agree / max(tot, 1), (num / max(den, 1e-300)) ** 0.5, dmax


def errors(eng, w, rec, new_ref, params, B, T):
    """Relative errors of the step's outputs, gradients and update against the oracle."""
    Z = eng.cfg.Z
    out = rec["out"]
    rel = lambda a, b: abs(a - b) / abs(b)
    e = {"loss": rel(w.loss[2].item(), out["loss"].item()),
         "kld_loss": rel(w.loss[0].item(), out["kld_loss"].item()),
         "recon_loss": rel(w.loss[1].item(), out["recon_loss"].item()),
         "mu": norm_rel(w.ML[:, :Z].reshape(B, T, Z), out["enc"]["mean"]),
         "log_var": norm_rel(w.ML[:, Z:].reshape(B, T, Z), out["enc"]["log_var"]),
         "mu_x": norm_rel(w.MUX.reshape(B, T, -1), out["dec"]["mean"]),
         "log_var_x": norm_rel(w.LVX.reshape(B, T, -1), out["dec"]["log_var"])}
    grads = {k: norm_rel(g, rec["grads"][k]) for k, g in eng.named_grads().items()}
    e["update_sign"], e["update_err"], e["param_maxabs"] = update_errors(eng, rec, new_ref, params)
    return e, grads


def report(tag, e, grads):
    worst = max(grads, key=grads.get)
    print(f"\n[{tag}] " + " ".join(f"{k} {v:.2e}" for k, v in e.items()) +
          f" | grads max {grads[worst]:.2e} ({worst}) median {float(np.median(list(grads.values()))):.2e}")
