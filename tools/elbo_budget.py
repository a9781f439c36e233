"""Where the bf16 step's ELBO error comes from: an fp64 emulation of the
fused bf16 forward with each rounding point of the engine switchable, on a model trained along the
trajectory test's data (tests/test_gpu_trajectory.py: c2 model, B=8, T=100, four learnable
batches).  The ELBO in a teacher-forced step is a pure forward quantity, so its error is the sum of
the forward's rounding effects; this attributes it to the operand that carries it.

Rounding points, as the kernels apply them (csrc/encoder.hip, lstm_wide.hip, gemm_fast.hip,
heads.hip):
  enc     x, the encoder weights and E1 / E2 as bf16 MFMA operands
  z       the latent z stored bf16 for the fused layer-0 projection
  wih0    W_ih_l0 as a bf16 operand
  rec0    layer 0: h and W_hh as bf16 operands of h W_hh^T
  proj1   dropout(h) and W_ih_l1 as bf16 operands of the layer-1 projection
  g16     the layer-1 projection stored in the fp16 gate buffer
  rec1    layer 1: h and W_hh as bf16 operands
  heads1  rnn_out and W1 bf16 operands, P1 stored bf16
  heads23 W2, W3 bf16 operands, P2 bf16

    python tools/elbo_budget.py [--steps 100]
"""
import argparse
import os
import sys
from collections import OrderedDict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import vae_cpu as O  # noqa: E402

F, E, Z, H, L, C = 80, 64, 32, 512, 2, 64
B, T = 8, 100
GROUPS = ["enc", "z", "wih0", "rec0", "proj1", "g16", "rec1", "heads1", "heads23"]


def batches(seed=5):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(8, F, generator=g) / 8 ** 0.5
    out = []
    for i in range(4):
        s = torch.cumsum(torch.randn(B, T, 8, generator=g), 1) / torch.arange(1, T + 1).sqrt().view(1, T, 1)
        x = s @ A + 0.1 * torch.randn(B, T, F, generator=g)
        lens = torch.ones(B) if i % 2 == 0 else torch.linspace(0.7, 1.0, B)
        out.append((x, lens))
    return out


def emulate(p, x, lens, eps, mask, on, split=(), wsplit=()):
    """ELBO of the bf16 forward in fp64 with the rounding points in `on` applied.  `split`: the
    groups whose bf16 operands are instead hi + lo pairs (three products: hi hi + hi lo + lo hi);
    `wsplit`: the groups whose WEIGHT operand alone is a hi + lo pair (two products a_bf16 (W_hi +
    W_lo): the activation stays a bf16 operand)."""
    d = lambda t: t.double()
    bf = lambda t: t.to(torch.bfloat16).double()
    f16 = lambda t: t.to(torch.float16).double()

    def r(t, g):            # an operand rounded at group g's point
        if g not in on:
            return d(t)
        if g in split:      # bf16x3: hi + lo with the lo*lo product dropped
            hi = bf(t)
            return hi + bf(t.double() - hi)
        return bf(t)

    def mm(a, w, g):        # a w^T with both operands rounded at g (split: drop lo*lo)
        if g in on and g in wsplit:
            wh = bf(w)
            return bf(a) @ (wh + bf(d(w) - wh)).t()
        if g in on and g in split:
            ah, wh = bf(a), bf(w)
            al, wl = bf(d(a) - ah), bf(d(w) - wh)
            return ah @ wh.t() + ah @ wl.t() + al @ wh.t()
        return r(a, g) @ r(w, g).t()

    P = {k: d(v) for k, v in p.items()}
    lr = lambda t: torch.where(t > 0, t, 0.01 * t)
    e1 = lr(mm(x, P["encoder.fc.0.blocks.0.weight"], "enc") + P["encoder.fc.0.blocks.0.bias"])
    e2 = lr(mm(e1, P["encoder.fc.0.blocks.2.weight"], "enc") + P["encoder.fc.0.blocks.2.bias"])
    mu = mm(e2, P["encoder.mean_fc.weight"], "enc") + P["encoder.mean_fc.bias"]
    lv = mm(e2, P["encoder.log_var_fc.weight"], "enc") + P["encoder.log_var_fc.bias"]
    z = d(eps) * torch.exp(0.5 * lv) + mu
    kld = -0.5 * (1 + lv - mu ** 2 - lv.exp())
    inp = r(z, "z") if "z" in on else z
    for li in range(L):
        outs = []
        for sfx, rev in (("", False), ("_reverse", True)):
            pre = f"decoder.rnn.weight_ih_l{li}{sfx}"
            wih, whh = P[pre], P[f"decoder.rnn.weight_hh_l{li}{sfx}"]
            bias = P[f"decoder.rnn.bias_ih_l{li}{sfx}"] + P[f"decoder.rnn.bias_hh_l{li}{sfx}"]
            gx = (mm(inp, wih, "wih0") if li == 0 else mm(inp, wih, "proj1")) + bias
            if li == 1 and "g16" in on:
                gx = f16(gx)
            h = torch.zeros(B, H, dtype=torch.float64)
            c = torch.zeros(B, H, dtype=torch.float64)
            o = [None] * T
            for t in (range(T - 1, -1, -1) if rev else range(T)):
                g = gx[:, t] + mm(h, whh, f"rec{li}")
                i, f, gg, og = g.split(H, 1)
                c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
                h = torch.sigmoid(og) * torch.tanh(c)
                o[t] = h
            outs.append(torch.stack(o, 1))
        y = torch.cat(outs, -1)
        if li < L - 1:
            y = y * d(mask)
            inp = bf(y) if "proj1" in on and "proj1" not in split else y
        else:
            inp = y
    heads = []
    for pfx in ("decoder.mean_fc", "decoder.log_var_fc"):
        p1 = lr(mm(inp, P[pfx + ".blocks.0.weight"], "heads1") + P[pfx + ".blocks.0.bias"])
        if "heads1" in on:
            p1 = r(p1, "heads1")
        p2 = lr(mm(p1, P[pfx + ".blocks.2.weight"], "heads23") + P[pfx + ".blocks.2.bias"])
        if "heads23" in on:
            p2 = r(p2, "heads23")
        heads.append(mm(p2, P[pfx + ".blocks.4.weight"], "heads23") + P[pfx + ".blocks.4.bias"])
    mean, log_var = heads
    rec = O.recon_loss(mean, log_var, d(x), "likelihood")
    lk = O.apply_lens_to_loss(kld, lens)
    lrc = O.apply_lens_to_loss(rec, lens)
    w_kld, w_rec = O.loss_weights(["kld_loss", "recon_loss"], {"kld_weight": 1e-3, "batch_size": B})
    return float(w_kld * lk + w_rec * lrc)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--every", type=int, default=20)
    a = ap.parse_args()
    torch.set_num_threads(8)
    data = batches()
    params = O.init_params(F, E, Z, H, L, C, seed=7)
    state = {}
    g = torch.Generator().manual_seed(11)
    cfg = dict(L=L, loss_type="likelihood", kld_weight=1e-3)
    for st in range(a.steps + 1):
        x, lens = data[st % 4]
        eps = torch.randn(B, T, Z, generator=g)
        mask = (torch.rand(B, T, 2 * H, generator=g) >= 0.15).float() / 0.85
        if st % a.every == 0 or st == a.steps:
            exact = emulate(params, x, lens, eps, mask, set())
            row = {grp: abs(emulate(params, x, lens, eps, mask, {grp}) - exact) / abs(exact) for grp in GROUPS}
            allr = abs(emulate(params, x, lens, eps, mask, set(GROUPS)) - exact) / abs(exact)
            spl = abs(emulate(params, x, lens, eps, mask, set(GROUPS), split=set(GROUPS)) - exact) / abs(exact)
            ws = abs(emulate(params, x, lens, eps, mask, set(GROUPS), wsplit={"enc", "heads1", "heads23"})
                     - exact) / abs(exact)
            print(f"step {st:4d} ELBO {exact:.5f} | all bf16 {allr:.2e} | all split {spl:.2e} | "
                  f"enc/heads weights split {ws:.2e} | " +
                  " ".join(f"{k} {v:.1e}" for k, v in row.items()), flush=True)
        params, _ = O.train_step(params, state, x, lens, eps, cfg, mask.unsqueeze(0), impl="aten")


if __name__ == "__main__":
    main()
