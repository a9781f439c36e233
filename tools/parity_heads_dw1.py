"""Diagnostic (round 5): where the fp32 mode's mean-head first-layer gradient error at B = 256
came from (the fp64-anchored whole-step test: engine 2.4e-5 / 2.0e-5 vs the fp32 oracle's
3.7e-7 / 1.1e-7 for mean_fc.blocks.0.weight / bias).  Runs the engine's fp32 step, then sums the
engine's own saved dP1 and rnn_out in fp64 on the host (equal to the engine's: the reductions were
exact), and counts the LeakyReLU-derivative flips of the heads' first layer against fp64.
Result: one flip in the engine's mean head (hardware tanh in the fp32 recurrence, rnn_out 1.2e-6
from fp64), one in the oracle's log_var head; with libm cell math the engine has none
(profiles/r05_fp32_mode_vs_fp64_B256.txt).
usage: python tools/parity_heads_dw1.py [B] [T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from step_parity import oracle_fp64, run_step  # noqa: E402


def nr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def main():
    from mlvae_hip.engine import VAEConfig
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    torch.set_num_threads(16)
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="fp32")
    lens = torch.linspace(0.6, 1.0, B)
    lens[3], lens[7] = 127 / 500, 254 / 500
    eng, w, rec, new_ref, params = run_step(cfg, B, T, 1303, lens)
    _, r64 = oracle_fp64(cfg, params, rec["inputs"])
    C, H = cfg.C, cfg.H
    dP1 = w.dP1.detach().cpu().double()            # [N, 2C] fp32 buffer of the engine
    R = w.rnn_out.detach().cpu().double()          # [N, 2H]
    g = eng.named_grads()
    for h, (name, sl) in enumerate((("mean_fc", slice(0, C)), ("log_var_fc", slice(C, 2 * C)))):
        gw64 = r64["grads"][f"decoder.{name}.blocks.0.weight"]
        gb64 = r64["grads"][f"decoder.{name}.blocks.0.bias"]
        gw32 = rec["grads"][f"decoder.{name}.blocks.0.weight"]
        gb32 = rec["grads"][f"decoder.{name}.blocks.0.bias"]
        hw = dP1[:, sl].t() @ R
        hb = dP1[:, sl].sum(0)
        print(f"{name}: weight  engine {nr(g[f'decoder.{name}.blocks.0.weight'], gw64):.2e}  "
              f"host-fp64(engine dP1, R) {nr(hw, gw64):.2e}  oracle32 {nr(gw32, gw64):.2e}  |g| {gw64.norm():.3e}")
        print(f"{name}: bias    engine {nr(g[f'decoder.{name}.blocks.0.bias'], gb64):.2e}  "
              f"host-fp64(engine dP1) {nr(hb, gb64):.2e}  oracle32 {nr(gb32, gb64):.2e}  |g| {gb64.norm():.3e}")
    # LeakyReLU derivative flips: first-layer pre-activations whose sign differs from fp64's, on
    # the valid frames (the padded ones carry no gradient)
    R64 = r64["out"]["dec"]["rnn_out"].reshape(B * T, -1)
    R32 = rec["out"]["dec"]["rnn_out"].reshape(B * T, -1).float()
    P1e = w.P1.detach().cpu().double()
    from oracle.vae_cpu import length_to_mask
    m = length_to_mask(rec["inputs"][1], T).reshape(-1) > 0
    for name, sl in (("mean_fc", slice(0, C)), ("log_var_fc", slice(C, 2 * C))):
        W = params[f"decoder.{name}.blocks.0.weight"]
        b = params[f"decoder.{name}.blocks.0.bias"]
        p64 = R64 @ W.double().t() + b.double()
        p32 = R32 @ W.t() + b
        fe = ((P1e[:, sl] > 0) != (p64 > 0))[m].sum().item()
        fo = ((p32 > 0) != (p64 > 0))[m].sum().item()
        print(f"{name}: lrelu' flips vs fp64 on {int(m.sum())} frames x {C}: engine {fe}  oracle32 {fo}")
    print("rnn_out engine vs fp64", nr(R.view(B, T, -1), r64["out"]["dec"]["rnn_out"]),
          " oracle32 vs fp64", nr(rec["out"]["dec"]["rnn_out"], r64["out"]["dec"]["rnn_out"]))


if __name__ == "__main__":
    main()
