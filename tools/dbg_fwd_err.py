"""Diagnostics: where a wide forward recurrence differs from the fp64 loop -- the first step with
an error, and the error by unit position inside a workgroup's 32-unit slice (which wave's tile),
by utterance and by direction.

    python tools/dbg_fwd_err.py --B 64 --T 11 --mode 2048
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from mlvae_hip._lib import check, lib  # noqa: E402

H = 512


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=11)
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    B, T = a.B, a.T
    torch.manual_seed(B + T)
    k = 1.0 / H ** 0.5
    w = [(torch.rand(4 * H, H, dtype=torch.float64) * 2 - 1) * k for _ in range(2)]
    gx = torch.randn(B, T, 8 * H, dtype=torch.float64) * 0.5
    ys, pre = [], torch.zeros(B, T, 8 * H, dtype=torch.float64)
    for d, rev in ((0, False), (1, True)):
        h = torch.zeros(B, H, dtype=torch.float64)
        c = torch.zeros(B, H, dtype=torch.float64)
        o = [None] * T
        for t in (range(T - 1, -1, -1) if rev else range(T)):
            g = gx[:, t, d * 4 * H:(d + 1) * 4 * H] + h @ w[d].t()
            pre[:, t, d * 4 * H:(d + 1) * 4 * H] = g
            i, f, gg, og = g.split(H, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(og) * torch.tanh(c)
            o[t] = h
        ys.append(torch.stack(o, 1))
    y = torch.cat(ys, -1)  # [B, T, 2H]
    N = B * T
    G = gx.reshape(N, 8 * H).to(torch.float16).cuda().contiguous()
    Cs = torch.empty(N, 2 * H, device="cuda")
    Y = torch.empty(N, 2 * H, device="cuda")
    Yb = torch.empty(N, 2 * H, device="cuda", dtype=torch.bfloat16)
    W0, W1 = w[0].float().cuda(), w[1].float().cuda()
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, 1, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    lib().mlvae_lstm_set_debug_mode(a.mode)
    P = lambda t: t.data_ptr()
    check(lib().mlvae_lstm_fwd_ex2(1, B, T, H, P(W0), P(W1), P(G), 1, P(Cs), P(Y), P(Yb), None, 0, 0, 0.0,
                                   P(xbuf), xb.value, P(err), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    lib().mlvae_lstm_set_debug_mode(0)
    e = (Y.view(B, T, 2 * H).double().cpu() - y).abs()
    print(f"B={B} T={T} mode={a.mode} err={err.item()} max|dY| {e.max():.3e}")
    for d in range(2):
        ed = e[..., d * H:(d + 1) * H]
        order = range(T) if d == 0 else range(T - 1, -1, -1)
        first = next((s for s, t in enumerate(order) if ed[:, t].max() > 2e-2), None)
        print(f" dir {d}: first step with |err| > 2e-2: {first}")
        if first is None:
            continue
        t = list(order)[first]
        et = ed[:, t]  # [B, H]
        bad = (et > 2e-2)
        print("   by unit mod 32 (bad count):", bad.view(B, H // 32, 32).sum((0, 1)).tolist())
        print("   by unit slice of 32 (bad count):", bad.view(B, H // 32, 32).sum((0, 2)).tolist())
        print("   by utterance (bad count):", bad.sum(1).tolist())
        # the input gate's pre-activation from the saved activated gate (fp16): what went into it
        gi = G.view(B, T, 8 * H)[:, t, d * 4 * H:d * 4 * H + H].double().cpu().clamp(1e-4, 1 - 1e-4)
        pg = torch.log(gi / (1 - gi))
        dp = pg - pre[:, t, d * 4 * H:d * 4 * H + H]
        bu, bj = torch.nonzero(bad, as_tuple=True)
        sel = dp[bu, bj]
        print(f"   input-gate pre-activation error at bad entries: mean {sel.mean():.3f} rms {sel.pow(2).mean().sqrt():.3f}"
              f" (good entries rms {dp[~bad].pow(2).mean().sqrt():.3f})")
        hpart = pre[:, t, d * 4 * H:d * 4 * H + H] - gx[:, t, d * 4 * H:d * 4 * H + H]
        for name, cand in [("-gx(t)", -gx[:, t, d * 4 * H:d * 4 * H + H]), ("-h.W", -hpart)] + \
                [(f"gx({u})-gx(t)", gx[:, u, d * 4 * H:d * 4 * H + H] - gx[:, t, d * 4 * H:d * 4 * H + H])
                 for u in range(T) if u != t]:
            r = (sel - cand[bu, bj]).pow(2).mean().sqrt() / max(sel.pow(2).mean().sqrt().item(), 1e-9)
            print(f"     residual vs {name}: {r:.3f}")


if __name__ == "__main__":
    main()
