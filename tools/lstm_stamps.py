"""Diagnostics: per-phase timing of one persistent LSTM recurrence launch (workgroup 0, thread 0
stamps s_memtime at the kernel's STAMP(0..4) points; ticks are shader cycles).

    python tools/lstm_stamps.py [--B 256] [--T 500] [--bwd] [--mode N]

Phases (batch-group and wide kernels alike):
  fwd: 0 step start | 1 poll done | 2 barrier / reduce | 3 MFMA done | 4 cell + publish done
  bwd: 0 step start | 1 poll done | 2 reduce done | 3 barrier | 4 MFMA + publish done
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402
from mlvae_hip._lib import check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--T", type=int, default=500)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--prec", type=int, default=1)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--mode", type=int, default=0, help="lstm debug mode bits")
    ap.add_argument("--noy", action="store_true", help="forward without the fp32 h output")
    ap.add_argument("--drop", type=float, default=0.0, help="forward with the fused bf16 dropout(h)")
    a = ap.parse_args()
    B, T, H, prec = a.B, a.T, a.H, a.prec
    P = lambda t: t.data_ptr()
    lib().mlvae_lstm_set_debug_mode(a.mode)
    g16 = lib().mlvae_lstm_gates_fp16(B, H, prec)  # wide-batch kernels: fp16 gate buffer
    G = (torch.randn(B * T, 8 * H, device="cuda") * 0.1).to(torch.float16 if g16 else torch.float32)
    Cs = torch.empty(B * T, 2 * H, device="cuda")
    Y = torch.empty(B * T, 2 * H, device="cuda")
    dGb = torch.empty(B * T, 8 * H, device="cuda", dtype=torch.bfloat16)
    Yb = torch.empty(B * T, 2 * H, device="cuda", dtype=torch.bfloat16)
    Ydb = torch.empty(B * T, 2 * H, device="cuda", dtype=torch.bfloat16)
    W0 = torch.randn(4 * H, H, device="cuda") * 0.04
    W1 = torch.randn(4 * H, H, device="cuda") * 0.04
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, prec, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    dbg = torch.zeros(T * 16, device="cuda", dtype=torch.int64)
    s = torch.cuda.current_stream().cuda_stream
    for it in range(4):
        if it == 3:
            lib().mlvae_lstm_set_debug(P(dbg))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if a.bwd:
            G.uniform_(0.05, 0.95)
            Cs.normal_()
        ev0.record()
        if a.bwd:
            check(lib().mlvae_lstm_bwd_ex2(prec, B, T, H, P(W0), P(W1), P(G), g16, P(Cs), P(Y), P(dGb), None,
                                           P(xbuf), xb.value, P(err), s))
        else:
            check(lib().mlvae_lstm_fwd_ex2(prec, B, T, H, P(W0), P(W1), P(G), g16, P(Cs),
                                           None if a.noy else P(Y), P(Yb), P(Ydb) if a.drop else None,
                                           7, 0, a.drop, P(xbuf), xb.value, P(err), s))
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1)
        print(f"{'bwd' if a.bwd else 'fwd'} B={B} T={T} launch {ms:.3f} ms ({ms / T * 1e3:.2f} us/step) "
              f"err={err.item()}")
    lib().mlvae_lstm_set_debug(None)
    lib().mlvae_lstm_set_debug_mode(0)
    d = dbg.view(T, 16).cpu().double()
    names = (["poll", "reduce", "barrier", "mfma+publish"] if a.bwd else
             ["poll", "barrier", "mfma", "cell+publish"])
    for b, nm in zip(range(1, 5), names):
        dd = d[2:, b] - d[2:, b - 1]
        print(f"{nm:14s} median {dd.median().item():8.0f} ticks  mean {dd.mean().item():8.0f}")
    # every stamp as an offset from the step start (extra stamps 5..7: see the STAMP sites)
    offs = [f"{b}:{(d[2:T - 1, b] - d[2:T - 1, 0]).median().item():.0f}" for b in range(1, 8)
            if (d[2:T - 1, b] != 0).all()]
    print("offsets from step start (median ticks) " + " ".join(offs))
    per = d[3:T - 1, 0] - d[2:T - 2, 0]     # step start to step start: the whole period
    tail = per - (d[2:T - 2, 4] - d[2:T - 2, 0])
    print(f"{'tail':14s} median {tail.median().item():8.0f} ticks  mean {tail.mean().item():8.0f}")
    print(f"{'step period':14s} median {per.median().item():8.0f} ticks  mean {per.mean().item():8.0f}")
    if a.mode & (1 << 22):  # interleaved forward: chain 1's stamps sit at slots 8..12
        for b, nm in zip(range(9, 13), names):
            dd = d[2:, b] - d[2:, b - 1]
            print(f"c1 {nm:11s} median {dd.median().item():8.0f} ticks  mean {dd.mean().item():8.0f}")
        print(f"{'c0 end->c1':14s} median {(d[2:, 8] - d[2:, 4]).median().item():8.0f}")
    if a.mode & (1 << 23):  # publish -> own stores acknowledged (slot 5)
        dd = d[2:, 5] - d[2:, 4]
        print(f"{'publish ack':14s} median {dd.median().item():8.0f} ticks  mean {dd.mean().item():8.0f}")
    nxt = d[3:, 0] - d[2:-1, 4]
    print(f"{'tail->next':14s} median {nxt.median().item():8.0f}")
    tot = d[3:, 0] - d[2:-1, 0]
    print(f"{'step total':14s} median {tot.median().item():8.0f} ticks")


if __name__ == "__main__":
    main()
