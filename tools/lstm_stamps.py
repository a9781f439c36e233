"""Diagnostics: per-phase timing of one persistent LSTM recurrence launch (workgroup 0, thread 0
stamps s_memtime at the kernel's STAMP(0..4) points; ticks are shader cycles).

    python tools/lstm_stamps.py [--B 256] [--T 500] [--bwd] [--mode N]

Phases (wide kernels; stamps of steps 64..95 buffered in LDS, lstm_common.h LSTAMP):
  fwd: 0 step start | 1 poll done | 2 barrier | 3 MFMA issued | 4 cell + publish | 6 out ring |
       7 drop bits (5: publish ack, debug bit 23)
  bwd: 0 step start | 1 poll done | 5 cell inputs staged | 6 prefetch issued | 2 reduce done |
       7 barrier | 3 prefetch issued (late, full-chip grids) | 4 MFMA + publish
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
    # the wide kernels stamp steps [STW0, STW0 + STWN) into LDS (lstm_common.h LSTAMP)
    w0, wn = 64, 32
    w = d[w0:w0 + wn]
    names = ({1: "poll done", 5: "cell inputs staged", 6: "prefetch issued", 2: "reduce done",
              7: "barrier", 3: "prefetch issued (late)", 4: "MFMA + publish"} if a.bwd else
             {1: "poll done", 2: "barrier", 3: "MFMA issued", 4: "cell + publish",
              5: "publish ack" if a.mode & (1 << 23) else "cell done",
              6: "out ring", 7: "drop bits"})
    order = sorted((b for b in names if (w[:, b] != 0).all()),
                   key=lambda b: (w[:, b] - w[:, 0]).median().item())
    prev = 0.0
    for b in order:
        off = (w[:, b] - w[:, 0]).median().item()
        print(f"{names[b]:20s} at {off:7.0f} ticks from the step start  (+{off - prev:6.0f})")
        prev = off
    if a.mode & 16 and not a.bwd:  # wave 4 (io) phases (debug bit 4, lstm_common.h IOSTAMP)
        io_names = ["io step start", "io vmcnt done", "io barrier", "io gx DMA issued", "io MFMA issued",
                    "io publish", "io stores issued"]
        for k, nm in enumerate(io_names):
            if (w[:, 8 + k] != 0).all():
                print(f"{nm:20s} at {(w[:, 8 + k] - w[:, 0]).median().item():7.0f} ticks from wave 0's step start")
        wv = []
    else:
        wv = [(w[:, 8 + k] - w[:, 0]).median().item() for k in range(8) if (w[:, 8 + k] != 0).all()]
    if wv:
        what = ("reduce done" if a.mode & (1 << 21) else "pre-barrier" if a.mode & (1 << 22) else "poll done")
        print(f"per-wave {what:11s} " + " ".join(f"w{k}:{v:.0f}" for k, v in enumerate(wv)))
        if len(wv) == 8:
            mx = (w[:, 8:16].max(dim=1).values - w[:, 0]).median().item()
            print(f"{'':20s} slowest wave per step: median {mx:.0f}")
    per = w[1:, 0] - w[:-1, 0]
    print(f"{'step period':20s} median {per.median().item():7.0f} ticks  mean {per.mean().item():7.0f}")
    last = order[-1] if order else 0
    print(f"{'tail (last -> next)':20s} median {(w[1:, 0] - w[:-1, last]).median().item():7.0f}")

if __name__ == "__main__":
    main()
