"""Hand-off latency of the wide forward recurrence from chip-wide realtime stamps (debug bit 3):
every workgroup records s_memrealtime (100 MHz, one clock for all CUs) at each wave's publish and
at each poller's poll completion for steps 64..95; for consumer c, poller w and step s the data
is ready once the LAST of its producers' waves published step s-1:

    latency = poll_done(c, w, s) - max_{p in producers(w), wave} publish(p, wave, s-1)

    python tools/lstm_handoff.py [--B 256] [--mode N] [--bwd]

--bwd (round 5): the BPTT.  Consumer workgroup c's partials all come from producer wave
c * HJ / 64 of every member (the reduce-scatter layout); every one of its 8 waves polls (slots
8 + w); the step's barrier waits for the last of them, so the per-wave latency spread -- and how
much of it is the wave's own poll phase rather than a later producer -- is what this prints."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402
from mlvae_hip._lib import check, lib  # noqa: E402

STW0, STWN = 64, 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--T", type=int, default=500)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--bwd", action="store_true")
    a = ap.parse_args()
    if a.bwd:
        return bwd(a)
    B, T, H = a.B, a.T, 512
    P = lambda t: t.data_ptr()
    NB = (B + 15) // 16
    tpw = 1 if 2 * NB * 16 <= 256 else 2
    HJ = 32 * tpw
    NJ = H // HJ
    gstride = (2 * NB + 7) & ~7
    grid = gstride * NJ
    G = (torch.randn(B * T, 8 * H, device="cuda") * 0.1).to(torch.float16)
    Cs = torch.empty(B * T, 2 * H, device="cuda")
    Yb = torch.empty(B * T, 2 * H, device="cuda", dtype=torch.bfloat16)
    Ydb = torch.empty(B * T, 2 * H, device="cuda", dtype=torch.bfloat16)
    W0 = torch.randn(4 * H, H, device="cuda") * 0.04
    W1 = torch.randn(4 * H, H, device="cuda") * 0.04
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, 1, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    dbg = torch.zeros(T * 16 + grid * STWN * 16, device="cuda", dtype=torch.int64)
    s = torch.cuda.current_stream().cuda_stream
    lib().mlvae_lstm_set_debug_mode(a.mode | 8)
    for it in range(4):
        if it == 3:
            lib().mlvae_lstm_set_debug(P(dbg))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lib().mlvae_lstm_fwd_ex2(1, B, T, H, P(W0), P(W1), P(G), 1, P(Cs), None, P(Yb), P(Ydb),
                                       7, 0, 0.15, P(xbuf), xb.value, P(err), s))
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
    lib().mlvae_lstm_set_debug(None)
    lib().mlvae_lstm_set_debug_mode(0)
    print(f"fwd B={B} T={T} mode {a.mode}: launch {ms:.3f} ms ({ms / T * 1e3:.2f} us/step), grid {grid}, "
          f"HJ {HJ}, NJ {NJ}, err {err.item()}")
    r = dbg[T * 16:].view(grid, STWN, 16).cpu().numpy().astype(np.int64)
    pub = r[:, :, 0:8]            # [wg][step][wave]
    done = r[:, :, 8:12]          # [wg][step][poller]
    lat, skew, last_wave = [], [], []
    period = []
    for b in range(grid):
        gid, js = b % gstride, b // gstride
        if gid >= 2 * NB:
            continue
        members = [gid + k * gstride for k in range(NJ)]
        period.append(np.median(np.diff(pub[b, :, 0])))
        for w in range(4):
            lo, hi = 128 * w // HJ, (128 * w + 127) // HJ
            prods = [members[p] for p in range(lo, hi + 1)]
            for si in range(1, STWN):
                pp = pub[prods, si - 1, :]          # [producers][waves]
                ready = pp.max()
                lat.append(done[b, si, w] - ready)
                skew.append(ready - pp.min())
                last_wave.append(int(np.argmax(pp.max(axis=0))))
    lat, skew = np.array(lat) * 10, np.array(skew) * 10   # ns
    print(f"step period (wave 0 publishes) median {np.median(period) * 10:.0f} ns")
    print(f"hand-off latency (last producer publish -> poll done) ns: p10 {np.percentile(lat, 10):.0f} "
          f"median {np.median(lat):.0f} p90 {np.percentile(lat, 90):.0f}")
    print(f"producer skew within a quarter (first -> last wave publish) ns: median {np.median(skew):.0f} "
          f"p90 {np.percentile(skew, 90):.0f}")
    print("last-publishing wave histogram:", np.bincount(last_wave, minlength=8).tolist())
    # one workgroup's step, realtime: the spread of its waves' publishes and its pollers' completions
    b0 = 0
    pw = (pub[b0, 10:30, :] - pub[b0, 10:30, :].min(axis=1, keepdims=True)) * 10
    print("WG 0 publish offsets within a step (ns, median per wave):", np.median(pw, axis=0).astype(int).tolist())


def bwd(a):
    B, T, H = a.B, a.T, 512
    P = lambda t: t.data_ptr()
    NB = (B + 15) // 16
    tpw = 1 if 2 * NB * 16 <= 256 else 2
    HJ = 32 * tpw
    NJ = H // HJ
    gstride = (2 * NB + 7) & ~7
    grid = gstride * NJ
    G = (torch.rand(B * T, 8 * H, device="cuda") * 0.9 + 0.05).to(torch.float16)
    Cs = torch.randn(B * T, 2 * H, device="cuda")
    Y = torch.randn(B * T, 2 * H, device="cuda") * 0.1
    dGb = torch.empty(B * T, 8 * H, device="cuda", dtype=torch.bfloat16)
    W0 = torch.randn(4 * H, H, device="cuda") * 0.04
    W1 = torch.randn(4 * H, H, device="cuda") * 0.04
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, 1, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    dbg = torch.zeros(T * 16 + grid * STWN * 16, device="cuda", dtype=torch.int64)
    s = torch.cuda.current_stream().cuda_stream
    lib().mlvae_lstm_set_debug_mode(a.mode | 8)
    for it in range(4):
        if it == 3:
            lib().mlvae_lstm_set_debug(P(dbg))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lib().mlvae_lstm_bwd_ex2(1, B, T, H, P(W0), P(W1), P(G), 1, P(Cs), P(Y), P(dGb), None,
                                       P(xbuf), xb.value, P(err), s))
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
    lib().mlvae_lstm_set_debug(None)
    lib().mlvae_lstm_set_debug_mode(0)
    print(f"bwd B={B} T={T} mode {a.mode}: launch {ms:.3f} ms ({ms / T * 1e3:.2f} us/step), grid {grid}, "
          f"HJ {HJ}, NJ {NJ}, err {err.item()}")
    pl = dbg[:grid].cpu().numpy()
    print(f"hand-off placement: {(pl == 1).sum()} workgroups with plain (same-XCD) publishes, "
          f"{(pl == 2).sum()} write-through")
    r = dbg[T * 16:].view(grid, STWN, 16).cpu().numpy().astype(np.int64)
    pub = r[:, :, 0:8]            # [wg][step][wave]  (publish done)
    done = r[:, :, 8:16]          # [wg][step][wave]  (poll done)
    lat = [[] for _ in range(8)]
    spread, last_minus_ready, ready_skew = [], [], []
    for b in range(grid):
        gid, js = b % gstride, b // gstride
        if gid >= 2 * NB:
            continue
        members = [gid + k * gstride for k in range(NJ)]
        pw = js * HJ // 64
        for si in range(1, STWN):
            pp = pub[members, si - 1, pw]
            ready = pp.max()
            ready_skew.append(ready - pp.min())
            d = done[b, si, :]
            for w in range(8):
                lat[w].append(d[w] - ready)
            spread.append(d.max() - d.min())
            last_minus_ready.append(d.max() - ready)
    ns = lambda v: np.array(v) * 10
    print("hand-off latency (last producer publish -> this wave's poll done), ns, per consumer wave:")
    for w in range(8):
        v = ns(lat[w])
        print(f"  w{w}: p10 {np.percentile(v, 10):5.0f}  median {np.median(v):5.0f}  p90 {np.percentile(v, 90):5.0f}")
    print(f"last wave's poll done - data ready, ns: median {np.median(ns(last_minus_ready)):.0f} "
          f"p90 {np.percentile(ns(last_minus_ready), 90):.0f}")
    print(f"poll-done spread over a workgroup's 8 waves (first -> last), ns: median {np.median(ns(spread)):.0f} "
          f"p90 {np.percentile(ns(spread), 90):.0f}")
    print(f"producer skew (first -> last member publish for one consumer), ns: median "
          f"{np.median(ns(ready_skew)):.0f} p90 {np.percentile(ns(ready_skew), 90):.0f}")
    period = [np.median(np.diff(pub[b, :, 0])) for b in range(grid) if b % gstride < 2 * NB]
    print(f"step period (wave 0 publishes) median {np.median(period) * 10:.0f} ns")


if __name__ == "__main__":
    main()
