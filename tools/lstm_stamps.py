"""Diagnostics: per-phase timing of the persistent LSTM forward step (workgroup 0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import ctypes
import torch
from mlvae_hip._lib import lib, check


def main(prec=1, B=32, T=500, H=512, bwd=False):
    P = lambda t: t.data_ptr()
    G = torch.randn(B * T, 8 * H, device="cuda") * 0.1
    Cs = torch.empty(B * T, 2 * H, device="cuda")
    Y = torch.empty(B * T, 2 * H, device="cuda")
    W0 = torch.randn(4 * H, H, device="cuda") * 0.04
    W1 = torch.randn(4 * H, H, device="cuda") * 0.04
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, prec, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    dbg = torch.zeros(T * 16, device="cuda", dtype=torch.int64)
    s = torch.cuda.current_stream().cuda_stream
    lib().mlvae_lstm_set_debug_mode(int(os.environ.get("LSTM_DBG_MODE", "0")))
    for it in range(3):
        if it == 2:
            lib().mlvae_lstm_set_debug(P(dbg))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        if bwd:
            G.uniform_(0.05, 0.95)
            Cs.normal_()
            check(lib().mlvae_lstm_bwd(prec, B, T, H, P(W0), P(W1), P(G), P(Cs), P(Y), P(xbuf),
                                       xb.value, P(err), s))
        else:
            check(lib().mlvae_lstm_fwd(prec, B, T, H, P(W0), P(W1), P(G), P(Cs), P(Y), P(xbuf),
                                       xb.value, P(err), s))
        ev1.record()
        torch.cuda.synchronize()
        print(f"{'bwd' if bwd else 'fwd'} launch {ev0.elapsed_time(ev1):.3f} ms ({ev0.elapsed_time(ev1) / T * 1e3:.2f} us/step)")
    lib().mlvae_lstm_set_debug(None)
    d = dbg.view(T, 16).cpu().double()
    names = (["poll+load", "mfma", "barrier", "cell+publish"] if bwd else
             ["poll+load", "mfma", "reduce", "cell+publish"])
    ph = [(1, 0), (2, 1), (3, 2), (4, 3)]
    for (b, a), nm in zip(ph, names):
        dd = (d[2:, b] - d[2:, a])
        print(f"{nm:14s} median {dd.median().item():8.0f} ticks  mean {dd.mean().item():8.0f}")
    nxt = d[3:, 0] - d[2:-1, 4]
    print(f"{'stores->next':14s} median {nxt.median().item():8.0f}")
    rt = d[2:, 1] - d[2:, 5]
    print(f"{'last poll RT':14s} median {rt.median().item():8.0f}")
    sp = d[2:, 6]
    print(f"{'spins':14s} median {sp.median().item():8.0f} mean {sp.mean().item():6.2f}")
    print(f"placement flags (bit0 plain same-XCD stores, bit1 xcd-local grid): {int(d[0, 7])}")
    if bwd:
        for w in range(4):
            pd = d[2:, 8 + w] - d[2:, 0]
            pb = d[2:, 12 + w] - d[2:, 0]
            print(f"wave {w}: poll done +{pd.median().item():6.0f}  at barrier +{pb.median().item():6.0f}")
    tot = d[3:, 0] - d[2:-1, 0]
    print(f"{'step total':14s} median {tot.median().item():8.0f}")


if __name__ == "__main__":
    main(prec=int(sys.argv[1]) if len(sys.argv) > 1 else 1,
         bwd=len(sys.argv) > 2 and sys.argv[2] == "bwd")
