"""Standalone timing of the Conv1d encoder's backward kernels at configs[3] (B=64, T=2000, F=80,
E=64, K=5), outside the train step (where they share the chip with the side-stream weight-gradient
GEMMs): mlvae_conv1d_dgrad + mlvae_conv1d_wgrad and the forward layers.  Algorithmic HBM bytes as bench.py (fp32 activations).
usage: python tools/conv_bench.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402

from mlvae_hip._lib import check, lib  # noqa: E402

B, T, F, E, K = 64, 2000, 80, 64, 5
N = B * T
HBM = 8000.0


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    l = lib()
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr() if t is not None else None
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(N, F, device="cuda", generator=g)
    e1 = torch.randn(N, E, device="cuda", generator=g)
    de2 = torch.randn(N, E, device="cuda", generator=g)
    w1 = torch.randn(E, F, K, device="cuda", generator=g) * 0.05
    w2 = torch.randn(E, E, K, device="cuda", generator=g) * 0.05
    b1 = torch.zeros(E, device="cuda")
    de1 = torch.empty(N, E, device="cuda")
    dw1, db1 = torch.empty_like(w1), torch.empty(E, device="cuda")
    nb = l.mlvae_conv1d_wgrad_workspace_size(B, T, F, E, K)
    ws = torch.empty(nb // 4 + 1, device="cuda")
    y1 = torch.empty(N, E, device="cuda")

    def two():
        check(l.mlvae_conv1d_dgrad(B, T, E, E, K, P(de2), E, P(w2), P(e1), E, P(de1), E, s))
        check(l.mlvae_conv1d_wgrad(B, T, F, E, K, P(de1), E, P(x), F, P(dw1), P(db1), P(ws), nb, s))

    def fwd1():
        check(l.mlvae_conv1d_fwd(B, T, F, E, K, P(x), F, P(w1), P(b1), 1, P(y1), E, s))

    for name, fn, nbytes in (("conv backward dgrad + wgrad", two, N * 4 * (4 * E + F)),
                             ("conv forward layer 1", fwd1, N * 4 * (F + E))):
        ms = timed(fn, iters)
        gbs = nbytes / (ms * 1e-3) / 1e9
        print(f"{name:30s} {ms * 1e3:8.1f} us  {nbytes / 1e6:7.1f} MB  {gbs:7.0f} GB/s = {100 * gbs / HBM:5.1f} % of HBM",
              flush=True)


if __name__ == "__main__":
    main()
