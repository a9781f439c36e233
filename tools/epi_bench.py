"""Cost of the dropout-mask recompute in the layer-1 dgrad epilogue (c3 shape: dX [128000 x 1024]
= dG [128000 x 4096] W_ih, bf16 out): the same GEMM with EPI_DROPOUT vs EPI_NONE, interleaved.
usage: python tools/epi_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402
from mlvae_hip._lib import check, lib  # noqa: E402

N, D, K = int(os.environ.get("GEMM_FRAMES", "128000")), 1024, 4096
EPI_DROPOUT, EPI_OUT_BF16 = 3, 32


def main():
    l = lib()
    A = torch.rand(N, K).sub(0.5).to(torch.bfloat16).cuda()
    B = torch.rand(D, K).sub(0.5).to(torch.bfloat16).cuda()      # W_ih^T copy: k-contiguous
    C = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
    ws = torch.empty(l.mlvae_gemm_bf16_workspace_size(N, D, K, 1) // 4 + 1, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def call(epi, p):
        check(l.mlvae_gemm_bf16(0, 1, N, D, K, 1, A.data_ptr(), K, 0, B.data_ptr(), K, 0, C.data_ptr(), D, 0,
                                0.0, None, None, epi, None, 0, 0, 0, 0, 12345, 0, p, ws.data_ptr(),
                                ws.numel() * 4, s))
    res = {0: [], 1: []}
    for rep in range(6):
        for k, (epi, p) in enumerate(((EPI_OUT_BF16, 0.0), (EPI_DROPOUT | EPI_OUT_BF16, 0.15))):
            for _ in range(2):
                call(epi, p)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(epi, p)
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 10)
    for k, name in ((0, "no dropout"), (1, "dropout epilogue")):
        ms = sorted(res[k])[len(res[k]) // 2]
        print(f"dgrad {name:18s} {ms:.3f} ms  {2.0 * N * D * K / ms / 1e9:.0f} TF/s")


if __name__ == "__main__":
    main()
