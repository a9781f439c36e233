"""Where a 256-squared GEMM tile's time goes: the layer-1 projection shape (M = 128,000 frames,
N = 4096) timed at K = 64 ... 2048 with fp16 (the step's projection epilogue) and fp32 output.
time(K) = tiles/CUs x (prologue + epilogue + K/64 x one K-step): the slope is the main loop, the
intercept the per-tile fixed cost (prologue latency + epilogue).  usage: python tools/gemm_kscan.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mlvae_hip._lib import check, lib  # noqa: E402

M, N = int(os.environ.get("GEMM_FRAMES", "128000")), 4096
KS = [64, 128, 256, 512, 1024, 2048]


def time_one(K, epi, var, iters=10):
    l = lib()
    A = torch.rand(M, K).sub(0.5).to(torch.bfloat16).cuda()
    B = torch.rand(N, K).sub(0.5).to(torch.bfloat16).cuda()
    C = torch.empty(M * N // (2 if epi else 1), device="cuda")
    bias = torch.rand(N, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    prev = l.mlvae_gemm_bf16_set_variant(var)
    wsz = l.mlvae_gemm_bf16_workspace_size(M, N, K, 1)
    ws = torch.empty(wsz // 4 + 1, device="cuda")

    def call():
        check(l.mlvae_gemm_bf16(0, 1, M, N, K, 1, A.data_ptr(), K, 0, B.data_ptr(), K, 0, C.data_ptr(), N, 0,
                                0.0, bias.data_ptr(), None, epi, None, 0, 0, 0, 0, 0, 0, 0.0,
                                ws.data_ptr(), ws.numel() * 4, s))
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    l.mlvae_gemm_bf16_set_variant(prev)
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    tiles = (M // 256) * (N // 256)
    waves = tiles / 256.0
    for var in [int(v) for v in os.environ.get("GEMM_VARS", "0,12").split(",")]:
        epis = [int(e) for e in os.environ.get("GEMM_EPIS", "16,0").split(",")]
        for epi, name in ((e, "fp16 out" if e == 16 else "fp32 out") for e in epis):
            us = [time_one(K, epi, var) for K in KS]
            ksteps = np.array(KS) / 64.0
            slope, icpt = np.polyfit(ksteps, np.array(us) / waves, 1)
            tf = [2.0 * M * N * K / (u * 1e-6) / 1e12 for K, u in zip(KS, us)]
            print(f"VAR {var:2d} {name} (MLVAE_GEMM_ABL={os.environ.get('MLVAE_GEMM_ABL', '0')} STAGGER={os.environ.get('MLVAE_GEMM_STAGGER', '1')}): " + " ".join(f"K{K}:{u:.0f}us({t:.0f}TF)" for K, u, t in zip(KS, us, tf)))
            print(f"   per tile: {slope:.2f} us per 64-deep K-step (MFMA floor at 2.4 GHz 0.85 us), "
                  f"fixed {icpt:.2f} us (prologue + epilogue); at K=1024 fixed share "
                  f"{icpt / (icpt + 16 * slope) * 100:.1f} %", flush=True)


if __name__ == "__main__":
    main()
