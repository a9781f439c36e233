"""Time the train step's big GEMM shapes (c2 or, GEMM_FRAMES=128000, c3; bf16 operands): mlvae_gemm_ex (128² register-staged)
against mlvae_gemm_bf16 (256² LDS-DMA), with torch.matmul (hipBLASLt, bf16 out) as the
library reference point.  usage: python tools/gemm_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402
from mlvae_hip._lib import check, lib  # noqa: E402

N = int(os.environ.get("GEMM_FRAMES", "16000"))   # B*T rows: 16,000 at c2, 128,000 at c3
H, D = 512, 1024
SHAPES = [  # name, ta, tb, M, Ncols, K
    ("fwd proj  Y=X W^T  ", 0, 1, N, 8 * H, D),
    ("proj l0   Y=Z W^T  ", 0, 1, N, 8 * H, 32),
    ("dgrad     dX=dG W  ", 0, 0, N, D, 8 * H),
    ("dgrad     dX=dG W^T", 0, 1, N, D, 8 * H),
    ("wgrad ih  dG^T X   ", 1, 0, 8 * H, D, N),
    ("wgrad hh  dG^T h   ", 1, 0, 4 * H, H, N),
    ("4096^3             ", 0, 1, 4096, 4096, 4096),
]


def run(ta, tb, M, Nc, K, fast, iters=10):
    l = lib()
    A = (torch.rand(K, M) if ta else torch.rand(M, K)).sub(0.5).to(torch.bfloat16).cuda()
    B = (torch.rand(Nc, K) if tb else torch.rand(K, Nc)).sub(0.5).to(torch.bfloat16).cuda()
    C = torch.empty(M, Nc, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if fast == 2:  # hipBLASLt through torch
        At, Bt = (A.t() if ta else A), (B.t() if tb else B)
        return _time(lambda: torch.matmul(At, Bt), iters, M, Nc, K)
    wsz = l.mlvae_gemm_bf16_workspace_size(M, Nc, K, 1) if fast else l.mlvae_gemm_ex_workspace_size(M, Nc, K)
    ws = torch.empty(wsz // 4 + 1, device="cuda")

    def call():
        if fast:
            check(l.mlvae_gemm_bf16(ta, tb, M, Nc, K, 1, A.data_ptr(), A.shape[1], 0, B.data_ptr(),
                                    B.shape[1], 0, C.data_ptr(), Nc, 0, 0.0, None, None, 0, None, 0,
                                    0, 0, 0, 0, 0, 0.0, ws.data_ptr(), ws.numel() * 4, s))
        else:
            check(l.mlvae_gemm_ex(ta, tb, M, Nc, K, 1.0, A.data_ptr(), 1, A.shape[1], B.data_ptr(),
                                  1, B.shape[1], 0.0, C.data_ptr(), Nc, None, None, 0, None, 0, 0, 0,
                                  ws.data_ptr(), ws.numel() * 4, s))
    return _time(call, iters, M, Nc, K)


def _time(call, iters, M, Nc, K):
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, 2.0 * M * Nc * K / ms / 1e9


def run_fp8(M, Nc, K, iters=10):
    """mlvae_gemm_fp8 (e4m3 operands A [M][K], B [N][K], fp16 C as the step's projection)"""
    l = lib()
    A = torch.randn(M, K, device="cuda").clamp(-448, 448).to(torch.float8_e4m3fn)
    B = torch.randn(Nc, K, device="cuda").clamp(-448, 448).to(torch.float8_e4m3fn)
    C = torch.empty(M, Nc, device="cuda", dtype=torch.float16)
    alpha = torch.ones(1, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def call():
        check(l.mlvae_gemm_fp8(M, Nc, K, A.data_ptr(), K, B.data_ptr(), K, C.data_ptr(), Nc, alpha.data_ptr(),
                               None, None, 16, s))
    return _time(call, iters, M, Nc, K)


def fp8_shapes():
    """fp8 k-contiguous products (GEMM_FP8=1): the projection and dgrad shapes on e4m3 operands"""
    for name, ta, tb, M, Nc, K in SHAPES:
        if ta or K == 32:
            continue
        ms = sorted(run_fp8(M, Nc, K)[0] for _ in range(3))
        print(f"fp8 {name} M={M:6d} N={Nc:5d} K={K:6d} | med {ms[1] * 1e3:7.1f} us min {ms[0] * 1e3:7.1f} us "
              f"{2.0 * M * Nc * K / ms[0] / 1e9:6.1f} TF", flush=True)


def ab(vars_, rounds=3):
    """Same-process A/B of gemm256 main-loop variants (GEMM_VARS=0,10): interleaved rounds, the
    median and min per variant (cdna_hip_programming.md §5.4 rule 24)."""
    l = lib()
    only = os.environ.get("GEMM_ONLY")
    for name, ta, tb, M, Nc, K in SHAPES:
        if (only and only not in name) or K == 32:
            continue
        res = {v: [] for v in vars_}
        for _ in range(rounds):
            for v in vars_:
                l.mlvae_gemm_bf16_set_variant(v)
                res[v].append(run(ta, tb, M, Nc, K, 1)[0])
        l.mlvae_gemm_bf16_set_variant(0)
        flops = 2.0 * M * Nc * K
        print(f"{name} M={M:6d} N={Nc:5d} K={K:6d} | " + " | ".join(
            f"VAR {v}: med {sorted(t)[len(t) // 2] * 1e3:7.1f} us min {min(t) * 1e3:7.1f} us "
            f"{flops / min(t) / 1e9:6.1f} TF" for v, t in res.items()), flush=True)


def main():
    if os.environ.get("GEMM_FP8"):
        return fp8_shapes()
    if os.environ.get("GEMM_VARS"):
        return ab([int(v) for v in os.environ["GEMM_VARS"].split(",")])
    only = os.environ.get("GEMM_ONLY")        # substring of a shape name: run just that one
    modes = [int(m) for m in os.environ.get("GEMM_MODES", "0,1,2").split(",")]
    for name, ta, tb, M, Nc, K in SHAPES:
        if only and only not in name:
            continue
        r = []
        for fast in modes:
            ms, tf = run(ta, tb, M, Nc, K, fast)
            r.append(f"{ms * 1e3:7.1f} us {tf:6.1f} TF")
        names = {0: "gemm_ex", 1: "gemm_bf16 256²", 2: "hipBLASLt"}
        print(f"{name} M={M:6d} N={Nc:5d} K={K:6d} | " +
              " | ".join(f"{names[m]}: {x}" for m, x in zip(modes, r)), flush=True)


if __name__ == "__main__":
    main()
