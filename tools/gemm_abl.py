"""GEMM ablation timing (diagnostics): the c3 projection / dgrad / wgrad shapes on the 256² kernel
with MLVAE_GEMM_ABL set by the caller (1: no MFMA, 2: no staging loads, 3: neither).
usage: MLVAE_GEMM_VAR=6 MLVAE_GEMM_ABL=N python tools/gemm_abl.py [proj dgrad wgrad]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gemm_bench as gb  # noqa: E402

N = 128000
want = sys.argv[1:] or ["proj", "dgrad", "wgrad"]
for name, ta, tb, M, Nc, K in [("proj", 0, 1, N, 4096, 1024), ("dgrad", 0, 1, N, 1024, 4096),
                               ("wgrad", 1, 0, 4096, 1024, N)]:
    if name not in want:
        continue
    ms, tf = gb.run(ta, tb, M, Nc, K, True)
    print(f"var={os.environ.get('MLVAE_GEMM_VAR', '0')} abl={os.environ.get('MLVAE_GEMM_ABL', '0')} {name:6s} "
          f"{ms:.3f} ms {tf:.0f} TF/s", flush=True)
