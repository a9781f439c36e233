"""One GEMM shape on the 256² kernel, a few timed launches (for rocprofv3 PMC passes).
usage: python tools/gemm_one.py proj|dgrad|wgrad"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gemm_bench as gb  # noqa: E402

N = 128000
SH = {"proj": (0, 1, N, 4096, 1024), "dgrad": (0, 1, N, 1024, 4096), "wgrad": (1, 0, 4096, 1024, N)}
ta, tb, M, Nc, K = SH[sys.argv[1] if len(sys.argv) > 1 else "proj"]
ms, tf = gb.run(ta, tb, M, Nc, K, True, iters=3)
print(f"{ms:.3f} ms {tf:.0f} TF/s")
