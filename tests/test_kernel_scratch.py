"""The hot-path kernels keep their state in registers / LDS: no scratch (private memory) use,
from the compiler's resource-usage remarks (tools/check_scratch.py).  A GEMM epilogue that
outgrew the unroller once put gemm256's accumulators in scratch and made every weight-gradient
GEMM 2-5x slower with no test failing.  CPU-only: it compiles, it runs nothing."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOT = ["gemm_fast.hip", "heads.hip", "lstm_wide.hip", "norm.hip", "encoder.hip", "skinny.hip",
       "optim.hip", "fp8.hip", "gemm_bf16.hip", "elbo.hip"]


@pytest.mark.skipif(not shutil.which(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")), reason="no hipcc")
def test_hot_path_kernels_use_no_scratch():
    csrc = os.path.join(ROOT, "ml-vae_amd", "csrc")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_scratch.py")] +
                       [os.path.join(csrc, f) for f in HOT], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
