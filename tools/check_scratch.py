"""Scratch (private-memory) use of the HIP kernels, from the compiler's resource-usage remarks.

    python tools/check_scratch.py [source.hip ...]      (default: every csrc/*.hip)

A kernel that needs scratch keeps registers (or a private array indexed at run time) in memory:
an epilogue that outgrew the unroller once moved gemm256's 128 accumulators to scratch and made
every GEMM 2-5x slower.  Prints `kernel scratch_bytes_per_lane vgprs` for each kernel; exit
status 1 when a kernel outside ALLOWED needs scratch."""
import glob
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ml-vae_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# kernels with a known, bounded scratch use (reloaded once in the prologue, not in the loop)
ALLOWED = ("lstm_bwd_wide_kernel",)
# the forward recurrence's stamp-instrumented debug instances (DBG = true: mode bits 1-4 only,
# never the timed path)
ALLOWED_RE = (re.compile(r"lstm_fwd_wide_kernelILi\d+ELi\d+ELi\d+ELb1E"),
              # the fp8-recurrence forward (F8R): the W_hh quantization in the prologue spills,
              # the step loop has no scratch access (checked in the ISA)
              re.compile(r"lstm_fwd_wide_kernelILi\d+ELi\d+ELi\d+ELb0ELb1ELb1E"))


def usage(src):
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "--cuda-device-only",
                          "-Rpass-analysis=kernel-resource-usage", "-I" + CSRC, "-o", os.devnull, src],
                         capture_output=True, text=True, check=True).stderr
    res, name = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            vg = None
            continue
        m = re.search(r"VGPRs: (\d+)", line)
        if m and name:
            vg = int(m.group(1))
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            res.append((name, int(m.group(1)), vg))
            name = None
    return res


def main(srcs):
    bad = []
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:   # one hipcc per source
        results = list(ex.map(usage, srcs))
    for src, res in zip(srcs, results):
        for name, scratch, vg in res:
            print(f"{os.path.basename(src):18s} {name[:90]:90s} scratch {scratch:5d} vgprs {vg}")
            if scratch and not any(a in name for a in ALLOWED) and not any(r.search(name) for r in ALLOWED_RE):
                bad.append(name)
    if bad:
        print("kernels with scratch:", *bad, sep="\n  ")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or sorted(glob.glob(os.path.join(CSRC, "*.hip")))))
