"""Build libmlvae.so (gfx950) in-tree with hipcc: one object per source, then link.

    python -m mlvae_hip.build          (from ml-vae_amd/)
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(HERE, "libmlvae.so")
# --diag: the diagnostics build (MLVAE_DIAG: recurrence phase stamps and debug-mode timing
# variants, csrc/lstm_common.h) -> libmlvae_diag.so, loaded by the tools through MLVAE_LIB_PATH
DIAG_OUT = os.path.join(HERE, "libmlvae_diag.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["capi.cpp", "gemm.hip", "gemm_bf16.hip", "gemm_fast.hip", "heads.hip", "skinny.hip", "encoder.hip", "lstm.hip", "lstm_wide.hip", "elbo.hip", "gmm.hip", "md.hip", "decode.hip", "conv.hip", "fp8.hip", "norm.hip", "optim.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
         "-I" + CSRC]


def _obj(src, diag=False):
    return os.path.join(CSRC, "build_diag" if diag else "build", os.path.splitext(src)[0] + ".o")


def _stale(src, diag=False):
    o = _obj(src, diag)
    if not os.path.exists(o):
        return True
    deps = [os.path.join(CSRC, src)] + glob.glob(os.path.join(CSRC, "*.h"))
    return any(os.path.getmtime(d) > os.path.getmtime(o) for d in deps)


def _compile(src, diag=False):
    o = _obj(src, diag)
    cmd = [HIPCC] + FLAGS + (["-DMLVAE_DIAG=1"] if diag else []) + ["-c", os.path.join(CSRC, src), "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return r.stderr


def build(force=False, verbose=False, diag=False):
    os.makedirs(os.path.join(CSRC, "build_diag" if diag else "build"), exist_ok=True)
    out = DIAG_OUT if diag else OUT
    todo = [s for s in SOURCES if force or _stale(s, diag)]
    if todo:
        with ThreadPoolExecutor(max_workers=min(len(todo), 8)) as ex:
            for src, err in zip(todo, ex.map(lambda s_: _compile(s_, diag), todo)):
                if verbose and err.strip():
                    print(f"[{src}] {err}", file=sys.stderr)
    objs = [_obj(s, diag) for s in SOURCES]
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
