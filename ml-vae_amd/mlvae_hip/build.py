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
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["capi.cpp", "gemm.hip", "gemm_bf16.hip", "gemm_fast.hip", "heads.hip", "skinny.hip", "encoder.hip", "lstm.hip", "lstm_wide.hip", "elbo.hip", "gmm.hip", "md.hip", "decode.hip", "conv.hip", "fp8.hip", "norm.hip", "optim.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
         "-I" + CSRC]


def _obj(src):
    return os.path.join(CSRC, "build", os.path.splitext(src)[0] + ".o")


def _stale(src):
    o = _obj(src)
    if not os.path.exists(o):
        return True
    deps = [os.path.join(CSRC, src)] + glob.glob(os.path.join(CSRC, "*.h"))
    return any(os.path.getmtime(d) > os.path.getmtime(o) for d in deps)


def _compile(src):
    o = _obj(src)
    cmd = [HIPCC] + FLAGS + ["-c", os.path.join(CSRC, src), "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return r.stderr


def build(force=False, verbose=False):
    os.makedirs(os.path.join(CSRC, "build"), exist_ok=True)
    todo = [s for s in SOURCES if force or _stale(s)]
    if todo:
        with ThreadPoolExecutor(max_workers=min(len(todo), 8)) as ex:
            for src, err in zip(todo, ex.map(_compile, todo)):
                if verbose and err.strip():
                    print(f"[{src}] {err}", file=sys.stderr)
    objs = [_obj(s) for s in SOURCES]
    if todo or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
