"""Same-process A/B of engine attributes (Python-side switches such as side_prep, zproj,
split_overlap): one engine per config, the variants alternated for ROUNDS rounds of K timed steps.
usage: python tools/step_ab.py <config> "<attr=val,...>" "<attr=val,...>" ...   ("" = defaults)"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

K, ROUNDS = 20, 4


def parse(spec):
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        out[k] = eval(v, {}, {})
    return out


def main():
    c, specs = sys.argv[1], sys.argv[2:]
    dev = torch.device("cuda:0")
    F, E, Z, H, L, C, B, T, _ = bench.CONFIGS[c]
    prec = "fp32" if c.endswith("_fp32") else "bf16"
    eng = bench.make_engine(c, prec, dev, 1, 0, B)
    x = bench.global_batch_shard(B, T, F, 0, dev)
    lens = torch.ones(B, device=dev)
    base = {k: getattr(eng, k) for s in specs for k in parse(s)}
    res = {s: [] for s in specs}
    for r in range(ROUNDS):
        for s in specs:
            for k, v in base.items():
                setattr(eng, k, v)
            for k, v in parse(s).items():
                setattr(eng, k, v)
            for _ in range(2):
                eng.train_step(x, lens)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                eng.train_step(x, lens)
            torch.cuda.synchronize()
            res[s].append((time.perf_counter() - t0) / K * 1e3)
    eng.check_errors()
    for s in specs:
        v = res[s]
        print(f"{c} [{s or 'default'}]: median {statistics.median(v):.3f} ms  ({' '.join(f'{t:.3f}' for t in v)})",
              flush=True)


if __name__ == "__main__":
    main()
