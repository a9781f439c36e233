"""Is the c3 train step host-bound anywhere?  Times the host side of eng.train_step (the Python
engine issuing ~50 launches) against the device's step time.  usage: python tools/cpu_overhead.py [cfg]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    dev = torch.device("cuda:0")
    F, E, Z, H, L, C, B, T, _ = bench.CONFIGS[cfg]
    eng = bench.make_engine(cfg, "bf16", dev, 1, 0, B)
    x = bench.global_batch_shard(B, T, F, 0, dev)
    lens = torch.ones(B, device=dev)
    from brain.features import InputNormalization
    norm = InputNormalization()
    for _ in range(5):
        eng.train_step(x, lens, normalizer=norm)
    torch.cuda.synchronize()
    n = 20
    host = []
    t0, c0 = time.perf_counter(), time.process_time()
    for _ in range(n):
        h0 = time.perf_counter()
        eng.train_step(x, lens, normalizer=norm)
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2, c2 = time.perf_counter(), time.process_time()
    host.sort()
    print(f"{cfg}: {n} steps wall {1e3 * (t2 - t0) / n:.3f} ms/step; host enqueue per step median "
          f"{1e3 * host[n // 2]:.3f} max {1e3 * host[-1]:.3f} ms; loop returned after {1e3 * (t1 - t0):.1f} ms, "
          f"drained at {1e3 * (t2 - t0):.1f} ms; process CPU {1e3 * (c2 - c0) / n:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
