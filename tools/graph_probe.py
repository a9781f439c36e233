"""Probe (round 5): what would capturing the whole train step in a HIP graph
save?  Times K eager train steps, then captures ONE step in a torch.cuda.CUDAGraph and times K
replays.  Timing only: a replay re-runs the captured step with its per-step host scalars frozen
(dropout / eps seeds), so it is not a training path.
usage: python tools/graph_probe.py [config ...]   (default c2 c3)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def main():
    cfgs = sys.argv[1:] or ["c2", "c3"]
    dev = torch.device("cuda:0")
    K = 20
    for c in cfgs:
        F, E, Z, H, L, C, B, T, _ = bench.CONFIGS[c]
        eng = bench.make_engine(c, "bf16", dev, 1, 0, B)
        x = bench.global_batch_shard(B, T, F, 0, dev)
        lens = torch.ones(B, device=dev)
        step = lambda: eng.train_step(x, lens)
        for _ in range(3):
            step()
        eager = [timed(step, K) for _ in range(2)]
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            step()
        torch.cuda.synchronize()
        eng.check_errors()
        graph = [timed(g.replay, K) for _ in range(2)]
        eager2 = timed(step, K)
        eng.check_errors()
        print(f"{c}: eager {eager[0]:.3f} / {eager[1]:.3f} / {eager2:.3f} ms   graph replay "
              f"{graph[0]:.3f} / {graph[1]:.3f} ms   (B={B} T={T})", flush=True)


if __name__ == "__main__":
    main()
