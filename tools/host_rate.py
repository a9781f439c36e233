"""Host enqueue time per training step vs GPU time (is the Python/ctypes host path ever the
bottleneck?).  usage: python tools/host_rate.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
import torch  # noqa: E402
from mlvae_hip.engine import VAEConfig, VAEEngine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = VAEEngine(VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16"), device="cuda:0")
eng.init_default(seed=123456)
x = torch.randn(32, 500, 80, device="cuda")
lens = torch.ones(32, device="cuda")
for _ in range(3):
    eng.train_step(x, lens)
torch.cuda.synchronize()
per = []
t0 = time.perf_counter()
for _ in range(steps):
    a = time.perf_counter()
    eng.train_step(x, lens)
    per.append(time.perf_counter() - a)
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"host enqueue {t_enq / steps * 1e3:.3f} ms/step (min {min(per) * 1e3:.3f}, max {max(per) * 1e3:.3f}); "
      f"wall {t_all / steps * 1e3:.3f} ms/step")
