"""Throughput of the Hierarchical-VAE encoder (VanillaVAE + GMMVAE + apply_weight mixing,
SURVEY.md 8(f) rank 1) on the HIP path, forward + backward, against the CPU oracle
(oracle/hvae_cpu.py, test infrastructure used here only as the timed baseline).

    python tools/bench_hvae.py [--B 32] [--T 500] [--N 4] [--steps 20]

Prints one JSON line: frames/s of modules.h_vae.HierarchicalVAE (fp32 module mode, library
Philox eps / Gumbel draws) and of the oracle on the host's threads, for the same shapes."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=500)
    ap.add_argument("--F", type=int, default=80)
    ap.add_argument("--E", type=int, default=64)
    ap.add_argument("--Z", type=int, default=32)
    ap.add_argument("--N", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from modules.h_vae import HierarchicalVAE
    torch.manual_seed(0)
    m = HierarchicalVAE([a.F, a.E, a.E], a.Z, a.N).cuda()
    x = torch.randn(a.B, a.T, a.F, device="cuda", requires_grad=True)
    pi = torch.softmax(torch.randn(a.B, a.T, 2, device="cuda"), -1).requires_grad_(True)

    def step():
        out = m(x, pi)
        loss = out["losses"]["vae_kld_loss"].sum() + out["sampled_h"].pow(2).sum()
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps

    # CPU oracle: same shapes, same work (forward + backward of the same scalar)
    from oracle import hvae_cpu as O
    threads = os.cpu_count() or 1  # the box's share: OMP_NUM_THREADS caps the machine count
    torch.set_num_threads(max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))))
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xc = x.detach().cpu().requires_grad_(True)
    pc = pi.detach().cpu().requires_grad_(True)
    eps_v, eps_g = torch.randn(a.B, a.T, a.Z), torch.randn(a.B, a.T, a.N * a.Z)
    expo = torch.empty(a.B, a.T, a.N).exponential_()
    n, t0 = 0, time.perf_counter()
    while True:
        out = O.hvae_forward(p, xc, pc, eps_v, eps_g, expo)
        (out["vae_kld_loss"].sum() + out["sampled_h"].pow(2).sum()).backward()
        n += 1
        if time.perf_counter() - t0 > 5.0 or n >= 20:
            break
    dc = (time.perf_counter() - t0) / n
    frames = a.B * a.T
    print(json.dumps({"workload": f"HierarchicalVAE enc [{a.F},{a.E},{a.E}] z={a.Z} N={a.N}, "
                                  f"B={a.B} T={a.T}, fwd+bwd, fp32 module mode",
                      "gpu_ms_per_step": dt * 1e3, "gpu_frames_per_s": frames / dt,
                      "cpu_ms_per_step": dc * 1e3, "cpu_frames_per_s": frames / dc,
                      "cpu_threads": torch.get_num_threads(), "cpu_steps": n}))


if __name__ == "__main__":
    main()
