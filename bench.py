"""Benchmark: spectrogram frames/s of the VAE training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--prec bf16|fp32] [--config c2]

N=1 workload = BASELINE.json configs[1]: full ML-VAE enc/dec on 80-d log-mel, T=500, B=32
per GPU, dropout 0.15 (train mode), Adam + clip 5.0 -- one step = one full fit_batch.
For N>1 (launched by torch.distributed.run) every rank trains its own B=32 shard of the
global batch (weak scaling; c3 = 8 x 32 = 256) and gradients are all-reduced over RCCL.
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

CONFIGS = {
    # name: (F, E, Z, H, L, C, B_per_gpu, T)
    "c1": (64, 128, 16, 128, 2, 128, 8, 200),
    "c2": (80, 64, 32, 512, 2, 64, 32, 500),
    "c4": (80, 64, 32, 512, 2, 64, 64, 2000),
}


def macs_per_frame(F, E, Z, H, L, C):
    enc = E * F + E * E + 2 * Z * E
    lstm = 0
    for l in range(L):
        din = Z if l == 0 else 2 * H
        lstm += 2 * (4 * H * din + 4 * H * H)
    heads = 2 * (C * 2 * H + C * C + F * C)
    return enc + lstm + heads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prec", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--config", default="c2", choices=list(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from mlvae_hip.engine import VAEConfig, VAEEngine
    F, E, Z, H, L, C, B, T = CONFIGS[args.config]
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec=args.prec)
    eng = VAEEngine(cfg)
    from oracle import vae_cpu as O  # only for the reference-default initial weights
    eng.load_reference_params(O.init_params(F, E, Z, H, L, C, seed=123456))
    if world > 1:
        from mlvae_hip import dist as mdist
        mdist.attach(eng, rank=rank, world=world, batch_per_rank=B)
    g = torch.Generator(device="cuda").manual_seed(123456 + rank)
    x = torch.randn(B, T, F, device="cuda", generator=g)
    lens = torch.ones(B, device="cuda")

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        eng.train_step(x, lens)
    barrier()
    eng.check_errors()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = eng.train_step(x, lens)
    barrier()
    dt = time.perf_counter() - t0
    eng.check_errors()
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    ms = dt / args.steps * 1e3
    frames = B * T * world * args.steps
    value = frames / dt
    lv = loss.tolist()
    if rank == 0:
        out = {
            "metric": "spectrogram frames/sec (VAE train step) + ELBO",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.prec,
            "data": "synthetic N(0,1) 80-d frames, lens=1, random-init weights",
            "config": {"workload": f"{args.config}: ML-VAE enc {E}x2, z={Z}, BiLSTM {L}x{H}, "
                                   f"dec-FC {C}, F={F}, T={T}, B={B}/GPU, Adam+clip5, dropout 0.15",
                       "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}"},
            "elbo": {"kld_loss": lv[0], "recon_loss": lv[1], "loss": lv[2]},
            "train_tflops": value * 6 * macs_per_frame(F, E, Z, H, L, C) / 1e12,
        }
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
