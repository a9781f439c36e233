"""Benchmark: spectrogram frames/s of the VAE training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--prec bf16|fp32] [--config c3]

Headline workload (``--config c3``, the default) = the metric's configuration: the full ML-VAE
(VanillaVAE enc [80,64,64] z=32, BiLSTM 2x512 decoder with dropout 0.15, dec-FC
[1024,64,64,80]) on 80-d log-mel at T=500 with a GLOBAL batch of 256 utterances, trained data
parallel over N GPUs (strong scaling: 256/N utterances per GPU; N=1 trains all 256 on one
MI355X).  One step = one full fit_batch of the fused HIP path: forward, Gaussian-NLL ELBO,
backward, global-norm clip 5.0, Adam.  The other configs (c1, c2 = configs[1] B=32/GPU, c4) are
per-GPU workloads (weak scaling) for A/B runs.

Process model: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) every process
is one rank.  Without it, ``--gpus N`` (N > 1) makes this process a launcher that starts N
worker processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment)
before it touches the GPU, waits for them and exits with their worst status.

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
  roofline          the dominant kernel -- whichever persistent BiLSTM recurrence (forward or
                    BPTT) took the most measured time per step: HIP-event time of its launches
                    on their stream, algorithmic bytes per launch, PMC traffic from the
                    committed rocprofv3 passes (profiles/pmc_traffic.json, source named) or
                    null, and its per-step latency against the inter-CU hand-off floor
  recurrences       the same fields for both recurrences
  kernels           secondary rooflines: the two big GEMMs against the bf16 MFMA peak, the fused
                    encoder (+reparameterisation + KL) and decoder-heads (+NLL) kernels against HBM
  cpu_baseline      the CPU oracle (oracle/vae_cpu.py, pinned to reference fixtures) timed on this
                    host's cores on a bounded sample of the same model (rank 0, N=1)
  extra (N=1 only)  c2 (configs[1], B=32, bf16) and the fp32 parity mode on the headline batch
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch does not initialise the GPU)

METRIC = "spectrogram frames/sec + ELBO; 80-d log-mel B=256 at 1/2/4/8 MI355X"
GLOBAL_BATCH = 256
# name: (F, E, Z, H, L, C, batch, T, batch_is_global)
CONFIGS = {
    "c1": (64, 128, 16, 128, 2, 128, 8, 200, False),
    "c2": (80, 64, 32, 512, 2, 64, 32, 500, False),
    "c3": (80, 64, 32, 512, 2, 64, GLOBAL_BATCH, 500, True),
    "c4": (80, 64, 32, 512, 2, 64, 64, 2000, False),
    "c5": (80, 64, 32, 512, 2, 64, 64, 500, False),   # configs[4]: B=512 over 8 GPUs = 64 per GPU
}
CONFIGS["c5bf16"] = CONFIGS["c5"]   # the same per-GPU shard in bf16 (the fp8 comparison)
CONFIGS["c3h"] = (80, 64, 32, 512, 2, 64, 128, 500, False)  # the metric's B=256 over 2 GPUs: one shard
FP8 = {"c5"}             # configs[4]: fp8 e4m3 layer-1 input projection (VAEConfig.fp8)
ENC_CONV = {"c4": 5}     # configs[3]: Conv1d encoder variant (kernel size 5), modules/conv_vae.py
TIMER_EVERY = 4          # time kernels with HIP events on every 4th timed step
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3, "fp8": 5000.0}
HANDOFF_FLOOR_US = 0.8   # MI355X_MICROARCH.md handoff-1to1, idle, 8 B


def macs_per_frame(F, E, Z, H, L, C):
    enc = E * F + E * E + 2 * Z * E
    lstm = sum(2 * (4 * H * (Z if l == 0 else 2 * H) + 4 * H * H) for l in range(L))
    heads = 2 * (C * 2 * H + C * C + F * C)
    return enc + lstm + heads


def lstm_launch_bytes(B, T, H, gate_bytes=4, dg_bytes=4, dy_bytes=4):
    """Algorithmic HBM bytes of one BPTT launch (both directions) per frame: read the saved gates
    [8H] (gate_bytes: 2 = the wide path's fp16 gate buffer, 4 = fp32), read c_{t-1} [2H] (fp32)
    and dY [2H] (dy_bytes: 2 = bf16, the engine's bf16 step), write dG [8H] (dg_bytes: 2 = bf16
    in bf16 mode)."""
    return B * T * (8 * H * gate_bytes + 2 * H * 4 + 2 * H * dy_bytes + 8 * H * dg_bytes)


def lstm_fwd_layer_bytes(B, T, H, L, gate_bytes=2, h_bytes=2, drop=True, fp8=False, zin=0):
    """Algorithmic HBM bytes of each layer's forward-recurrence launch (both directions).  Per
    frame: read the input projection [8H] (gate_bytes: 2 = fp16 on the wide path), write the
    activated gates [8H] (same width), c [2H] fp32 and h [2H] (h_bytes: 2 = the bf16 GEMM
    operand); layers below the top also write dropout(h) [2H] bf16 (drop) and, in fp8 mode, its
    e4m3 copy [2H].  zin > 0: layer 0 computes its projection itself (mlvae_lstm_fwd_z) and
    reads the bf16 latent [zin]."""
    return [B * T * ((zin * 2 if (zin and l == 0) else 8 * H * gate_bytes) + 8 * H * gate_bytes + 2 * H * 4 +
                     2 * H * h_bytes + ((2 * H * 2 + (2 * H if fp8 else 0)) if (drop and l < L - 1) else 0))
            for l in range(L)]


def lstm_fwd_launch_bytes(*args, **kw):
    """The layers' forward launches averaged (the HIP-event timer averages them too)."""
    per = lstm_fwd_layer_bytes(*args, **kw)
    return sum(per) / len(per)


def lstm_launch_flops(B, T, H):
    """Recurrent MACs: per frame and direction 4H x H (h W_hh^T, or dG W_hh in BPTT)."""
    return 2 * B * T * 2 * 4 * H * H


def encoder_fwd_bytes(N, F, E, Z):
    """encoder_fwd_kernel: reads x (F fp32); writes E1, E2 (bf16, the backward's operands),
    [mu | log_var] (2Z fp32), z (Z fp32), z as bf16 [z | 1 | 0..] (Z+16 bf16) and eps (Z fp32)."""
    return N * (4 * F + 2 * 2 * E + 4 * 2 * Z + 4 * Z + 2 * (Z + 16) + 4 * Z)


def encoder_bwd_bytes(N, F, E, Z):
    """encoder_bwd_kernel: reads dz, [mu | log_var], eps (fp32), E1, E2 (bf16), x (fp32);
    writes per-block weight-gradient partials (negligible per frame)."""
    return N * (4 * Z + 4 * 2 * Z + 4 * Z + 2 * 2 * E + 4 * F)


def heads_bytes(N, F, C, H, dy_bytes=4, wg_fused=False):
    """The heads (train, the engine's fused mode): reads h (2H bf16) and x (F fp32); writes
    mu_x, log_var_x (F each, fp32), dY (2H; dy_bytes 2 = bf16, the engine's bf16 step) and, as
    bf16 (the weight-gradient GEMMs' operand precision), P1 (2C), P2m, P2v (C each), d mu_x,
    d log_var_x (F each), dP2m, dP2v (C each), dP1 (2C).  wg_fused (round 5, the heads' dW3 / dW2
    inside the heads kernel): P2, d mu_x, d log_var_x and dP2 are no longer written."""
    saved = 2 * C + 2 * C if wg_fused else 2 * C + 2 * C + 2 * F + 2 * C + 2 * C
    return N * (2 * 2 * H + 4 * F + 4 * 2 * F + dy_bytes * 2 * H + 2 * saved)


def conv_fwd_bytes(N, F, E):
    """Both Conv1d encoder layers forward (conv.hip): read x (F fp32), write E1; read E1, write E2."""
    return N * 4 * (F + 3 * E)


def conv_bwd_bytes(N, F, E):
    """The Conv1d backward region below the top layer (fp32 activations): the layer-2 input
    gradient dE1 = conv^T(dE2) * lrelu'(E1) (read dE2, E1, write dE1) and the layer-1 weight
    gradient dE1^T x (read dE1, x).  (Through round 4 this counted 5E + F per frame -- one E too
    many.)"""
    return N * 4 * (4 * E + F)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(cfg_name, budget_s=15.0):
    """The CPU oracle (torch CPU, ATen LSTM as the reference calls it) on this host, on a
    bounded sample of the same workload: whole train steps at the benchmarked shape (the
    headline's B=256, T=500), as many as fit the budget (at least one)."""
    from oracle import vae_cpu as O
    F, E, Z, H, L, C, B, T, _ = CONFIGS[cfg_name]
    threads = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", threads))
    torch.set_num_threads(max(1, min(threads, cap)))
    g = torch.Generator().manual_seed(1)
    params = O.init_params(F, E, Z, H, L, C, seed=123456, enc_conv=ENC_CONV.get(cfg_name, 0))
    x = torch.randn(B, T, F, generator=g)
    lens = torch.ones(B)
    cfg = dict(L=L, loss_type="likelihood", kld_weight=1e-3)
    state, steps, t0 = {}, 0, time.perf_counter()
    masks_shape = (L - 1, B, T, 2 * H)
    while True:
        eps = torch.randn(B, T, Z, generator=g)
        masks = (torch.rand(masks_shape, generator=g) > 0.15).float() / 0.85 if L > 1 else None
        params, _ = O.train_step(params, state, x, lens, eps, cfg, masks, impl="aten")
        steps += 1
        dt = time.perf_counter() - t0
        if dt > budget_s or steps >= 20:
            break
    return {"value": steps * B * T / dt, "unit": "frames/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu": cpu_model(),
            "sample": f"{steps} full train steps of the same model (B={B}, T={T}, fp32, ATen LSTM, "
                      f"dropout 0.15, clip+Adam) in {dt:.1f} s on {torch.get_num_threads()} host threads"}


def _pmc_table():
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def pmc_traffic(key):
    """HBM bytes per launch of kernel "<config>/<kernel>" from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, written by tools/gpu_pmc.sh + tools/pmc_summary.py), or None."""
    cfg, _, kern = key.partition("/")
    try:
        return _pmc_table().get(cfg, {}).get(kern, {}).get("hbm_bytes_per_launch")
    except AttributeError:
        return None


def pmc_source(cfg):
    """Which rocprofv3 PMC passes the config's traffic numbers came from."""
    src = _pmc_table().get(cfg, {}).get("_source")
    return {"file": "profiles/pmc_traffic.json", "config": cfg, **(src or {})}


def pmc_sum(cfg_name, roles):
    """Summed PMC bytes per launch of the launches `roles` (one region of the step), or None."""
    v = [pmc_traffic(f"{cfg_name}/{r}") for r in roles]
    return None if any(x is None for x in v) else sum(v)


def recurrence_roofline(name, what, layer_bytes, flops, ms, launches, T, cfg_name, prec):
    """HBM roofline (algorithmic bytes / HIP-event launch time) + per-step latency of one
    persistent recurrence kernel.  layer_bytes: algorithmic bytes of each layer's launch; the
    HIP-event time averages the layers' launches, so `algorithmic_bytes_per_launch` and the PMC
    `traffic` are the same layer means (per layer in `per_layer`: l0 = the bottom layer)."""
    nbytes = sum(layer_bytes) / len(layer_bytes)
    dur_s = ms * 1e-3
    achieved = nbytes / dur_s / 1e9
    step_us = ms * 1e3 / T
    per_layer = {f"l{l}": {"algorithmic_bytes": b, "traffic": pmc_traffic(f"{cfg_name}/{name}_l{l}")}
                 for l, b in enumerate(layer_bytes)}
    tl = [v["traffic"] for v in per_layer.values()]
    traffic = None if any(t is None for t in tl) else sum(tl) / len(tl)
    return {"kernel": name, "what": what, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_source": pmc_source(cfg_name), "per_layer": per_layer,
            "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": ms, "launches": launches,
            "mfma_frac": flops / dur_s / 1e12 / MFMA_PEAK_TFLOPS[prec],
            "step_latency_us": step_us, "handoff_floor_us": HANDOFF_FLOOR_US,
            "latency_frac": HANDOFF_FLOOR_US / step_us}


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_workers(n, argv):
    """Launcher mode: N worker processes of this script, one per GPU (started before this
    process touches the GPU; no exec).  Returns the worst exit status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):  # one rank failed: stop the others
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def dry_run(rank, world):
    """Process-model check without a GPU: gloo group, one all-reduce, rank 0 reports."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t)
        total = t.item()
        dist.destroy_process_group()
    else:
        total = 1.0
    if rank == 0:
        print(json.dumps({"dry_run": True, "world": world, "rank_sum": total,
                          "per_rank_batch": GLOBAL_BATCH // world}))


def make_engine(cfg_name, prec, device, world, rank, B):
    from mlvae_hip.engine import VAEConfig, VAEEngine
    F, E, Z, H, L, C, _, T, _ = CONFIGS[cfg_name]
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec=prec, enc_conv=ENC_CONV.get(cfg_name, 0),
                    fp8=cfg_name in FP8 and prec != "fp32")
    eng = VAEEngine(cfg, device=device)
    eng.init_default(seed=123456)
    if world > 1:
        from mlvae_hip import dist as mdist
        mdist.attach(eng, rank=rank, world=world, batch_per_rank=B)
    return eng


def global_batch_shard(B, T, F, rank, device):
    """This rank's utterances of the synthetic global batch (seeded, identical for every N)."""
    g = torch.Generator(device=device).manual_seed(123456)
    xg = torch.randn(B * (rank + 1), T, F, device=device, generator=g)  # rows < rank*B discarded
    return xg[rank * B:].contiguous()


def timed_run(eng, x, lens, steps, warmup, world, timers=None, norm=None):
    """Warm up, then time exactly `steps` fused train steps between barrier + synchronize
    brackets.  norm: the recipe's InputNormalization, run on the device inside every step
    (ref:src/models/test_vanilla_vae/model.py:24-25 normalises each batch before the encoder)."""
    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(warmup):
        eng.train_step(x, lens, normalizer=norm)
    barrier()
    eng.check_errors()
    t0 = time.perf_counter()
    loss = None
    for i in range(steps):
        eng.kernel_timers = timers if (timers is not None and i % TIMER_EVERY == 0) else None
        loss = eng.train_step(x, lens, normalizer=norm)
    barrier()
    dt = time.perf_counter() - t0
    eng.kernel_timers = None
    eng.check_errors()
    # a step whose numbers went non-finite is not a measurement (NaN data also draws less power,
    # so such a run can even look faster): refuse to report it
    if loss is not None and not bool(torch.isfinite(loss).all()):
        raise SystemExit(f"bench: non-finite ELBO {loss.tolist()} -- invalid run, not reported")
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], device=x.device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    return dt, loss


def secondary(kern, B, T, cfg_name, dy_bytes=4, wg_fused=False):
    """Per-kernel rooflines of the timed secondary launches (HIP events, main stream); dy_bytes:
    the width of dY the engine's heads write (2 = bf16); wg_fused: the heads computed their small
    weight gradients in-kernel (VAEEngine.heads_wgrad)."""
    F, E, Z, H, L, C, _, _, _ = CONFIGS[cfg_name]
    N = B * T
    out = {}
    gemm_flops = 2.0 * N * 8 * H * 2 * H
    wg_flops = {"wgrad_ih_l1": 2.0 * N * 8 * H * 2 * H,           # dW_ih_l1 = dG^T X   (K = frames)
                "wgrad_hh_l1": 2.0 * N * 8 * H * H,               # both directions' dW_hh_l1
                "wgrad_hh_l0": 2.0 * N * 8 * H * H}
    for name, what in (("proj_l1", "layer-1 input projection [N x 2H] x [2H x 8H] (gemm256)"),
                       ("dgrad_l1", "layer-1 dgrad [N x 8H] x [8H x 2H] + dropout bwd (gemm256)"),
                       ("wgrad_ih_l1", "layer-1 weight gradient dW_ih = dG^T X, K = frames, split-K (gemm256)"),
                       ("wgrad_hh_l1", "layer-1 dW_hh, both directions, time-shifted h (gemm256, batch 2)"),
                       ("wgrad_hh_l0", "layer-0 dW_hh, both directions, time-shifted h (gemm256, batch 2)")):
        if name in kern:
            tf = wg_flops.get(name, gemm_flops) / (kern[name] * 1e-3) / 1e12
            out[name] = {"what": what, "bound": "mfma", "avg_launch_ms": kern[name],
                         "achieved": tf, "peak": MFMA_PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
                         "frac": tf / MFMA_PEAK_TFLOPS["bf16"], "traffic": pmc_traffic(f"{cfg_name}/{name}")}
    # HBM-bound regions: the timed region's launches (PMC roles, tools/pmc_summary.py) summed, beside
    # the same region's algorithmic bytes
    for name, nbytes, roles in (
            ("encoder_fwd", encoder_fwd_bytes(N, F, E, Z), ["encoder_fwd"]),
            ("encoder_bwd", encoder_bwd_bytes(N, F, E, Z), ["encoder_bwd"]),
            ("conv_fwd", conv_fwd_bytes(N, F, E), ["conv_fwd_l1", "conv_fwd_l2"]),
            ("conv_bwd", conv_bwd_bytes(N, F, E), ["conv_dgrad", "conv_wgrad_l1"]),
            ("heads", heads_bytes(N, F, C, H, dy_bytes, wg_fused), ["heads_p1", "heads_mid", "heads_dy"])):
        if name in kern:
            gbs = nbytes / (kern[name] * 1e-3) / 1e9
            out[name] = {"bound": "hbm", "avg_launch_ms": kern[name], "achieved": gbs,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_launch": nbytes,
                         "traffic": pmc_sum(cfg_name, roles), "traffic_launches": roles}
    return out


def conv_standalone(cfg_name, device, iters=50):
    """The Conv1d encoder's kernels timed alone (HIP events) at the config's shapes on synthetic
    data: in the train step the backward shares the chip with the side-stream weight-gradient
    GEMMs, so its in-step time measures that contention, not the kernels."""
    from mlvae_hip._lib import check, lib
    F, E, Z, H, L, C, B, T, _ = CONFIGS[cfg_name]
    K, N, l = ENC_CONV[cfg_name], B * T, lib()
    s = torch.cuda.current_stream(device).cuda_stream
    g = torch.Generator(device=device).manual_seed(5)
    x, e1, de2 = (torch.randn(N, c, device=device, generator=g) for c in (F, E, E))
    w1, w2 = torch.randn(E, F, K, device=device) * 0.05, torch.randn(E, E, K, device=device) * 0.05
    b1, de1, y1 = torch.zeros(E, device=device), torch.empty(N, E, device=device), torch.empty(N, E, device=device)
    dw1, db1 = torch.empty_like(w1), torch.empty(E, device=device)
    nb = l.mlvae_conv1d_wgrad_workspace_size(B, T, F, E, K)
    ws = torch.empty(nb // 4 + 1, device=device)

    def bwd():
        check(l.mlvae_conv1d_dgrad(B, T, E, E, K, de2.data_ptr(), E, w2.data_ptr(), e1.data_ptr(), E,
                                   de1.data_ptr(), E, s))
        check(l.mlvae_conv1d_wgrad(B, T, F, E, K, de1.data_ptr(), E, x.data_ptr(), F, dw1.data_ptr(),
                                   db1.data_ptr(), ws.data_ptr(), nb, s))

    def fwd():
        check(l.mlvae_conv1d_fwd(B, T, F, E, K, x.data_ptr(), F, w1.data_ptr(), b1.data_ptr(), 1, y1.data_ptr(), E, s))

    out = {}
    for name, fn, nbytes, what in (
            ("conv_bwd", bwd, conv_bwd_bytes(N, F, E),
             "layer-2 input gradient + layer-1 weight gradient (+ slab reduce), alone"),
            ("conv_fwd_layer1", fwd, N * 4 * (F + E), "layer-1 forward (+ LeakyReLU), alone")):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(device)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize(device)
        ms = a.elapsed_time(b) / iters
        gbs = nbytes / (ms * 1e-3) / 1e9
        out[name] = {"what": what, "bound": "hbm", "avg_launch_ms": ms, "achieved": gbs, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": nbytes}
    return out


def extra_runs(args, device):
    """N=1 extras: configs[1] (c2, B=32 bf16), configs[3] (c4: Conv1d encoder, T=2000, B=64,
    bf16) and the fp32 parity mode on the headline batch."""
    out = {}
    runs = [("c2_bf16", "c2", "bf16", 10, 2), ("c4_conv_bf16", "c4", "bf16", 4, 2),
            ("c5_fp8_per_gpu", "c5", "bf16", 10, 2), ("c5_bf16_per_gpu", "c5bf16", "bf16", 10, 2)]
    if args.prec != "fp32":
        runs.append((f"{args.config}_fp32", args.config, "fp32", 3, 1))
    for key, cname, prec, steps, warm in runs:
        F, E, Z, H, L, C, B, T, _ = CONFIGS[cname]
        eng = make_engine(cname, prec, device, 1, 0, B)
        x = global_batch_shard(B, T, F, 0, device)
        lens = torch.ones(B, device=device)
        timers = {}
        from brain.features import InputNormalization
        dt, loss = timed_run(eng, x, lens, steps, warm, 1, timers if cname in ("c4", "c5", "c5bf16") else None,
                             InputNormalization())
        dyb = 2 if getattr(eng, "dy_bf16", False) else 4
        lv = loss.tolist()
        out[key] = {"global_batch": B, "seq_len": T,
                    "dtype": "fp8-e4m3 layer-1 projection/dgrad/dW_ih/dW_hh, layer-0 dW_hh, both layers' dG (layer-0 dZ / dW_ih read it), bf16 elsewhere" if cname in FP8 else prec,
                    "steps": steps,
                    "ms_per_step": dt / steps * 1e3, "frames_per_s": B * T * steps / dt,
                    "loss": lv[2]}
        if timers:
            kern = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) for k, v in timers.items()}
            if cname in ENC_CONV:
                out[key]["encoder"] = f"Conv1d K={ENC_CONV[cname]} [{F},{E},{E}]"
                out[key]["kernels"] = {k: v for k, v in secondary(kern, B, T, cname, dyb, getattr(eng, 'heads_wgrad', False)).items()
                                       if k.startswith("conv")}
                # PMC HBM bytes per launch of each conv kernel (profiles/pmc_traffic.json[c4])
                out[key]["pmc_bytes_per_launch"] = {k: pmc_traffic(f"{cname}/{k}") for k in
                                                    ("conv_fwd_l1", "conv_fwd_l2", "conv_dgrad", "conv_wgrad_l1",
                                                     "conv_wgrad_l2")}
                out[key]["pmc_source"] = pmc_source(cname)
                out[key]["kernels_standalone"] = conv_standalone(cname, device)
            else:
                sec = secondary(kern, B, T, cname, dyb, getattr(eng, 'heads_wgrad', False))
                if cname in FP8:  # against the fp8 (block-scaled) MFMA peak
                    what = {"proj_l1": "layer-1 input projection on fp8 e4m3 operands (incl. the W_ih "
                                       "scale + casts; the input arrives as e4m3 from the recurrence)",
                            "dgrad_l1": "layer-1 dgrad on fp8 e4m3 operands (dG from the BPTT, delayed "
                                        "scaling) + dropout bwd"}
                    for kk in ("proj_l1", "dgrad_l1"):
                        if kk in sec:
                            sec[kk].update(what=what[kk], peak=MFMA_PEAK_TFLOPS["fp8"])
                            sec[kk]["frac"] = sec[kk]["achieved"] / MFMA_PEAK_TFLOPS["fp8"]
                out[key]["kernels"] = {k: v for k, v in sec.items() if k in ("proj_l1", "dgrad_l1")}
                out[key]["fp8"] = cname in FP8
            out[key]["kernel_ms"] = kern
        del eng, x
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prec", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--config", default="c3", choices=list(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the N=1 c2 / fp32 extra runs")
    ap.add_argument("--dry-run", action="store_true", help="process model only (gloo, no GPU)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend of the ranks (nccl = RCCL over xGMI; gloo: the "
                         "one-GPU rehearsal of the worker path in tests/test_gpu_bench_dp.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_workers(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(rank, world)

    # one GPU per rank; ranks beyond the visible devices share them (the gloo rehearsal on a
    # one-GPU box: device_count() does not initialise the GPU)
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev
    torch.cuda.set_device(local)
    device = f"cuda:{local}"
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    F, E, Z, H, L, C, batch, T, is_global = CONFIGS[args.config]
    if is_global:
        if batch % world:
            raise SystemExit(f"global batch {batch} does not split over {world} GPUs")
        B = batch // world
    else:
        B = batch
    eng = make_engine(args.config, args.prec, device, world, rank, B)
    x = global_batch_shard(B, T, F, rank, device)   # synthetic log-mel stand-in
    lens = torch.ones(B, device=device)
    timers = {}
    from brain.features import InputNormalization   # the recipe's normaliser (model.yaml:14-15)
    norm = InputNormalization()
    dt, loss = timed_run(eng, x, lens, args.steps, args.warmup, world, timers, norm)
    ms = dt / args.steps * 1e3
    value = B * T * world * args.steps / dt
    lv = loss.tolist()
    kern = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) for k, v in timers.items()}
    launches = {k: len(v) for k, v in timers.items()}
    dyb = 2 if getattr(eng, "dy_bf16", False) else 4   # dY width the engine's bf16 step used
    zp = bool(getattr(eng, "zproj", False))             # layer 0's projection inside its forward
    wgf = bool(getattr(eng, "heads_wgrad", False))      # the heads' small weight gradients in-kernel
    del eng
    torch.cuda.empty_cache()
    if rank == 0:
        from mlvae_hip._lib import lib
        g16 = bool(lib().mlvae_lstm_gates_fp16_t(B, T, H, 1 if args.prec == "bf16" else 0))
        bf = args.prec == "bf16"
        recs = {
            "lstm_fwd": recurrence_roofline(
                "lstm_fwd", "persistent BiLSTM forward recurrence, both directions, one launch per layer",
                lstm_fwd_layer_bytes(B, T, H, L, 2 if g16 else 4, 2 if bf else 4, True,
                                     args.config in FP8 and bf, Z if (zp and g16 and bf and Z == 32) else 0),
                lstm_launch_flops(B, T, H), kern["lstm_fwd"], launches["lstm_fwd"], T, args.config, args.prec),
            "lstm_bwd": recurrence_roofline(
                "lstm_bwd", "persistent BiLSTM BPTT recurrence, both directions, one launch per layer",
                [lstm_launch_bytes(B, T, H, 2 if g16 else 4, 2 if bf else 4, dyb if g16 else 4)] * L,
                lstm_launch_flops(B, T, H), kern["lstm_bwd"], launches["lstm_bwd"], T, args.config, args.prec),
        }
        # the bench line's roofline names the kernel with the most measured time per step (both
        # recurrences run once per layer per step)
        dom = max(recs, key=lambda k: kern[k] * launches[k])
        enc_desc = f"Conv1d(K={ENC_CONV[args.config]})" if args.config in ENC_CONV else "VanillaVAE"
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong" if is_global else "weak",
            "vs_baseline": None,
            "dtype": args.prec,
            "data": "synthetic N(0,1) 80-d frames (log-mel stand-in), lens=1, globally normalised "
                    "inside every timed step by the recipe's InputNormalization on the device, "
                    "random-init weights (PyTorch default init, seed 123456)",
            "config": {"workload": f"{args.config}: {enc_desc} enc [{F},{E},{E}] z={Z}, BiLSTM "
                                   f"{L}x{H} (dropout 0.15), dec-FC [{2 * H},{C},{C},{F}], T={T}, "
                                   f"global batch {B * world} = {B}/GPU x {world}, Gaussian-NLL ELBO, "
                                   f"clip 5.0 + Adam 1e-3",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": T,
                       "parallelism": f"dp{world}"},
            "elbo": {"kld_loss": lv[0], "recon_loss": lv[1], "loss": lv[2]},
            "train_tflops": value * 6 * macs_per_frame(F, E, Z, H, L, C) / 1e12,
            "roofline": recs[dom],
            "recurrences": recs,
            "kernels": secondary(kern, B, T, args.config, dyb, wgf) if args.prec == "bf16" else {},
            "kernel_ms": kern,
        }
        if world == 1 and not args.no_extra:
            out["extra"] = extra_runs(args, device)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.config)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
