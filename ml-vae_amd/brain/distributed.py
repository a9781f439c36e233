"""Data-parallel launch for the recipe (the reference's run_opts surface: --distributed_launch,
--distributed_backend, ref:src/prepare_experiment.py:12,55 and SpeechBrain 0.5's DDP launch).

One process per GPU under ``python -m torch.distributed.run --nproc-per-node N train.py ...``
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the environment, MASTER_ADDR 127.0.0.1).  The
fused engine then all-reduces its flat gradient (mlvae_hip.dist); each rank reads its slice of
every global batch (world x batch_size utterances, utils/data_io); the input normaliser's batch
statistics are all-reduced; rank 0 alone writes checkpoints and logs."""
import os

import torch
import torch.distributed as dist


def init_from_env(run_opts):
    """Initialise the process group when launched distributed; sets run_opts['rank'],
    ['world_size'] and, on a GPU box, ['device'] = cuda:LOCAL_RANK.  Returns (rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 and not run_opts.get("distributed_launch", False):
        run_opts.setdefault("rank", 0)
        run_opts.setdefault("world_size", 1)
        return 0, 1
    if world <= 1:
        raise RuntimeError("--distributed_launch needs torch.distributed.run (WORLD_SIZE unset)")
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    use_gpu = torch.cuda.is_available()
    backend = run_opts.get("distributed_backend") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        local = local % torch.cuda.device_count()  # ranks beyond the visible GPUs share them (tests)
        torch.cuda.set_device(local)
        run_opts["device"] = f"cuda:{local}"
    if not dist.is_initialized():
        kw = {"device_id": torch.device("cuda", local)} if (use_gpu and backend == "nccl") else {}
        dist.init_process_group(backend, **kw)
    run_opts["rank"], run_opts["world_size"] = rank, world
    return rank, world


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_main():
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def all_reduce_sum_(t):
    """In-place sum over ranks (no-op single-process)."""
    if world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def barrier():
    if world_size() > 1:
        dist.barrier()
