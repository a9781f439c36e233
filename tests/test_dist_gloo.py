"""Data-parallel logic (mlvae_hip/dist.py) with the gloo backend, world size 2, on CPU:
summing per-rank shares built with the global frame count reproduces the single-process
gradient of the global masked mean."""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import vae_cpu as O


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mlvae_hip import dist as mdist
    torch.manual_seed(0)
    B, T, C = 4, 10, 3
    loss = torch.rand(B, T, C)
    lens = torch.tensor([1.0, 0.7, 0.5, 0.3])
    shard = slice(rank * B // world, (rank + 1) * B // world)
    mask = O.length_to_mask(lens[shard], T)
    count = torch.tensor([int(mask.sum().item())])
    mdist.allreduce_count(count)
    # rank's share of the global masked mean and of its gradient
    share = (loss[shard] * mask.unsqueeze(-1)).sum() / (count.item() * C)
    grad = torch.zeros(B, T, C)
    grad[shard] = mask.unsqueeze(-1).expand(-1, -1, C) / (count.item() * C)
    loss3 = torch.tensor([0.0, share.item(), share.item()])
    flat = grad.reshape(-1).clone()
    buckets = grad.reshape(-1).clone()
    mdist.allreduce_step(flat, loss3)
    # the engine's two buckets (suffix during the BPTT, prefix in optimizer_step) sum the same
    split = 37
    mdist.allreduce_grad_bucket(buckets[split:])
    mdist.allreduce_grad_bucket(buckets[:split])
    assert torch.equal(buckets, flat)
    params = torch.full((5,), float(rank))
    mdist.broadcast_params(params)
    # the recurrence timeout word: set on rank 1 only, every rank must see it (and skip Adam
    # together) -- the MAX all-reduce the engine runs before the fused Adam
    err = torch.tensor([1 if rank == 1 else 0], dtype=torch.int32)
    mdist.allreduce_err(err)
    # numpy copies pickle by value (a CPU tensor is shared by fd via this process's resource
    # sharer, which may be gone before the parent unpickles it)
    q.put((rank, loss3[2].item(), flat.reshape(B, T, C).numpy().copy(), params.numpy().copy(),
           int(err.item())))
    dist.destroy_process_group()


def _free_port():
    """A port the OS reports free on 127.0.0.1 (a fixed base can collide with a lingering
    socket of an earlier run)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_two_rank_allreduce_matches_global_masked_mean():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    torch.manual_seed(0)
    B, T, C = 4, 10, 3
    loss = torch.rand(B, T, C)
    lens = torch.tensor([1.0, 0.7, 0.5, 0.3])
    ref = O.apply_lens_to_loss(loss, lens)
    lr = loss.clone().requires_grad_(True)
    O.apply_lens_to_loss(lr, lens).backward()
    for rank, l, g, params, err in res:
        g, params = torch.from_numpy(g), torch.from_numpy(params)
        assert abs(l - ref.item()) < 1e-6
        assert torch.allclose(g, lr.grad, atol=1e-7)
        assert torch.equal(params, torch.zeros(5))
        assert err == 1   # rank 0 sees rank 1's timeout: both skip the update
