"""Runtime behaviour of the fused step on the GPU: failure detection (non-finite skip and
patience, the recurrence err word), workspace reuse across padded lengths, Adam state
save/load against torch.optim.Adam, and data parallelism through the real engine with a real
collective (two gloo ranks sharing the one GPU)."""
import os

import pytest
import torch

from gpu_utils import need_gpu
from mlvae_hip.engine import VAEConfig, VAEEngine
from oracle import vae_cpu as O

pytestmark = pytest.mark.gpu

TINY = dict(F=16, E=16, Z=8, H=32, L=2, C=16)


def _tiny_cfg(prec="fp32", dropout=0.0):
    return VAEConfig(dropout=dropout, prec=prec, **TINY)


def test_nonfinite_loss_skips_update_and_patience_raises():
    """check_gradients on the fused path (ref:src/models/md_model.py:82): a NaN loss leaves the
    parameters and Adam state untouched and advances the device counter; more than
    nonfinite_patience of them in a stage raises ValueError at the stage-end check."""
    need_gpu()
    cfg = _tiny_cfg()
    params = O.init_params(16, 16, 8, 32, 2, 16, seed=3)
    eng = VAEEngine(cfg, params=params)
    B, T = 3, 10
    x = torch.randn(B, T, cfg.F).cuda()
    lens = torch.ones(B).cuda()
    eng.train_step(x, lens)
    torch.cuda.synchronize()
    before = (eng.flat.clone(), eng.exp_avg.clone(), int(eng.step_ctr.item()))
    xbad = x.clone()
    xbad[1, 4, 2] = float("nan")
    for i in range(3):
        loss = eng.train_step(xbad, lens)
        torch.cuda.synchronize()
        assert not torch.isfinite(loss[2]).item()
        assert torch.equal(eng.flat, before[0]) and torch.equal(eng.exp_avg, before[1])
        assert int(eng.step_ctr.item()) == before[2] and int(eng.nonfinite_ctr.item()) == i + 1
    assert eng.check_health(nonfinite_patience=3) == 3      # 3 <= patience: no raise
    for _ in range(4):
        eng.train_step(xbad, lens)
    with pytest.raises(ValueError, match="patience"):
        eng.check_health(nonfinite_patience=3)
    eng.train_step(x, lens)                                  # a finite batch trains again
    torch.cuda.synchronize()
    assert int(eng.step_ctr.item()) == before[2] + 1


def test_err_word_raises_at_the_stage_check():
    need_gpu()
    eng = VAEEngine(_tiny_cfg())
    eng.err.fill_(1)
    with pytest.raises(RuntimeError, match="timed out"):
        eng.check_health()


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_err_word_mid_stage_leaves_weights_and_adam_state_untouched(prec):
    """A recurrence hand-off timeout (the err word, set here as the kernels would set it) in the
    middle of a stage: the fused Adam reads the word on the device and skips every update from
    then on, counted in err_skips apart from non-finite losses; the stage-end check raises."""
    need_gpu()
    eng = VAEEngine(_tiny_cfg(prec), params=O.init_params(16, 16, 8, 32, 2, 16, seed=4))
    B, T = 3, 10
    x = torch.randn(B, T, 16).cuda()
    lens = torch.ones(B).cuda()
    eng.train_step(x, lens)                 # a good step first: the state moves
    torch.cuda.synchronize()
    before = [t.clone() for t in (eng.flat, eng.exp_avg, eng.exp_avg_sq)]
    step = int(eng.step_ctr.item())
    eng.err.fill_(1)                         # the timeout
    for _ in range(3):
        eng.train_step(x, lens)
    torch.cuda.synchronize()
    for a, b in zip(before, (eng.flat, eng.exp_avg, eng.exp_avg_sq)):
        assert torch.equal(a, b)
    assert int(eng.step_ctr.item()) == step and int(eng.err_skips.item()) == 3
    assert int(eng.nonfinite_ctr.item()) == 0
    with pytest.raises(RuntimeError, match="skipped \\(3 steps\\)"):
        eng.check_health()


def test_varying_padded_length_reuses_workspace_and_matches_oracle():
    """PaddedBatch's Tmax changes every batch: the engine reuses its pooled workspace (no
    reallocation once the largest B*T has been seen) and each step still matches the oracle,
    Adam state carried across steps."""
    need_gpu()
    cfg = _tiny_cfg()
    params = O.init_params(16, 16, 8, 32, 2, 16, seed=11)
    eng = VAEEngine(cfg, params=params)
    g = torch.Generator().manual_seed(4)
    state, ref = {}, params
    sizes = []
    for T in (20, 35, 12, 35, 28):
        x = torch.randn(3, T, 16, generator=g)
        eps = torch.randn(3, T, 8, generator=g)
        lens = torch.tensor([1.0, 0.6, 0.85])
        eng.train_step(x.cuda(), lens.cuda(), eps=eps.cuda())
        torch.cuda.synchronize()
        eng.check_errors()
        ref, _ = O.train_step(ref, state, x, lens, eps, dict(L=2, loss_type="likelihood", kld_weight=1e-3))
        worst = max((eng.view(k).cpu() - v).abs().max().item() for k, v in ref.items())
        assert worst < 2e-5, (T, worst)
        sizes.append(eng._pool.nbytes())
    assert sizes[2] == sizes[1] and sizes[3] == sizes[1] and sizes[4] == sizes[1]


def test_hip_adam_save_load_matches_torch_adam():
    """mlvae_hip.optim.Adam: two parameter groups with different lr, save -> load into a fresh
    optimizer -> keep stepping; must track torch.optim.Adam (bias corrections resume)."""
    need_gpu()
    from mlvae_hip.optim import Adam
    torch.manual_seed(0)
    init = [torch.randn(37, 5), torch.randn(64), torch.randn(8, 8)]
    grads = [[torch.randn_like(t) for t in init] for _ in range(6)]

    def run(opt_cls, steps, params=None, sd=None):
        ps = params or [torch.nn.Parameter(t.clone().cuda()) for t in init]
        opt = opt_cls([{"params": ps[:2], "lr": 1e-2}, {"params": ps[2:], "lr": 3e-3}])
        if sd is not None:
            opt.load_state_dict(sd)
        for gs in steps:
            for p, gr in zip(ps, gs):
                p.grad = gr.cuda()
            opt.step()
        return ps, opt
    ref_p, _ = run(torch.optim.Adam, grads)
    p1, o1 = run(Adam, grads[:3])
    sd = o1.state_dict()
    p2, _ = run(Adam, grads[3:], params=[torch.nn.Parameter(p.detach().clone()) for p in p1], sd=sd)
    for a, b in zip(p2, ref_p):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()
    # and a torch.optim.Adam checkpoint resumes in the HIP Adam
    t_p, t_o = run(torch.optim.Adam, grads[:3])
    p3, _ = run(Adam, grads[3:], params=[torch.nn.Parameter(p.detach().clone()) for p in t_p],
                sd=t_o.state_dict())
    for a, b in zip(p3, ref_p):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------- data parallel, real collective
def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlvae_hip import dist as mdist
    from mlvae_hip.engine import VAEConfig, VAEEngine
    from oracle import vae_cpu as O
    cfg = VAEConfig(F=16, E=16, Z=8, H=32, L=2, C=16, dropout=0.15, prec="fp32")
    params = O.init_params(16, 16, 8, 32, 2, 16, seed=21 + rank)   # rank 1 differs: broadcast fixes it
    eng = VAEEngine(cfg, params=params, seed=99)
    B, T = 2, 14
    mdist.attach(eng, rank=rank, world=world, batch_per_rank=B)
    g = torch.Generator().manual_seed(8)
    xg = torch.randn(B * world, T, 16, generator=g)
    lg = torch.tensor([1.0, 0.7, 0.45, 0.9])
    sl = slice(rank * B, (rank + 1) * B)
    losses = []
    for _ in range(2):
        losses.append(eng.train_step(xg[sl].cuda(), lg[sl].cuda()).clone())
    torch.cuda.synchronize()
    eng.check_errors()
    # numpy copies pickle by value: a CPU tensor in a spawn queue is shared by file descriptor
    # through this process's resource sharer, which is gone once it exits (GPUTEST r05)
    q.put((rank, eng.flat.cpu().numpy().copy(), torch.stack(losses).cpu().numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def _err_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlvae_hip import dist as mdist
    from mlvae_hip.engine import VAEConfig, VAEEngine
    from oracle import vae_cpu as O
    cfg = VAEConfig(F=16, E=16, Z=8, H=32, L=2, C=16, dropout=0.0, prec="fp32")
    eng = VAEEngine(cfg, params=O.init_params(16, 16, 8, 32, 2, 16, seed=5), seed=3)
    B, T = 2, 10
    mdist.attach(eng, rank=rank, world=world, batch_per_rank=B)
    g = torch.Generator().manual_seed(2)
    xg = torch.randn(B * world, T, 16, generator=g)
    sl = slice(rank * B, (rank + 1) * B)
    eng.train_step(xg[sl].cuda(), torch.ones(B).cuda())   # a good step: both replicas move
    torch.cuda.synchronize()
    before = eng.flat.cpu()
    if rank == 1:
        eng.err.fill_(1)                                   # rank 1's recurrence timed out
    for _ in range(2):
        eng.train_step(xg[sl].cuda(), torch.ones(B).cuda())
    torch.cuda.synchronize()
    q.put((rank, before.numpy().copy(), eng.flat.cpu().numpy().copy(), int(eng.err.item()),
           int(eng.err_skips.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_a_timeout_on_one_rank_skips_the_update_on_every_rank():
    """the fused Adam's skip-on-timeout decision must be global.  Rank 1's err word
    is set after one good step; both ranks then skip every update (the word is MAX-reduced with
    the gradients), so the replicas keep identical weights instead of diverging."""
    need_gpu()
    import torch.multiprocessing as mp
    from test_dist_gloo import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_err_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    res = [(r[0], torch.from_numpy(r[1]), torch.from_numpy(r[2])) + tuple(r[3:]) for r in res]
    for rank, before, after, err, skips in res:
        assert err == 1 and skips == 2, (rank, err, skips)
        assert torch.equal(before, after), rank
    assert torch.equal(res[0][2], res[1][2])


def test_two_gloo_ranks_through_the_engine_equal_one_engine_on_the_global_batch():
    """SURVEY.md 8(e)(i)-(iii) with a real collective: two ranks (gloo on CUDA tensors, one GPU)
    each train their shard with the bucketed all-reduce live (suffix bucket on the comm stream
    during the lower layer's BPTT); after two steps their parameters equal one engine's on the
    whole batch (same global eps / dropout streams, global masked mean, global clip)."""
    need_gpu()
    import torch.multiprocessing as mp
    from test_dist_gloo import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    cfg = VAEConfig(F=16, E=16, Z=8, H=32, L=2, C=16, dropout=0.15, prec="fp32")
    eng = VAEEngine(cfg, params=O.init_params(16, 16, 8, 32, 2, 16, seed=21), seed=99)
    g = torch.Generator().manual_seed(8)
    xg = torch.randn(4, 14, 16, generator=g).cuda()
    lg = torch.tensor([1.0, 0.7, 0.45, 0.9]).cuda()
    losses = [eng.train_step(xg, lg).clone() for _ in range(2)]
    torch.cuda.synchronize()
    full = eng.flat.cpu()
    for rank, flat, ls in res:
        flat, ls = torch.from_numpy(flat), torch.from_numpy(ls)
        assert torch.allclose(ls, torch.stack(losses).cpu(), rtol=2e-5, atol=1e-7), (rank, ls, losses)
        assert (flat - full).abs().max().item() < 2e-6, (rank, (flat - full).abs().max().item())
