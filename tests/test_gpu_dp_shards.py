"""Data-parallel exactness on one GPU: two VAEEngine shards with the data-parallel hooks
(global utterance offset for eps, all-reduced valid-frame count) whose summed gradients and
losses must equal one engine on the whole batch.  The collective
itself is replaced by an explicit sum; its gloo path is tests/test_dist_gloo.py."""
import pytest
import torch

from gpu_utils import need_gpu
from mlvae_hip import dist as mdist
from mlvae_hip.engine import VAEConfig, VAEEngine
from oracle import vae_cpu as O

pytestmark = pytest.mark.gpu


def test_two_shards_sum_to_full_batch(monkeypatch):
    need_gpu()
    F, E, Z, H, L, C, B, T = 16, 16, 8, 32, 2, 16, 6, 20
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.0, prec="fp32")
    params = O.init_params(F, E, Z, H, L, C, seed=3)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, T, F, generator=g).cuda()
    lens = torch.tensor([1.0, 0.8, 0.55, 1.0, 0.3, 0.9]).cuda()

    full = VAEEngine(cfg, params=params)
    wf = full.forward(x, lens, train=True)
    full.backward(wf)
    torch.cuda.synchronize()

    # the all-reduce of the frame count, done by hand: every shard sees the global count
    total = int(O.length_to_mask(lens.cpu(), T).sum().item())
    monkeypatch.setattr(mdist, "allreduce_count", lambda c, group=None: c.fill_(total))
    grads, losses = [], []
    for r, sl in enumerate((slice(0, B // 2), slice(B // 2, B))):
        eng = VAEEngine(cfg, params=params)
        eng.world, eng.rank = 2, r   # equal shards: the engine starts rank r's at r * B/2
        eng.bucket_allreduce = False  # no collective here: the shards are summed by hand
        w = eng.forward(x[sl].contiguous(), lens[sl].contiguous(), train=True)
        eng.backward(w)
        torch.cuda.synchronize()
        eng.check_errors()
        assert eng.global_offset == sl.start
        grads.append(eng.grad.clone())
        losses.append(w.loss.clone())
    gsum = grads[0] + grads[1]
    lsum = losses[0] + losses[1]
    assert torch.allclose(lsum, wf.loss, rtol=1e-5, atol=1e-7), (lsum, wf.loss)
    scale = full.grad.abs().max().item()
    assert (gsum - full.grad).abs().max().item() <= 1e-5 * scale


def test_bucketed_allreduce_sees_final_gradients(monkeypatch):
    """world = 2 on one GPU with a stand-in collective that doubles its bucket on the stream it
    is issued on: the suffix bucket (top LSTM layer + heads) goes out on the communication
    stream during the bottom layer's BPTT, the prefix in optimizer_step.  Both must see the
    final gradients: the result is exactly 2x a single engine's (bf16 path, side streams on)."""
    need_gpu()
    F, E, Z, H, L, C, B, T = 80, 64, 32, 128, 2, 64, 4, 60
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.0, prec="bf16")
    params = O.init_params(F, E, Z, H, L, C, seed=3)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B, T, F, generator=g).cuda()
    eps = torch.randn(B, T, Z, generator=g).cuda()
    lens = torch.tensor([1.0, 0.8, 0.55, 0.9]).cuda()
    ref = VAEEngine(cfg, params=params)
    wr = ref.forward(x, lens, eps=eps, train=True)
    ref.backward(wr)
    torch.cuda.synchronize()
    monkeypatch.setattr(mdist, "allreduce_count", lambda c, group=None: c)
    monkeypatch.setattr(mdist, "allreduce_grad_bucket", lambda b, group=None: b.mul_(2.0))
    monkeypatch.setattr(mdist, "allreduce_loss", lambda l, group=None: l.mul_(2.0))
    monkeypatch.setattr(mdist, "allreduce_err", lambda e, group=None: e)
    eng = VAEEngine(cfg, params=params)
    eng.world = 2
    w = eng.forward(x, lens, eps=eps, train=True)
    eng.backward(w)
    assert eng._ar_pending
    eng._allreduce_grads(w)
    torch.cuda.synchronize()
    eng.check_errors()
    assert torch.equal(eng.grad, 2.0 * ref.grad)
    assert torch.equal(w.loss, 2.0 * wr.loss)
