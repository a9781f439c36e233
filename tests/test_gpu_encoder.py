"""Fused encoder (encoder.hip): forward and backward against an fp64 autograd restatement of
ref:src/modules/vanilla_vae.py:13-45 (+ FCBlock ref:src/modules/fc_block.py:4-21) on the same
bf16 GEMM operands (x, weights and the two hidden activations rounded as the kernel rounds them,
straight-through for the gradient); the in-kernel noise against mlvae_randn, bit for bit."""
import math

import pytest
import torch

from gpu_utils import P, need_gpu, norm_rel, rel_err, stream
from mlvae_hip._lib import check, lib

pytestmark = pytest.mark.gpu
E, Z, ZA = 64, 32, 48


def _params(F, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(E, F, generator=g) / math.sqrt(F), torch.randn(E, generator=g) * 0.1,
            torch.randn(E, E, generator=g) / 8, torch.randn(E, generator=g) * 0.1,
            torch.randn(2 * Z, E, generator=g) / 8, torch.randn(2 * Z, generator=g) * 0.1]


def _mask(lens, T):
    """SpeechBrain length_to_mask in fp32 (ref:src/utils/data_utils.py:86-87), flattened."""
    return (torch.arange(T).float()[None, :] < (lens.float() * T)[:, None]).reshape(-1)


def _reference(x, prm, eps, mask, dz, kl_scale):
    rnd = lambda v: v + (v.to(torch.bfloat16).double() - v).detach()
    lrelu = lambda v: torch.nn.functional.leaky_relu(v, 0.01)
    W0, b0, W1, b1, Wml, bml = [p.double().requires_grad_(True) for p in prm]
    e1 = lrelu(rnd(x.double()) @ rnd(W0).t() + b0)
    e2 = lrelu(rnd(e1) @ rnd(W1).t() + b1)
    ml = rnd(e2) @ rnd(Wml).t() + bml
    mu, lv = ml[:, :Z], ml[:, Z:]
    z = eps.double() * torch.exp(0.5 * lv) + mu
    kl = (-0.5 * (1 + lv - mu * mu - torch.exp(lv))) * mask.double()[:, None]
    count = int(mask.sum().item())
    ((z * dz.double()).sum() + kl_scale * kl.sum() / (count * Z)).backward()
    return dict(e1=e1.detach(), e2=e2.detach(), ml=ml.detach(), z=z.detach(), kl=kl.sum().item(),
                grads=[W0.grad, b0.grad, W1.grad, b1.grad, Wml.grad, bml.grad])


def _forward(B, T, F, x, prm, lens, eps=None, seed=0, offset=0, split=0):
    l = lib()
    N = B * T
    bf = dict(device="cuda", dtype=torch.bfloat16)
    o = dict(e1=torch.empty(N, E, **bf), e2=torch.empty(N, E, **bf),
             ml=torch.empty(N, 2 * Z, device="cuda"), z=torch.empty(N, Z, device="cuda"),
             zb=torch.full((N, ZA), 7.0, **bf), eps=torch.empty(N, Z, device="cuda"),
             parts=torch.empty(l.mlvae_encoder_partials_count(B, T), device="cuda"))
    d = [p.cuda() for p in prm]
    dx, dl = x.cuda(), lens.cuda()
    de = eps.cuda() if eps is not None else None
    check(l.mlvae_encoder_fwd_ex(B, T, F, E, Z, P(dx), *[P(t) for t in d],
                                 P(de) if de is not None else None, seed, offset, P(dl),
                                 o["e1"].data_ptr(), o["e2"].data_ptr(), P(o["ml"]), P(o["z"]),
                                 o["zb"].data_ptr(), ZA, None if de is not None else P(o["eps"]),
                                 P(o["parts"]), split, stream()))
    torch.cuda.synchronize()
    o["keep"] = (d, dx, dl, de)
    return o


CASES = [(3, 50, 80), (4, 300, 64), (32, 500, 80)]


def _inputs(B, T, F, seed):
    torch.manual_seed(seed)
    N = B * T
    lens = torch.rand(B) * 0.8 + 0.2
    lens[0] = 1.0
    return torch.randn(N, F), _params(F, seed), lens, torch.randn(N, Z)


@pytest.mark.parametrize("B,T,F", CASES)
def test_encoder_forward(B, T, F):
    need_gpu()
    x, prm, lens, eps = _inputs(B, T, F, B + T + F)
    ref = _reference(x, prm, eps, _mask(lens, T), torch.zeros(B * T, Z), 1.0)
    o = _forward(B, T, F, x, prm, lens, eps=eps)
    assert rel_err(o["e1"].float(), ref["e1"]) < 1e-2
    assert rel_err(o["e2"].float(), ref["e2"]) < 1e-2
    assert rel_err(o["ml"], ref["ml"]) < 5e-3
    assert rel_err(o["z"], ref["z"]) < 5e-3
    assert abs(o["parts"].double().sum().item() - ref["kl"]) <= 2e-3 * abs(ref["kl"])
    zb = o["zb"].cpu()
    assert torch.equal(zb[:, :Z], o["z"].cpu().to(torch.bfloat16))
    assert torch.all(zb[:, Z] == 1.0) and torch.all(zb[:, Z + 1:] == 0.0)


@pytest.mark.parametrize("B,T,F", CASES)
def test_encoder_forward_split_bf16(B, T, F):
    """The split-bf16 forward (mlvae_encoder_fwd_ex split = 1: every product a_hi W_hi + a_hi W_lo +
    a_lo W_hi) against the fp64 forward WITHOUT operand rounding: mu / log_var / z and the KL sums
    to ~1e-5 of fp64 (the plain bf16 forward is ~3e-3 away), e1 / e2 still saved as bf16."""
    need_gpu()
    x, prm, lens, eps = _inputs(B, T, F, 3 + B + T + F)
    mask = _mask(lens, T)
    lrelu = lambda v: torch.nn.functional.leaky_relu(v, 0.01)
    W0, b0, W1, b1, Wml, bml = [p.double() for p in prm]
    e1 = lrelu(x.double() @ W0.t() + b0)
    e2 = lrelu(e1 @ W1.t() + b1)
    ml = e2 @ Wml.t() + bml
    mu, lv = ml[:, :Z], ml[:, Z:]
    z = eps.double() * torch.exp(0.5 * lv) + mu
    kl = ((-0.5 * (1 + lv - mu * mu - torch.exp(lv))) * mask.double()[:, None]).sum().item()
    o = _forward(B, T, F, x, prm, lens, eps=eps, split=1)
    p = _forward(B, T, F, x, prm, lens, eps=eps, split=0)
    e_ml, e_plain = rel_err(o["ml"], ml), rel_err(p["ml"], ml)
    e_kl = abs(o["parts"].double().sum().item() - kl) / abs(kl)
    print(f"\nsplit encoder B={B} T={T} F={F}: ml {e_ml:.2e} (plain bf16 {e_plain:.2e}) z {rel_err(o['z'], z):.2e} "
          f"KL {e_kl:.2e}")
    assert e_ml < 5e-5 and rel_err(o["z"], z) < 5e-5 and e_kl < 2e-5
    assert e_ml < 0.05 * e_plain
    assert rel_err(o["e1"].float(), e1) < 1e-2 and rel_err(o["e2"].float(), e2) < 1e-2
    zb = o["zb"].cpu()
    assert torch.equal(zb[:, :Z], o["z"].cpu().to(torch.bfloat16))


def test_encoder_noise_matches_randn():
    need_gpu()
    B, T, F = 5, 77, 80
    x, prm, lens, _ = _inputs(B, T, F, 1)
    seed, offset = 1234567, (3 << 40) + 4160
    o = _forward(B, T, F, x, prm, lens, seed=seed, offset=offset)
    ref = torch.empty(B * T * Z, device="cuda")
    check(lib().mlvae_randn(B * T * Z, seed, offset, P(ref), stream()))
    torch.cuda.synchronize()
    assert torch.equal(o["eps"].view(-1), ref)
    mu, lv = o["ml"][:, :Z], o["ml"][:, Z:]
    assert rel_err(o["z"], o["eps"] * torch.exp(0.5 * lv) + mu) < 1e-6


@pytest.mark.parametrize("B,T,F", CASES)
def test_encoder_backward(B, T, F):
    need_gpu()
    x, prm, lens, eps = _inputs(B, T, F, 7 + B + T + F)
    N = B * T
    dz = torch.randn(N, Z) * 0.05
    kl_scale = 0.37
    mask = _mask(lens, T)
    ref = _reference(x, prm, eps, mask, dz, kl_scale)
    o = _forward(B, T, F, x, prm, lens, eps=eps)
    l = lib()
    d, dx, dl, de = o["keep"]
    ddz = dz.cuda()
    ws = torch.empty(l.mlvae_encoder_workspace_size(B, T, F, E, Z) // 4 + 1, device="cuda")
    count = torch.tensor([int(mask.sum())], dtype=torch.int32, device="cuda")
    runs = []
    for cnt in (None, count):  # count from lens, or the (data-parallel) global count
        g = [torch.full_like(t, float("nan")) for t in d]
        check(l.mlvae_encoder_bwd(B, T, F, E, Z, P(ddz), P(o["ml"]), P(de), o["e1"].data_ptr(),
                                  o["e2"].data_ptr(), P(dx), P(d[4]), P(d[2]), P(dl),
                                  cnt.data_ptr() if cnt is not None else None, kl_scale,
                                  P(g[4]), P(g[5]), P(g[2]), P(g[3]), P(g[0]), P(g[1]), P(ws),
                                  ws.numel() * 4, stream()))
        torch.cuda.synchronize()
        runs.append([t.cpu() for t in g])
    for name, gk, r in zip(("W0", "b0", "W1", "b1", "Wml", "bml"), runs[0], ref["grads"]):
        assert norm_rel(gk, r) < 2e-2, (name, norm_rel(gk, r))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
