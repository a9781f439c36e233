"""GMM-VAE / Hierarchical-VAE encoders on the HIP path (modules/gmm_vae.py, modules/h_vae.py over
libmlvae's gmm_latent + apply_weight kernels) against the reference's own numbers
(tests/golden/make_golden_hvae.py fixtures, eps and Gumbel draws injected), fp32.

Tolerances: outputs 1e-5 relative-max, parameter / input gradients 1e-4 relative-max."""
import json
import os

import numpy as np
import pytest
import torch

from gpu_utils import P, need_gpu, rel_err, stream
from test_oracle_hvae_golden import GMM_CASES, HVAE_CASES, load

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _module(meta, params):
    if meta["kind"] == "gmm":
        from modules.gmm_vae import GMMVAE
        m = GMMVAE([meta["F"], meta["E"], meta["E"]], meta["Z"], meta["N"])
    else:
        from modules.h_vae import HierarchicalVAE
        m = HierarchicalVAE([meta["F"], meta["E"], meta["E"]], meta["Z"], meta["N"])
    m.load_state_dict(dict(params))
    return m.cuda()


@pytest.mark.parametrize("case", GMM_CASES + HVAE_CASES)
def test_forward_backward_match_reference(case):
    need_gpu()
    meta, params, ins, outs, cots, grads, grads_in = load(case)
    m = _module(meta, params)
    x = ins["x"].cuda().requires_grad_(True)
    leaves = {"x": x}
    if meta["kind"] == "gmm":
        out = m(x, eps=ins["eps"].cuda(), expo=ins["expo"].cuda())
    else:
        pi = ins["pi"].cuda().requires_grad_(True)
        leaves["pi"] = pi
        out = m(x, pi, eps_v=ins["eps_v"].cuda(), eps_g=ins["eps_g"].cuda(),
                expo=ins["expo"].cuda())
        out = {**{k: v for k, v in out.items() if k != "losses"}, **out["losses"]}
    assert set(out) == set(outs)
    for k, v in outs.items():
        assert rel_err(out[k], v) < 1e-5, k
    total = sum((out[k] * cots[k].cuda()).sum() for k in outs)
    total.backward()
    torch.cuda.synchronize()
    named = dict(m.named_parameters())
    for k, g in grads.items():
        got = named[k].grad if named[k].grad is not None else torch.zeros_like(named[k])
        assert rel_err(got, g) < 1e-4, k
    for k, g in grads_in.items():
        assert rel_err(leaves[k].grad, g) < 1e-4, k


def test_apply_weight_matches_reference_and_torch():
    need_gpu()
    from utils.data_utils import apply_weight
    d = np.load(os.path.join(GOLDEN, "apply_weight.npz"), allow_pickle=False)
    for tag in ("flat", "split"):
        x, w, y = (torch.from_numpy(d[f"{tag}/{k}"]) for k in "xwy")
        assert rel_err(apply_weight(x.cuda(), w.cuda()), y) < 1e-6
    # gradients against a plain torch fp32 restatement, ragged C (not a multiple of 64)
    g = torch.Generator().manual_seed(3)
    B, T, N, C = 3, 33, 5, 70
    x = torch.randn(B, T, N * C, generator=g)
    w = torch.softmax(torch.randn(B, T, N, generator=g), -1)
    dy = torch.randn(B, T, C, generator=g)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    (wr.unsqueeze(-1) * xr.view(B, T, N, C)).sum(2).backward(dy)
    xd, wd = x.cuda().requires_grad_(True), w.cuda().requires_grad_(True)
    apply_weight(xd, wd).backward(dy.cuda())
    assert rel_err(xd.grad, xr.grad) < 1e-6
    assert rel_err(wd.grad, wr.grad) < 1e-5


def test_philox_gumbel_draw_is_categorical():
    """Library Gumbel draws (no injection): hard weights are one-hot and, by the Gumbel-max
    property, argmax frequencies follow softmax(logits) whatever tau is."""
    need_gpu()
    from mlvae_hip._lib import check, lib
    rows, N, Z = 200_000, 4, 1
    logits = torch.tensor([0.0, 1.0, 2.0, -1.0])
    Pm = torch.zeros(rows, 4 * N * Z + N)
    Pm[:, 4 * N * Z:] = logits
    Pm = Pm.cuda()
    eps = torch.zeros(rows, N * Z, device="cuda")
    z, kl = torch.empty_like(eps), torch.empty_like(eps)
    w = torch.empty(rows, N, device="cuda")
    ys = torch.empty_like(w)
    check(lib().mlvae_gmm_latent_fwd(rows, N, Z, P(Pm), Pm.shape[1], P(eps), None, 1234, 0, 0.1,
                                     P(z), P(kl), P(w), P(ys), stream()), "gmm_latent_fwd")
    torch.cuda.synchronize()
    w = w.cpu()
    assert torch.isfinite(w).all()
    assert ((w - w.round()).abs() < 1e-6).all()
    assert torch.allclose(w.sum(-1), torch.ones(rows), atol=1e-6)
    freq = w.round().mean(0)
    assert (freq - torch.softmax(logits, 0)).abs().max() < 0.01, freq


def test_gmm_latent_rejects_bad_shapes():
    need_gpu()
    from mlvae_hip._lib import lib
    l = lib()
    assert l.mlvae_gmm_latent_fwd(4, 0, 2, None, 10, None, None, 0, 0, 0.1, None, None, None,
                                  None, stream()) != 0
    assert l.mlvae_gmm_latent_fwd(4, 2, 2, None, 9, None, None, 0, 0, 0.1, None, None, None,
                                  None, stream()) != 0  # ldp < 4*N*Z + N
    assert l.mlvae_apply_weight_fwd(4, 2, 3, None, 5, None, None, 3, stream()) != 0
