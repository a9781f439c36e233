"""MD-VAE upstream LSTMs on the HIP path:

* the unidirectional persistent recurrence (mlvae_lstm1_fwd / _bwd) against an fp64 loop, fp32
  and bf16, including a batch past one launch (chunked);
* PhonemeRecognizer and BoundaryDetector (modules/*.py over LSTMFn + csrc/md.hip) against the
  reference's own numbers (tests/golden/make_golden_md.py; Kumaraswamy uniforms injected), fp32:
  outputs 1e-5 relative-max, parameter / input gradients 1e-4 relative-max;
* the reference's boundary assert as an AssertionError.
Reference ops: ref:src/modules/phoneme_recognizer.py:9-81, ref:src/modules/boundary_detector.py:15-103."""
import ctypes

import numpy as np
import pytest
import torch

from gpu_utils import P, need_gpu, rel_err, stream
from mlvae_hip._lib import check, lib
from test_oracle_md_golden import load

pytestmark = pytest.mark.gpu


def _loop(gx, w_hh, H):
    B, T, _ = gx.shape
    h = torch.zeros(B, H, dtype=torch.float64)
    c = torch.zeros(B, H, dtype=torch.float64)
    o = []
    for t in range(T):
        g = gx[:, t] + h @ w_hh.t()
        i, f, gc, og = g.split(H, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gc)
        h = torch.sigmoid(og) * torch.tanh(c)
        o.append(h)
    return torch.stack(o, 1)


@pytest.mark.parametrize("prec,tol", [(0, 2e-5), (1, 3e-2)])
@pytest.mark.parametrize("B,T,H", [(3, 17, 16), (20, 33, 64), (32, 40, 512), (70, 9, 512), (9, 12, 128)])
def test_unidirectional_recurrence_matches_fp64_loop(prec, tol, B, T, H):
    need_gpu()
    torch.manual_seed(B * 3 + T + H)
    k = 1.0 / H ** 0.5
    w = ((torch.rand(4 * H, H) * 2 - 1) * k).double().requires_grad_(True)
    gx = (torch.randn(B, T, 4 * H, dtype=torch.float64) * 0.5).requires_grad_(True)
    y = _loop(gx, w, H)
    dy = torch.randn_like(y)
    dG, dW = torch.autograd.grad((y * dy).sum(), [gx, w])
    N = B * T
    G = gx.detach().float().reshape(N, 4 * H).cuda().contiguous()
    Cs = torch.empty(N, H, device="cuda")
    Y = torch.empty(N, H, device="cuda")
    W = w.detach().float().cuda()
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, prec, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    check(lib().mlvae_lstm1_fwd(prec, B, T, H, P(W), P(G), P(Cs), P(Y), None, P(xbuf), xb.value,
                                P(err), stream()))
    torch.cuda.synchronize()
    assert err.item() == 0
    assert rel_err(Y.view(B, T, H), y) < tol
    dY = dy.float().reshape(N, H).cuda().contiguous()
    check(lib().mlvae_lstm1_bwd(prec, B, T, H, P(W), P(G), P(Cs), P(dY), None, P(xbuf), xb.value,
                                P(err), stream()))
    torch.cuda.synchronize()
    assert err.item() == 0
    assert rel_err(G.view(B, T, 4 * H), dG) < tol * 5
    # dW_hh = sum_t dG_t^T h_{t-1}: the time-shifted weight-gradient GEMM on the 4H-wide buffers
    ws = torch.empty(lib().mlvae_gemm_workspace_size(4 * H, H, N) // 4 + 1, device="cuda")
    out = torch.empty(4 * H, H, device="cuda")
    check(lib().mlvae_gemm(prec, 1, 0, 4 * H, H, N, 1.0, P(G), 4 * H, P(Y), H, 0.0, P(out), H, None,
                           None, 0, None, 0, T, -1, P(ws), ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert rel_err(out, dW) < tol * 5


def _state(rec):
    return {k[len("param/"):]: torch.from_numpy(v) for k, v in rec.items() if k.startswith("param/")}


def _compare_grads(m, rec, x):
    named = dict(m.named_parameters())
    for k in rec:
        if k.startswith("grad/"):
            n = k[len("grad/"):]
            got = named[n].grad if named[n].grad is not None else torch.zeros_like(named[n])
            assert rel_err(got, torch.from_numpy(rec[k])) < 1e-4, n
    assert rel_err(x.grad, torch.from_numpy(rec["grad_in/x"])) < 1e-4


@pytest.mark.parametrize("name", ["md_phn_tiny", "md_phn_mid"])
def test_phoneme_recognizer_matches_reference(name):
    need_gpu()
    from modules.phoneme_recognizer import PhonemeRecognizer
    rec = load(name)
    B, T, D, H, NL, FC, n_ph, Lmax = (int(v) for v in rec["dims"])
    m = PhonemeRecognizer(D, H, NL, [H, FC, FC, n_ph + 2], n_ph)
    m.load_state_dict(_state(rec))
    m = m.cuda()
    x = torch.from_numpy(rec["x"]).cuda().requires_grad_(True)
    o = m(x, torch.from_numpy(rec["feat_lens"]).cuda(), torch.from_numpy(rec["phn"]).cuda(),
          torch.from_numpy(rec["phn_lens"]).cuda(), torch.from_numpy(rec["boundary"]).cuda())
    outs = {"out": o["out"], "bce": o["losses"]["phn_recog_bce_loss"]}
    for k, v in outs.items():
        assert rel_err(v, torch.from_numpy(rec[f"out/{k}"])) < 1e-5, k
    total = sum((v * torch.from_numpy(rec[f"cot/{k}"]).cuda()).sum() for k, v in outs.items())
    total.backward()
    torch.cuda.synchronize()
    _compare_grads(m, rec, x)


@pytest.mark.parametrize("name", ["md_bnd_tiny", "md_bnd_mid"])
def test_boundary_detector_matches_reference(name):
    need_gpu()
    from modules.boundary_detector import BoundaryDetector
    rec = load(name)
    B, T, D, H, NL, FC = (int(v) for v in rec["dims"])
    m = BoundaryDetector(D, H, NL, [H, FC, FC, 1])
    m.load_state_dict(_state(rec))
    m = m.cuda()
    x = torch.from_numpy(rec["x"]).cuda().requires_grad_(True)
    o = m(x, torch.from_numpy(rec["feat_lens"]).cuda(), torch.from_numpy(rec["boundary"]).cuda(),
          uniform_u=torch.from_numpy(rec["u"]).cuda())
    outs = {"boundary_v": o["boundary_v"], "bce": o["losses"]["boundary_bce_loss"],
            "kld": o["losses"]["boundary_kld_loss"]}
    for k, v in outs.items():
        assert rel_err(v, torch.from_numpy(rec[f"out/{k}"])) < 1e-5, k
    total = sum((v * torch.from_numpy(rec[f"cot/{k}"]).cuda()).sum() for k, v in outs.items())
    total.backward()
    torch.cuda.synchronize()
    _compare_grads(m, rec, x)


def test_boundary_philox_draws_are_uniform_and_deterministic():
    """Without injected uniforms the draws come from Philox keyed by element index: the same
    seed gives the same outputs, and the mean sample of Kumaraswamy(1, 1) is ~U(0,1)'s 1/2."""
    need_gpu()
    from mlvae_hip import ops
    n = 1 << 16
    z = torch.full((n,), 0.5413, device="cuda")  # softplus(z) = 1: alpha = beta = 1 (+1e-5)
    y = torch.zeros(n, device="cuda")
    v1, b1, k1 = ops.BoundaryHeadsFn.apply(z, z, y, None, 1234)
    v2, _, _ = ops.BoundaryHeadsFn.apply(z, z, y, None, 1234)
    torch.cuda.synchronize()
    assert torch.equal(v1, v2)
    assert abs(v1.mean().item() - 0.5) < 5e-3
    from oracle import md_cpu as M
    a = torch.nn.functional.softplus(z[:1].cpu().double()) + 1e-5
    assert rel_err(k1[:1], M.beta_kl(a, a)) < 1e-5


def test_phoneme_boundary_mismatch_raises():
    need_gpu()
    from mlvae_hip import ops
    rec = load("md_phn_tiny")
    bnd = torch.from_numpy(rec["boundary"]).clone()
    bnd[0, 1] = 1 - bnd[0, 1]
    out = torch.zeros(3, 20, 7, device="cuda")
    with pytest.raises(AssertionError):
        ops.phn_bce(out, torch.from_numpy(rec["feat_lens"]).cuda(), torch.from_numpy(rec["phn"]).cuda(),
                    torch.from_numpy(rec["phn_lens"]).cuda(), bnd.cuda())
    # and the error word was cleared: a valid call passes afterwards
    ops.phn_bce(out, torch.from_numpy(rec["feat_lens"]).cuda(), torch.from_numpy(rec["phn"]).cuda(),
                torch.from_numpy(rec["phn_lens"]).cuda(), torch.from_numpy(rec["boundary"]).cuda())
