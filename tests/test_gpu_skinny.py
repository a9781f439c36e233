"""Skinny products of the bottom LSTM layer (skinny.hip): dZ = dG W_ih (NT) and
dW_ih | bias = dG^T [z | 1] (TN, fixed-order frame-split reduce), against fp64 products of the
same bf16 operands (ref:src/modules/decoder.py:14-15,22, the layer-0 input projection's autograd)."""
import pytest
import torch

from gpu_utils import P, need_gpu, rel_err, stream
from mlvae_hip._lib import check, lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(16000, 32, 4096), (1000, 16, 64), (77, 48, 256), (300, 64, 96),
                                   (65637, 32, 1024), (66000, 48, 256), (65536, 16, 512)])
def test_skinny_nt(M, N, K):
    need_gpu()
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K).to(torch.bfloat16)
    Bt = torch.randn(N, K).to(torch.bfloat16)
    ref = A.double() @ Bt.double().t()
    dA, dB = A.cuda(), Bt.cuda()
    C = torch.full((M, N), float("nan"), device="cuda")
    check(lib().mlvae_skinny_nt(M, N, K, dA.data_ptr(), K, dB.data_ptr(), K, P(C), N, stream()))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 1e-5


@pytest.mark.parametrize("M,K,nw,NB,bias", [(4096, 16000, 32, 48, True), (2048, 1000, 32, 48, True),
                                            (512, 130, 16, 16, False), (256, 64, 40, 64, True)])
def test_skinny_tn(M, K, nw, NB, bias):
    need_gpu()
    torch.manual_seed(M + K + nw)
    A = torch.randn(K, M).to(torch.bfloat16)          # dG [frames, gate rows]
    Bm = torch.zeros(K, NB)
    Bm[:, :nw] = torch.randn(K, nw)
    if bias:
        Bm[:, nw] = 1.0                                # the ones column of [z | 1 | 0 ...]
    Bm = Bm.to(torch.bfloat16)
    ref = A.double().t() @ Bm.double()                # [M, NB]
    l = lib()
    dA, dB = A.cuda(), Bm.cuda()
    ws = torch.empty(l.mlvae_skinny_tn_workspace_size(M, NB, K) // 4 + 1, device="cuda")
    outs = []
    for _ in range(2):
        W = torch.full((M, nw), float("nan"), device="cuda")
        b1 = torch.full((M,), float("nan"), device="cuda")
        b2 = torch.full((M,), float("nan"), device="cuda")
        check(l.mlvae_skinny_tn(M, NB, K, dA.data_ptr(), M, dB.data_ptr(), NB, nw, P(W),
                                P(b1) if bias else None, P(b2) if bias else None, P(ws),
                                ws.numel() * 4, stream()))
        torch.cuda.synchronize()
        outs.append((W.cpu(), b1.cpu(), b2.cpu()))
    W, b1, b2 = outs[0]
    assert rel_err(W, ref[:, :nw]) < 1e-5
    if bias:
        assert rel_err(b1, ref[:, nw]) < 1e-5
        assert torch.equal(b1, b2)
    else:
        assert torch.isnan(b1).all()                   # no bias output requested: untouched
    assert torch.equal(outs[0][0], outs[1][0])         # fixed-order reduce: bit-identical reruns


@pytest.mark.parametrize("M,N,K,lda", [(16000, 4096, 32, 48), (1000, 4096, 16, 32), (77, 48, 24, 24)])
def test_skinny_proj_matches_fp32_reference(M, N, K, lda):
    """Layer-0 input projection z W_ih^T + b_ih + b_hh (K = latent width, A rows strided like
    the engine's [z | 1 | 0..] operand) against a torch fp32 product of the same bf16 values."""
    need_gpu()
    l = lib()
    g = torch.Generator().manual_seed(21)
    A = torch.randn(M, lda, generator=g).to(torch.bfloat16)
    B = torch.randn(N, K, generator=g).to(torch.bfloat16)
    b1, b2 = torch.randn(N, generator=g), torch.randn(N, generator=g)
    ref = A[:, :K].float() @ B.float().t() + b1 + b2
    Ad, Bd, C = A.cuda(), B.cuda(), torch.empty(M, N, device="cuda")
    b1d, b2d = b1.cuda(), b2.cuda()  # held: a freed temporary's block would be reused
    check(l.mlvae_skinny_proj(M, N, K, Ad.data_ptr(), lda, Bd.data_ptr(), K, P(b1d), P(b2d), P(C),
                              N, stream()))
    # fp16 output (the wide recurrence's gate buffer): the fp32 result rounded once
    C16 = torch.empty(M, N, device="cuda", dtype=torch.float16)
    check(l.mlvae_skinny_proj_ex(M, N, K, Ad.data_ptr(), lda, Bd.data_ptr(), K, P(b1d), P(b2d),
                                 C16.data_ptr(), N, 1, stream()))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 1e-5
    assert torch.equal(C16, C.to(torch.float16))
    # bad shapes are refused, not launched
    assert l.mlvae_skinny_proj(M, N, 40, Ad.data_ptr(), lda, Bd.data_ptr(), 40, None, None, P(C),
                               N, stream()) != 0


@pytest.mark.parametrize("M,K8", [(16000, 4096), (1000, 4096), (333, 512), (128000, 4096)])
def test_skinny_dzw_matches_fp64(M, K8):
    """mlvae_skinny_dzw: dZ = dG W_ih_l0 and dW_ih_l0 | biases = dG^T [z | 1] from one pass over dG,
    against fp64 products of the same bf16 operands (ragged M; the c3 shape N = 128,000), and bit-
    identical reruns (fixed-order slab reduce)."""
    need_gpu()
    torch.manual_seed(M + K8)
    Z, NB = 32, 48
    dG = torch.randn(M, K8).to(torch.bfloat16)
    Wt = torch.randn(Z, K8).to(torch.bfloat16)                 # W_ih_l0^T
    zb = torch.zeros(M, NB)
    zb[:, :Z] = torch.randn(M, Z)
    zb[:, Z] = 1.0
    zb = zb.to(torch.bfloat16)
    dGd, Wd, zd = dG.cuda(), Wt.cuda(), zb.cuda()
    ref_dz = (dGd.double() @ Wd.double().t()).cpu()
    ref_w = (dGd.double().t() @ zd.double()).cpu()             # [K8, NB]
    l = lib()
    ws = torch.empty(l.mlvae_skinny_dzw_workspace_size(M, K8) // 4 + 1, device="cuda")
    outs = []
    for _ in range(2):
        dZ = torch.full((M, Z), float("nan"), device="cuda")
        W = torch.full((K8, Z), float("nan"), device="cuda")
        b1 = torch.full((K8,), float("nan"), device="cuda")
        b2 = torch.full((K8,), float("nan"), device="cuda")
        check(l.mlvae_skinny_dzw(M, K8, dGd.data_ptr(), K8, Wd.data_ptr(), K8, zd.data_ptr(), NB, Z, P(dZ), Z, P(W),
                                 P(b1), P(b2), P(ws), ws.numel() * 4, stream()))
        torch.cuda.synchronize()
        outs.append((dZ.cpu(), W.cpu(), b1.cpu(), b2.cpu()))
    dZ, W, b1, b2 = outs[0]
    assert rel_err(dZ, ref_dz) < 1e-5
    assert rel_err(W, ref_w[:, :Z]) < 1e-5
    assert rel_err(b1, ref_w[:, Z]) < 1e-5 and torch.equal(b1, b2)
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    assert l.mlvae_skinny_dzw(M, K8, dGd.data_ptr(), K8, Wd.data_ptr(), K8, zd.data_ptr(), NB, 16, P(dZ), Z, P(W),
                              None, None, P(ws), ws.numel() * 4, stream()) != 0
