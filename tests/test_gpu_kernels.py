"""Kernel-level parity on the GPU: MFMA GEMM and the persistent BiLSTM recurrence against
plain PyTorch CPU references (fp64 where that is the cleaner bar)."""
import pytest
import torch

from gpu_utils import P, need_gpu, rel_err, stream
from mlvae_hip._lib import check, lib
from oracle import vae_cpu as O

pytestmark = pytest.mark.gpu


def _ref_gemm(A, B, ta, tb, kshift_T=0, kshift=0):
    a = A.double().t() if ta else A.double()
    b = B.double().t() if tb else B.double()
    if kshift:
        K = b.shape[0]
        t = torch.arange(K) % kshift_T + kshift
        ok = (t >= 0) & (t < kshift_T)
        idx = torch.arange(K) + kshift
        bs = torch.zeros_like(b)
        bs[ok] = b[idx[ok]]
        b = bs
    return a @ b


@pytest.mark.parametrize("prec,tol", [(0, 2e-6), (1, 2e-2)])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 72), (37, 5, 3), (129, 257, 1000), (64, 80, 4000)])
def test_gemm(prec, tol, ta, tb, M, N, K):
    need_gpu()
    torch.manual_seed(M * 7 + N + K)
    A = torch.randn(K, M) if ta else torch.randn(M, K)
    B = torch.randn(N, K) if tb else torch.randn(K, N)
    bias1, bias2 = torch.randn(N), torch.randn(N)
    ref = _ref_gemm(A, B, ta, tb) + bias1.double() + bias2.double()
    dev = [t.cuda() for t in (A, B, bias1, bias2)]
    C = torch.empty(M, N, device="cuda")
    ws = torch.empty(lib().mlvae_gemm_workspace_size(M, N, K) // 4 + 1, device="cuda")
    check(lib().mlvae_gemm(prec, ta, tb, M, N, K, 1.0, P(dev[0]), dev[0].shape[1], P(dev[1]),
                           dev[1].shape[1], 0.0, P(C), N, P(dev[2]), P(dev[3]), 0, None, 0, 0, 0,
                           P(ws), ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < tol


@pytest.mark.parametrize("prec,tol", [(0, 2e-6), (1, 2e-2)])
def test_gemm_epilogues_and_shift(prec, tol):
    need_gpu()
    torch.manual_seed(3)
    M, N, K, T = 96, 48, 300, 25
    A = torch.randn(K, M)
    B = torch.randn(K, N)
    aux = torch.randn(M, N)
    Cin = torch.randn(M, N)
    l = lib()
    ws = torch.empty(l.mlvae_gemm_workspace_size(M, N, K) // 4 + 1, device="cuda")
    dA, dB, daux = A.cuda(), B.cuda(), aux.cuda()
    for epi, shift in [(1, 0), (2, 0), (0, -1), (0, 1)]:
        C = Cin.cuda()
        check(l.mlvae_gemm(prec, 1, 0, M, N, K, 0.5, P(dA), M, P(dB), N, 2.0, P(C), N, None, None,
                           epi, P(daux), N, T if shift else 0, shift, P(ws), ws.numel() * 4, stream()))
        torch.cuda.synchronize()
        ref = 0.5 * _ref_gemm(A, B, 1, 0, T, shift) + 2.0 * Cin.double()
        if epi == 1:
            ref = torch.nn.functional.leaky_relu(ref, 0.01)
        if epi == 2:
            ref = ref * torch.where(aux > 0, 1.0, 0.01).double()
        assert rel_err(C, ref) < tol, (epi, shift)


def _as_bf16(t, on):
    """(device tensor handed to the kernel, fp64 values the kernel sees)."""
    if on:
        b = t.to(torch.bfloat16)
        return b.cuda(), b.double()
    return t.cuda(), t.double()


@pytest.mark.parametrize("abf,bbf", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 72), (40, 24, 8), (136, 264, 1000), (64, 80, 4000)])
def test_gemm_ex_bf16_operands(abf, bbf, ta, tb, M, N, K):
    """mlvae_gemm_ex: bf16 MFMA over bf16- or fp32-stored operands, every transpose."""
    need_gpu()
    torch.manual_seed(M + 3 * N + K)
    A = torch.randn(K, M) if ta else torch.randn(M, K)
    B = torch.randn(N, K) if tb else torch.randn(K, N)
    bias1 = torch.randn(N)
    dA, A64 = _as_bf16(A, abf)
    dB, B64 = _as_bf16(B, bbf)
    a = A64.t() if ta else A64
    b = B64.t() if tb else B64
    # fp32 operands are rounded to bf16 while staging: compare against the rounded product
    if not abf:
        a = a.to(torch.bfloat16).double()
    if not bbf:
        b = b.to(torch.bfloat16).double()
    ref = a @ b + bias1.double()
    C = torch.empty(M, N, device="cuda")
    l = lib()
    ws = torch.empty(l.mlvae_gemm_ex_workspace_size(M, N, K) // 4 + 1, device="cuda")
    check(l.mlvae_gemm_ex(ta, tb, M, N, K, 1.0, P(dA), abf, dA.shape[1], P(dB), bbf, dB.shape[1],
                          0.0, P(C), N, P(bias1.cuda()), None, 0, None, 0, 0, 0, P(ws),
                          ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 1e-4


@pytest.mark.parametrize("bf", [0, 1])
def test_gemm_ex_epilogues_and_shift(bf):
    need_gpu()
    torch.manual_seed(4)
    M, N, K, T = 96, 48, 304, 19
    A = torch.randn(K, M)
    B = torch.randn(K, N)
    aux = torch.randn(M, N)
    Cin = torch.randn(M, N)
    dA, A64 = _as_bf16(A, bf)
    dB, B64 = _as_bf16(B, bf)
    A64, B64 = A64.to(torch.bfloat16).double(), B64.to(torch.bfloat16).double()
    l = lib()
    ws = torch.empty(l.mlvae_gemm_ex_workspace_size(M, N, K) // 4 + 1, device="cuda")
    daux = aux.cuda()
    for epi, shift in [(1, 0), (2, 0), (0, -1), (0, 1)]:
        C = Cin.cuda()
        check(l.mlvae_gemm_ex(1, 0, M, N, K, 0.5, P(dA), bf, M, P(dB), bf, N, 2.0, P(C), N, None,
                              None, epi, P(daux), N, T if shift else 0, shift, P(ws),
                              ws.numel() * 4, stream()))
        torch.cuda.synchronize()
        ref = 0.5 * _ref_gemm(A64, B64, 1, 0, T, shift) + 2.0 * Cin.double()
        if epi == 1:
            ref = torch.nn.functional.leaky_relu(ref, 0.01)
        if epi == 2:
            ref = ref * torch.where(aux > 0, 1.0, 0.01).double()
        assert rel_err(C, ref) < 1e-4, (epi, shift)


def test_cast_bf16():
    need_gpu()
    x = torch.randn(1003) * 100
    y = torch.empty(1003, dtype=torch.bfloat16, device="cuda")
    xd = x.cuda()
    check(lib().mlvae_cast_bf16(x.numel(), P(xd), P(y), stream()))
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), x.to(torch.bfloat16))


@pytest.mark.parametrize("rows,cols", [(4096, 1024), (4096, 32), (37, 70)])
def test_cast_bf16_transposed(rows, cols):
    need_gpu()
    x = torch.randn(rows, cols)
    y = torch.empty(cols, rows, dtype=torch.bfloat16, device="cuda")
    xd = x.cuda()
    check(lib().mlvae_cast_bf16_t(rows, cols, P(xd), P(y), stream()))
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), x.t().contiguous().to(torch.bfloat16))


def _lstm_ref(x, p, H):
    """One bidirectional layer from the oracle's explicit loop; returns y and autograd fn."""
    outs = []
    for sfx, rev in (("", False), ("_reverse", True)):
        outs.append(O.lstm_direction_loop(x, p["w_ih" + sfx], p["w_hh" + sfx], p["b_ih" + sfx],
                                          p["b_hh" + sfx], rev))
    return torch.cat(outs, -1)


@pytest.mark.parametrize("prec,tol", [(0, 2e-5), (1, 3e-2)])
@pytest.mark.parametrize("B,T,H,D", [(3, 17, 8, 4), (20, 33, 64, 16), (32, 40, 512, 32), (40, 9, 128, 8),
                                     (17, 21, 256, 8), (5, 12, 1024, 8)])
def test_lstm_layer_fwd_bwd(prec, tol, B, T, H, D):
    need_gpu()  # fp32 at H > 512: the stepwise BPTT (lstm.hip lstm_bwd_step_f32)
    torch.manual_seed(B + T + H)
    k = 1.0 / H ** 0.5
    p = {}
    for sfx in ("", "_reverse"):
        p["w_ih" + sfx] = (torch.rand(4 * H, D) * 2 - 1) * k
        p["w_hh" + sfx] = (torch.rand(4 * H, H) * 2 - 1) * k
        p["b_ih" + sfx] = (torch.rand(4 * H) * 2 - 1) * k
        p["b_hh" + sfx] = (torch.rand(4 * H) * 2 - 1) * k
    x = torch.randn(B, T, D, dtype=torch.float64)
    pd = {kk: v.double().requires_grad_(True) for kk, v in p.items()}
    y = _lstm_ref(x, pd, H)
    dy = torch.randn_like(y)
    gx = torch.cat([x @ pd["w_ih"].t() + pd["b_ih"] + pd["b_hh"],
                    x @ pd["w_ih_reverse"].t() + pd["b_ih_reverse"] + pd["b_hh_reverse"]], -1)
    # gradient wrt the input projection G (what the kernel's dG is)
    gxl = gx.detach().requires_grad_(True)
    # recompute y from gx via a loop with w_hh only
    def from_gx(gxv):
        outs = []
        for d, (sfx, rev) in enumerate((("", False), ("_reverse", True))):
            g4 = gxv[..., d * 4 * H:(d + 1) * 4 * H]
            h = torch.zeros(B, H, dtype=torch.float64)
            c = torch.zeros(B, H, dtype=torch.float64)
            o = [None] * T
            for t in (range(T - 1, -1, -1) if rev else range(T)):
                gg = g4[:, t] + h @ pd["w_hh" + sfx].t()
                i, f, gc, og = gg.split(H, 1)
                c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gc)
                h = torch.sigmoid(og) * torch.tanh(c)
                o[t] = h
            outs.append(torch.stack(o, 1))
        return torch.cat(outs, -1)
    y2 = from_gx(gxl)
    assert (y2 - y).abs().max() < 1e-10
    (dG_ref, dWhh0, dWhh1) = torch.autograd.grad((y2 * dy).sum(), [gxl, pd["w_hh"], pd["w_hh_reverse"]])

    N = B * T
    G = gx.detach().float().reshape(N, 8 * H).cuda().contiguous()
    Cs = torch.empty(N, 2 * H, device="cuda")
    Y = torch.empty(N, 2 * H, device="cuda")
    W0, W1 = p["w_hh"].cuda(), p["w_hh_reverse"].cuda()
    import ctypes
    xb = ctypes.c_size_t()
    check(lib().mlvae_lstm_workspace_size(B, H, prec, ctypes.byref(xb)))
    xbuf = torch.empty(xb.value, device="cuda", dtype=torch.uint8)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    check(lib().mlvae_lstm_fwd(prec, B, T, H, P(W0), P(W1), P(G), P(Cs), P(Y), P(xbuf), xb.value,
                               P(err), stream()))
    torch.cuda.synchronize()
    assert err.item() == 0
    assert rel_err(Y.view(B, T, 2 * H), y) < tol
    dY = dy.float().reshape(N, 2 * H).cuda().contiguous()
    check(lib().mlvae_lstm_bwd(prec, B, T, H, P(W0), P(W1), P(G), P(Cs), P(dY), P(xbuf), xb.value,
                               P(err), stream()))
    torch.cuda.synchronize()
    assert err.item() == 0
    assert rel_err(G.view(B, T, 8 * H), dG_ref) < tol * 5
    # recurrent weight grads through the shifted wgrad GEMM
    ws = torch.empty(lib().mlvae_gemm_workspace_size(4 * H, H, N) // 4 + 1, device="cuda")
    for d, (ref, shift) in enumerate(((dWhh0, -1), (dWhh1, 1))):
        out = torch.empty(4 * H, H, device="cuda")
        check(lib().mlvae_gemm(prec, 1, 0, 4 * H, H, N, 1.0, P(G, d * 4 * H), 8 * H, P(Y, d * H),
                               2 * H, 0.0, P(out), H, None, None, 0, None, 0, T, shift, P(ws),
                               ws.numel() * 4, stream()))
        torch.cuda.synchronize()
        assert rel_err(out, ref) < tol * 5


def test_dropout_mask_statistics_and_fused_backward():
    """Inter-layer dropout (ref:src/modules/decoder.py:14, nn.LSTM dropout=0.15 in train mode):
    the forward kernel keeps ~85 % of elements scaled by 1/0.85, and the dgrad GEMM epilogue
    (mlvae_gemm_ex_drop, epilogue 3) applies bit-for-bit the same mask to its output."""
    need_gpu()
    l = lib()
    torch.manual_seed(11)
    p, seed = 0.15, 987654321
    M, N, K = 300, 136, 256
    x = torch.ones(M * N, device="cuda")
    y = torch.empty_like(x)
    check(l.mlvae_dropout_ex(x.numel(), P(x), P(y), None, None, seed, 0, p, stream()))
    torch.cuda.synchronize()
    vals = sorted(set(torch.unique(y).tolist()))
    assert len(vals) == 2 and vals[0] == 0.0 and abs(vals[1] - 1.0 / (1.0 - p)) < 1e-6, vals
    keep = (y != 0).double().mean().item()
    assert abs(keep - (1 - p)) < 0.01, keep
    # fused epilogue == GEMM then dropout kernel (same seed, same flat index row*N + col)
    A = torch.randn(M, K).to(torch.bfloat16).cuda()
    B = torch.randn(K, N).to(torch.bfloat16).cuda()
    ws = torch.empty(l.mlvae_gemm_ex_workspace_size(M, N, K) // 4 + 1, device="cuda")
    C0 = torch.empty(M, N, device="cuda")
    C1 = torch.empty(M, N, device="cuda")
    check(l.mlvae_gemm_ex(0, 0, M, N, K, 1.0, A.data_ptr(), 1, K, B.data_ptr(), 1, N, 0.0, P(C0), N,
                          None, None, 0, None, 0, 0, 0, P(ws), ws.numel() * 4, stream()))
    check(l.mlvae_dropout(C0.numel(), P(C0), P(C0), None, seed, p, stream()))
    check(l.mlvae_gemm_ex_drop(0, 0, M, N, K, 1.0, A.data_ptr(), 1, K, B.data_ptr(), 1, N, 0.0,
                               P(C1), N, None, None, 3, None, 0, 0, 0, seed, 0, p, P(ws),
                               ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)


def test_dropout_vector_and_scalar_paths_agree():
    """mlvae_dropout_ex's 16-byte path (aligned) and its element path (unaligned views) give the
    same masked values, fp32 and bf16, for a length that is not a multiple of 4."""
    need_gpu()
    l = lib()
    n, seed, p = 100_003, 4242, 0.15
    x = torch.randn(n + 1, device="cuda")
    outs = []
    for off in (0, 1):  # element offset 1 = 4-byte misaligned pointers: element path
        y = torch.zeros(n + 1, device="cuda")
        yb = torch.zeros(n + 1, device="cuda", dtype=torch.bfloat16)
        xs = x.clone()
        if off:
            xs[1:] = x[:n]
        check(l.mlvae_dropout_ex(n, P(xs, off), P(y, off), yb.data_ptr() + 2 * off, None, seed, 0, p,
                                 stream()))
        torch.cuda.synchronize()
        outs.append((y[off:off + n].cpu(), yb[off:off + n].view(torch.int16).cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    kept = (outs[0][0] != 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.01


def test_dropout_offset_is_the_shard_of_the_global_mask():
    """A data-parallel shard passes the global index of its first element: its masks are the
    matching slice of the single-GPU masks, in the dropout kernel and in both fused dgrad
    epilogues (mlvae_gemm_ex_drop, mlvae_gemm_bf16)."""
    need_gpu()
    l = lib()
    seed, p = 20241016, 0.15
    M, N, K = 96, 64, 64
    x = torch.randn(M * N, device="cuda")
    full = torch.empty_like(x)
    check(l.mlvae_dropout_ex(x.numel(), P(x), P(full), None, None, seed, 0, p, stream()))
    r0 = 40   # shard = rows 40.. of the [M, N] layer output
    part = torch.empty(M * N - r0 * N, device="cuda")
    check(l.mlvae_dropout_ex(part.numel(), P(x, r0 * N), P(part), None, None, seed, r0 * N, p, stream()))
    torch.cuda.synchronize()
    assert torch.equal(part, full[r0 * N:])
    A = torch.randn(M - r0, K).to(torch.bfloat16).cuda()
    Bt = torch.randn(N, K).to(torch.bfloat16).cuda()
    Bk = Bt.t().contiguous()
    ws = torch.empty(1 << 16, device="cuda")
    C0, C1, C2, C3 = (torch.empty(M - r0, N, device="cuda") for _ in range(4))
    check(l.mlvae_gemm_ex(0, 0, M - r0, N, K, 1.0, A.data_ptr(), 1, K, Bk.data_ptr(), 1, N, 0.0, P(C0), N,
                          None, None, 0, None, 0, 0, 0, P(ws), ws.numel() * 4, stream()))
    check(l.mlvae_dropout_ex(C0.numel(), P(C0), P(C0), None, None, seed, r0 * N, p, stream()))
    check(l.mlvae_gemm_ex_drop(0, 0, M - r0, N, K, 1.0, A.data_ptr(), 1, K, Bk.data_ptr(), 1, N, 0.0,
                               P(C1), N, None, None, 3, None, 0, 0, 0, seed, r0 * N, p, P(ws),
                               ws.numel() * 4, stream()))
    for C, epi in ((C2, 0), (C3, 3)):
        check(l.mlvae_gemm_bf16(0, 1, M - r0, N, K, 1, A.data_ptr(), K, 0, Bt.data_ptr(), K, 0, P(C), N,
                                0, 0.0, None, None, epi, None, 0, 0, 0, 0, seed, r0 * N, p, P(ws),
                                ws.numel() * 4, stream()))
    check(l.mlvae_dropout_ex(C2.numel(), P(C2), P(C2), None, None, seed, r0 * N, p, stream()))
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)
    assert torch.equal(C2, C3)
