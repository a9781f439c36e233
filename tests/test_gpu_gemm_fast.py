"""mlvae_gemm_bf16 (256 x 256 LDS-DMA tiles): every operand layout, batch, time shift, split-K
and the epilogues, against an fp64 product of the same bf16 operands."""
import pytest
import torch

from gpu_utils import P, need_gpu, rel_err, stream
from mlvae_hip._lib import check, lib

pytestmark = pytest.mark.gpu


def _shift_rows(b, T, shift):
    """rows k of B -> k + shift when 0 <= k % T + shift < T, else zero (the recurrent dW_hh)."""
    K = b.shape[0]
    t = torch.arange(K) % T + shift
    ok = (t >= 0) & (t < T)
    idx = torch.arange(K) + shift
    out = torch.zeros_like(b)
    out[ok] = b[idx[ok]]
    return out


def _run(ta, tb, M, N, K, batch=1, kshift_T=0, kshift=0, kstep=0, epi=0, beta=0.0, bias=True,
         seed=0):
    torch.manual_seed(seed + M + 3 * N + 7 * K + 11 * ta + 13 * tb)
    A = [(torch.randn(K, M) if ta else torch.randn(M, K)).to(torch.bfloat16) for _ in range(batch)]
    B = [(torch.randn(N, K) if tb else torch.randn(K, N)).to(torch.bfloat16) for _ in range(batch)]
    Cin = torch.randn(batch, M, N)
    aux = torch.randn(M, N)
    b1, b2 = torch.randn(N), torch.randn(N)
    refs = []
    for z in range(batch):
        a = A[z].double().t() if ta else A[z].double()
        b = B[z].double().t() if tb else B[z].double()
        if kshift_T:
            b = _shift_rows(b, kshift_T, kshift + z * kstep)
        r = a @ b
        if bias:
            r = r + b1.double() + b2.double()
        r = r + beta * Cin[z].double()
        if epi == 1:
            r = torch.nn.functional.leaky_relu(r, 0.01)
        if epi == 2:
            r = r * torch.where(aux > 0, 1.0, 0.01).double()
        refs.append(r)
    dA = torch.stack(A).cuda()
    dB = torch.stack(B).cuda()
    C = Cin.clone().cuda()
    db1, db2, daux = b1.cuda(), b2.cuda(), aux.cuda()  # kept alive across the launch
    l = lib()
    ws = torch.empty(l.mlvae_gemm_bf16_workspace_size(M, N, K, batch) // 4 + 1, device="cuda")
    lda, ldb = A[0].shape[1], B[0].shape[1]
    check(l.mlvae_gemm_bf16(ta, tb, M, N, K, batch, dA.data_ptr(), lda, A[0].numel(), dB.data_ptr(),
                            ldb, B[0].numel(), P(C), N, M * N, beta,
                            P(db1) if bias else None, P(db2) if bias else None, epi,
                            P(daux), N, kshift_T, kshift, kstep, 0, 0, 0.0, P(ws),
                            ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    return C.cpu(), torch.stack(refs)


@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(304, 136, 200), (520, 264, 1000), (8, 16, 64), (256, 256, 40),
                                   (304, 136, 256), (256, 256, 128)])
def test_layouts(ta, tb, M, N, K):
    need_gpu()
    C, ref = _run(ta, tb, M, N, K)
    assert rel_err(C, ref) < 1e-5


@pytest.mark.parametrize("ta,tb", [(1, 0), (0, 0)])
def test_split_k_long(ta, tb):
    """K = frames: split-K partial slabs + fixed-order reduce."""
    need_gpu()
    C, ref = _run(ta, tb, 512, 256, 8000, bias=False)
    assert rel_err(C, ref) < 1e-5


def test_batched_time_shift():
    """Both directions' dW_hh in one launch: shift -1 for batch 0, +1 for batch 1."""
    need_gpu()
    C, ref = _run(1, 0, 264, 128, 2000, batch=2, kshift_T=25, kshift=-1, kstep=2, bias=False)
    assert rel_err(C, ref) < 1e-5


@pytest.mark.parametrize("epi", [1, 2])
def test_epilogues(epi):
    need_gpu()
    C, ref = _run(0, 1, 304, 200, 128, epi=epi, beta=0.5)
    assert rel_err(C, ref) < 1e-5


def test_dropout_epilogue_matches_dropout_kernel():
    need_gpu()
    l = lib()
    torch.manual_seed(5)
    M, N, K, p, seed = 700, 264, 512, 0.15, 4242
    A = torch.randn(M, K).to(torch.bfloat16).cuda()
    B = torch.randn(N, K).to(torch.bfloat16).cuda()
    C0 = torch.empty(M, N, device="cuda")
    C1 = torch.empty(M, N, device="cuda")
    ws = torch.empty(16, device="cuda")
    for C, epi in ((C0, 0), (C1, 3)):
        check(l.mlvae_gemm_bf16(0, 1, M, N, K, 1, A.data_ptr(), K, 0, B.data_ptr(), K, 0, P(C), N, 0,
                                0.0, None, None, epi, None, 0, 0, 0, 0, seed, 0, p, P(ws), 64, stream()))
    check(l.mlvae_dropout(C0.numel(), P(C0), P(C0), None, seed, p, stream()))
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)


@pytest.mark.parametrize("K", [512, 8000])
def test_fp16_output(K):
    """EPI_OUT_F16 (the input projection into the wide recurrence's fp16 gate buffer): the fp32
    result + biases rounded once to fp16, through the staged epilogue and the split-K reduce."""
    need_gpu()
    l = lib()
    torch.manual_seed(K)
    M, N = 600, 4096 if K == 512 else 256
    A = torch.randn(M, K).to(torch.bfloat16).cuda()
    B = torch.randn(N, K).to(torch.bfloat16).cuda()
    b1, b2 = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    C16 = torch.empty(M, N, device="cuda", dtype=torch.float16)
    ws = torch.empty(l.mlvae_gemm_bf16_workspace_size(M, N, K, 1) // 4 + 1, device="cuda")
    for out, epi in ((C, 0), (C16, 16)):
        check(l.mlvae_gemm_bf16(0, 1, M, N, K, 1, A.data_ptr(), K, 0, B.data_ptr(), K, 0, out.data_ptr(), N,
                                0, 0.0, P(b1), P(b2), epi, None, 0, 0, 0, 0, 0, 0, 0.0, P(ws),
                                ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert torch.equal(C16, C.to(torch.float16))
    # fp16 C with an activation epilogue is refused
    assert l.mlvae_gemm_bf16(0, 1, M, N, K, 1, A.data_ptr(), K, 0, B.data_ptr(), K, 0, C16.data_ptr(), N,
                             0, 0.0, None, None, 16 | 1, None, 0, 0, 0, 0, 0, 0, 0.0, P(ws),
                             ws.numel() * 4, stream()) != 0
