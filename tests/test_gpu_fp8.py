"""fp8 GEMM mode (BASELINE.json configs[4]) kernels through the C ABI:

* mlvae_cast_fp8 equals torch's float8_e4m3fn (OCP) rounding of the scaled, saturated input, bit
  for bit, from fp32 and from bf16 sources;
* mlvae_fp8_scale: q = 448 / max|x|, alpha = 1 / (q * other);
* mlvae_gemm_fp8 (block-scaled 16x16x128 MFMA, unit block scales) against an fp64 product of the
  SAME fp8 operands (decoded by torch) times alpha, + biases: 1e-4 max-relative, fp32 and fp16 C,
  partial K-tiles and edge tiles."""
import pytest
import torch

from gpu_utils import P, need_gpu, rel_err, stream
from mlvae_hip._lib import check, lib

pytestmark = pytest.mark.gpu


def _f8(t):
    return t.view(torch.float8_e4m3fn).double()


def test_cast_fp8_matches_torch_e4m3fn():
    need_gpu()
    torch.manual_seed(0)
    x = torch.randn(4096, device="cuda") * 3
    x[:8] = torch.tensor([0.0, -0.0, 1e-9, 500.0, -1e4, 448.0, 0.0017, -0.3])
    out = torch.empty(4096, dtype=torch.uint8, device="cuda")
    check(lib().mlvae_cast_fp8(x.numel(), P(x), 0, None, 2.0, out.data_ptr(), stream()))
    torch.cuda.synchronize()
    ref = (x.double() * 2).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(out.cpu(), ref.cpu())
    xb = torch.randn(4096, device="cuda").to(torch.bfloat16)
    sc = torch.tensor([16.0], device="cuda")
    check(lib().mlvae_cast_fp8(xb.numel(), xb.data_ptr(), 1, P(sc), 0.0, out.data_ptr(), stream()))
    torch.cuda.synchronize()
    ref = (xb.double() * 16).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(out.cpu(), ref.cpu())


def test_fp8_scale():
    need_gpu()
    x = torch.randn(100003, device="cuda")
    x[777] = -9.5
    out = torch.zeros(2, device="cuda")
    ws = torch.empty(lib().mlvae_fp8_scale_workspace_size() // 4 + 1, device="cuda")
    check(lib().mlvae_fp8_scale(x.numel(), P(x), 256.0, P(out), P(ws), ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    q = 448.0 / 9.5
    assert abs(out[0].item() - q) / q < 1e-6 and abs(out[1].item() - 1 / (q * 256)) * q * 256 < 1e-6
    z = torch.zeros(64, device="cuda")
    check(lib().mlvae_fp8_scale(z.numel(), P(z), 1.0, P(out), P(ws), ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert out.tolist() == [1.0, 1.0]


@pytest.mark.parametrize("M,N,K,f16", [(300, 260, 256, False), (1000, 512, 1024, True), (256, 4096, 1024, True),
                                       (513, 132, 144, False), (4000, 1024, 2048, False)])
def test_gemm_fp8_matches_fp64_on_the_same_operands(M, N, K, f16):
    need_gpu()
    torch.manual_seed(M + N + K)
    A = (torch.randn(M, K, device="cuda") * 4).clamp(-448, 448).to(torch.float8_e4m3fn)
    B = (torch.randn(N, K, device="cuda") * 4).clamp(-448, 448).to(torch.float8_e4m3fn)
    b1 = torch.randn(N, device="cuda")
    b2 = torch.randn(N, device="cuda")
    alpha = torch.tensor([0.037], device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=torch.float16 if f16 else torch.float32)
    check(lib().mlvae_gemm_fp8(M, N, K, A.data_ptr(), K, B.data_ptr(), K, C.data_ptr(), N, P(alpha), P(b1), P(b2),
                               16 if f16 else 0, stream()))
    torch.cuda.synchronize()
    ref = (A.cpu().double() @ B.cpu().double().t()) * 0.037 + b1.cpu().double() + b2.cpu().double()
    # fp32 C: 1e-4 (measured <= 2.6e-5: the block-scaled MFMA's internal sums are not a k-ordered
    # fp32 fma chain); fp16 C: its own rounding
    assert rel_err(C.float(), ref) < (1e-3 if f16 else 1e-4)
