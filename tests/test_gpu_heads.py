"""Fused decoder heads (heads.hip) against an fp64 autograd restatement of
ref:src/modules/decoder.py:24-25,37-53 + ref:src/modules/fc_block.py on the same bf16 operands.
Tolerances: the kernel feeds bf16 MFMAs (activations rounded to bf16 between layers)."""
import math

import pytest
import torch

from gpu_utils import P, need_gpu, norm_rel, rel_err, stream
from mlvae_hip._lib import check, lib

pytestmark = pytest.mark.gpu


def _valid(lens, T):
    """SpeechBrain length_to_mask in fp32 (ref:src/utils/data_utils.py:86-87)."""
    lim = (lens.float() * T)
    return (torch.arange(T).float()[None, :] < lim[:, None])


@pytest.mark.parametrize("loss_type", [0, 1])
@pytest.mark.parametrize("B,T,F,H2,train", [(3, 50, 80, 256, 1), (2, 64, 64, 384, 1), (3, 50, 80, 256, 0)])
def test_heads_fused(loss_type, B, T, F, H2, train):
    need_gpu()
    torch.manual_seed(B * 1000 + T + F + H2 + loss_type)
    C, N = 64, B * T
    rec_scale = 0.7
    Y = torch.randn(N, H2).to(torch.bfloat16)
    W1 = (torch.randn(2 * C, H2) / math.sqrt(H2)).to(torch.bfloat16)
    b1 = torch.randn(2 * C) * 0.1
    W2 = [torch.randn(C, C) / 8 for _ in range(2)]
    b2 = [torch.randn(C) * 0.1 for _ in range(2)]
    W3 = [torch.randn(F, C) / 8 for _ in range(2)]
    b3 = [torch.randn(F) * 0.1 for _ in range(2)]
    x = torch.randn(N, F)
    lens = torch.tensor([1.0, 0.7, 0.31][:B])
    mask = _valid(lens, T).reshape(N, 1).double()
    count = int(mask.sum().item())

    # fp64 reference
    Yd = Y.double().requires_grad_(True)
    lrelu = lambda v: torch.nn.functional.leaky_relu(v, 0.01)
    P1 = lrelu(Yd @ W1.double().t() + b1.double())
    outs, p2s = [], []
    for h in range(2):
        p2 = lrelu(P1[:, h * C:(h + 1) * C] @ W2[h].double().t() + b2[h].double())
        p2s.append(p2)
        outs.append(p2 @ W3[h].double().t() + b3[h].double())
    for o in outs:
        o.retain_grad()
    mu, lv = outs
    d = x.double() - mu
    if loss_type == 0:
        r = 0.5 * (math.log(2 * math.pi) + lv + d * d / (torch.exp(lv) + 1e-5))
    else:
        r = d * d
    lsum = (r * mask).sum()
    (rec_scale * lsum / (count * F)).backward()

    l = lib()
    dev = lambda t: t.contiguous().cuda()
    dY, dW1 = dev(Y), dev(W1)
    dW1t = dev(W1.t())
    db1 = dev(b1)
    dW2, db2, dW3, db3 = [dev(t) for t in W2], [dev(t) for t in b2], [dev(t) for t in W3], [dev(t) for t in b3]
    dx, dlens = dev(x), dev(lens)
    f = dict(device="cuda", dtype=torch.float32)
    o = {k: torch.zeros(N, n, **f) for k, n in (("p1", 2 * C), ("p2m", C), ("p2v", C), ("mux", F),
                                                  ("lvx", F), ("dmux", F), ("dlvx", F), ("dp2m", C),
                                                  ("dp2v", C), ("dp1", 2 * C), ("dy", H2))}
    parts = torch.zeros(l.mlvae_heads_partials_count(B, T), **f)
    assert l.mlvae_heads_supported(C, F, H2)
    tr = lambda k: P(o[k]) if train else None
    check(l.mlvae_heads_fused(B, T, F, C, H2, loss_type, train, dY.data_ptr(), dW1.data_ptr(),
                              dW1t.data_ptr() if train else None, P(db1), P(dW2[0]), P(db2[0]),
                              P(dW3[0]), P(db3[0]), P(dW2[1]), P(db2[1]), P(dW3[1]), P(db3[1]),
                              P(dx), P(dlens), None, rec_scale, tr("p1"), tr("p2m"), tr("p2v"),
                              P(o["mux"]), P(o["lvx"]), tr("dmux"),
                              P(o["dlvx"]) if (train and loss_type == 0) else None, tr("dp2m"),
                              tr("dp2v"), tr("dp1"), tr("dy"), P(parts), stream()))
    torch.cuda.synchronize()
    assert rel_err(o["mux"], mu) < 2e-2
    assert rel_err(o["lvx"], lv) < 2e-2
    assert abs(parts.sum().item() - lsum.item()) / abs(lsum.item()) < 1e-2
    if not train:
        return
    assert rel_err(o["p1"], P1) < 1e-2
    assert rel_err(o["p2m"], p2s[0]) < 2e-2
    assert norm_rel(o["dmux"], mu.grad) < 2e-2
    if loss_type == 0:
        assert norm_rel(o["dlvx"], lv.grad) < 2e-2
    assert norm_rel(o["dy"], Yd.grad) < 3e-2
    if loss_type == 1:  # mse: the log_var head gets no gradient
        assert o["dp1"][:, C:].abs().max().item() == 0.0


@pytest.mark.parametrize("loss_type", [0, 1])
@pytest.mark.parametrize("B,T,F,H2", [(3, 50, 80, 256), (5, 77, 64, 128)])
def test_heads_fused_bias_sums(loss_type, B, T, F, H2):
    """mlvae_heads_fused_ex: the five head bias gradients from in-kernel column sums equal the
    column sums of the kernel's own dOUT / dP2 / dP1 outputs (fp32, fixed-order reduce); mse
    leaves the log_var head's biases untouched."""
    need_gpu()
    torch.manual_seed(B + T + F + loss_type)
    C, N = 64, B * T
    l = lib()
    f = dict(device="cuda", dtype=torch.float32)
    Y = torch.randn(N, H2).to(torch.bfloat16).cuda()
    W1 = (torch.randn(2 * C, H2) / math.sqrt(H2)).to(torch.bfloat16)
    dW1, dW1t = W1.cuda(), W1.t().contiguous().cuda()
    b1 = (torch.randn(2 * C) * 0.1).cuda()
    W2 = [(torch.randn(C, C) / 8).cuda() for _ in range(2)]
    b2 = [(torch.randn(C) * 0.1).cuda() for _ in range(2)]
    W3 = [(torch.randn(F, C) / 8).cuda() for _ in range(2)]
    b3 = [(torch.randn(F) * 0.1).cuda() for _ in range(2)]
    x = torch.randn(N, F).cuda()
    lens = torch.tensor([1.0, 0.7, 0.31, 0.9, 0.5][:B]).cuda()
    o = {k: torch.zeros(N, n, **f) for k, n in (("p1", 2 * C), ("p2m", C), ("p2v", C), ("mux", F),
                                                  ("lvx", F), ("dmux", F), ("dlvx", F), ("dp2m", C),
                                                  ("dp2v", C), ("dp1", 2 * C), ("dy", H2))}
    parts = torch.zeros(l.mlvae_heads_partials_count(B, T), **f)
    ws = torch.zeros(l.mlvae_heads_bias_workspace_size(B, T, F, C) // 4 + 1, **f)
    nan = lambda n: torch.full((n,), float("nan"), **f)
    db3m, db3v, db2m, db2v, db1 = nan(F), nan(F), nan(C), nan(C), nan(2 * C)
    lik = loss_type == 0
    check(l.mlvae_heads_fused_ex(B, T, F, C, H2, loss_type, 1, Y.data_ptr(), dW1.data_ptr(), dW1t.data_ptr(),
                                 P(b1), P(W2[0]), P(b2[0]), P(W3[0]), P(b3[0]), P(W2[1]), P(b2[1]),
                                 P(W3[1]), P(b3[1]), P(x), P(lens), None, 0.7, P(o["p1"]), P(o["p2m"]),
                                 P(o["p2v"]), P(o["mux"]), P(o["lvx"]), P(o["dmux"]),
                                 P(o["dlvx"]) if lik else None, P(o["dp2m"]), P(o["dp2v"]), P(o["dp1"]),
                                 P(o["dy"]), P(parts), P(ws), ws.numel() * 4, P(db3m), P(db3v), P(db2m),
                                 P(db2v), P(db1), 0, stream()))
    torch.cuda.synchronize()
    cs = lambda t: t.double().sum(0)
    assert rel_err(db3m, cs(o["dmux"])) < 1e-5
    assert rel_err(db2m, cs(o["dp2m"])) < 1e-5
    if lik:
        assert rel_err(db3v, cs(o["dlvx"])) < 1e-5
        assert rel_err(db2v, cs(o["dp2v"])) < 1e-5
        assert rel_err(db1, cs(o["dp1"])) < 1e-5
    else:
        assert torch.isnan(db3v).all() and torch.isnan(db2v).all() and torch.isnan(db1[C:]).all()
        assert rel_err(db1[:C], cs(o["dp1"][:, :C])) < 1e-5
    # the same launch twice: bit-identical (fixed-order sums)
    first = db1.clone()
    check(l.mlvae_heads_fused_ex(B, T, F, C, H2, loss_type, 1, Y.data_ptr(), dW1.data_ptr(), dW1t.data_ptr(),
                                 P(b1), P(W2[0]), P(b2[0]), P(W3[0]), P(b3[0]), P(W2[1]), P(b2[1]),
                                 P(W3[1]), P(b3[1]), P(x), P(lens), None, 0.7, P(o["p1"]), P(o["p2m"]),
                                 P(o["p2v"]), P(o["mux"]), P(o["lvx"]), P(o["dmux"]),
                                 P(o["dlvx"]) if lik else None, P(o["dp2m"]), P(o["dp2v"]), P(o["dp1"]),
                                 P(o["dy"]), P(parts), P(ws), ws.numel() * 4, P(db3m), P(db3v), P(db2m),
                                 P(db2v), P(db1), 0, stream()))
    torch.cuda.synchronize()
    assert torch.equal(first[:C], db1[:C])
    # saved_bf16: the five saved intermediates as bf16 = the fp32 ones rounded once; the bias
    # sums (taken from the fp32 registers) and everything else unchanged
    ob = {k: torch.zeros(N, o[k].shape[1], device="cuda", dtype=torch.bfloat16)
          for k in ("p1", "p2m", "p2v", "dmux", "dlvx", "dp2m", "dp2v", "dp1")}
    dy2, mux2 = torch.zeros_like(o["dy"]), torch.zeros_like(o["mux"])
    b1b = db1.clone().fill_(float("nan"))
    check(l.mlvae_heads_fused_ex(B, T, F, C, H2, loss_type, 1, Y.data_ptr(), dW1.data_ptr(), dW1t.data_ptr(),
                                 P(b1), P(W2[0]), P(b2[0]), P(W3[0]), P(b3[0]), P(W2[1]), P(b2[1]),
                                 P(W3[1]), P(b3[1]), P(x), P(lens), None, 0.7, P(ob["p1"]), P(ob["p2m"]),
                                 P(ob["p2v"]), P(mux2), P(o["lvx"]), P(ob["dmux"]),
                                 P(ob["dlvx"]) if lik else None, P(ob["dp2m"]), P(ob["dp2v"]), P(ob["dp1"]),
                                 P(dy2), P(parts), P(ws), ws.numel() * 4, P(db3m), P(db3v), P(db2m),
                                 P(db2v), P(b1b), 1, stream()))
    torch.cuda.synchronize()
    for k in ("p1", "p2m", "dmux", "dp2m", "dp1") + (("p2v", "dlvx", "dp2v") if lik else ()):
        assert torch.equal(ob[k], o[k].to(torch.bfloat16)), k
    assert torch.equal(dy2, o["dy"]) and torch.equal(mux2, o["mux"])
    # saved_bf16 + bias sums runs the split form (P1 / dY GEMMs around heads_mid_kernel): every
    # output above is bit-identical; its bias sums agree to fp32 rounding (1 ulp seen in tiles
    # with masked frames)
    assert rel_err(b1b[:C], first[:C]) < 1e-6


@pytest.mark.parametrize("loss_type", [0, 1])
@pytest.mark.parametrize("B,T,F,H2", [(3, 50, 80, 256), (5, 77, 64, 128), (40, 500, 80, 1024)])
def test_heads_fused_weight_gradients(loss_type, B, T, F, H2):
    """mlvae_heads_fused_ex2: dW3 = dOUT_h^T P2_h and dW2 = dP2_h^T P1_h of both heads, accumulated
    inside the heads' middle kernel, against the fp64 products of the bf16 intermediates the split
    form saves (the kernel's LDS images hold exactly those values) -- ragged tiles, masked frames,
    N = 20,000 frames on the full persistent grid; mse writes nothing for the log_var head; the
    other outputs are bit-identical to mlvae_heads_fused_ex's and two launches are bit-identical."""
    need_gpu()
    torch.manual_seed(B + T + F + loss_type + 7)
    C, N = 64, B * T
    l = lib()
    f = dict(device="cuda", dtype=torch.float32)
    Y = torch.randn(N, H2).to(torch.bfloat16).cuda()
    W1 = (torch.randn(2 * C, H2) / math.sqrt(H2)).to(torch.bfloat16)
    dW1, dW1t = W1.cuda(), W1.t().contiguous().cuda()
    b1 = (torch.randn(2 * C) * 0.1).cuda()
    W2 = [(torch.randn(C, C) / 8).cuda() for _ in range(2)]
    b2 = [(torch.randn(C) * 0.1).cuda() for _ in range(2)]
    W3 = [(torch.randn(F, C) / 8).cuda() for _ in range(2)]
    b3 = [(torch.randn(F) * 0.1).cuda() for _ in range(2)]
    x = torch.randn(N, F).cuda()
    lens = torch.linspace(0.3, 1.0, B).cuda()
    lik = loss_type == 0
    ws = torch.zeros(l.mlvae_heads_bias_workspace_size(B, T, F, C) // 4 + 1, **f)
    wgs = torch.zeros(l.mlvae_heads_wgrad_workspace_size(B, T, F, C) // 4 + 1, **f)
    nan = lambda *s: torch.full(s, float("nan"), **f)

    def run(wg):
        o = {k: torch.zeros(N, n, device="cuda", dtype=torch.bfloat16)
             for k, n in (("p1", 2 * C), ("p2m", C), ("p2v", C), ("dmux", F), ("dlvx", F),
                          ("dp2m", C), ("dp2v", C), ("dp1", 2 * C))}
        o.update(mux=torch.zeros(N, F, **f), lvx=torch.zeros(N, F, **f), dy=torch.zeros(N, H2, **f),
                 parts=torch.zeros(l.mlvae_heads_partials_count(B, T), **f))
        db = [nan(F), nan(F), nan(C), nan(C), nan(2 * C)]
        dw = [nan(F, C), nan(F, C), nan(C, C), nan(C, C)]
        wg_args = (P(wgs), wgs.numel() * 4, P(dw[0]), P(dw[1]) if lik else None, P(dw[2]),
                   P(dw[3]) if lik else None) if wg else (None, 0, None, None, None, None)
        check(l.mlvae_heads_fused_ex2(B, T, F, C, H2, loss_type, 1, Y.data_ptr(), dW1.data_ptr(),
                                      dW1t.data_ptr(), P(b1), P(W2[0]), P(b2[0]), P(W3[0]), P(b3[0]),
                                      P(W2[1]), P(b2[1]), P(W3[1]), P(b3[1]), P(x), P(lens), None, 0.7,
                                      P(o["p1"]), P(o["p2m"]), P(o["p2v"]), P(o["mux"]), P(o["lvx"]),
                                      P(o["dmux"]), P(o["dlvx"]) if lik else None, P(o["dp2m"]),
                                      P(o["dp2v"]), P(o["dp1"]), P(o["dy"]), P(o["parts"]), P(ws),
                                      ws.numel() * 4, *[P(t) for t in db], 1, *wg_args, stream()))
        torch.cuda.synchronize()
        return o, db, dw

    ref, dbr, _ = run(False)
    o, db, dw = run(True)
    # outputs the fused form still writes: bit-identical
    for k in ("p1", "mux", "lvx", "dy", "dp1", "parts"):
        assert torch.equal(o[k], ref[k]), k
    for a_, b_ in zip(db, dbr):
        assert torch.equal(torch.nan_to_num(a_, 7.0), torch.nan_to_num(b_, 7.0))
    d = lambda t: t.double()
    heads = [(0, "p2m", "dmux", "dp2m")] + ([(1, "p2v", "dlvx", "dp2v")] if lik else [])
    for h, p2, dout, dp2 in heads:
        want3 = d(ref[dout]).t() @ d(ref[p2])
        want2 = d(ref[dp2]).t() @ d(ref["p1"][:, h * C:(h + 1) * C])
        assert rel_err(dw[h], want3) < 1e-5, (h, rel_err(dw[h], want3))
        assert rel_err(dw[2 + h], want2) < 1e-5, (h, rel_err(dw[2 + h], want2))
    if not lik:
        assert torch.isnan(dw[1]).all() and torch.isnan(dw[3]).all()
    first = [t.clone() for t in dw]
    _, _, dw2 = run(True)
    for a_, b_ in zip(first, dw2):
        assert torch.equal(torch.nan_to_num(a_, 7.0), torch.nan_to_num(b_, 7.0))


@pytest.mark.parametrize("loss_type", [0, 1])
@pytest.mark.parametrize("B,T,F,H2", [(3, 50, 80, 256), (5, 77, 64, 128), (40, 500, 80, 1024), (140, 500, 80, 1024)])
def test_heads_nt_products_match_the_gemm_bit_for_bit(loss_type, B, T, F, H2):
    """The split form's P1 = LReLU(Y W1^T + b1) and dY = dP1 W1 on the 128-row kernel
    (mlvae_heads_set_nt_mode 2; the default from 64K frames -- the last shape) against the 256²
    GEMM (mode 0): every output of the heads launch bit-identical (the same k-order per output),
    ragged 128-row blocks included."""
    need_gpu()
    torch.manual_seed(B + T + F + H2 + loss_type)
    C, N = 64, B * T
    l = lib()
    f = dict(device="cuda", dtype=torch.float32)
    Y = torch.randn(N, H2).to(torch.bfloat16).cuda()
    W1 = (torch.randn(2 * C, H2) / math.sqrt(H2)).to(torch.bfloat16)
    dW1, dW1t = W1.cuda(), W1.t().contiguous().cuda()
    b1 = (torch.randn(2 * C) * 0.1).cuda()
    W2 = [(torch.randn(C, C) / 8).cuda() for _ in range(2)]
    b2 = [(torch.randn(C) * 0.1).cuda() for _ in range(2)]
    W3 = [(torch.randn(F, C) / 8).cuda() for _ in range(2)]
    b3 = [(torch.randn(F) * 0.1).cuda() for _ in range(2)]
    x = torch.randn(N, F).cuda()
    lens = (torch.rand(B) * 0.7 + 0.3).cuda()
    lik = loss_type == 0

    def run(mode):
        check(l.mlvae_heads_set_nt_mode(mode))
        o = {k: torch.zeros(N, n, device="cuda", dtype=torch.bfloat16)
             for k, n in (("p1", 2 * C), ("p2m", C), ("p2v", C), ("dmux", F), ("dlvx", F), ("dp2m", C),
                          ("dp2v", C), ("dp1", 2 * C))}
        o.update({k: torch.zeros(N, n, **f) for k, n in (("mux", F), ("lvx", F), ("dy", H2))})
        parts = torch.zeros(l.mlvae_heads_partials_count(B, T), **f)
        ws = torch.zeros(l.mlvae_heads_bias_workspace_size(B, T, F, C) // 4 + 1, **f)
        db = [torch.zeros(n, **f) for n in (F, F, C, C, 2 * C)]
        check(l.mlvae_heads_fused_ex(B, T, F, C, H2, loss_type, 1, Y.data_ptr(), dW1.data_ptr(), dW1t.data_ptr(),
                                     P(b1), P(W2[0]), P(b2[0]), P(W3[0]), P(b3[0]), P(W2[1]), P(b2[1]),
                                     P(W3[1]), P(b3[1]), P(x), P(lens), None, 0.7, P(o["p1"]), P(o["p2m"]),
                                     P(o["p2v"]), P(o["mux"]), P(o["lvx"]), P(o["dmux"]),
                                     P(o["dlvx"]) if lik else None, P(o["dp2m"]), P(o["dp2v"]), P(o["dp1"]),
                                     P(o["dy"]), P(parts), P(ws), ws.numel() * 4, P(db[0]), P(db[1]), P(db[2]),
                                     P(db[3]), P(db[4]), 1, stream()))
        torch.cuda.synchronize()
        return o, parts, db

    try:
        ref, ref_parts, ref_db = run(0)
        new, new_parts, new_db = run(2)
    finally:
        check(l.mlvae_heads_set_nt_mode(1))
    assert new["p1"].float().abs().sum() > 0 and new["dy"].abs().sum() > 0
    for k in ref:
        assert torch.equal(ref[k], new[k]), k
    assert torch.equal(ref_parts, new_parts)
    for a, b in zip(ref_db, new_db):
        assert torch.equal(a, b)
    with pytest.raises(Exception):
        check(l.mlvae_heads_set_nt_mode(3))


@pytest.mark.parametrize("loss_type", [0, 1])
@pytest.mark.parametrize("B,T,F,H2", [(3, 50, 80, 256), (5, 77, 64, 128), (40, 500, 80, 1024), (140, 500, 80, 1024)])
def test_heads_split_bf16_forward(loss_type, B, T, F, H2):
    """mlvae_heads_fused_ex3 with w1_split (the accurate-ELBO forward): P1 = LReLU(Y (W1_hi + W1_lo)^T
    + b1) on the 128-row kernel, then stages 2-3 on split W2 / W3 / P2.  Against fp64 on the fp32
    weights (no operand rounding but the bf16 input Y): P1 within rounding of its bf16 storage, and
    mu_x / log_var_x -- from the saved bf16 P1 -- and the loss partials to ~1e-5 (plain bf16: ~1e-3).
    The backward outputs and the bias / weight gradients are the plain split form's (bf16)."""
    need_gpu()
    torch.manual_seed(B + T + F + H2 + loss_type + 11)
    C, N = 64, B * T
    l = lib()
    f = dict(device="cuda", dtype=torch.float32)
    Y = torch.randn(N, H2).to(torch.bfloat16).cuda()
    W1 = torch.randn(2 * C, H2) / math.sqrt(H2)
    W1b = W1.to(torch.bfloat16)
    dW1, dW1t = W1b.cuda(), W1b.t().contiguous().cuda()
    W1f = W1.cuda()
    b1 = (torch.randn(2 * C) * 0.1).cuda()
    W2 = [(torch.randn(C, C) / 8).cuda() for _ in range(2)]
    b2 = [(torch.randn(C) * 0.1).cuda() for _ in range(2)]
    W3 = [(torch.randn(F, C) / 8).cuda() for _ in range(2)]
    b3 = [(torch.randn(F) * 0.1).cuda() for _ in range(2)]
    x = torch.randn(N, F).cuda()
    lens = torch.linspace(0.3, 1.0, B).cuda()
    lik = loss_type == 0
    ws = torch.zeros(l.mlvae_heads_bias_workspace_size(B, T, F, C) // 4 + 1, **f)
    wgs = torch.zeros(l.mlvae_heads_wgrad_workspace_size(B, T, F, C) // 4 + 1, **f)
    w1s = torch.empty(2 * C, 2 * H2, device="cuda", dtype=torch.bfloat16)
    check(l.mlvae_bf16_split_rows(P(W1f), 2 * C, H2, 64, w1s.data_ptr(), stream()))

    def run(split):
        o = {k: torch.zeros(N, n, device="cuda", dtype=torch.bfloat16)
             for k, n in (("p1", 2 * C), ("p2m", C), ("p2v", C), ("dmux", F), ("dlvx", F),
                          ("dp2m", C), ("dp2v", C), ("dp1", 2 * C))}
        o.update(mux=torch.zeros(N, F, **f), lvx=torch.zeros(N, F, **f), dy=torch.zeros(N, H2, **f),
                 parts=torch.zeros(l.mlvae_heads_partials_count(B, T), **f))
        db = [torch.zeros(n, **f) for n in (F, F, C, C, 2 * C)]
        dw = [torch.zeros(F, C, **f), torch.zeros(F, C, **f), torch.zeros(C, C, **f), torch.zeros(C, C, **f)]
        check(l.mlvae_heads_fused_ex3(B, T, F, C, H2, loss_type, 1, Y.data_ptr(), dW1.data_ptr(),
                                      dW1t.data_ptr(), P(b1), P(W2[0]), P(b2[0]), P(W3[0]), P(b3[0]),
                                      P(W2[1]), P(b2[1]), P(W3[1]), P(b3[1]), P(x), P(lens), None, 0.7,
                                      P(o["p1"]), P(o["p2m"]), P(o["p2v"]), P(o["mux"]), P(o["lvx"]),
                                      P(o["dmux"]), P(o["dlvx"]) if lik else None, P(o["dp2m"]),
                                      P(o["dp2v"]), P(o["dp1"]), P(o["dy"]), P(o["parts"]), P(ws),
                                      ws.numel() * 4, *[P(t) for t in db], 1, P(wgs), wgs.numel() * 4,
                                      P(dw[0]), P(dw[1]) if lik else None, P(dw[2]), P(dw[3]) if lik else None,
                                      w1s.data_ptr() if split else None, stream()))
        torch.cuda.synchronize()
        return o, db, dw

    o, db, dw = run(True)
    p, _, _ = run(False)
    d = lambda t: t.detach().double().cpu()
    lr = lambda t: torch.where(t > 0, t, 0.01 * t)
    pre64 = d(Y) @ d(W1).t() + d(b1)
    p1_64 = lr(pre64)
    # relative to |P1| with a floor (an entry near 0 after cancellation carries the fp32 sum's
    # absolute error): the split P1 is within half a bf16 ulp of fp64, the plain one is not
    den = p1_64.abs() + 1e-3 * p1_64.abs().max()
    ulp = (d(o["p1"]) - p1_64).abs() / den
    ulp_plain = (d(p["p1"]) - p1_64).abs() / den
    # stages 2-3 from the kernel's own bf16 P1 (the mid kernel's input)
    outs, rec_sum = [], 0.0
    for h in range(2):
        p2 = lr(d(o["p1"])[:, h * C:(h + 1) * C] @ d(W2[h]).t() + d(b2[h]))
        outs.append(p2 @ d(W3[h]).t() + d(b3[h]))
    e_mu, e_mu_plain = rel_err(o["mux"], outs[0]), rel_err(p["mux"], outs[0])
    e_lv = rel_err(o["lvx"], outs[1])
    T_ = T
    valid = (torch.arange(T_).double()[None, :] < (lens.cpu().float() * T_)[:, None].double()).reshape(-1)
    xx = d(x)
    if lik:
        nll = 0.5 * (1.8378770351409912 + outs[1] + (xx - outs[0]) ** 2 / (torch.exp(outs[1]) + 1e-5))
    else:
        nll = (xx - outs[0]) ** 2
    rec_sum = (nll * valid[:, None]).sum().item()
    e_rec = abs(o["parts"].double().sum().item() - rec_sum) / abs(rec_sum)
    e_rec_plain = abs(p["parts"].double().sum().item() - rec_sum) / abs(rec_sum)
    print(f"\nsplit heads lt={loss_type} B={B} T={T} H2={H2}: P1 max {ulp.max():.2e} (plain {ulp_plain.max():.2e}) "
          f"mu_x {e_mu:.2e} (plain {e_mu_plain:.2e}) log_var_x {e_lv:.2e} rec sum {e_rec:.2e} (plain {e_rec_plain:.2e})")
    assert ulp.max() <= 1.1 * 2.0 ** -8 and ulp_plain.max() > ulp.max()   # half a bf16 ulp (+ fp32 sums)
    assert e_mu < 5e-5 and e_lv < 5e-5 and e_rec < 2e-5
    assert e_mu < 0.1 * e_mu_plain
    # the backward stays the plain split form's bf16 products, on this forward's (more exact) P1 /
    # P2: dY agrees with the plain form's to the bf16-forward differences (incl. LeakyReLU branches
    # the plain forward's weight rounding flips); the whole-step tests bound it against the oracle
    assert norm_rel(o["dy"], p["dy"]) < 0.1
    for a_ in db + dw[:1] + dw[2:3]:
        assert torch.isfinite(a_).all()
