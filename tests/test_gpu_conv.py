"""Conv1d encoder variant (BASELINE.json configs[3]) on the HIP path (csrc/conv.hip).

* kernels, through the C ABI, against fp64 restatements on the SAME bf16-rounded operands (the
  kernels multiply bf16 operands and accumulate in fp32): forward (+ LeakyReLU), input gradient
  (+ the LeakyReLU derivative of the layer below), weight + bias gradients -- 2e-5 max-relative,
  including T shorter than the kernel, utterances ending mid-tile and a K = 1 layer;
* modules.conv_vae.ConvVAE against the oracle encoder (torch conv1d, fp32) at bf16 tolerance;
* the whole fused training step at configs[3]'s utterance length (T = 2000; B = 16 to bound the
  oracle's CPU time) against oracle.vae_cpu.train_step, with the bf16 bounds of
  test_gpu_parity_workload.py.
The reference has no Conv1d: parity is against torch.nn.Conv1d semantics (unpinned)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from gpu_utils import P, need_gpu, norm_rel, rel_err, stream
from mlvae_hip._lib import check, lib

pytestmark = pytest.mark.gpu

SHAPES = [(3, 70, 80, 64, 5), (2, 130, 64, 64, 3), (2, 5, 16, 16, 9), (4, 64, 48, 32, 1), (1, 2000, 80, 64, 5),
          (5, 129, 64, 128, 7)]


def _bf(t):
    return t.to(torch.bfloat16).double()


def _conv64(x, w, b=None):
    return Fn.conv1d(x.transpose(1, 2), w, b, padding=w.shape[2] // 2).transpose(1, 2)


@pytest.mark.parametrize("B,T,Cin,Cout,K", SHAPES)
def test_conv1d_forward_and_dgrad(B, T, Cin, Cout, K):
    need_gpu()
    torch.manual_seed(B * 7 + T + K)
    x = torch.randn(B, T, Cin)
    w = torch.randn(Cout, Cin, K) / (Cin * K) ** 0.5
    b = torch.randn(Cout)
    y = torch.empty(B, T, Cout, device="cuda")
    xd, wd, bd = x.cuda(), w.cuda(), b.cuda()   # (device copies held until the launch has run)
    check(lib().mlvae_conv1d_fwd(B, T, Cin, Cout, K, P(xd), Cin, P(wd), P(bd), 1, P(y), Cout, stream()))
    torch.cuda.synchronize()
    ref = Fn.leaky_relu(_conv64(_bf(x), _bf(w), b.double()), 0.01)
    assert rel_err(y, ref) < 2e-5
    # dx = conv^T(dy) * lrelu'(aux): aux = a LeakyReLU output of the layer below
    dy = torch.randn(B, T, Cout)
    aux = torch.randn(B, T, Cin)
    dx = torch.empty(B, T, Cin, device="cuda")
    dyd, auxd = dy.cuda(), aux.cuda()
    check(lib().mlvae_conv1d_dgrad(B, T, Cin, Cout, K, P(dyd), Cout, P(wd), P(auxd), Cin, P(dx), Cin, stream()))
    torch.cuda.synchronize()
    xv = torch.zeros(B, T, Cin, dtype=torch.float64, requires_grad=True)
    (_conv64(xv, _bf(w)) * _bf(dy)).sum().backward()
    ref = xv.grad * torch.where(aux > 0, 1.0, 0.01).double()
    assert rel_err(dx, ref) < 2e-5


@pytest.mark.parametrize("B,T,Cin,Cout,K", [s for s in SHAPES if s[3] <= 64 and s[4] * ((s[2] + 15) // 16 * 16) <= 512])
def test_conv1d_weight_gradient(B, T, Cin, Cout, K):
    need_gpu()
    assert lib().mlvae_conv1d_supported(Cin, Cout, K)
    torch.manual_seed(B + T * 3 + Cin)
    x = torch.randn(B, T, Cin)
    dy = torch.randn(B, T, Cout)
    nb = lib().mlvae_conv1d_wgrad_workspace_size(B, T, Cin, Cout, K)
    ws = torch.empty(nb // 4 + 1, device="cuda")
    dw = torch.empty(Cout, Cin, K, device="cuda")
    db = torch.empty(Cout, device="cuda")
    dyd, xd = dy.cuda(), x.cuda()
    check(lib().mlvae_conv1d_wgrad(B, T, Cin, Cout, K, P(dyd), Cout, P(xd), Cin, P(dw), P(db),
                                   P(ws), ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    wv = torch.zeros(Cout, Cin, K, dtype=torch.float64, requires_grad=True)
    (_conv64(_bf(x), wv) * _bf(dy)).sum().backward()
    assert rel_err(dw, wv.grad) < 2e-5
    assert rel_err(db, dy.double().sum((0, 1))) < 1e-5
    # deterministic: a second launch gives the same bits
    dw2 = torch.empty_like(dw)
    check(lib().mlvae_conv1d_wgrad(B, T, Cin, Cout, K, P(dyd), Cout, P(xd), Cin, P(dw2), P(db),
                                   P(ws), ws.numel() * 4, stream()))
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2)


def _encoder_bf16_operands(p, x, eps):
    """oracle.vae_cpu.encoder_forward in fp64 with every matrix-product operand rounded to bf16
    as the kernels round them (activations, weights; biases and the reparameterisation stay
    exact).  With iid random cotangents the plain fp32 oracle differs from ANY bf16-operand
    encoder by 5-6 % in the conv-layer gradients (LeakyReLU derivative flips of near-zero
    pre-activations; reproduced on the CPU by this same emulation), so the tight comparison is
    against this restatement."""
    r = lambda t: t.to(torch.bfloat16).double()
    h = x
    for i in (0, 2):
        w = p[f"encoder.conv.0.blocks.{i}.weight"]
        h = Fn.leaky_relu(_conv64(r(h), r(w), p[f"encoder.conv.0.blocks.{i}.bias"]), 0.01)
    mean = Fn.linear(r(h), r(p["encoder.mean_fc.weight"]), p["encoder.mean_fc.bias"])
    lv = Fn.linear(r(h), r(p["encoder.log_var_fc.weight"]), p["encoder.log_var_fc.bias"])
    return {"mean": mean, "log_var": lv, "sampled_h": eps * torch.exp(0.5 * lv) + mean,
            "loss": -0.5 * (1 + lv - mean.pow(2) - lv.exp())}


def test_conv_vae_module_matches_oracle():
    need_gpu()
    from mlvae_hip import ops
    from modules.conv_vae import ConvVAE
    from oracle import vae_cpu as O
    prev = ops.get_precision()
    ops.set_precision("bf16")
    try:
        torch.manual_seed(3)
        enc = ConvVAE([80, 64, 64], 32, kernel_size=5)
        p32 = {f"encoder.{k}": v.detach().clone() for k, v in enc.named_parameters()}
        p = {k: v.double().requires_grad_(True) for k, v in p32.items()}
        enc = enc.cuda()
        B, T = 4, 333
        x = torch.randn(B, T, 80)
        eps = torch.randn(B, T, 32)
        xd = x.cuda().requires_grad_(True)
        out = enc(xd, eps=eps.cuda())
        plain = O.encoder_forward(p32, x, eps)
        for k in ("mean", "log_var", "sampled_h", "loss"):
            assert norm_rel(out[k], plain[k]) < 1e-2, k
        xv = x.double().requires_grad_(True)
        ref = _encoder_bf16_operands(p, xv, eps.double())
        for k in ("mean", "log_var", "sampled_h", "loss"):
            assert norm_rel(out[k], ref[k]) < 1e-4, k   # (bf16 ties of fp32 vs fp64 sums)
        cot = {k: torch.randn(ref[k].shape, dtype=torch.float64) for k in ("sampled_h", "loss")}
        sum((out[k] * cot[k].float().cuda()).sum() for k in cot).backward()
        sum((ref[k] * cot[k]).sum() for k in cot).backward()
        errs = {k: norm_rel(v.grad, p[f"encoder.{k}"].grad) for k, v in enc.named_parameters()}
        errs["x"] = norm_rel(xd.grad, xv.grad)
        print("\n[ConvVAE module bf16 vs bf16-operand oracle] " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
        for k, v in errs.items():   # what remains is the backward's own bf16 operand rounding
            assert v < 2e-2, k
    finally:
        ops.set_precision(prev)


def test_c4_conv_encoder_training_step_matches_oracle():
    """configs[3]: Conv1d encoder (K = 5), long utterances (T = 2000), the whole fused step
    (conv encoder + reparam/KL + BiLSTM 2x512 with dropout + heads + clip + Adam) vs the oracle."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig, VAEEngine
    from oracle import vae_cpu as O
    from philox_np import dropout_mask
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16", enc_conv=5)
    B, T, seed = 16, 2000, 4242
    g = torch.Generator().manual_seed(seed)
    params = O.init_params(cfg.F, cfg.E, cfg.Z, cfg.H, cfg.L, cfg.C, seed=seed, enc_conv=5)
    x = torch.randn(B, T, cfg.F, generator=g)
    lens = torch.linspace(0.55, 1.0, B)
    eng = VAEEngine(cfg, params=params, seed=seed)
    eng.train_step(x.cuda(), lens.cuda())
    torch.cuda.synchronize()
    eng.check_errors()
    w = eng.work(B, T)
    eps = w.eps_used.detach().cpu().view(B, T, cfg.Z)
    s = (eng.seed * 1000003 + 0) & ((1 << 63) - 1)
    masks = torch.from_numpy(dropout_mask(s, B * T * 2 * cfg.H, cfg.dropout)).view(1, B, T, 2 * cfg.H)
    new_ref, rec = O.train_step(params, {}, x, lens, eps, dict(L=cfg.L, loss_type="likelihood", kld_weight=1e-3),
                                masks, impl="aten")
    out = rec["out"]
    e_loss = abs(w.loss[2].item() - out["loss"].item()) / abs(out["loss"].item())
    e_mu = norm_rel(w.ML[:, :cfg.Z].reshape(B, T, cfg.Z), out["enc"]["mean"])
    e_lv = norm_rel(w.ML[:, cfg.Z:].reshape(B, T, cfg.Z), out["enc"]["log_var"])
    e_mux = norm_rel(w.MUX.reshape(B, T, -1), out["dec"]["mean"])
    grads = {k: norm_rel(gr, rec["grads"][k]) for k, gr in eng.named_grads().items()}
    par = max((eng.view(k).cpu() - v).abs().max().item() for k, v in new_ref.items())
    worst = max(grads, key=grads.get)
    print(f"\n[c4 conv K=5 B={B} T={T}] loss {e_loss:.2e} mu {e_mu:.2e} log_var {e_lv:.2e} mu_x {e_mux:.2e} "
          f"grads max {grads[worst]:.2e} ({worst}) median {float(np.median(list(grads.values()))):.2e} "
          f"params {par:.2e}")
    assert e_loss <= 1e-3
    assert e_mu <= 1e-2 and e_lv <= 1e-2 and e_mux <= 1e-2
    print(" ".join(f"{k} {v:.2e}" for k, v in grads.items() if k.startswith("encoder.")))
    for k, v in grads.items():
        assert v <= 3e-2, (k, v)
        if k.startswith("decoder.rnn."):  # (a one-step time shift of h in dW_hh_l0 gave 4.6e-2)
            assert v <= 1.5e-2, (k, v)
    assert par <= 2.5e-3
