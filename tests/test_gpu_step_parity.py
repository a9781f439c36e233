"""Whole-train-step parity: VAEEngine (HIP path, via the C ABI) vs the reference's own
numbers (tests/golden, produced by the reference modules) and vs the CPU oracle."""
import pytest
import torch

from golden_utils import CASES, cfg_of, load_case
from gpu_utils import need_gpu, norm_rel, rel_err
from mlvae_hip.engine import VAEConfig, VAEEngine
from oracle import vae_cpu as O

pytestmark = pytest.mark.gpu

# fp32 parity mode tolerances (north_star: ELBO within 1e-4 relative)
TOL_LOSS = 1e-5
TOL_OUT = 1e-4
TOL_GRAD = 1e-3
TOL_PARAM = 1e-5  # absolute, after Adam (lr 1e-3)


def _cfg(meta, prec="fp32"):
    return VAEConfig(F=meta["F"], E=meta["enc"], Z=meta["z"], H=meta["H"], L=meta["L"],
                     C=meta["dec_fc"], dropout=meta["dropout"] if meta["train_dropout"] else 0.0,
                     loss_type=meta["loss_type"], kld_weight=meta["kld_weight"], prec=prec)


@pytest.mark.parametrize("case", CASES)
def test_train_steps_match_golden(case):
    need_gpu()
    meta, x, lens, params, steps = load_case(case)
    eng = VAEEngine(_cfg(meta), params=params)
    xd, ld = x.cuda(), lens.cuda()
    for st in steps:
        masks = st["dropout_mask"].cuda() if meta["train_dropout"] else None
        loss = eng.train_step(xd, ld, eps=st["eps"].cuda(), dropout_masks=masks)
        torch.cuda.synchronize()
        eng.check_errors()
        w = eng.work(meta["B"], meta["T"])
        for i, k in enumerate(("kld_loss", "recon_loss", "loss")):
            assert abs(loss[i].item() - st[k].item()) <= TOL_LOSS * abs(st[k].item()), k
        B, T = meta["B"], meta["T"]
        Z = meta["z"]
        assert rel_err(w.ML[:, :Z].view(B, T, Z), st["enc_mean"]) < TOL_OUT
        assert rel_err(w.ML[:, Z:].view(B, T, Z), st["enc_log_var"]) < TOL_OUT
        assert rel_err(w.MUX.view(B, T, -1), st["dec_mean"]) < TOL_OUT
        assert rel_err(w.LVX.view(B, T, -1), st["dec_log_var"]) < TOL_OUT
        for k, g in eng.named_grads().items():
            assert rel_err(g, st["grads"][k]) < TOL_GRAD, k
        assert abs(eng.grad_norm.item() - st["grad_norm"].item()) < 1e-4 * st["grad_norm"].item()
        for k, v in eng.named_parameters().items():
            assert (v.cpu() - st["params"][k]).abs().max().item() < TOL_PARAM, k


@pytest.mark.parametrize("prec,tol_loss", [("fp32", 1e-5), ("bf16", 3e-3)])
def test_c2_shape_matches_oracle(prec, tol_loss):
    """c2 dimensions (F=80, enc 64, z=32, BiLSTM 2x512, dec-FC 64) at B=4, T=48."""
    need_gpu()
    torch.manual_seed(0)
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.0, prec=prec)
    params = O.init_params(80, 64, 32, 512, 2, 64, seed=1)
    B, T = 4, 48
    x = torch.randn(B, T, 80)
    lens = torch.tensor([1.0, 0.75, 0.5, 0.25])
    eps = torch.randn(B, T, 32)
    new_ref, rec = O.train_step(params, {}, x, lens, eps,
                                dict(L=2, loss_type="likelihood", kld_weight=1e-3), impl="aten")
    eng = VAEEngine(cfg, params=params)
    loss = eng.train_step(x.cuda(), lens.cuda(), eps=eps.cuda())
    torch.cuda.synchronize()
    eng.check_errors()
    assert abs(loss[2].item() - rec["out"]["loss"].item()) <= tol_loss * abs(rec["out"]["loss"].item())
    for k, g in eng.named_grads().items():
        if prec == "fp32":
            assert rel_err(g, rec["grads"][k]) < 1e-3, k
        else:  # bf16 operands: ||g - ref|| / ||ref|| (deep in the BPTT chain bf16 rounding adds up)
            assert norm_rel(g, rec["grads"][k]) < 0.1, (k, norm_rel(g, rec["grads"][k]))
