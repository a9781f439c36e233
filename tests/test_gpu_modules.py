"""Module-level drop-in path (modules/*.py over mlvae_hip.ops autograd Functions) against the
reference's own numbers (golden fixtures) and against the fused engine."""
import pytest
import torch

from golden_utils import load_case
from gpu_utils import need_gpu, rel_err

pytestmark = pytest.mark.gpu


def _build(meta, params):
    from modules.decoder import Decoder
    from modules.vanilla_vae import VanillaVAE
    enc = VanillaVAE([meta["F"], meta["enc"], meta["enc"]], meta["z"])
    dec = Decoder(meta["z"], meta["H"], meta["L"], meta["dropout"],
                  [2 * meta["H"], meta["dec_fc"], meta["dec_fc"], meta["F"]], meta["loss_type"])
    mods = torch.nn.ModuleDict({"encoder": enc, "decoder": dec})
    mods.load_state_dict({k: v for k, v in params.items()})
    return mods.cuda()


@pytest.mark.parametrize("case", ["tiny_likelihood", "tiny_mse", "tiny_quirk_lens", "mid_likelihood"])
def test_modules_forward_backward_match_reference(case):
    need_gpu()
    from utils.data_utils import apply_lens_to_loss
    meta, x, lens, params, steps = load_case(case)
    mods = _build(meta, params)
    mods.eval()  # fixtures are eval-mode LSTM (no inter-layer dropout)
    st = steps[0]
    xd, ld = x.cuda(), lens.cuda()
    enc = mods["encoder"](xd, eps=st["eps"].cuda())
    dec = mods["decoder"](enc["sampled_h"], xd)
    kld = apply_lens_to_loss(enc["loss"], ld)
    rec = apply_lens_to_loss(dec["losses"]["recon_loss"], ld)
    loss = meta["kld_weight"] * kld + rec
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - st["loss"].item()) <= 1e-5 * abs(st["loss"].item())
    assert rel_err(enc["mean"], st["enc_mean"]) < 1e-5
    assert rel_err(enc["log_var"], st["enc_log_var"]) < 1e-5
    assert rel_err(dec["mean"], st["dec_mean"]) < 1e-4
    assert rel_err(dec["losses"]["recon_loss"], st["dec_recon"]) < 1e-4
    for k, p in mods.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        assert rel_err(g, st["grads"][k]) < 1e-3, k


def test_invalid_loss_type_raises():
    need_gpu()
    from modules.decoder import Decoder
    dec = Decoder(4, 8, 1, 0.0, [16, 8, 8, 6], loss_type="l1").cuda()
    with pytest.raises(ValueError, match="Invalid loss type"):
        dec(torch.randn(2, 5, 4, device="cuda"), torch.randn(2, 5, 6, device="cuda"))


def test_module_path_optimizer_matches_reference_step():
    """modules + mlvae_hip.optim (clip_grad_norm_ + Adam) reproduce the reference's post-Adam
    parameters of step 0."""
    need_gpu()
    from mlvae_hip import optim
    from utils.data_utils import apply_lens_to_loss
    meta, x, lens, params, steps = load_case("tiny_likelihood")
    mods = _build(meta, params)
    mods.eval()
    opt = optim.Adam(mods.parameters(), lr=1e-3)
    st = steps[0]
    xd, ld = x.cuda(), lens.cuda()
    enc = mods["encoder"](xd, eps=st["eps"].cuda())
    dec = mods["decoder"](enc["sampled_h"], xd)
    loss = meta["kld_weight"] * apply_lens_to_loss(enc["loss"], ld) + apply_lens_to_loss(
        dec["losses"]["recon_loss"], ld)
    loss.backward()
    norm = optim.clip_grad_norm_(list(mods.parameters()), 5.0)
    opt.step()
    torch.cuda.synchronize()
    assert abs(norm.item() - st["grad_norm"].item()) < 1e-4 * st["grad_norm"].item()
    for k, p in mods.named_parameters():
        assert (p.detach().cpu() - st["params"][k]).abs().max().item() < 1e-5, k


def test_engine_and_modules_agree_and_share_storage():
    """VAEEngine.from_modules: module parameters become views of the engine's flat buffer;
    one fused train step == module forward/backward + clip + Adam."""
    need_gpu()
    from mlvae_hip.engine import VAEEngine
    meta, x, lens, params, steps = load_case("mid_likelihood")
    a = _build(meta, params)
    b = _build(meta, params)
    st = steps[0]
    eng = VAEEngine.from_modules(a["encoder"], a["decoder"], prec="fp32")
    eng.cfg.dropout = 0.0
    eng.train_step(x.cuda(), lens.cuda(), eps=st["eps"].cuda())
    torch.cuda.synchronize()
    # engine updated the modules' own parameters in place
    for k, p in a.named_parameters():
        assert (p.detach().cpu() - st["params"][k]).abs().max().item() < 1e-5, k
    assert a["encoder"].mean_fc.weight.data_ptr() == eng.view("encoder.mean_fc.weight").data_ptr()
