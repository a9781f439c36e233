"""auto_mix_prec (ref:src/models/md_model.py:60-76: autocast forward, GradScaler-scaled backward,
unscale, check_gradients, scaler.step, scaler.update) on the HIP path.

* module mode (autograd over the HIP ops): the autocast region is the ops' bf16-operand mode;
  the loss scale is a power of two, so a scaled-and-unscaled step equals the plain bf16 step --
  checked against a run without AMP in bf16 mode (post-Adam parameters), and the scaler is a
  checkpoint recoverable;
* the fused engine: auto_mix_prec selects its bf16 operand mode."""
import functools

import pytest
import torch

from gpu_utils import need_gpu

pytestmark = pytest.mark.gpu


def _model(tmp_path, amp, fused, tag):
    from brain import EpochCounter, InputNormalization
    from models.test_vanilla_vae.model import SBModel
    from modules.decoder import Decoder
    from modules.vanilla_vae import VanillaVAE
    torch.manual_seed(5)
    enc = VanillaVAE([16, 32, 32], 8)
    dec = Decoder(8, 32, 2, 0.0, [64, 16, 16, 16])
    hp = dict(normalizer=InputNormalization(), epoch_counter=EpochCounter(1),
              optimizer=functools.partial(torch.optim.Adam, lr=1e-3), metric_keys=["kld_loss", "recon_loss"],
              min_key="loss", output_dir=str(tmp_path / tag), precision="fp32" if amp else "bf16",
              kld_loss_weight=1e-3)
    m = SBModel(modules={"encoder": enc, "decoder": dec}, hparams=hp,
                run_opts={"device": "cuda", "auto_mix_prec": amp})
    m.use_fused_step = fused
    return m


def _fit(m):
    from utils.data_io import SyntheticSet
    from mlvae_hip import ops
    prev = ops.get_precision()
    ops.set_precision(m.hparams.precision)
    torch.manual_seed(11)   # the same eps draws in every run
    try:
        ds = SyntheticSet(24, 16, 30, 50, seed=2)
        m.fit(m.hparams.epoch_counter, ds, None, train_loader_kwargs={"batch_size": 8})
    finally:
        ops.set_precision(prev)
    torch.cuda.synchronize()
    return {k: v.detach().cpu().clone() for k, v in m.modules.state_dict().items()}


def test_module_mode_amp_step_equals_bf16_step(tmp_path):
    need_gpu()
    amp = _model(tmp_path, True, False, "amp")
    ref = _model(tmp_path, False, False, "ref")
    pa, pr = _fit(amp), _fit(ref)
    assert amp.engine is None and amp.scaler.get_scale() == 65536.0  # no overflow: scale kept
    assert amp.optimizer_step == 3
    for k in pa:
        assert torch.allclose(pa[k], pr[k], rtol=0, atol=1e-6), k
    init = _model(tmp_path, False, False, "init").modules.state_dict()
    assert any(not torch.equal(pa[k], init[k].cpu()) for k in pa)   # the steps were taken


def test_fused_engine_amp_selects_bf16_mode(tmp_path):
    need_gpu()
    m = _model(tmp_path, True, True, "fused")
    _fit(m)
    assert m.engine is not None and m.engine.cfg.prec == "bf16"


def test_amp_scaler_state_survives_resume(tmp_path):
    """The GradScaler is registered before on_fit_start's recovery (SpeechBrain builds it with
    the Brain), so a resumed run restores the loss scale and the growth tracker."""
    need_gpu()
    from brain.checkpoints import Checkpointer
    a = _model(tmp_path, True, False, "amp_a")
    a.checkpointer = Checkpointer(tmp_path / "ckpt")
    _fit(a)
    a.scaler.update(new_scale=1024.0)  # a state the defaults cannot reproduce
    scale, tracker = a.scaler.get_scale(), a.scaler.state_dict()["_growth_tracker"]
    a.checkpointer.save_checkpoint(meta={"loss": 1.0})
    b = _model(tmp_path, True, False, "amp_b")
    b.checkpointer = Checkpointer(tmp_path / "ckpt")
    b.on_fit_start()
    sd = b.scaler.state_dict()
    assert sd["scale"] == scale == 1024.0 and sd["_growth_tracker"] == tracker
