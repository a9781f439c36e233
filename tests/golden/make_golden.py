"""Generate the golden fixtures that pin ``oracle/`` to the reference.

TEST INFRASTRUCTURE ONLY.  This script runs in the build container (never on
the GPU box: ``/root/reference`` does not exist there).  It imports the
reference's own modules from ``/root/reference/src`` and records their
outputs on small seeded inputs as ``.npz`` fixtures next to this file.  Only
the fixtures (data) are committed alongside this script; no reference source
is copied.

Reference code exercised (read-only):
  * ``modules.vanilla_vae.VanillaVAE``   ref:src/modules/vanilla_vae.py:9-45
  * ``modules.decoder.Decoder``          ref:src/modules/decoder.py:10-53
  * ``modules.fc_block.FCBlock``         ref:src/modules/fc_block.py:4-21
  * ``utils.data_utils.apply_lens_to_loss`` ref:src/utils/data_utils.py:67-104
  * ``models.md_model.MDModel.compute_and_save_losses``
                                          ref:src/models/md_model.py:189-213
  * Adam from the recipe yaml (``!name:torch.optim.Adam lr: 1e-3``)
                                          ref:src/models/test_vanilla_vae/model.yaml:45-47

Two things the reference imports are not in this container and are supplied
by small stand-ins *inside this script only*:
  * ``speechbrain.nnet.losses.length_to_mask`` (SpeechBrain 0.5.x semantics:
    ``arange(T, dtype=lens.dtype) < lens*T``) -- this boundary is "parity
    unpinned" (no reference test pins it).
  * ``ruamel.yaml`` for ``hyperpyyaml`` -- the conda pure-python
    ``ruamel_yaml`` 0.15.100 is aliased, as SURVEY.md section 8(c) describes.
SpeechBrain's ``check_gradients`` is un-vendored; it is restated here as
``torch.nn.utils.clip_grad_norm_(params, 5.0)`` (SB default max_grad_norm).

Usage (from /tmp, no bytecode written anywhere):
    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden.py
"""
import importlib.util
import json
import os
import sys
import types
import warnings

sys.dont_write_bytecode = True

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# import shims (generator-only)
# --------------------------------------------------------------------------
def _install_ruamel():
    path = "/opt/conda/lib/python3.9/site-packages/ruamel_yaml/__init__.py"
    spec = importlib.util.spec_from_file_location(
        "ruamel_yaml", path, submodule_search_locations=[os.path.dirname(path)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ruamel_yaml"] = mod
    spec.loader.exec_module(mod)
    ruamel = types.ModuleType("ruamel")
    ruamel.yaml = mod
    sys.modules["ruamel"] = ruamel
    sys.modules["ruamel.yaml"] = mod
    sys.modules["ruamel.yaml.comments"] = importlib.import_module("ruamel_yaml.comments")


def _length_to_mask(length, max_len=None, dtype=None, device=None):
    assert len(length.shape) == 1
    if max_len is None:
        max_len = length.max().long().item()
    mask = torch.arange(max_len, device=length.device, dtype=length.dtype).expand(
        len(length), max_len) < length.unsqueeze(1)
    return torch.as_tensor(mask, dtype=dtype or length.dtype, device=device or length.device)


class _Recorder:
    def __init__(self, *a, **k):
        self.args, self.kwargs = a, k


def _install_speechbrain():
    sb = types.ModuleType("speechbrain")
    sb.__path__ = []

    class Brain:  # only what MDModel's class body needs
        pass

    class Stage:
        TRAIN, VALID, TEST = 1, 2, 3

    sb.Brain, sb.Stage = Brain, Stage
    mods = {"speechbrain": sb}
    for name in ["nnet", "nnet.losses", "utils", "utils.train_logger", "utils.epoch_loop",
                 "utils.checkpoints", "processing", "processing.features", "lobes",
                 "lobes.features"]:
        m = types.ModuleType("speechbrain." + name)
        m.__path__ = []
        mods["speechbrain." + name] = m
    mods["speechbrain.nnet.losses"].length_to_mask = _length_to_mask
    mods["speechbrain.nnet.losses"].compute_masked_loss = lambda *a, **k: None
    mods["speechbrain.utils.train_logger"].FileTrainLogger = _Recorder
    mods["speechbrain.utils.epoch_loop"].EpochCounter = type("EpochCounter", (_Recorder,), {})
    mods["speechbrain.utils.checkpoints"].Checkpointer = type("Checkpointer", (_Recorder,), {})
    mods["speechbrain.processing.features"].InputNormalization = type(
        "InputNormalization", (_Recorder,), {})
    mods["speechbrain.lobes.features"].Fbank = type("Fbank", (_Recorder,), {})
    sys.modules.update(mods)
    for full, m in mods.items():  # parent.child attributes so pydoc.locate can walk them
        if "." in full:
            parent, child = full.rsplit(".", 1)
            setattr(mods[parent], child, m)
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = _Recorder
    sys.modules["torch.utils.tensorboard"] = tb


_install_ruamel()
_install_speechbrain()
sys.path.insert(0, REF_SRC)

from modules.vanilla_vae import VanillaVAE  # noqa: E402  (reference)
from modules.decoder import Decoder  # noqa: E402  (reference)
from utils.data_utils import apply_lens_to_loss  # noqa: E402  (reference)
from models.md_model import MDModel  # noqa: E402  (reference)


class _FakeBrain:
    """Just enough of `self` for MDModel.compute_and_save_losses."""

    def __init__(self, kld_weight, batch_size):
        self.hparams = types.SimpleNamespace(kld_weight=kld_weight, batch_size=batch_size)
        self.stats_loggers = {}


def fp32_quirk_lens(T, count=2):
    """Lengths L whose fp32(L/T)*T lands above L (mask admits one more frame)."""
    out = []
    for L in range(1, T):
        rel = torch.tensor([L / T], dtype=torch.float32)
        if (rel * T).item() > L:
            out.append(L)
        if len(out) == count:
            break
    return out


def run_case(name, B, T, F, enc, z, H, L, dec_fc, loss_type, train_dropout, seed,
             n_steps=2, lens=None, kld_weight=1e-3, dropout=0.15):
    torch.manual_seed(seed)
    encoder = VanillaVAE(fc_sizes=[F, enc, enc], latent_size=z)
    decoder = Decoder(input_size=z, rnn_hidden_size=H, rnn_num_layers=L, rnn_dropout=dropout,
                      fc_sizes=[2 * H, dec_fc, dec_fc, F], loss_type=loss_type)
    modules = torch.nn.ModuleDict({"encoder": encoder, "decoder": decoder})
    # Parameter order = Brain's self.modules.parameters() order.
    names = [n for n, _ in modules.named_parameters()]
    init = {n: p.detach().clone() for n, p in modules.named_parameters()}
    opt = torch.optim.Adam(modules.parameters(), lr=1e-3)
    if train_dropout:
        modules.train()
    else:
        modules.eval()  # eval: LSTM inter-layer dropout off, eps still sampled

    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, T, F, generator=g)
    if lens is None:
        lens = torch.linspace(0.5, 1.0, B)
    lens = torch.as_tensor(lens, dtype=torch.float32)

    rec = {"x": x.numpy(), "lens": lens.numpy()}
    for k, v in init.items():
        rec["init/" + k] = v.numpy()

    real_randn_like = torch.randn_like
    for step in range(n_steps):
        eps = torch.randn(B, T, z, generator=g)
        torch.randn_like = lambda t, _e=eps: _e.clone()  # inject eps into reparameterize
        try:
            drop_seed = seed * 100 + step
            torch.manual_seed(drop_seed)
            enc_out = encoder(x)
            dec_out = decoder(enc_out["sampled_h"], x)
        finally:
            torch.randn_like = real_randn_like
        losses = {
            "kld_loss": apply_lens_to_loss(enc_out["loss"], lens),
            "recon_loss": apply_lens_to_loss(dec_out["losses"]["recon_loss"], lens),
        }
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            loss = MDModel.compute_and_save_losses(_FakeBrain(kld_weight, B), losses)
        opt.zero_grad()
        loss.backward()
        # A parameter with no gradient (e.g. the log-variance head under
        # loss_type='mse') is skipped by Adam and by clip_grad_norm_; that is
        # numerically identical to a zero gradient, which is what we record.
        grads = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
                 for n, p in modules.named_parameters()}
        total_norm = torch.nn.utils.clip_grad_norm_(modules.parameters(), 5.0)
        opt.step()
        pre = f"step{step}/"
        rec[pre + "eps"] = eps.numpy()
        rec[pre + "drop_seed"] = np.array(drop_seed)
        for k in ["mean", "log_var", "sampled_h", "loss"]:
            rec[pre + "enc_" + k] = enc_out[k].detach().numpy()
        rec[pre + "dec_mean"] = dec_out["mean"].detach().numpy()
        rec[pre + "dec_log_var"] = dec_out["log_var"].detach().numpy()
        rec[pre + "dec_recon"] = dec_out["losses"]["recon_loss"].detach().numpy()
        rec[pre + "kld_loss"] = losses["kld_loss"].detach().numpy()
        rec[pre + "recon_loss"] = losses["recon_loss"].detach().numpy()
        rec[pre + "loss"] = loss.detach().numpy()
        rec[pre + "grad_norm"] = total_norm.detach().numpy()
        for k, v in grads.items():
            rec[pre + "grad/" + k] = v.numpy()
        for n, p in modules.named_parameters():
            rec[pre + "param/" + n] = p.detach().clone().numpy()  # clone: Adam updates in place
        if train_dropout:
            # Reproduce nn.LSTM's inter-layer dropout draw: same seed, same
            # bernoulli_ over the TIME-MAJOR [T,B,2H] layer output (ATen runs
            # the stack time-major even with batch_first; checked below).
            torch.manual_seed(drop_seed)
            masks = [(torch.empty(T, B, 2 * H).bernoulli_(1 - dropout) / (1 - dropout))
                     .transpose(0, 1).contiguous() for _ in range(L - 1)]
            rec[pre + "dropout_mask"] = torch.stack(masks).numpy()
    meta = dict(B=B, T=T, F=F, enc=enc, z=z, H=H, L=L, dec_fc=dec_fc, loss_type=loss_type,
                train_dropout=train_dropout, seed=seed, n_steps=n_steps, kld_weight=kld_weight,
                dropout=dropout, lr=1e-3, max_grad_norm=5.0, param_names=names)
    rec["meta_json"] = np.array(json.dumps(meta))
    path = os.path.join(OUT_DIR, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"wrote {path}: loss step0 {rec['step0/loss']:.8f}")
    return rec


def mask_fixture():
    """length_to_mask at the T=500 quirk points and at T=17 (ref:src/utils/data_utils.py:86-92)."""
    out = {}
    for T in (17, 50, 500):
        q = fp32_quirk_lens(T, 3)
        Ls = sorted(set(q + [1, T // 2, T - 1, T]))
        lens = torch.tensor([L / T for L in Ls], dtype=torch.float32)
        loss = torch.ones(len(Ls), T, 3)
        mask = _length_to_mask(lens * T, max_len=T)
        out[f"T{T}/lens"] = lens.numpy()
        out[f"T{T}/valid_frames"] = mask.sum(1).numpy()
        out[f"T{T}/maskmean_of_ones"] = apply_lens_to_loss(loss, lens).numpy()
        g = torch.Generator().manual_seed(T)
        r = torch.rand(len(Ls), T, 3, generator=g)
        out[f"T{T}/rand"] = r.numpy()
        out[f"T{T}/maskmean_rand"] = apply_lens_to_loss(r, lens).numpy()
        out[f"T{T}/batchmean_rand"] = apply_lens_to_loss(r, lens, "batchmean").numpy()
        out[f"T{T}/batch_rand"] = apply_lens_to_loss(r, lens, "batch").numpy()
    path = os.path.join(OUT_DIR, "masks.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v for k, v in out.items() if k.endswith("valid_frames")})


def weights_fixture():
    """_kld rescale in compute_and_save_losses (ref:src/models/md_model.py:189-213)."""
    cases = []
    for keys, hp in [
        (["kld_loss", "recon_loss"], dict(kld_weight=1e-3, batch_size=32)),
        (["vae_kld_loss", "recon_loss"], dict(vae_kld_weight=0.5, batch_size=32)),
        (["kld_loss", "recon_loss"], dict(batch_size=8)),
    ]:
        fb = types.SimpleNamespace(hparams=types.SimpleNamespace(**hp), stats_loggers={})
        losses = {k: torch.tensor(float(i + 2)) for i, k in enumerate(keys)}
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            total = MDModel.compute_and_save_losses(fb, losses)
        cases.append(dict(keys=keys, hparams=hp, values=[float(v) for v in losses.values()],
                          total=float(total)))
    path = os.path.join(OUT_DIR, "loss_weights.json")
    with open(path, "w") as f:
        json.dump(cases, f, indent=1)
    print("wrote", path)


def config_fixture():
    """Resolved run.yaml + !include test_vanilla_vae/model.yaml (ref:src/prepare_experiment.py:15-25)."""
    import ruamel.yaml
    from hyperpyyaml import load_hyperpyyaml
    from hyperpyyaml.core import recursive_update

    overrides_str = ("dataset: SynAudioMNIST\nmodel_class: test_vanilla_vae\nmodel_name: vae\n"
                     "model: !include:../models/test_vanilla_vae/model.yaml\n"
                     "extra_overrides: {model: {n_epochs: 1, input_size: 80}}\n")
    overrides = ruamel.yaml.YAML().load(overrides_str)
    extra = overrides.pop("extra_overrides", {})
    cwd = os.getcwd()
    os.chdir(REF_SRC)
    try:
        with open("config/run.yaml") as fin:
            hp = load_hyperpyyaml(fin, [extra, overrides])
        recursive_update(hp, extra)
    finally:
        os.chdir(cwd)

    def plain(v):
        if isinstance(v, (int, float, str, bool)) or v is None:
            return v
        if isinstance(v, dict):
            return {str(k): plain(x) for k, x in v.items()}
        if isinstance(v, (list, tuple)):
            return [plain(x) for x in v]
        if isinstance(v, torch.nn.Module):
            return {"__module__": type(v).__name__, "repr": repr(v)}
        if hasattr(v, "func"):
            return {"__partial__": v.func.__module__ + "." + v.func.__qualname__,
                    "keywords": plain(dict(v.keywords))}
        return {"__object__": type(v).__name__,
                "kwargs": plain(getattr(v, "kwargs", {}))}

    out = plain(hp)
    path = os.path.join(OUT_DIR, "resolved_config.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


def dropout_replay_check(rec):
    """Check the replayed dropout mask reproduces nn.LSTM train-mode output."""
    meta = json.loads(str(rec["meta_json"]))
    H, L = meta["H"], meta["L"]
    lstm = torch.nn.LSTM(meta["z"], H, L, dropout=meta["dropout"], bidirectional=True,
                         batch_first=True)
    sd = {k[len("decoder.rnn."):]: torch.from_numpy(v) for k, v in
          ((k[len("init/"):], v) for k, v in rec.items() if k.startswith("init/"))
          if k.startswith("decoder.rnn.")}
    lstm.load_state_dict(sd)
    lstm.train()
    zin = torch.from_numpy(rec["step0/enc_sampled_h"])
    torch.manual_seed(int(rec["step0/drop_seed"]))
    ref_out = lstm(zin)[0]
    # manual two-layer with explicit mask
    mask = torch.from_numpy(rec["step0/dropout_mask"])
    h = zin
    for layer in range(L):
        one = torch.nn.LSTM(h.shape[-1], H, 1, bidirectional=True, batch_first=True)
        one.load_state_dict({k.replace(f"_l{layer}", "_l0"): v for k, v in sd.items()
                             if f"_l{layer}" in k})
        h = one(h)[0]
        if layer < L - 1:
            h = h * mask[layer]
    err = (h - ref_out).abs().max().item()
    print("dropout replay max err", err)
    assert err < 1e-6, err


if __name__ == "__main__":
    torch.set_num_threads(1)
    cfgs = dict(
        tiny_likelihood=dict(B=3, T=17, F=8, enc=16, z=4, H=8, L=2, dec_fc=16,
                             loss_type="likelihood", train_dropout=False, seed=11),
        tiny_mse=dict(B=3, T=17, F=8, enc=16, z=4, H=8, L=2, dec_fc=16, loss_type="mse",
                      train_dropout=False, seed=12),
        tiny_dropout=dict(B=3, T=17, F=8, enc=16, z=4, H=8, L=2, dec_fc=16,
                          loss_type="likelihood", train_dropout=True, seed=13),
        tiny_quirk_lens=dict(B=4, T=50, F=8, enc=16, z=4, H=8, L=2, dec_fc=16,
                             loss_type="likelihood", train_dropout=False, seed=14,
                             lens=[L / 50 for L in fp32_quirk_lens(50, 2)] + [1.0, 0.5]),
        mid_likelihood=dict(B=4, T=40, F=80, enc=64, z=32, H=32, L=2, dec_fc=64,
                            loss_type="likelihood", train_dropout=False, seed=15),
        one_layer=dict(B=2, T=9, F=8, enc=16, z=4, H=16, L=1, dec_fc=16,
                       loss_type="likelihood", train_dropout=False, seed=16),
    )
    recs = {k: run_case(k, **v) for k, v in cfgs.items()}
    dropout_replay_check(recs["tiny_dropout"])
    mask_fixture()
    weights_fixture()
    config_fixture()
