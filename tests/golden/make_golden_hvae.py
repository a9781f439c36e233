"""Golden fixtures for the GMM-VAE and Hierarchical-VAE encoders.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (never on the GPU box).  It reuses the
import shims of ``make_golden.py`` (speechbrain stand-ins, aliased ruamel) and calls the
reference's own modules from ``/root/reference/src``; only ``.npz`` data is written.

Reference code exercised (read-only):
  * ``modules.gmm_vae.GMMVAE``            ref:src/modules/gmm_vae.py:8-67
  * ``modules.h_vae.HierarchicalVAE``     ref:src/modules/h_vae.py:12-72
  * ``utils.data_utils.apply_weight``     ref:src/utils/data_utils.py:32-64

Randomness is injected so the GPU path can replay it:
  * ``torch.randn_like`` (reparameterise, ref:src/modules/gmm_vae.py:52, vanilla_vae.py:39)
    returns recorded eps tensors, in call order;
  * ``Tensor.exponential_`` (the draw inside ``F.gumbel_softmax``, ref:src/modules/gmm_vae.py:31)
    fills recorded Exp(1) samples, so gumbels = -log(E).
Gradients are recorded for a scalar sum(out_k * cot_k) over every output with seeded cotangents.

Usage:  cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden_hvae.py
"""
import json
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden  # noqa: E402,F401  (installs the generator-only shims, puts ref src on path)
from modules.gmm_vae import GMMVAE  # noqa: E402  (reference)
from modules.h_vae import HierarchicalVAE  # noqa: E402  (reference)
from utils.data_utils import apply_weight  # noqa: E402  (reference)

OUT_DIR = make_golden.OUT_DIR


class _Inject:
    """Replay eps (randn_like, in order) and Exp(1) draws (exponential_, in order)."""

    def __init__(self, eps_list, exp_list):
        self.eps, self.exp = list(eps_list), list(exp_list)

    def __enter__(self):
        self._rl, self._ex = torch.randn_like, torch.Tensor.exponential_
        eps, exp = self.eps, self.exp
        torch.randn_like = lambda t, *a, **k: eps.pop(0).clone()
        torch.Tensor.exponential_ = lambda self_, *a, **k: self_.copy_(exp.pop(0))
        return self

    def __exit__(self, *exc):
        torch.randn_like, torch.Tensor.exponential_ = self._rl, self._ex
        assert not self.eps and not self.exp, "not every injected draw was consumed"


def _record(rec, prefix, module, outs, inputs, g):
    """Outputs, cotangents and d(sum out*cot)/d(params, inputs)."""
    total = 0.0
    for k, v in outs.items():
        cot = torch.randn(v.shape, generator=g)
        rec[f"{prefix}cot/{k}"] = cot.numpy()
        rec[f"{prefix}out/{k}"] = v.detach().numpy()
        total = total + (v * cot).sum()
    params = list(module.named_parameters())
    grads = torch.autograd.grad(total, [p for _, p in params] + list(inputs.values()),
                                allow_unused=True)
    for (n, p), gr in zip(params, grads[:len(params)]):
        rec[f"{prefix}grad/{n}"] = (gr if gr is not None else torch.zeros_like(p)).numpy()
    for k, gr in zip(inputs, grads[len(params):]):
        rec[f"{prefix}grad_in/{k}"] = gr.numpy()


def gmm_case(name, B, T, F, E, Z, N, seed):
    torch.manual_seed(seed)
    m = GMMVAE(fc_sizes=[F, E, E], latent_size=Z, num_components=N)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, T, F, generator=g).requires_grad_(True)
    eps = torch.randn(B, T, N * Z, generator=g)
    expo = torch.empty(B, T, N).exponential_(generator=g)
    rec = {"x": x.detach().numpy(), "eps": eps.numpy(), "expo": expo.numpy()}
    for n, p in m.named_parameters():
        rec["init/" + n] = p.detach().numpy()
    with _Inject([eps], [expo]):
        out = m(x)
    _record(rec, "", m, out, {"x": x}, g)
    meta = dict(kind="gmm", B=B, T=T, F=F, E=E, Z=Z, N=N, seed=seed, tau=0.1,
                param_names=[n for n, _ in m.named_parameters()])
    rec["meta_json"] = np.array(json.dumps(meta))
    path = os.path.join(OUT_DIR, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print("wrote", path)


def hvae_case(name, B, T, F, E, Z, N, seed):
    torch.manual_seed(seed)
    m = HierarchicalVAE(fc_sizes=[F, E, E], latent_size=Z, num_components=N)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, T, F, generator=g).requires_grad_(True)
    pi = torch.softmax(torch.randn(B, T, 2, generator=g), -1).requires_grad_(True)
    eps_v = torch.randn(B, T, Z, generator=g)
    eps_g = torch.randn(B, T, N * Z, generator=g)
    expo = torch.empty(B, T, N).exponential_(generator=g)
    rec = {"x": x.detach().numpy(), "pi": pi.detach().numpy(), "eps_v": eps_v.numpy(),
           "eps_g": eps_g.numpy(), "expo": expo.numpy()}
    for n, p in m.named_parameters():
        rec["init/" + n] = p.detach().numpy()
    with _Inject([eps_v, eps_g], [expo]):
        out = m(x, pi)
    flat = {k: v for k, v in out.items() if k != "losses"}
    flat["vae_kld_loss"] = out["losses"]["vae_kld_loss"]
    _record(rec, "", m, flat, {"x": x, "pi": pi}, g)
    meta = dict(kind="hvae", B=B, T=T, F=F, E=E, Z=Z, N=N, seed=seed, tau=0.1,
                param_names=[n for n, _ in m.named_parameters()])
    rec["meta_json"] = np.array(json.dumps(meta))
    path = os.path.join(OUT_DIR, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print("wrote", path)


def apply_weight_case(name, seed):
    g = torch.Generator().manual_seed(seed)
    rec = {}
    for tag, shape in (("flat", (2, 5, 3 * 4)), ("split", (2, 5, 3, 4))):
        x = torch.randn(*shape, generator=g)
        w = torch.softmax(torch.randn(2, 5, 3, generator=g), -1)
        rec[f"{tag}/x"], rec[f"{tag}/w"] = x.numpy(), w.numpy()
        rec[f"{tag}/y"] = apply_weight(x, w).numpy()
    path = os.path.join(OUT_DIR, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print("wrote", path)


if __name__ == "__main__":
    torch.set_num_threads(1)
    gmm_case("gmm_tiny", B=3, T=7, F=8, E=16, Z=4, N=3, seed=21)
    gmm_case("gmm_mid", B=2, T=40, F=80, E=64, Z=32, N=4, seed=22)
    hvae_case("hvae_tiny", B=3, T=7, F=8, E=16, Z=4, N=3, seed=23)
    hvae_case("hvae_mid", B=2, T=40, F=80, E=64, Z=32, N=2, seed=24)
    apply_weight_case("apply_weight", seed=25)
