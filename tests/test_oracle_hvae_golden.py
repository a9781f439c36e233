"""Pin the GMM-VAE / H-VAE oracle (oracle/hvae_cpu.py) to fixtures produced by the reference
modules themselves (tests/golden/make_golden_hvae.py).  CPU only."""
import json
import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

from oracle import hvae_cpu as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GMM_CASES = ["gmm_tiny", "gmm_mid"]
HVAE_CASES = ["hvae_tiny", "hvae_mid"]


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(d["meta_json"]))
    t = lambda k: torch.from_numpy(np.array(d[k]))
    params = OrderedDict((k, t("init/" + k)) for k in meta["param_names"])
    sub = lambda pre: {k[len(pre):]: t(k) for k in d.files if k.startswith(pre)}
    return meta, params, {k: t(k) for k in d.files if "/" not in k and k != "meta_json"}, \
        sub("out/"), sub("cot/"), sub("grad/"), sub("grad_in/")


def rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def run_oracle(meta, params, ins):
    p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    x = ins["x"].clone().requires_grad_(True)
    if meta["kind"] == "gmm":
        out = O.gmm_vae_forward(p, x, ins["eps"], ins["expo"])
        leaves = {"x": x}
    else:
        pi = ins["pi"].clone().requires_grad_(True)
        out = O.hvae_forward(p, x, pi, ins["eps_v"], ins["eps_g"], ins["expo"])
        leaves = {"x": x, "pi": pi}
    return p, leaves, out


@pytest.mark.parametrize("case", GMM_CASES + HVAE_CASES)
def test_oracle_matches_reference(case):
    meta, params, ins, outs, cots, grads, grads_in = load(case)
    p, leaves, out = run_oracle(meta, params, ins)
    assert set(out) == set(outs)
    for k, v in outs.items():
        assert rel(out[k].detach(), v) < 1e-6, k
    total = sum((out[k] * cots[k]).sum() for k in outs)
    total.backward()
    for k, g in grads.items():
        got = p[k].grad if p[k].grad is not None else torch.zeros_like(g)
        assert rel(got, g) < 1e-5, k
    for k, g in grads_in.items():
        assert rel(leaves[k].grad, g) < 1e-5, k


def test_gumbel_weights_are_one_hot():
    for case in GMM_CASES:
        _, _, _, outs, *_ = load(case)
        w = outs["gmm_weight"]
        assert torch.allclose(w.sum(-1), torch.ones(w.shape[:-1]), atol=1e-6)
        assert ((w - w.round()).abs() < 1e-6).all()


def test_apply_weight_matches_reference():
    d = np.load(os.path.join(GOLDEN, "apply_weight.npz"), allow_pickle=False)
    for tag in ("flat", "split"):
        x, w, y = (torch.from_numpy(d[f"{tag}/{k}"]) for k in "xwy")
        assert rel(O.apply_weight(x, w), y) < 1e-6


@pytest.mark.parametrize("case", ["gmm_tiny", "hvae_tiny"])
def test_module_state_dict_matches_reference(case):
    """The HIP-backed modules keep the reference's parameter names and shapes (checkpoints load)."""
    from modules.gmm_vae import GMMVAE
    from modules.h_vae import HierarchicalVAE
    meta, params, *_ = load(case)
    cls = GMMVAE if meta["kind"] == "gmm" else HierarchicalVAE
    m = cls([meta["F"], meta["E"], meta["E"]], meta["Z"], meta["N"])
    sd = m.state_dict()
    assert list(sd) == meta["param_names"]
    assert all(sd[k].shape == params[k].shape for k in sd)
    m.load_state_dict(dict(params))
