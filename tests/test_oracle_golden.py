"""Pin the CPU oracle (oracle/vae_cpu.py) to fixtures produced by the reference
itself (tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from golden_utils import CASES, GOLDEN, cfg_of, load_case
from oracle import vae_cpu as O


def _rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("impl", ["loop", "aten"])
@pytest.mark.parametrize("case", CASES)
def test_train_steps_match_reference(case, impl):
    meta, x, lens, params, steps = load_case(case)
    cfg = cfg_of(meta)
    state = {}
    p = params
    for st in steps:
        masks = st.get("dropout_mask") if meta["train_dropout"] else None
        p, rec = O.train_step(p, state, x, lens, st["eps"], cfg, masks, impl)
        out = rec["out"]
        # fp32 forward: exact algorithmic restatement -> tight bounds
        assert _rel(out["enc"]["mean"], st["enc_mean"]) < 1e-6
        assert _rel(out["enc"]["log_var"], st["enc_log_var"]) < 1e-6
        assert _rel(out["enc"]["sampled_h"], st["enc_sampled_h"]) < 1e-6
        assert _rel(out["dec"]["mean"], st["dec_mean"]) < 1e-5
        assert _rel(out["dec"]["log_var"], st["dec_log_var"]) < 1e-5
        assert _rel(out["dec"]["losses"]["recon_loss"], st["dec_recon"]) < 1e-5
        for k in ("kld_loss", "recon_loss", "loss"):
            assert abs(out[k].item() - st[k].item()) <= 1e-6 * abs(st[k].item()), k
        for k, g in rec["grads"].items():
            assert _rel(g, st["grads"][k]) < 1e-4, k
        assert abs(rec["grad_norm"].item() - st["grad_norm"].item()) < 1e-5 * st["grad_norm"].item()
        for k, v in p.items():
            assert (v - st["params"][k]).abs().max().item() < 2e-6, k


def test_length_mask_quirk():
    d = np.load(os.path.join(GOLDEN, "masks.npz"))
    for T in (17, 50, 500):
        lens = torch.from_numpy(d[f"T{T}/lens"])
        m = O.length_to_mask(lens, T)
        np.testing.assert_array_equal(m.sum(1).numpy(), d[f"T{T}/valid_frames"])
        r = torch.from_numpy(d[f"T{T}/rand"])
        for red, key in (("mean", "maskmean_rand"), ("batchmean", "batchmean_rand"),
                         ("batch", "batch_rand")):
            np.testing.assert_allclose(O.apply_lens_to_loss(r, lens, red).numpy(),
                                       d[f"T{T}/{key}"], rtol=1e-6)
    # the T=500 quirk named in SURVEY.md 8(a) row 9: 127 -> 128 valid frames
    assert O.length_to_mask(torch.tensor([127 / 500]), 500).sum().item() == 128


def test_loss_weights():
    with open(os.path.join(GOLDEN, "loss_weights.json")) as f:
        cases = json.load(f)
    for c in cases:
        ws = O.loss_weights(c["keys"], c["hparams"])
        total = sum(torch.tensor(w, dtype=torch.float32) * torch.tensor(v)
                    for w, v in zip(ws, c["values"]))
        assert abs(float(total) - c["total"]) < 1e-6


def test_loop_matches_aten_fp64():
    torch.manual_seed(0)
    p = O.init_params(8, 16, 4, 8, 2, 16, dtype=torch.float64)
    x = torch.randn(2, 9, 8, dtype=torch.float64)
    eps = torch.randn(2, 9, 4, dtype=torch.float64)
    cfg = dict(L=2, loss_type="likelihood")
    a = O.forward_loss(p, x, torch.tensor([1.0, 0.6]), eps, cfg, impl="loop")["loss"]
    b = O.forward_loss(p, x, torch.tensor([1.0, 0.6]), eps, cfg, impl="aten")["loss"]
    assert abs(a.item() - b.item()) < 1e-12
