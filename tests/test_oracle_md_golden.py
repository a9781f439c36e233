"""The MD-VAE upstream-LSTM oracle (oracle/md_cpu.py) against fixtures produced by the reference
modules themselves (tests/golden/make_golden_md.py): PhonemeRecognizer
(ref:src/modules/phoneme_recognizer.py:9-81) and BoundaryDetector
(ref:src/modules/boundary_detector.py:15-103), outputs and gradients of sum(out * cot)."""
import os

import numpy as np
import pytest
import torch

from oracle import md_cpu as M

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, f"{name}.npz")))


def params(rec):
    return {k[len("param/"):]: torch.from_numpy(v).requires_grad_(True)
            for k, v in rec.items() if k.startswith("param/")}


def rel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def check_grads(rec, p, x, outs, tol):
    total = sum((outs[k] * torch.from_numpy(rec[f"cot/{k}"])).sum() for k in outs)
    names = list(p)
    grads = torch.autograd.grad(total, [p[n] for n in names] + [x])
    for n, g in zip(names, grads[:-1]):
        assert rel(g, rec[f"grad/{n}"]) < tol, n
    assert rel(grads[-1], rec["grad_in/x"]) < tol


@pytest.mark.parametrize("name", ["md_phn_tiny", "md_phn_mid"])
def test_phoneme_recognizer_matches_reference(name):
    rec = load(name)
    B, T, D, H, NL, FC, n_ph, Lmax = (int(v) for v in rec["dims"])
    p = params(rec)
    x = torch.from_numpy(rec["x"]).requires_grad_(True)
    o = M.phoneme_recognizer(p, x, torch.from_numpy(rec["feat_lens"]), torch.from_numpy(rec["phn"]),
                             torch.from_numpy(rec["phn_lens"]), torch.from_numpy(rec["boundary"]), NL, 3)
    assert rel(o["out"], rec["out/out"]) < 1e-5
    assert rel(o["bce"], rec["out/bce"]) < 1e-5
    check_grads(rec, p, x, o, 1e-4)


@pytest.mark.parametrize("name", ["md_bnd_tiny", "md_bnd_mid"])
def test_boundary_detector_matches_reference(name):
    rec = load(name)
    B, T, D, H, NL, FC = (int(v) for v in rec["dims"])
    p = params(rec)
    x = torch.from_numpy(rec["x"]).requires_grad_(True)
    o = M.boundary_detector(p, x, torch.from_numpy(rec["boundary"]), torch.from_numpy(rec["u"]), NL, 3)
    for k in ("boundary_v", "bce", "kld"):
        assert rel(o[k], rec[f"out/{k}"]) < 1e-5, k
    check_grads(rec, p, x, o, 1e-4)


def test_boundary_mismatch_raises_like_the_reference():
    """The reference asserts len(boundaries) == L_i (phoneme_recognizer.py:65)."""
    rec = load("md_phn_tiny")
    bnd = torch.from_numpy(rec["boundary"]).clone()
    bnd[0, 1] = 1 - bnd[0, 1]
    out = torch.zeros(3, 20, 7)
    with pytest.raises(AssertionError):
        M.phn_bce(out, torch.from_numpy(rec["feat_lens"]), torch.from_numpy(rec["phn"]),
                  torch.from_numpy(rec["phn_lens"]), bnd)
