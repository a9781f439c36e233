"""Golden fixtures for the MD-VAE upstream LSTMs.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (never on the GPU box).  It reuses the
import shims of ``make_golden.py`` (speechbrain stand-ins, aliased ruamel) and calls the
reference's own modules from ``/root/reference/src``; only ``.npz`` data is written.

Reference code exercised (read-only):
  * ``modules.phoneme_recognizer.PhonemeRecognizer``   ref:src/modules/phoneme_recognizer.py:9-81
    (unidirectional nn.LSTM + FCBlock + the per-utterance duration-expanded BCE-with-logits)
  * ``modules.boundary_detector.BoundaryDetector``     ref:src/modules/boundary_detector.py:15-103
    (unidirectional nn.LSTM + two FCBlock/Softplus heads, Beta(1,9) KL, 10 Kumaraswamy draws)

Randomness is injected: ``torch.rand_like`` (the Kumaraswamy uniforms, boundary_detector.py:60)
returns recorded tensors in call order.  Gradients are recorded for sum(out_k * cot_k) over every
output with seeded cotangents.

Usage:  cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden_md.py
"""
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden  # noqa: E402,F401  (installs the generator-only shims, puts ref src on path)
from modules.boundary_detector import BoundaryDetector  # noqa: E402  (reference)
from modules.phoneme_recognizer import PhonemeRecognizer  # noqa: E402  (reference)

OUT_DIR = make_golden.OUT_DIR


def _segments(B, T, L, rel, g):
    """Per utterance: T_i = round(T * rel_i) frames split into L_i phoneme segments (first
    boundary at frame 0), and the phoneme labels.  Returns boundary [B, T] (float 0/1), phoneme
    ids [B, L] (long, zero padded), L_i / L."""
    bnd = torch.zeros(B, T)
    n_l = []
    for b in range(B):
        Ti = int(torch.round(torch.tensor(T * rel[b], dtype=torch.float32)).item())
        Li = int(torch.randint(2, min(L, Ti) + 1, (1,), generator=g).item())
        cuts = torch.randperm(Ti - 1, generator=g)[:Li - 1] + 1
        bnd[b, 0] = 1.0
        bnd[b, cuts] = 1.0
        n_l.append(Li)
    return bnd, torch.tensor(n_l)


def _record(rec, module, outs, inputs, g):
    total = 0.0
    for k, v in outs.items():
        cot = torch.randn(v.shape, generator=g)
        rec[f"cot/{k}"] = cot.numpy()
        rec[f"out/{k}"] = v.detach().numpy()
        total = total + (v * cot).sum()
    params = list(module.named_parameters())
    grads = torch.autograd.grad(total, [p for _, p in params] + list(inputs.values()), allow_unused=True)
    for (n, p), gr in zip(params, grads[:len(params)]):
        rec[f"param/{n}"] = p.detach().numpy()
        rec[f"grad/{n}"] = (gr if gr is not None else torch.zeros_like(p)).numpy()
    for k, gr in zip(inputs, grads[len(params):]):
        rec[f"grad_in/{k}"] = gr.numpy()


def phn_case(name, B, T, D, H, NL, FC, n_ph, Lmax, rel, seed):
    torch.manual_seed(seed)
    m = PhonemeRecognizer(D, H, NL, [H, FC, FC, n_ph + 2], n_ph)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, T, D, generator=g).requires_grad_(True)
    rel = torch.tensor(rel, dtype=torch.float32)
    bnd, n_l = _segments(B, T, Lmax, rel.tolist(), g)
    phn = torch.randint(0, n_ph + 2, (B, Lmax), generator=g)
    for b in range(B):
        phn[b, n_l[b]:] = 0
    phn_rel = n_l.float() / Lmax
    out = m(x, rel, phn, phn_rel, bnd)
    rec = {"x": x.detach().numpy(), "feat_lens": rel.numpy(), "phn": phn.numpy(),
           "phn_lens": phn_rel.numpy(), "boundary": bnd.numpy(),
           "dims": np.array([B, T, D, H, NL, FC, n_ph, Lmax])}
    _record(rec, m, {"out": out["out"], "bce": out["losses"]["phn_recog_bce_loss"]}, {"x": x}, g)
    np.savez(os.path.join(OUT_DIR, f"{name}.npz"), **rec)
    print(name, {k: v.shape for k, v in rec.items() if k.startswith("out/")})


def boundary_case(name, B, T, D, H, NL, FC, rel, seed):
    torch.manual_seed(seed)
    m = BoundaryDetector(D, H, NL, [H, FC, FC, 1])
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, T, D, generator=g).requires_grad_(True)
    rel = torch.tensor(rel, dtype=torch.float32)
    bnd, _ = _segments(B, T, T // 2, rel.tolist(), g)
    us = [torch.rand(B, T, generator=g) for _ in range(10)]
    queue = list(us)
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **k: queue.pop(0).clone()
    try:
        out = m(x, rel, bnd)
    finally:
        torch.rand_like = orig
    assert not queue
    rec = {"x": x.detach().numpy(), "feat_lens": rel.numpy(), "boundary": bnd.numpy(),
           "u": torch.stack(us).numpy(), "dims": np.array([B, T, D, H, NL, FC])}
    _record(rec, m, {"boundary_v": out["boundary_v"], "bce": out["losses"]["boundary_bce_loss"],
                     "kld": out["losses"]["boundary_kld_loss"]}, {"x": x}, g)
    np.savez(os.path.join(OUT_DIR, f"{name}.npz"), **rec)
    print(name, {k: v.shape for k, v in rec.items() if k.startswith("out/")})


if __name__ == "__main__":
    phn_case("md_phn_tiny", B=3, T=20, D=8, H=16, NL=2, FC=12, n_ph=5, Lmax=6,
             rel=[1.0, 0.85, 0.6], seed=11)
    phn_case("md_phn_mid", B=4, T=120, D=80, H=64, NL=2, FC=32, n_ph=40, Lmax=30,
             rel=[1.0, 0.9, 0.75, 127 / 120 * 0.5], seed=12)
    boundary_case("md_bnd_tiny", B=3, T=20, D=8, H=16, NL=2, FC=12, rel=[1.0, 0.85, 0.6], seed=21)
    boundary_case("md_bnd_mid", B=4, T=120, D=80, H=64, NL=2, FC=32, rel=[1.0, 0.9, 0.75, 0.5], seed=22)
