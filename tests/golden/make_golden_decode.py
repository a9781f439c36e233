"""Golden fixtures for the MD-VAE Viterbi decode.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (never on the GPU box): it calls the
reference's own ``utils.decode_utils.decode_plvl_md_lbl_seqs_full`` (ref:src/utils/decode_utils.py:
374-565, the function ref:src/models/MD_VAE/model.py:20,133-141 runs inside the training forward)
on seeded synthetic model outputs and writes its decoded sequences as padded ``.npz`` arrays.

Cases: random logits / boundary posteriors / pi logits; ragged frame and phoneme lengths; a case
with saturated probabilities (exact 0 / 1, the eps clamp of decode_utils.log) and a dec_weight != 1.

Usage:  cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden_decode.py
"""
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden  # noqa: E402,F401  (generator-only shims, reference src on sys.path)
from utils.decode_utils import decode_plvl_md_lbl_seqs_full  # noqa: E402  (reference)

OUT_DIR = make_golden.OUT_DIR


def case(name, B, T, L, N, rel_t, rel_l, weight, seed, saturate=False):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, T, N, generator=g) * 3
    bv = torch.rand(B, T, generator=g)
    pi = torch.randn(B, T, 2, generator=g) * 2
    prior = torch.rand(N, generator=g) * 0.5
    if saturate:
        logits[:, ::3] = 200.0   # sigmoid -> exactly 1: 1 - p = 0 -> eps clamp
        bv[:, ::4] = 0.0
        bv[:, 1::5] = 1.0
        prior[0] = 0.0
    seqs = torch.randint(0, N, (B, L), generator=g)
    rel_t = torch.tensor(rel_t, dtype=torch.float32)
    rel_l = torch.tensor(rel_l, dtype=torch.float32)
    pred = {"phn_recog_out": logits, "boundary_v": bv, "pi_logits": pi}
    bnd, flvl, plvl = decode_plvl_md_lbl_seqs_full(pred, [f"u{i}" for i in range(B)], rel_t, seqs,
                                                  rel_l, prior, weight=weight)
    Tl = [len(b) for b in bnd]
    Ll = [len(p) for p in plvl]
    pad = lambda seqs_, n: np.stack([np.pad(np.asarray(s, dtype=np.int64), (0, n - len(s)),
                                            constant_values=-1) for s in seqs_])
    np.savez(os.path.join(OUT_DIR, f"{name}.npz"), logits=logits.numpy(), boundary_v=bv.numpy(),
             pi_logits=pi.numpy(), prior=prior.numpy(), seqs=seqs.numpy(), feat_lens=rel_t.numpy(),
             seq_lens=rel_l.numpy(), weight=np.array(weight), T_i=np.array(Tl), L_i=np.array(Ll),
             boundary=pad(bnd, T), flvl=pad(flvl, T), plvl=pad(plvl, L))
    print(name, "T_i", Tl, "L_i", Ll)


if __name__ == "__main__":
    case("decode_tiny", B=3, T=24, L=6, N=7, rel_t=[1.0, 0.75, 0.5], rel_l=[1.0, 5 / 6, 0.5],
         weight=1.0, seed=31)
    case("decode_mid", B=6, T=300, L=40, N=42, rel_t=[1.0, 0.9, 0.8, 0.7, 0.6, 0.5],
         rel_l=[1.0, 0.9, 0.75, 0.7, 0.5, 0.45], weight=0.7, seed=32)
    case("decode_saturated", B=3, T=60, L=12, N=9, rel_t=[1.0, 0.95, 0.6], rel_l=[1.0, 0.75, 0.5],
         weight=1.3, seed=33, saturate=True)
