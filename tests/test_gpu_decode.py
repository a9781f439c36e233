"""The MD-VAE Viterbi decode on the GPU (csrc/decode.hip via utils.decode_utils) against the
reference's own outputs (tests/golden/make_golden_decode.py; ref:src/utils/decode_utils.py:374-565)
and, at the metric's frame counts (T = 500, 2000), against the pinned oracle (oracle/decode_cpu.py):
decoded boundaries, frame-level and phoneme-level labels, exactly."""
import numpy as np
import pytest
import torch

from gpu_utils import need_gpu
from oracle import decode_cpu as D
from test_oracle_decode_golden import CASES, expected, load

pytestmark = pytest.mark.gpu


def _gpu_decode(t, weight):
    from utils.decode_utils import decode_plvl_md_lbl_seqs_full
    pred = {"phn_recog_out": t["logits"].cuda(), "boundary_v": t["boundary_v"].cuda(),
            "pi_logits": t["pi_logits"].cuda()}
    return decode_plvl_md_lbl_seqs_full(pred, list(range(t["logits"].shape[0])), t["feat_lens"].cuda(),
                                        t["seqs"].cuda(), t["seq_lens"].cuda(), t["prior"].cuda(), weight)


def _same(got, exp):
    for g_list, e_list in zip(got, exp):
        assert len(g_list) == len(e_list)
        for g, e in zip(g_list, e_list):
            assert np.array_equal(np.asarray(g), np.asarray(e))


@pytest.mark.parametrize("name", CASES)
def test_decode_matches_reference(name):
    need_gpu()
    r, t = load(name)
    _same(_gpu_decode(t, float(r["weight"])), expected(r))


@pytest.mark.parametrize("B,T,L,N,seed", [(8, 500, 60, 42, 1), (2, 2000, 250, 42, 2)])
def test_decode_matches_oracle_at_metric_lengths(B, T, L, N, seed):
    need_gpu()
    g = torch.Generator().manual_seed(seed)
    t = {"logits": torch.randn(B, T, N, generator=g) * 3, "boundary_v": torch.rand(B, T, generator=g),
         "pi_logits": torch.randn(B, T, 2, generator=g), "prior": torch.rand(N, generator=g) * 0.5,
         "seqs": torch.randint(0, N, (B, L), generator=g),
         "feat_lens": torch.linspace(0.6, 1.0, B), "seq_lens": torch.linspace(0.5, 1.0, B)}
    ref = D.decode(t["logits"], t["boundary_v"], t["pi_logits"], t["prior"], t["seqs"], t["feat_lens"],
                   t["seq_lens"], 0.9)
    _same(_gpu_decode(t, 0.9), ref)
