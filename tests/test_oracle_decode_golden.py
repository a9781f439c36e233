"""The Viterbi MD decode oracle (oracle/decode_cpu.py) against the reference's own outputs
(tests/golden/make_golden_decode.py; ref:src/utils/decode_utils.py:374-565): decoded boundary
sequences, frame-level and phoneme-level mispronunciation labels, exactly."""
import os

import numpy as np
import pytest
import torch

from oracle import decode_cpu as D

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["decode_tiny", "decode_mid", "decode_saturated"]


def load(name):
    r = dict(np.load(os.path.join(GOLD, f"{name}.npz")))
    t = {k: torch.from_numpy(r[k]) for k in ("logits", "boundary_v", "pi_logits", "prior", "seqs",
                                             "feat_lens", "seq_lens")}
    return r, t


def expected(r):
    B = len(r["T_i"])
    return ([r["boundary"][i, :r["T_i"][i]] for i in range(B)],
            [r["flvl"][i, :r["T_i"][i]] for i in range(B)],
            [r["plvl"][i, :r["L_i"][i]] for i in range(B)])


@pytest.mark.parametrize("name", CASES)
def test_decode_matches_reference(name):
    r, t = load(name)
    got = D.decode(t["logits"], t["boundary_v"], t["pi_logits"], t["prior"], t["seqs"], t["feat_lens"],
                   t["seq_lens"], float(r["weight"]))
    for g_list, e_list in zip(got, expected(r)):
        assert len(g_list) == len(e_list)
        for g, e in zip(g_list, e_list):
            assert np.array_equal(np.asarray(g), e)
