"""The host restatement of the library's dropout-mask generator (tests/philox_np.py, replaying
ml-vae_amd/csrc/common.h drop_quad / dropout_scale) against published SplitMix64 outputs, and the
mask's keep rate -- the GPU parity tests replay every in-kernel mask through it."""
import numpy as np

from philox_np import G64, dropout_mask, mix64


def test_mix64_reproduces_the_splitmix64_reference_sequence():
    # SplitMix64 (Steele, Lea, Flood 2014; Vigna's splitmix64.c) seeded with 1234567: the first
    # outputs are mix64(state + k * gamma), k = 1, 2, 3
    st = np.uint64(1234567)
    with np.errstate(over="ignore"):
        out = [int(mix64(np.array([st + G64 * np.uint64(k)], dtype=np.uint64))[0]) for k in (1, 2, 3)]
    assert out == [6457827717110365317, 3203168211198807973, 9817491932198370423]


def test_dropout_mask_keep_rate_scale_and_seed_dependence():
    p, n = 0.15, 1 << 20
    m = dropout_mask(77, n, p)
    kept = m > 0
    assert abs(kept.mean() - (1 - p)) < 4 * (p * (1 - p) / n) ** 0.5
    assert np.all(m[kept] == np.float32(1.0) / np.float32(1 - p))
    m2 = dropout_mask(78, n, p)
    assert 0.2 < (kept != (m2 > 0)).mean() < 0.3         # independent seeds: 2 p (1-p) = 0.255
    assert np.array_equal(dropout_mask(77, 1000, p), m[:1000])   # a prefix is the same mask
