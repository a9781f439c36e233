"""Numpy restatement of the library's counter-based generators (ml-vae_amd/csrc/common.h): the
Philox-4x32-10 that draws eps and the other sampled noise, and the SplitMix64 quads of the
inter-layer dropout mask (dropout_scale), so a test can replay the exact masks the fused train
step drew in-kernel and hand them to the CPU oracle."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4(seed, ctr):
    """ctr: uint64 array of counters -> 4 uint32 arrays."""
    ctr = np.asarray(ctr, dtype=np.uint64)
    c0 = (ctr & MASK32).astype(np.uint64)
    c1 = (ctr >> np.uint64(32)).astype(np.uint64)
    c2 = np.full_like(c0, 0x243F6A88)
    c3 = np.full_like(c0, 0x85A308D3)
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0
            p1 = M1 * c2
            n0 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)
            n2 = (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)
            c0, c1, c2, c3 = n0 & MASK32, p1 & MASK32, n2 & MASK32, p0 & MASK32
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return [c.astype(np.uint32) for c in (c0, c1, c2, c3)]


G64 = np.uint64(0x9E3779B97F4A7C15)


def mix64(z):
    """SplitMix64's output function (common.h mix64) on a uint64 array."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def drop_quads(seed, q):
    """64 random bits of each element quad q (common.h drop_quad(drop_key(seed), q))."""
    k = mix64(np.array([(seed ^ 0x6A09E667F3BCC909) & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))[0]
    with np.errstate(over="ignore"):
        return mix64(k + np.asarray(q, dtype=np.uint64) * G64)


def dropout_mask(seed, n, p):
    """Scaled keep mask (0 or 1/(1-p)) of flat elements 0..n-1 (common.h dropout_scale): element
    i keeps iff the 16-bit uniform in bits [16 (i & 3), +16) of drop_quad(drop_key(seed), i >> 2)
    is < 1-p."""
    nq = (n + 3) // 4
    r = drop_quads(seed, np.arange(nq, dtype=np.uint64))
    lanes = np.stack([(r >> np.uint64(16 * e)) & np.uint64(0xFFFF) for e in range(4)], axis=1).reshape(-1)[:n]
    keep = np.float32(1.0 - p)
    u = lanes.astype(np.float32) * np.float32(1.0 / 65536.0)
    return np.where(u < keep, np.float32(1.0) / keep, np.float32(0.0)).astype(np.float32)
