"""CPU oracle for the MD-VAE Viterbi decode -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, as the checker.

Own-code restatement (numpy, float64 DP over float32 log terms) of
``decode_plvl_md_lbl_seqs_full`` (ref:src/utils/decode_utils.py:374-565; the eps-clamped log at
:8-14).  For each utterance, states (l = canonical phoneme, beta = correct / mispronounced) over
frames t: hold (boundary b = 0) or advance from phoneme l-1 in either state (b = 1, weighted pi
term); ties keep the first candidate (np.argmax); backtracking emits the boundary frames, the
frame-level and phoneme-level mispronunciation labels.  The DP runs a whole column of l at once
per t (the GPU kernel's wavefront order); the recurrence and tie rules are the reference's.

Pinned by ``tests/test_oracle_decode_golden.py`` against the reference's outputs
(``tests/golden/make_golden_decode.py``).
"""
import numpy as np
import torch

EPS = 1e-5


def clamp_log(x):
    """decode_utils.log (ref:src/utils/decode_utils.py:8-14): values in [0, eps) -> eps, fp32 log."""
    r = x.detach().cpu().clone()
    r[(r >= 0) & (r < EPS)] = EPS
    return torch.log(r).numpy()


def log_terms(logits, boundary_v, pi_logits, prior):
    p = torch.sigmoid(logits)
    log_p_yx = clamp_log(torch.stack([p, 1 - p], dim=3))               # [B, T, N, 2]
    log_p_y = clamp_log(torch.stack([prior, 1 - prior], dim=1))        # [N, 2]
    log_p_b = clamp_log(torch.stack([boundary_v, 1 - boundary_v], 2))  # [B, T, 2]
    log_p_pi = clamp_log(torch.softmax(pi_logits, dim=-1))             # [B, T, 2]
    return log_p_yx, log_p_y, log_p_b, log_p_pi


def decode_one(lyx, lpy, lpb, lpi, y, weight):
    """One utterance: lyx [T, N, 2], lpy [N, 2], lpb [T, 2], lpi [T, 2], y [L] phoneme ids."""
    T, L = lyx.shape[0], len(y)
    # (the reference sums left to right: ((dp + log_p_b) [+ w log_p_pi]) + log_p_yx - log_p_y)
    val = np.full((L, 2), -np.inf)
    path = np.full((T, L, 2), -1, dtype=np.int8)
    w32 = np.float32(weight)  # NumPy 2 (NEP 50): a Python float times a float32 stays float32
    for b in range(2):  # the reference's first column is all-float32 arithmetic
        val[0, b] = np.float64((w32 * lpi[0, b] + lyx[0, y[0], b]) - lpy[y[0], b])
    for t in range(1, T):
        new = np.empty_like(val)
        lb0, lb1 = np.float64(lpb[t, 0]), np.float64(lpb[t, 1])
        for b in range(2):
            ex = lyx[t, y, b].astype(np.float64)
            py = lpy[y, b].astype(np.float64)
            hold = val[:, b] + lb0 + ex - py
            new[:, b] = hold
            path[t, :, b] = 0
            if L > 1:
                wp = np.float64(w32 * lpi[t, b])  # float32 product, then float64 sums
                fc = val[:-1, 0] + lb1 + wp + ex[1:] - py[1:]
                fi = val[:-1, 1] + lb1 + wp + ex[1:] - py[1:]
                cand = np.stack([hold[1:], fc, fi])          # first max wins, as np.argmax
                arg = np.argmax(cand, axis=0)
                new[1:, b] = cand[arg, np.arange(L - 1)]
                path[t, 1:, b] = arg
        val = new
    # backtracking (ref:src/utils/decode_utils.py:500-537)
    l, t = L - 1, T - 1
    beta = 0 if val[l, 0] > val[l, 1] else 1
    frame, phone, bidx = [beta], [beta], []
    while t > 0:
        p = path[t, l, beta]
        if p == 1 or p == 2:
            l -= 1
            bidx.append(t)
            beta = 0 if p == 1 else 1
            frame.append(beta)
            phone.append(beta)
        else:
            frame.append(frame[-1])
        t -= 1
    bidx.append(t)
    if not (l == 0 and t == 0):
        raise AssertionError(f"l = {l}, t = {t}")
    bnd = np.zeros(T, dtype=np.int64)
    bnd[bidx] = 1
    return bnd, frame[::-1], phone[::-1]


def decode(logits, boundary_v, pi_logits, prior, seqs, feat_lens, seq_lens, weight=1.0):
    """Batch: returns lists (decoded boundary seqs, frame-level labels, phoneme-level labels)."""
    T_i = torch.round(feat_lens * logits.shape[1]).int().numpy()
    L_i = torch.round(seq_lens * seqs.shape[1]).int().numpy()
    lyx, lpy, lpb, lpi = log_terms(logits, boundary_v, pi_logits, prior)
    y = seqs.numpy()
    out = [decode_one(lyx[i, :T_i[i]], lpy, lpb[i, :T_i[i]], lpi[i, :T_i[i]], y[i, :L_i[i]], weight)
           for i in range(len(T_i))]
    return [o[0] for o in out], [o[1] for o in out], [o[2] for o in out]
