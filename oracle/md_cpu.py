"""CPU oracle for the MD-VAE upstream LSTMs -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, as the checker.  The product path (``ml-vae_amd/``)
never imports it.

Own-code restatement, in plain PyTorch on the CPU (fp32, or fp64 for self-checks), of:

  PhonemeRecognizer  ref:src/modules/phoneme_recognizer.py:9-81
      unidirectional nn.LSTM (batch_first) -> FCBlock -> per-utterance BCE-with-logits against
      the canonical phoneme sequence expanded by the boundary durations (:42-79)
  BoundaryDetector   ref:src/modules/boundary_detector.py:15-103
      unidirectional nn.LSTM -> two FCBlock + Softplus heads -> alpha, beta (+1e-5) ->
      KL(Beta(alpha, beta) || Beta(1, 9)) (:88-97) and ten Kumaraswamy draws
      v = (1 - u^(1/beta))^(1/alpha), u = 0.01 + 0.98 * U(0,1), BCE(v, boundary) averaged (:54-84)

Pinned by ``tests/test_oracle_md_golden.py`` against fixtures the reference modules produced
(``tests/golden/make_golden_md.py``).  Parameters are dicts keyed by the reference state_dict
names (``rnn.weight_ih_l0``, ``fc.blocks.0.weight``, ``fc_alpha.0.blocks.0.weight`` ...).
"""
import torch
import torch.nn.functional as Fn

from oracle.vae_cpu import NEG_SLOPE, lstm_direction_loop

PRIOR_A, PRIOR_B = 1.0, 9.0   # ref:src/modules/boundary_detector.py:91-92
EPS_AB = 1e-5                 # ref:src/modules/boundary_detector.py:46-48
EPS_V = 1e-5                  # ref:src/modules/boundary_detector.py:66-67
N_SAMPLES = 10                # ref:src/modules/boundary_detector.py:55


def uni_lstm(p, x, L, prefix="rnn.", dropout_masks=None):
    """Unidirectional L-layer nn.LSTM, batch_first, h0 = c0 = 0
    (ref:src/modules/phoneme_recognizer.py:13; boundary_detector.py:19; the MD-VAE's 512-unit
    rnn ref:src/models/MD_VAE/model.yaml:78-83).  dropout_masks[l] (scaled keep masks of layer
    l's output, l < L-1): nn.LSTM's train-mode inter-layer dropout with injected masks."""
    h = x
    for li in range(L):
        h = lstm_direction_loop(h, p[f"{prefix}weight_ih_l{li}"], p[f"{prefix}weight_hh_l{li}"],
                                p[f"{prefix}bias_ih_l{li}"], p[f"{prefix}bias_hh_l{li}"], False)
        if dropout_masks is not None and li < L - 1:
            h = h * dropout_masks[li]
    return h


def fc_block(p, prefix, x, n_linear, end_activation=False):
    """FCBlock (ref:src/modules/fc_block.py:4-21): Linear / LeakyReLU pairs; blocks.{2i}."""
    for i in range(n_linear):
        x = Fn.linear(x, p[f"{prefix}blocks.{2 * i}.weight"], p[f"{prefix}blocks.{2 * i}.bias"])
        if i < n_linear - 1 or end_activation:
            x = Fn.leaky_relu(x, NEG_SLOPE)
    return x


def frame_targets(boundary, phn, T_lens, L_lens):
    """Per frame the index of its phoneme in the canonical sequence: (number of boundaries in
    [0, t]) - 1, valid for t < T_i (ref:src/modules/phoneme_recognizer.py:61-71 builds the same
    expansion with repeat_interleave over the boundary durations).  Raises as the reference's
    asserts do when the boundaries do not give exactly L_i segments starting at frame 0."""
    B, T = boundary.shape
    cls = torch.zeros(B, T, dtype=torch.long)
    for b in range(B):
        Ti, Li = int(T_lens[b]), int(L_lens[b])
        bi = boundary[b, :Ti]
        if int((bi == 1).sum()) != Li or (Ti > 0 and bi[0] != 1):
            raise AssertionError("boundaries do not match the phoneme sequence")
        idx = torch.cumsum((bi == 1).long(), 0) - 1
        cls[b, :Ti] = phn[b, idx]
    return cls


def phn_bce(out, feat_lens, phn, phn_lens, boundary):
    """PhonemeRecognizer.compute_losses (ref:src/modules/phoneme_recognizer.py:35-81): [B,T,C]
    BCE-with-logits against one-hot(phoneme of the frame), zero past each utterance's T_i."""
    B, T, C = out.shape
    T_lens = torch.round(T * feat_lens).int()
    L_lens = torch.round(phn.shape[1] * phn_lens).int()
    cls = frame_targets(boundary, phn, T_lens, L_lens)
    y = Fn.one_hot(cls, num_classes=C).to(out.dtype)
    loss = Fn.binary_cross_entropy_with_logits(out, y, reduction="none")
    valid = (torch.arange(T)[None, :] < T_lens[:, None].long()).to(out.dtype)[..., None]
    return loss * valid


def phoneme_recognizer(p, x, feat_lens, phn, phn_lens, boundary, L, n_fc):
    out = fc_block(p, "fc.", uni_lstm(p, x, L), n_fc)
    return {"out": out, "bce": phn_bce(out, feat_lens, phn, phn_lens, boundary)}


def beta_kl(a, b):
    """KL(Beta(a, b) || Beta(1, 9)) (torch.distributions _kl_beta_beta, used at
    ref:src/modules/boundary_detector.py:94-95)."""
    qa, qb = torch.tensor(PRIOR_A, dtype=a.dtype), torch.tensor(PRIOR_B, dtype=a.dtype)
    t1 = torch.lgamma(qa) + torch.lgamma(qb) + torch.lgamma(a + b)
    t2 = torch.lgamma(a) + torch.lgamma(b) + torch.lgamma(qa + qb)
    return (t1 - t2 + (a - qa) * torch.digamma(a) + (b - qb) * torch.digamma(b)
            + (qa + qb - a - b) * torch.digamma(a + b))


def boundary_heads(za, zb, boundary, u):
    """Everything after the two FCBlock heads (ref:src/modules/boundary_detector.py:42-86):
    za, zb = pre-Softplus head outputs [B, T]; u = the ten U(0,1) draws [10, B, T]."""
    a = Fn.softplus(za) + EPS_AB
    b = Fn.softplus(zb) + EPS_AB
    kld = beta_kl(a, b)
    bce = torch.zeros_like(a)
    v = torch.zeros_like(a)
    for s in range(N_SAMPLES):
        us = u[s] * 0.98 + 0.01
        vs = (1 - us ** (1 / b)) ** (1 / a)
        vs = vs * (1 - 2 * EPS_V) + EPS_V
        v = v + vs
        bce = bce + Fn.binary_cross_entropy(vs, boundary, reduction="none")
    return {"boundary_v": v / N_SAMPLES, "bce": bce / N_SAMPLES, "kld": kld}


def boundary_detector(p, x, boundary, u, L, n_fc):
    r = uni_lstm(p, x, L)
    za = fc_block(p, "fc_alpha.0.", r, n_fc).squeeze(-1)
    zb = fc_block(p, "fc_beta.0.", r, n_fc).squeeze(-1)
    return boundary_heads(za, zb, boundary, u)
