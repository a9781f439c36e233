"""CPU oracle for the ML-VAE training step -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the *checker* (or the
timed CPU baseline).  The product path (``ml-vae_amd/``) never imports it and
fails loudly when its HIP library is missing.

This is an own-code restatement, in plain PyTorch on the CPU, fp32 (or fp64
for self-checks), of the reference's hot path:

  encoder   ref:src/modules/vanilla_vae.py:9-45   (FCBlock ref:src/modules/fc_block.py:4-21)
  decoder   ref:src/modules/decoder.py:10-53      (nn.LSTM bidirectional, batch_first, no packing)
  masking   ref:src/utils/data_utils.py:67-104    (+ SpeechBrain 0.5 length_to_mask, un-vendored)
  weights   ref:src/models/md_model.py:189-213    (compute_and_save_losses)
  objective ref:src/models/test_vanilla_vae/model.py:37-55
  step      ref:src/models/md_model.py:54-88      (backward, check_gradients -> clip 5.0, Adam)
  optimizer ref:src/models/test_vanilla_vae/model.yaml:45-47 (Adam lr 1e-3, torch defaults)

Parity pinning: ``tests/test_oracle_golden.py`` checks this module against the
fixtures in ``tests/golden/`` that ``tests/golden/make_golden.py`` produced by
running the reference modules themselves in the build container.  The
SpeechBrain pieces (length_to_mask, check_gradients) are un-vendored in the
reference, so those two are restated from SpeechBrain 0.5 semantics and are
"parity unpinned" beyond what the fixtures exercise.

Parameters are held in an ordered dict keyed by the reference state_dict names
(``encoder.fc.0.blocks.0.weight`` ... ``decoder.log_var_fc.blocks.4.bias``),
in ``self.modules.parameters()`` order.
"""
import math
from collections import OrderedDict

import torch
import torch.nn.functional as Fn

LOG_2PI_F32 = float(torch.log(2 * torch.tensor(math.pi)).item())  # ref:src/modules/decoder.py:42 (fp32 log 2pi)
NEG_SLOPE = 0.01  # nn.LeakyReLU default, ref:src/modules/fc_block.py:11


# --------------------------------------------------------------------------
# configuration / parameter naming
# --------------------------------------------------------------------------
def param_shapes(F, enc, z, H, L, dec_fc, enc_conv=0):
    """Reference parameter names and shapes, in Brain.modules.parameters() order.
    enc_conv = K > 0: the Conv1d encoder variant (configs[3]; no reference counterpart --
    ml-vae_amd/modules/conv_vae.py), Conv1d weights [Cout, Cin, K] under ``encoder.conv.0``."""
    s = OrderedDict()
    pre, k = ("encoder.conv.0.blocks", (enc_conv,)) if enc_conv else ("encoder.fc.0.blocks", ())
    s[f"{pre}.0.weight"] = (enc, F) + k
    s[f"{pre}.0.bias"] = (enc,)
    s[f"{pre}.2.weight"] = (enc, enc) + k
    s[f"{pre}.2.bias"] = (enc,)
    s["encoder.mean_fc.weight"] = (z, enc)
    s["encoder.mean_fc.bias"] = (z,)
    s["encoder.log_var_fc.weight"] = (z, enc)
    s["encoder.log_var_fc.bias"] = (z,)
    for layer in range(L):
        din = z if layer == 0 else 2 * H
        for sfx in ("", "_reverse"):
            s[f"decoder.rnn.weight_ih_l{layer}{sfx}"] = (4 * H, din)
            s[f"decoder.rnn.weight_hh_l{layer}{sfx}"] = (4 * H, H)
            s[f"decoder.rnn.bias_ih_l{layer}{sfx}"] = (4 * H,)
            s[f"decoder.rnn.bias_hh_l{layer}{sfx}"] = (4 * H,)
    for head in ("mean_fc", "log_var_fc"):
        dims = [2 * H, dec_fc, dec_fc, F]
        for i in range(3):
            s[f"decoder.{head}.blocks.{2 * i}.weight"] = (dims[i + 1], dims[i])
            s[f"decoder.{head}.blocks.{2 * i}.bias"] = (dims[i + 1],)
    return s


def init_params(F, enc, z, H, L, dec_fc, seed=123456, dtype=torch.float32, enc_conv=0):
    """PyTorch-default init (kaiming-uniform Linear, U(-1/sqrt(H),1/sqrt(H)) LSTM).

    Same distributions the reference gets from nn.Linear/nn.LSTM constructors
    under torch.manual_seed(seed) (ref:src/config/run.yaml:2-3); values are not
    claimed bit-identical to the reference's construction order.
    """
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for name, shp in param_shapes(F, enc, z, H, L, dec_fc, enc_conv).items():
        if ".rnn." in name:
            bound = 1.0 / math.sqrt(H)
        else:
            fan_in = math.prod(shp[1:]) if len(shp) >= 2 else None  # Conv1d: Cin * K
            if fan_in is None:  # bias: use the weight's fan_in
                wname = name[:-4] + "weight"
                fan_in = math.prod(out[wname].shape[1:])
            bound = 1.0 / math.sqrt(fan_in)
        out[name] = (torch.rand(shp, generator=g, dtype=torch.float64) * 2 - 1).mul(bound).to(dtype)
    return out


# --------------------------------------------------------------------------
# forward pieces
# --------------------------------------------------------------------------
def length_to_mask(lens, T):
    """SpeechBrain 0.5 ``length_to_mask(lens*T, max_len=T)`` as used at
    ref:src/utils/data_utils.py:87: ``arange(T, dtype=lens.dtype) < lens*T``.
    Note the fp32 quirk: fp32(127/500)*500 > 127 so 128 frames are valid."""
    lens = lens.to(torch.float32)
    abs_len = lens * T
    return (torch.arange(T, dtype=torch.float32).unsqueeze(0) < abs_len.unsqueeze(1)).to(torch.float32)


def apply_lens_to_loss(loss, lens, reduction="mean"):
    """ref:src/utils/data_utils.py:67-104."""
    B, T = loss.shape[0], loss.shape[1]
    m = length_to_mask(lens, T).to(loss.dtype)
    while m.dim() < loss.dim():
        m = m.unsqueeze(-1)
    mask = torch.ones_like(loss) * m
    lm = loss * mask
    if reduction == "mean":
        return lm.sum() / mask.sum()
    if reduction == "batchmean":
        return lm.sum() / B
    if reduction == "batch":
        return lm.reshape(B, -1).sum(-1) / mask.reshape(B, -1).sum(-1)
    raise ValueError(reduction)


def lrelu(x):
    return Fn.leaky_relu(x, NEG_SLOPE)


def encoder_forward(p, x, eps):
    """VanillaVAE.forward with injected eps (ref:src/modules/vanilla_vae.py:21-45).
    fc = Seq(FCBlock([F,enc,enc]), LeakyReLU): Linear-LReLU-Linear, then LReLU.
    Conv1d variant (``encoder.conv.0.*`` present): the same with Conv1d(K, padding (K-1)/2)
    over time on the [B, C, T] transpose (torch's own conv1d, cross-checked by conv1d_numpy)."""
    if "encoder.conv.0.blocks.0.weight" in p:
        h = x.transpose(1, 2)
        for i in (0, 2):
            wt = p[f"encoder.conv.0.blocks.{i}.weight"]
            h = lrelu(Fn.conv1d(h, wt, p[f"encoder.conv.0.blocks.{i}.bias"], padding=wt.shape[2] // 2))
        h = h.transpose(1, 2)
    else:
        h = lrelu(Fn.linear(x, p["encoder.fc.0.blocks.0.weight"], p["encoder.fc.0.blocks.0.bias"]))
        h = lrelu(Fn.linear(h, p["encoder.fc.0.blocks.2.weight"], p["encoder.fc.0.blocks.2.bias"]))
    mean = Fn.linear(h, p["encoder.mean_fc.weight"], p["encoder.mean_fc.bias"])
    log_var = Fn.linear(h, p["encoder.log_var_fc.weight"], p["encoder.log_var_fc.bias"])
    std = torch.exp(0.5 * log_var)
    z = eps * std + mean
    kld = -0.5 * (1 + log_var - mean.pow(2) - log_var.exp())
    return {"mean": mean, "log_var": log_var, "sampled_h": z, "loss": kld}


def conv1d_numpy(x, w, b):
    """Explicit restatement of Conv1d over time for batch-first frames: x [B, T, Cin] (numpy),
    w [Cout, Cin, K], b [Cout]; y[b, t] = b + sum_j W[:, :, j] x[b, t + j - (K-1)/2] with zeros
    outside [0, T) (the semantics torch.nn.Conv1d(padding=(K-1)/2) has on [B, C, T])."""
    import numpy as np
    B, T, _ = x.shape
    K = w.shape[2]
    p = (K - 1) // 2
    xp = np.zeros((B, T + 2 * p, x.shape[2]), dtype=np.float64)
    xp[:, p:p + T] = x
    y = np.broadcast_to(np.asarray(b, dtype=np.float64), (B, T, w.shape[0])).copy()
    for j in range(K):
        y += xp[:, j:j + T] @ np.asarray(w[:, :, j], dtype=np.float64).T
    return y


def lstm_direction_loop(x, w_ih, w_hh, b_ih, b_hh, reverse):
    """One direction of one nn.LSTM layer, explicit time loop, h0=c0=0, no packing
    (the reverse direction starts at the padded tail, t=T-1).  Gate order i,f,g,o."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    gx = Fn.linear(x, w_ih, b_ih + b_hh)  # [B,T,4H]
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    outs = [None] * T
    order = range(T - 1, -1, -1) if reverse else range(T)
    for t in order:
        g = gx[:, t] + h @ w_hh.t()
        i, f, gg, o = g.split(H, dim=1)
        i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
        c = f * c + i * gg
        h = o * torch.tanh(c)
        outs[t] = h
    return torch.stack(outs, dim=1)


def bilstm(p, x, L, dropout_masks=None, impl="loop"):
    """Bidirectional L-layer nn.LSTM (ref:src/modules/decoder.py:14-15,22).
    dropout_masks[l] (already scaled by 1/(1-p)) multiplies layer l's output
    for l < L-1 (train mode); None = eval mode."""
    H = p["decoder.rnn.weight_hh_l0"].shape[1]
    h = x
    for layer in range(L):
        if impl == "aten":  # the ATen LSTM op the reference itself calls, one layer at a time
            names = [f"weight_ih_l{layer}", f"weight_hh_l{layer}", f"bias_ih_l{layer}",
                     f"bias_hh_l{layer}"]
            flat = [p["decoder.rnn." + n + s] for s in ("", "_reverse") for n in names]
            h0 = h.new_zeros(2, h.shape[0], H)
            h = torch.lstm(h, (h0, h0), flat, True, 1, 0.0, False, True, True)[0]
            if dropout_masks is not None and layer < L - 1:
                h = h * dropout_masks[layer]
            continue
        outs = []
        for sfx, rev in (("", False), ("_reverse", True)):
            outs.append(lstm_direction_loop(
                h, p[f"decoder.rnn.weight_ih_l{layer}{sfx}"], p[f"decoder.rnn.weight_hh_l{layer}{sfx}"],
                p[f"decoder.rnn.bias_ih_l{layer}{sfx}"], p[f"decoder.rnn.bias_hh_l{layer}{sfx}"], rev))
        h = torch.cat(outs, dim=-1)
        if dropout_masks is not None and layer < L - 1:
            h = h * dropout_masks[layer]
    return h


class _LReLUKink(torch.autograd.Function):
    """LeakyReLU whose derivative takes the other branch where `flip` is set (test infrastructure
    for the fp64-anchored parity tests: at a pre-activation within rounding of 0 either slope is
    a valid derivative of the computed value, so an fp32 implementation that lands on the other
    side of the kink is compared with the fp64 step that takes the same branch there)."""

    @staticmethod
    def forward(ctx, x, flip):
        ctx.save_for_backward(x, flip)
        return Fn.leaky_relu(x, NEG_SLOPE)

    @staticmethod
    def backward(ctx, g):
        x, flip = ctx.saved_tensors
        pos = (x > 0) ^ flip
        return g * torch.where(pos, torch.ones_like(g), torch.full_like(g, NEG_SLOPE)), None


def fc_head(p, prefix, r, kink=None, pre_out=None):
    """FCBlock([2H, fc, fc, F]) (ref:src/modules/fc_block.py:9-16): no end activation.
    kink (tests): bool [.., fc] -- the first layer's LeakyReLU derivative branch flipped there;
    pre_out (tests): dict receiving the first layer's pre-activation under `prefix`."""
    pre = Fn.linear(r, p[prefix + ".blocks.0.weight"], p[prefix + ".blocks.0.bias"])
    if pre_out is not None:
        pre_out[prefix] = pre.detach()
    h = lrelu(pre) if kink is None else _LReLUKink.apply(pre, kink)
    h = lrelu(Fn.linear(h, p[prefix + ".blocks.2.weight"], p[prefix + ".blocks.2.bias"]))
    return Fn.linear(h, p[prefix + ".blocks.4.weight"], p[prefix + ".blocks.4.bias"])


def recon_loss(mean, log_var, target, loss_type):
    """ref:src/modules/decoder.py:37-53 (the unused Normal.log_prob is dead code)."""
    if loss_type == "likelihood":
        return 0.5 * (LOG_2PI_F32 + log_var + (target - mean) ** 2 / (torch.exp(log_var) + 1e-5))
    if loss_type == "mse":
        return (target - mean) ** 2
    raise ValueError(f"Invalid loss type: {loss_type}")


def decoder_forward(p, z, x, L, loss_type, dropout_masks=None, impl="loop", head_kink=None):
    r = bilstm(p, z, L, dropout_masks, impl)
    kink = head_kink or {}
    pre = {}
    mean = fc_head(p, "decoder.mean_fc", r, kink.get("decoder.mean_fc"), pre)
    log_var = fc_head(p, "decoder.log_var_fc", r, kink.get("decoder.log_var_fc"), pre)
    return {"rnn_out": r, "mean": mean, "log_var": log_var, "p1_pre": pre,
            "losses": {"recon_loss": recon_loss(mean, log_var, x, loss_type)}}


def loss_weights(keys, hparams):
    """compute_and_save_losses weighting (ref:src/models/md_model.py:189-213)."""
    ws = []
    for k in keys:
        wk = k.replace("_loss", "_weight")
        w = hparams.get(wk, "none")
        if w == "none":
            w = 1
        if "_kld" in wk:
            w = w / (2249 / hparams["batch_size"])
        ws.append(w)
    return ws


def forward_loss(p, x, lens, eps, cfg, dropout_masks=None, impl="loop"):
    """compute_forward + compute_objectives (ref:src/models/test_vanilla_vae/model.py:19-55),
    normaliser omitted (identity)."""
    enc = encoder_forward(p, x, eps)
    dec = decoder_forward(p, enc["sampled_h"], x, cfg["L"], cfg["loss_type"], dropout_masks, impl,
                          cfg.get("head_kink"))
    kld = apply_lens_to_loss(enc["loss"], lens)
    rec = apply_lens_to_loss(dec["losses"]["recon_loss"], lens)
    w_kld, w_rec = loss_weights(["kld_loss", "recon_loss"],
                                {"kld_weight": cfg.get("kld_weight", 1e-3),
                                 "batch_size": cfg.get("batch_size", x.shape[0])})
    loss = 0
    loss = loss + w_kld * kld
    loss = loss + w_rec * rec
    return {"enc": enc, "dec": dec, "kld_loss": kld, "recon_loss": rec, "loss": loss}


# --------------------------------------------------------------------------
# optimizer pieces
# --------------------------------------------------------------------------
def clip_grad_norm(grads, max_norm=5.0):
    """torch.nn.utils.clip_grad_norm_ as SpeechBrain's check_gradients calls it
    (max_grad_norm=5.0): total = ||(||g_i||_2)_i||_2, coef = max/(total+1e-6),
    grads *= min(coef, 1)."""
    norms = torch.stack([g.norm(2) for g in grads.values()])
    total = norms.norm(2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return OrderedDict((k, g * coef) for k, g in grads.items()), total


def adam_step(params, grads, state, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam (no weight decay, amsgrad off) single-tensor semantics."""
    b1, b2 = betas
    state["step"] = state.get("step", 0) + 1
    t = state["step"]
    bc1 = 1 - b1 ** t
    bc2 = 1 - b2 ** t
    out = OrderedDict()
    for k, p in params.items():
        g = grads[k]
        m = state.setdefault("m", {}).get(k, torch.zeros_like(p))
        v = state.setdefault("v", {}).get(k, torch.zeros_like(p))
        m = m * b1 + g * (1 - b1)
        v = v * b2 + g * g * (1 - b2)
        state["m"][k], state["v"][k] = m, v
        denom = v.sqrt() / math.sqrt(bc2) + eps
        out[k] = p - (lr / bc1) * m / denom
    return out


def train_step(params, state, x, lens, eps, cfg, dropout_masks=None, impl="loop", max_norm=5.0):
    """One MDModel.fit_batch (ref:src/models/md_model.py:77-88): forward,
    backward, check_gradients (finite check + clip), Adam step.
    Returns (new_params, record)."""
    leaf = OrderedDict((k, v.detach().clone().requires_grad_(True)) for k, v in params.items())
    out = forward_loss(leaf, x, lens, eps, cfg, dropout_masks, impl)
    loss = out["loss"]
    gl = torch.autograd.grad(loss, list(leaf.values()), allow_unused=True)
    grads = OrderedDict((k, (g if g is not None else torch.zeros_like(leaf[k])).detach())
                        for k, g in zip(leaf.keys(), gl))
    rec = {"out": out, "grads": grads}
    if not torch.isfinite(loss):
        rec["skipped"] = True
        return OrderedDict((k, v.detach()) for k, v in params.items()), rec
    clipped, total = clip_grad_norm(grads, max_norm)
    rec["grad_norm"] = total
    new = adam_step(OrderedDict((k, v.detach()) for k, v in params.items()), clipped, state,
                    lr=cfg.get("lr", 1e-3))
    rec["skipped"] = False
    return new, rec
