"""The VAE training step on MI355X: flat parameter/gradient/Adam buffers plus a fixed
sequence of libmlvae.so launches (no autograd, no torch compute kernels on the path).

One ``train_step`` = the reference's ``MDModel.fit_batch`` for the test_vanilla_vae
recipe (ref:src/models/md_model.py:54-88 with
ref:src/models/test_vanilla_vae/model.py:19-55):

  encoder   FC(F->E) LReLU FC(E->E) LReLU -> [mu | log_var] FC(E->2Z)       (3 GEMMs)
  ELBO-1    z = eps*exp(lv/2) + mu ; KL ; masked partial sums                (1 kernel)
  decoder   L x [input-projection GEMM + persistent BiLSTM recurrence]      (2L launches)
            (+ inter-layer dropout in train mode)
  heads     FC(2H->2C) fused for both heads, then FC(C->C), FC(C->F) per head
  ELBO-2    reconstruction NLL/MSE + masked sums + d/d(mu_x, lv_x)           (1 kernel)
  backward  dgrad/wgrad GEMMs, BPTT recurrence, column sums for biases
  step      grad sum-of-squares -> clip(5.0) + Adam + device step counter  (no host sync)

Every tensor is row-major [B*T, C]; the flat parameter buffer keeps pairs that a fused
launch reads as one matrix adjacent (mean/log_var heads, both LSTM directions).
"""
import math
import os
from collections import OrderedDict
from dataclasses import dataclass, field

import torch

from . import _lib
from ._lib import check, lib

PREC = {"fp32": 0, "bf16": 1}
LOSS = {"likelihood": 0, "mse": 1}
EPI_NONE, EPI_LRELU, EPI_DLRELU, EPI_DROPOUT = 0, 1, 2, 3
EPI_OUT_F16 = 16  # flag: mlvae_gemm_bf16 stores C as fp16
EPI_OUT_BF16 = 32  # flag: mlvae_gemm_bf16 stores C as bf16
G8_MARGIN = 2.0   # fp8 mode: headroom of the delayed dG scale over the previous step's amax


def x8_scale(p):
    """fp8 mode: the fixed e4m3 scale of a layer input dropout(h): |h| < 1, so |dropout(h)| <=
    1/(1-p); the largest power of two keeping that under e4m3's 448 (256 at p = 0.15)."""
    s, lim = 1.0, 448.0 * (1.0 - p)
    while s * 2.0 <= lim:
        s *= 2.0
    return s


@dataclass
class VAEConfig:
    """Dimensions/hyper-parameters of the recipe (ref:src/models/test_vanilla_vae/model.yaml:17-54)."""
    F: int = 80             # input_size (feature dim)
    E: int = 64             # enc_fc_size
    Z: int = 32             # latent_size
    H: int = 512            # dec_rnn_hidden_size
    L: int = 2              # dec_rnn_num_layers
    C: int = 64             # dec_fc_size
    dropout: float = 0.15   # dec_rnn_dropout
    loss_type: str = "likelihood"
    kld_weight: float = 1e-3
    recon_weight: float = 1.0
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    adam_eps: float = 1e-8
    max_grad_norm: float = 5.0
    prec: str = "fp32"      # "fp32" (exact parity mode) or "bf16" (bf16 MFMA operands)
    enc_conv: int = 0       # Conv1d encoder kernel size (modules/conv_vae.py, configs[3]); 0 = Linear
    fp8: bool = False       # configs[4]: the layer >= 1 input projections on fp8 e4m3 operands (bf16 mode)

    @property
    def enc_prefix(self):
        return "encoder.conv.0.blocks" if self.enc_conv else "encoder.fc.0.blocks"

    def check(self):
        for k in ("F", "E", "Z", "H", "C"):
            v = getattr(self, k)
            if v <= 0 or v % 4:
                raise ValueError(f"{k}={v}: every width must be a positive multiple of 4")
        if self.loss_type not in LOSS:
            raise ValueError(f"Invalid loss type: {self.loss_type}")
        if self.prec not in PREC:
            raise ValueError(f"prec must be one of {list(PREC)}")
        if self.fp8 and self.prec != "bf16":
            raise ValueError("fp8 projections run inside the bf16 mode: prec must be 'bf16'")
        if self.fp8 and not (0.0 <= self.dropout < 0.99):
            raise ValueError("fp8 mode: the layer-input scale needs dropout p < 0.99")
        if self.enc_conv:
            if self.enc_conv % 2 != 1:
                raise ValueError("enc_conv: the Conv1d kernel size must be odd")
            if self.prec != "bf16":
                raise ValueError("the Conv1d encoder kernels use bf16 operands: prec must be 'bf16'")
            if not (lib().mlvae_conv1d_supported(self.F, self.E, self.enc_conv) and
                    lib().mlvae_conv1d_supported(self.E, self.E, self.enc_conv)):
                raise ValueError(f"Conv1d encoder F={self.F} E={self.E} K={self.enc_conv} not supported "
                                 "(include/mlvae.h mlvae_conv1d_supported)")
        return self


def reference_shapes(cfg):
    """Reference parameter names/shapes in Brain.modules.parameters() order
    (encoder: ref:src/modules/vanilla_vae.py:13-19; decoder: ref:src/modules/decoder.py:14-17)."""
    F, E, Z, H, L, C = cfg.F, cfg.E, cfg.Z, cfg.H, cfg.L, cfg.C
    s = OrderedDict()
    k, ep = (cfg.enc_conv,), cfg.enc_prefix
    s[f"{ep}.0.weight"] = (E, F) + (k if cfg.enc_conv else ())
    s[f"{ep}.0.bias"] = (E,)
    s[f"{ep}.2.weight"] = (E, E) + (k if cfg.enc_conv else ())
    s[f"{ep}.2.bias"] = (E,)
    s["encoder.mean_fc.weight"] = (Z, E)
    s["encoder.mean_fc.bias"] = (Z,)
    s["encoder.log_var_fc.weight"] = (Z, E)
    s["encoder.log_var_fc.bias"] = (Z,)
    for l in range(L):
        din = Z if l == 0 else 2 * H
        for sfx in ("", "_reverse"):
            s[f"decoder.rnn.weight_ih_l{l}{sfx}"] = (4 * H, din)
            s[f"decoder.rnn.weight_hh_l{l}{sfx}"] = (4 * H, H)
            s[f"decoder.rnn.bias_ih_l{l}{sfx}"] = (4 * H,)
            s[f"decoder.rnn.bias_hh_l{l}{sfx}"] = (4 * H,)
    for head in ("mean_fc", "log_var_fc"):
        dims = [2 * H, C, C, F]
        for i in range(3):
            s[f"decoder.{head}.blocks.{2 * i}.weight"] = (dims[i + 1], dims[i])
            s[f"decoder.{head}.blocks.{2 * i}.bias"] = (dims[i + 1],)
    return s


def _engine_order(cfg):
    """Flat-buffer order: groups listed together are laid out back to back (no padding),
    so one launch can read them as a single stacked matrix/vector."""
    ep = cfg.enc_prefix
    g = [[f"{ep}.0.weight"], [f"{ep}.0.bias"], [f"{ep}.2.weight"], [f"{ep}.2.bias"],
         ["encoder.mean_fc.weight", "encoder.log_var_fc.weight"],
         ["encoder.mean_fc.bias", "encoder.log_var_fc.bias"]]
    for l in range(cfg.L):
        for kind in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
            g.append([f"decoder.rnn.{kind}_l{l}", f"decoder.rnn.{kind}_l{l}_reverse"])
    g.append(["decoder.mean_fc.blocks.0.weight", "decoder.log_var_fc.blocks.0.weight"])
    g.append(["decoder.mean_fc.blocks.0.bias", "decoder.log_var_fc.blocks.0.bias"])
    for head in ("mean_fc", "log_var_fc"):
        for i in (2, 4):
            g.append([f"decoder.{head}.blocks.{i}.weight"])
            g.append([f"decoder.{head}.blocks.{i}.bias"])
    return g


class ParamLayout:
    def __init__(self, cfg):
        self.shapes = reference_shapes(cfg)
        self.offsets = {}
        off = 0
        for group in _engine_order(cfg):
            off = (off + 3) // 4 * 4  # 16-byte aligned group start
            for name in group:
                self.offsets[name] = off
                n = 1
                for d in self.shapes[name]:
                    n *= d
                off += n
        self.total = (off + 3) // 4 * 4
        assert set(self.offsets) == set(self.shapes)

    def numel(self, name):
        n = 1
        for d in self.shapes[name]:
            n *= d
        return n


class _Pool:
    """Named device buffers that only grow: a _Work for a new (B, T) takes views of them, so a
    recipe whose padded length changes every batch reuses one allocation (sized by the largest
    B*T seen, grown by >= 25 % at a time) instead of reallocating ~GBs per batch."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}

    def __call__(self, name, shape, dtype=torch.float32):
        if isinstance(shape, int):
            shape = (shape,)
        n = 1
        for d in shape:
            n *= int(d)
        key = (name, dtype)
        cur = self.bufs.get(key)
        if cur is None or cur.numel() < n:
            cap = n if cur is None else max(n, cur.numel() * 5 // 4)
            cur = torch.empty(max(cap, 1), device=self.device, dtype=dtype)
            self.bufs[key] = cur
        return cur[:n].view(shape)

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.bufs.values())


class _Work:
    """Activation/gradient workspaces for one (B, T): views of the engine's growing pool."""

    def __init__(self, cfg, B, T, device, enc_fused=False, pool=None, f8_l0=False):
        N = B * T
        F, E, Z, H, L, C = cfg.F, cfg.E, cfg.Z, cfg.H, cfg.L, cfg.C
        pool = pool or _Pool(device)
        self.B, self.T, self.N = B, T, N

        class _Alloc:  # torch.empty-like front end of the pool: every buffer gets its own name
            def __init__(self):
                self.i = 0

            def __call__(self, *shape, dtype=torch.float32, **_):
                self.i += 1
                return pool(f"w{self.i}", shape, dtype)
        empty = _Alloc()
        f = dict(dtype=torch.float32)
        self.E1 = empty(N, E, **f)
        self.E2 = empty(N, E, **f)
        self.ML = empty(N, 2 * Z, **f)
        self.Zs = empty(N, Z, **f)
        self.eps = empty(N, Z, **f)
        # gate buffer [N, 8H]: fp32, or fp16 where the recurrence runs the wide-batch kernels
        # (halves the projection's write and the recurrences' reads; include/mlvae.h)
        self.g16 = bool(lib().mlvae_lstm_gates_fp16_t(B, T, H, PREC[cfg.prec]))
        self.G = [empty(N, 8 * H, dtype=torch.float16 if self.g16 else torch.float32) for _ in range(L)]
        # wide BPTT: per batch group rows of the bias gradients (summed over groups by colsum)
        self.NBG = (B + 15) // 16
        self.dbias_rows = [empty(self.NBG, 8 * H, **f) if self.g16 else None for _ in range(L)]
        self.Cs = [empty(N, 2 * H, **f) for _ in range(L)]
        self.Y = [empty(N, 2 * H, **f) for _ in range(L)]
        self.Yd = [empty(N, 2 * H, **f) if cfg.dropout > 0 else None for _ in range(L - 1)]
        # bf16 mode: bf16 copies of the big GEMM operands (h, dropout output, dG)
        self.bf = cfg.prec == "bf16"
        b16 = dict(dtype=torch.bfloat16)
        self.Yb = [empty(N, 2 * H, **b16) for _ in range(L)] if self.bf else None
        self.Ydb = ([empty(N, 2 * H, **b16) if cfg.dropout > 0 else None for _ in range(L - 1)]
                    if self.bf else None)
        self.dGb = [empty(N, 8 * H, **b16) for _ in range(L)] if self.bf else None
        # fused encoder (encoder.hip): z as bf16 [N, Z + 16] = [z | 1 | 0 ...], the ones column
        # feeding the bottom layer's bias gradient (skinny.hip); bf16 hidden activations
        self.enc_fused = self.bf and enc_fused
        self.ZA = Z + 16 if self.enc_fused else Z
        self.Zb = empty(N, self.ZA, **b16) if self.bf else None  # first layer's GEMM operand
        # fp8 mode, per layer li >= 1: X8[li] the e4m3 layer input (written by layer li-1's
        # forward recurrence or a cast), dG8[li] the layer's e4m3 dG (written by its BPTT); both
        # per layer, because layer li's weight gradient on the side stream still reads them while
        # the layers below run (one shared pair was overwritten at L >= 3)
        f8 = self.bf and cfg.fp8
        self.X8 = {li: empty(N, 2 * H, dtype=torch.uint8) for li in range(1, L)} if f8 else None
        # (layer 0 too when its dG readers can take e4m3: the skinny dZ / dW_ih_l0 kernels, i.e. the
        # fused encoder without the one-pass skinny_dzw form, engine.py _f8_layer0)
        self.dG8 = {li: empty(N, 8 * H, dtype=torch.uint8) for li in range(0 if f8_l0 else 1, L)} if f8 else None
        # ... and H8[li] the e4m3 copy of layer li's own h (x-scale), dW_hh's operand: the fp8 BPTT
        # then writes dG as e4m3 only (12 -> 4 KB per frame)
        self.H8 = {li: empty(N, 2 * H, dtype=torch.uint8) for li in range(0 if f8_l0 else 1, L)} if f8 else None
        self.E1b = empty(N, E, **b16) if self.enc_fused else None
        self.E2b = empty(N, E, **b16) if self.enc_fused else None
        if self.bf:
            self.Yd = [None] * (L - 1)  # the dropout output exists as bf16 only
        self.P1 = empty(N, 2 * C, **f)
        self.P2m = empty(N, C, **f)
        self.P2v = empty(N, C, **f)
        self.MUX = empty(N, F, **f)
        self.LVX = empty(N, F, **f)
        # backward
        self.dMUX = empty(N, F, **f)
        self.dLVX = empty(N, F, **f)
        self.dP2m = empty(N, C, **f)
        self.dP2v = empty(N, C, **f)
        self.dP1 = empty(N, 2 * C, **f)
        # fused heads: per-workgroup bias-gradient column sums (the five head biases)
        self.heads_bws = empty(lib().mlvae_heads_bias_workspace_size(B, T, F, C) // 4 + 1, **f) \
            if self.bf else None
        # ... and the heads' four small weight gradients accumulated inside the heads kernel
        nwg = lib().mlvae_heads_wgrad_workspace_size(B, T, F, C) if self.bf else 0
        self.heads_wgws = empty(nwg // 4 + 1, **f) if nwg else None
        self.dY = [empty(N, 2 * H, **f) for _ in range(L)]
        self.dZs = empty(N, Z, **f)
        self.dML = empty(N, 2 * Z, **f)
        self.dE2 = empty(N, E, **f)
        self.dE1 = empty(N, E, **f)
        l = lib()
        self.nk = l.mlvae_elbo_partials_count(B, T, Z)
        self.nr = l.mlvae_elbo_partials_count(B, T, F)
        self.pk = empty(self.nk, **f)
        self.pr = empty(self.nr, **f)
        self.nh = l.mlvae_heads_partials_count(B, T)
        self.ph = empty(self.nh, **f)   # fused heads' recon partials
        self.nke = l.mlvae_encoder_partials_count(B, T) if self.enc_fused else 0
        self.pke = empty(max(self.nke, 1), **f)  # fused encoder's KL partials
        ewb = l.mlvae_encoder_workspace_size(B, T, F, E, Z) if self.enc_fused else 0
        self.enc_ws = empty(ewb // 4 + 1, **f)
        # Conv1d encoder: weight-gradient slabs of the two layers (main and side stream)
        self.conv_ws = ([empty(l.mlvae_conv1d_wgrad_workspace_size(B, T, cin, E, cfg.enc_conv) // 4 + 1, **f)
                         for cin in (F, E)] if cfg.enc_conv else None)
        self.loss = torch.zeros(3, device=device, dtype=torch.float32)  # own tensor: returned to the caller   # [kld_loss, recon_loss, total]
        self.count = torch.zeros(1, device=device, dtype=torch.int32)
        # GEMM split-K workspace: the largest any call of the step asks for
        shapes = [(N, E, F), (N, E, E), (N, 2 * Z, E), (N, 2 * C, 2 * H), (N, C, C), (N, F, C),
                  (F, C, N), (C, C, N), (2 * C, 2 * H, N), (2 * Z, E, N), (E, E, N), (E, F, N),
                  (N, 2 * H, 8 * H), (N, Z, 8 * H), (4 * H, H, N)]
        for li in range(L):
            din = Z if li == 0 else 2 * H
            shapes += [(N, 8 * H, din), (8 * H, din, N)]
        ws = max(max(l.mlvae_gemm_workspace_size(m, n, k), l.mlvae_gemm_ex_workspace_size(m, n, k),
                     l.mlvae_gemm_bf16_workspace_size(m, n, k, 1))
                 for m, n, k in shapes)
        ws = max(ws, l.mlvae_gemm_bf16_workspace_size(4 * H, H, N, 2))  # both directions' dW_hh
        if self.enc_fused:
            ws = max(ws, l.mlvae_skinny_tn_workspace_size(8 * H, self.ZA, N))
            if Z == 32 and (8 * H) % 256 == 0:
                ws = max(ws, l.mlvae_skinny_dzw_workspace_size(N, 8 * H))
        cs = max(l.mlvae_colsum_workspace_size(N, c) for c in (F, C, 2 * C, 8 * H, 2 * Z, E))
        self.gws = empty(max(ws, cs, 16) // 4 + 1, **f)
        self.gws_side = empty(max(ws, cs, 16) // 4 + 1, **f)  # for the wgrad side stream
        self.gws_bytes = self.gws.numel() * 4
        xb = _lib.SZ()
        check(l.mlvae_lstm_workspace_size(B, H, PREC[cfg.prec], _lib.C.byref(xb)), "lstm_workspace_size")
        self.xbuf = empty(max(xb.value, 16), dtype=torch.uint8)


def _aligned(ptr, ld, bf):
    return ptr is not None and ptr % 16 == 0 and ld % (8 if bf else 4) == 0


def _pb(t, off=0):
    """address of element off of a bf16 tensor"""
    return t.data_ptr() + 2 * off


def _p(t, off=0):
    return t.data_ptr() + 4 * off


class VAEEngine:
    """MI355X-native train/eval step of the VanillaVAE + BiLSTM-decoder recipe."""

    def __init__(self, cfg, device="cuda", params=None, seed=123456):
        self.cfg = cfg.check()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("VAEEngine runs on the HIP device only (no CPU fallback)")
        lib()
        self.layout = ParamLayout(cfg)
        n = self.layout.total
        f = dict(device=self.device, dtype=torch.float32)
        self.flat = torch.zeros(n, **f)
        # the flat gradient sits behind a 4-float header: in data parallel the step's loss shares
        # and err word ride in the last gradient bucket's all-reduce (mlvae_dp_scalars)
        self._grad_ext = torch.zeros(4 + n, **f)
        self.grad = self._grad_ext[4:]
        self.exp_avg = torch.zeros(n, **f)
        self.exp_avg_sq = torch.zeros(n, **f)
        self.step_ctr = torch.zeros(1, device=self.device, dtype=torch.int32)
        self.nonfinite_ctr = torch.zeros(1, device=self.device, dtype=torch.int32)
        self.grad_norm = torch.zeros(1, **f)
        self.hyp = torch.zeros(4, **f)
        # spin-timeout word of the persistent recurrences (set on a hand-off timeout; the
        # launch then completes with undefined outputs): checked by check_errors()
        self.err = torch.zeros(1, device=self.device, dtype=torch.int32)
        # optimizer steps skipped because `err` was set (their gradients are undefined): the
        # fused Adam reads the word on the device, so a timeout never reaches the weights
        self.err_skips = torch.zeros(1, device=self.device, dtype=torch.int32)
        self._nonfinite_seen = 0   # nonfinite_ctr value at the last check_health()
        # bf16 mode: bf16 copy of the weights, refreshed at the start of every forward
        self.flat_bf = torch.empty(n, device=self.device, dtype=torch.bfloat16) if cfg.prec == "bf16" else None
        # bf16 mode: k-contiguous W_ih^T [din, 8H] of the layers whose dgrad runs on the 256² GEMM
        self.wih_t = {}
        # bf16 mode: the heads run as one fused kernel (heads.hip) when the shape is supported
        self.fused_heads = (cfg.prec == "bf16" and bool(lib().mlvae_heads_supported(cfg.C, cfg.F, 2 * cfg.H)))
        # fused heads: in-kernel bias sums + bf16 saved intermediates (False: the colsum passes
        # over fp32 intermediates; same box 12.30 -> 12.17 ms/step with them)
        self.heads_bias_sums = True
        # dY (the layer outputs' gradients) in bf16 where its producers can write it: the heads'
        # split form and the bf16 dgrad, into the wide-batch BPTT (mlvae_lstm_bwd_ex3 / _fp8_ex)
        self.dy_bf16 = cfg.prec == "bf16"
        self.w1_t = (torch.empty(2 * cfg.C * 2 * cfg.H, device=self.device, dtype=torch.bfloat16)
                     if self.fused_heads else None)
        # the split-bf16 forward of the encoder and the heads (bf16 hi + lo operand pairs: the ELBO,
        # mu and log_var without the bf16 rounding of those weights -- the bulk of the bf16 step's
        # ELBO error, tools/elbo_budget.py); False: plain bf16 operands
        self.split_fwd = cfg.prec == "bf16"
        self.w1_split = (torch.empty(2 * cfg.C * 4 * cfg.H, device=self.device, dtype=torch.bfloat16)
                         if self.fused_heads else None)
        # bf16 mode: the encoder (+ reparameterisation + KL) runs as two fused kernels
        # (encoder.hip) and the bottom layer's products on skinny kernels (skinny.hip)
        self.fused_encoder = (cfg.prec == "bf16" and not cfg.enc_conv and
                              bool(lib().mlvae_encoder_supported(cfg.F, cfg.E, cfg.Z)))
        if cfg.prec == "bf16":
            for li in range(1, cfg.L):
                self.wih_t[li] = torch.empty(2 * cfg.H * 8 * cfg.H, device=self.device, dtype=torch.bfloat16)
            if cfg.fp8:  # fp8 e4m3 copies of W_ih_l{>=1} (both directions) and their scales
                self.w8 = {li: torch.empty(8 * cfg.H * 2 * cfg.H, device=self.device, dtype=torch.uint8)
                           for li in range(1, cfg.L)}
                self.w8s = {li: torch.zeros(2, device=self.device) for li in range(1, cfg.L)}
                # the fp8 dgrad: W_ih^T as e4m3 (scale w8s[li][0]), [q_dG, alpha] from delayed
                # scaling, and the amax words the BPTT writes (two: this step's / the last step's)
                self.w8t = {li: torch.empty(2 * cfg.H * 8 * cfg.H, device=self.device, dtype=torch.uint8)
                            for li in range(1, cfg.L)}
                self.g8 = {li: torch.zeros(2, device=self.device) for li in range(0, cfg.L)}
                self.g8_amax = {li: torch.zeros(2, device=self.device, dtype=torch.int32) for li in range(0, cfg.L)}
                # the fp8 weight gradient dW_ih = dG^T X (e4m3 dG and layer input): alpha =
                # 1 / (q_dG * x-scale) (False: bf16)
                self.fp8_wgrad = True
                # ... and dW_hh = sum_t dG_t^T h_{t-/+1} on e4m3 dG and h (time-shifted rows in the
                # fp8 TN kernel), so that no bf16 dG is written (False: bf16 dW_hh and dG)
                self.fp8_whh = True
                # ... and layer 0's dG readers (dZ, dW_ih_l0, dW_hh_l0) on e4m3 as well (False: bf16)
                self.fp8_l0 = True
                self.one1 = torch.ones(1, device=self.device)  # layer 0's "other" scale: alpha = 1 / q_dG
                # ... and then (from the second step) the recurrence below writes the e4m3 layer
                # input alone: no bf16 GEMM reads dropout(h) (False: both copies every step)
                self.fp8_skip_ydb = True
                self.x8s = torch.tensor([x8_scale(cfg.dropout)], device=self.device)
                self.g8w = {li: torch.zeros(2, device=self.device) for li in range(0, cfg.L)}
                self.g8_ready = False  # a previous step's amax exists (the first step's dgrad is bf16)
                self.g8_par = 0
                self.f8ws = torch.empty(lib().mlvae_fp8_scale_workspace_size() // 4 + 1, device=self.device)
            if self.fused_encoder:  # dZ = dG W_ih_l0 over its k-contiguous transpose
                self.wih_t[0] = torch.empty(cfg.Z * 8 * cfg.H, device=self.device, dtype=torch.bfloat16)
        self.nparts = lib().mlvae_sumsq_partials_count(n)
        self.sq_parts = torch.zeros(self.nparts, device=self.device, dtype=torch.float64)
        self.seed = seed
        self.rng_step = 0
        self._work = {}
        self._T = 0
        self._pool = _Pool(self.device)
        # weight-gradient GEMMs on a side stream, unless the recurrences fill the chip
        # (_full_chip; force_overlap True / False overrides the choice)
        self.force_overlap = None
        self.overlap = True
        # split-K workgroup targets of the weight-gradient GEMMs (mlvae_gemm_bf16): those that
        # overlap a recurrence / those in the step's tail
        self.split_overlap = 128
        self.split_tail = 160
        # layer-0 input projection (K = latent width) fused into the layer-0 forward recurrence
        # (mlvae_lstm_fwd_z: the 8H-wide fp16 projection is never written); where that form does
        # not apply, on the skinny projection kernel (skinny_proj False: the 256² GEMM)
        self.zproj = True
        self.skinny_proj = True
        # layer 0's dZ and dW_ih_l0 from one pass over dG (False: the NT + TN pair)
        self.dzw = True
        # dW_hh as unshifted products minus the utterance-boundary terms (_whh_bf16; False: the
        # time-shifted batched product), and layer 0's bf16 h written pre-shifted (False: as h_t)
        self.whh_unshift = True
        self.yb_prev = True
        # the wide recurrence writes dropout(h) itself (False: a separate dropout pass)
        self._fuse_drop = True
        self.side_stream = torch.cuda.Stream(self.device)
        # the step's critical path (recurrences, dgrads) runs on a high-priority stream so the
        # dispatcher prefers its workgroups over the side stream's weight-gradient GEMMs
        self.prioritize = False   # measured no gain at c2 (8.44 vs 8.39 ms); kept as an option
        self.main_stream = torch.cuda.Stream(self.device, priority=-1)
        self._on_side = False
        self.side_prep = True      # weight prep beside the layer-0 recurrence (when it leaves CUs free)
        self.heads_wgrad = True    # the heads' dW3 / dW2 inside the heads kernel (mlvae_heads_fused_ex2)
        self.kernel_timers = None   # {name: [(start_event, end_event), ...]} when profiling
        self.process_group = None   # set by mlvae_hip.dist for data parallel
        self.world = 1
        self.rank = 0
        self.global_offset = 0      # first global utterance index of this shard
        # data parallel: the gradient suffix from the top LSTM layer on (top layer + heads) is
        # all-reduced on comm_stream during the lower layers' BPTT, the prefix in optimizer_step
        self.bucket_allreduce = True
        self.comm_stream = None
        self._ar_pending = False
        self.ar_split = self.layout.offsets[f"decoder.rnn.weight_ih_l{cfg.L - 1}"]
        if params is not None:
            self.load_reference_params(params)

    # ------------------------------------------------------------------ parameters
    def view(self, name, buf=None):
        buf = self.flat if buf is None else buf
        o = self.layout.offsets[name]
        return buf[o:o + self.layout.numel(name)].view(self.layout.shapes[name])

    def named_parameters(self):
        return OrderedDict((k, self.view(k)) for k in self.layout.shapes)

    def named_grads(self):
        return OrderedDict((k, self.view(k, self.grad)) for k in self.layout.shapes)

    @classmethod
    def from_modules(cls, encoder, decoder, device="cuda", prec="fp32", kld_weight=1e-3,
                     recon_weight=1.0, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                     max_grad_norm=5.0, seed=123456, fp8=False):
        """Build an engine whose flat buffer becomes the storage of the given modules'
        parameters (VanillaVAE + Decoder, as the recipe yaml builds them): after this call
        module.parameters() are views of engine.flat and their .grad views of engine.grad."""
        heads = decoder.mean_fc.linear_plan()
        if hasattr(encoder, "conv"):  # modules/conv_vae.py ConvVAE
            c0 = encoder.conv[0].conv_plan()[0][0]
            F, E, kconv = c0.in_channels, c0.out_channels, c0.kernel_size[0]
        else:
            lin0 = encoder.fc[0].linear_plan()[0][0]
            F, E, kconv = lin0.in_features, lin0.out_features, 0
        cfg = VAEConfig(F=F, E=E, enc_conv=kconv,
                        Z=encoder.mean_fc.out_features, H=decoder.rnn.hidden_size,
                        L=decoder.rnn.num_layers, C=heads[0][0].out_features,
                        dropout=float(decoder.rnn.dropout), loss_type=decoder.loss_type,
                        kld_weight=kld_weight, recon_weight=recon_weight, lr=lr, betas=tuple(betas),
                        adam_eps=eps, max_grad_norm=max_grad_norm, prec=prec, fp8=fp8)
        params = OrderedDict()
        for pre, mod in (("encoder.", encoder), ("decoder.", decoder)):
            for n, p in mod.named_parameters():
                params[pre + n] = p.detach()
        eng = cls(cfg, device=device, params=params, seed=seed)
        for pre, mod in (("encoder.", encoder), ("decoder.", decoder)):
            for n, p in mod.named_parameters():
                p.data = eng.view(pre + n)
                p.grad = eng.view(pre + n, eng.grad)
        return eng

    def init_default(self, seed=None):
        """PyTorch-default initialisation, drawn on the device: U(-1/sqrt(fan_in), +) for
        Linear weights and biases (nn.Linear.reset_parameters) and U(-1/sqrt(H), +) for every
        LSTM tensor (nn.LSTM.reset_parameters) -- the distributions the reference's modules
        get from their constructors (ref:src/modules/fc_block.py, src/modules/decoder.py)."""
        g = torch.Generator(device=self.device).manual_seed(self.seed if seed is None else seed)
        with torch.no_grad():
            for name, shp in self.layout.shapes.items():
                if ".rnn." in name:
                    bound = 1.0 / math.sqrt(self.cfg.H)
                else:
                    wshape = self.layout.shapes[name[:-4] + "weight"] if name.endswith("bias") else shp
                    bound = 1.0 / math.sqrt(math.prod(wshape[1:]))  # fan_in (Conv1d: Cin * K)
                v = self.view(name)
                v.uniform_(-bound, bound, generator=g)
        return self

    def load_reference_params(self, params):
        with torch.no_grad():
            for k, v in params.items():
                self.view(k).copy_(torch.as_tensor(v, dtype=torch.float32))

    def _ptr(self, name, buf=None):
        return _p(self.flat if buf is None else buf, self.layout.offsets[name])

    def _wb(self, name):
        """bf16 copy of a weight (bf16 mode), else None."""
        if self.flat_bf is None:
            return None
        return _pb(self.flat_bf, self.layout.offsets[name])

    def _fp8_whh(self, w, li, N, T, gp, shifted=False):
        """fp8 mode: both directions' dW_hh_l{li} = sum_t dG_t^T h_{t-1} / h_{t+1} on e4m3 operands in
        one batched launch (mlvae_gemm_fp8_tn_ex, time-shifted rows): the layer's e4m3 dG from its
        BPTT and h cast to e4m3 with the layer-input scale (|h| < 1), so alpha = 1 / (q_dG x-scale)"""
        H = self.cfg.H
        l = lib()
        ws = w.gws_side if self._on_side else w.gws
        st = self._stream()
        check(l.mlvae_cast_fp8(N * 2 * H, _pb(w.Yb[li]), 1, None, x8_scale(self.cfg.dropout), w.H8[li].data_ptr(),
                               st), "cast_fp8")
        check(l.mlvae_gemm_fp8_tn_ex(4 * H, H, N, 2, w.dG8[li].data_ptr(), 8 * H, 4 * H, w.H8[li].data_ptr(), 2 * H, H,
                                     gp(f"decoder.rnn.weight_hh_l{li}"), H, 4 * H * H, _p(self.g8w[li], 1),
                                     0 if shifted else T, 0 if shifted else -1, 0 if shifted else 2,
                                     _p(ws), w.gws_bytes, st), "gemm_fp8_tn_ex")

    def _whh_bf16(self, w, li, N, T, dG_bf, Yb, gp):
        """Both directions' dW_hh_l{li} = sum_t dG_t^T h_{t-1} (forward) / h_{t+1} (reverse) as
        UNSHIFTED products (the m/n-contiguous eight-phase loop; with time-shifted rows it spills and
        runs on the older loop): over all N frames the operands offset by one row pair dG row k with
        h row k -/+ 1, which at each utterance's first (forward) / last (reverse) step is the
        neighbouring utterance's h -- those B - 1 terms are summed first by a small strided product
        (rows T apart) and subtracted by the main product's beta = -1."""
        H = self.cfg.H
        if not getattr(self, "whh_unshift", True):  # (A/B: the time-shifted batched product)
            self._fast(w, 1, 0, 4 * H, H, N, _pb(dG_bf), 8 * H, _pb(Yb), 2 * H, gp(f"decoder.rnn.weight_hh_l{li}"),
                       H, batch=2, a_bs=4 * H, b_bs=H, c_bs=4 * H * H, kshift_T=T, kshift=-1, kstep=2)
            return
        nb = N // T
        ld, lh = 8 * H, 2 * H
        C = gp(f"decoder.rnn.weight_hh_l{li}")  # the reverse direction's gradient follows it
        # both directions in one batched launch each (batch strides: the reverse entry's offsets
        # minus the forward one's): forward dG from row 1 with h from row 0, reverse dG from row 0
        # with h from row 1; the boundary terms at rows T apart: forward (dG row bT, h row bT - 1),
        # reverse (dG row bT + T - 1, h row (b + 1) T)
        if nb > 1:
            ca0, cb0 = T * ld, (T - 1) * lh
            self._fast(w, 1, 0, 4 * H, H, nb - 1, _pb(dG_bf, ca0), T * ld, _pb(Yb, cb0), T * lh, C, H, batch=2,
                       a_bs=(T - 1) * ld + 4 * H - ca0, b_bs=T * lh + H - cb0, c_bs=4 * H * H)
        self._fast(w, 1, 0, 4 * H, H, N - 1, _pb(dG_bf, ld), ld, _pb(Yb), lh, C, H, batch=2,
                   a_bs=4 * H - ld, b_bs=lh + H, c_bs=4 * H * H, beta=-1.0 if nb > 1 else 0.0)

    def _dzw_path(self, N):
        """dZ and dW_ih_l0 from the one-pass skinny_dzw kernel (bf16 dG only)"""
        cfg = self.cfg
        return bool(self.dzw and cfg.Z == 32 and (8 * cfg.H) % 256 == 0 and N >= 65536)

    def _f8_layer0(self, N):
        """fp8 mode: layer 0's BPTT writes its dG as e4m3 alone from the second step on, and dZ,
        dW_ih_l0 (+ biases) and dW_hh_l0 read that copy -- the skinny e4m3 kernels (skinny.hip) and
        the time-shifted fp8 TN GEMM; needs the fused encoder without the one-pass skinny_dzw form"""
        cfg = self.cfg
        return bool(cfg.fp8 and cfg.prec == "bf16" and getattr(self, "fp8_l0", False) and self.fused_encoder
                    and not self._dzw_path(N) and N >= 4096 and (8 * cfg.H) % 256 == 0 and cfg.H % 16 == 0)

    def work(self, B, T):
        key = (B, T)
        if key not in self._work:
            self._work = {key: _Work(self.cfg, B, T, self.device,  # views of the growing pool
                                     enc_fused=self.fused_encoder, pool=self._pool, f8_l0=self._f8_layer0(B * T))}
        return self._work[key]

    # ------------------------------------------------------------------ launch helpers
    def _stream(self):
        if self._on_side:
            return self.side_stream.cuda_stream
        return torch.cuda.current_stream(self.device).cuda_stream

    def _gemm(self, w, ta, tb, M, N, K, A, lda, B, ldb, C, ldc, bias1=None, bias2=None, epi=0,
              aux=None, ldaux=0, kshift_T=0, kshift=0, beta=0.0):
        ws = w.gws_side if self._on_side else w.gws
        check(lib().mlvae_gemm(PREC[self.cfg.prec], ta, tb, M, N, K, 1.0, A, lda, B, ldb, beta, C,
                               ldc, bias1, bias2, epi, aux, ldaux, kshift_T, kshift,
                               _p(ws), w.gws_bytes, self._stream()), "mlvae_gemm")

    def _mm(self, w, ta, tb, M, N, K, A, lda, B, ldb, C, ldc, A_bf=None, B_bf=None, bias1=None,
            bias2=None, epi=0, aux=None, ldaux=0, kshift_T=0, kshift=0, beta=0.0, drop_seed=None):
        """GEMM with each operand given as fp32 (A, B) and/or bf16 (A_bf, B_bf) pointer.
        bf16 mode runs mlvae_gemm_ex (bf16 operands preferred); fp32 mode the exact kernel.
        drop_seed: fuse the inter-layer dropout backward into the epilogue (bf16 path only).
        Returns True when that fusion happened."""
        if self.cfg.prec == "bf16":
            a, abf = (A_bf, 1) if A_bf is not None else (A, 0)
            b, bbf = (B_bf, 1) if B_bf is not None else (B, 0)
            if _aligned(a, lda, abf) and _aligned(b, ldb, bbf):
                ws = w.gws_side if self._on_side else w.gws
                if drop_seed is not None:
                    check(lib().mlvae_gemm_ex_drop(ta, tb, M, N, K, 1.0, a, abf, lda, b, bbf, ldb, beta,
                                                   C, ldc, bias1, bias2, EPI_DROPOUT, aux, ldaux,
                                                   kshift_T, kshift, drop_seed, self._drop_off,
                                                   self.cfg.dropout,
                                                   _p(ws), w.gws_bytes, self._stream()),
                          "mlvae_gemm_ex_drop")
                    return True
                check(lib().mlvae_gemm_ex(ta, tb, M, N, K, 1.0, a, abf, lda, b, bbf, ldb, beta, C,
                                          ldc, bias1, bias2, epi, aux, ldaux, kshift_T, kshift,
                                          _p(ws), w.gws_bytes, self._stream()), "mlvae_gemm_ex")
                return False
        if A is None or B is None:
            raise RuntimeError("GEMM operand exists only as bf16 but is not 16-byte aligned")
        self._gemm(w, ta, tb, M, N, K, A, lda, B, ldb, C, ldc, bias1=bias1, bias2=bias2, epi=epi,
                   aux=aux, ldaux=ldaux, kshift_T=kshift_T, kshift=kshift, beta=beta)
        return False

    def _fast(self, w, ta, tb, M, N, K, A_bf, lda, B_bf, ldb, C, ldc, batch=1, a_bs=0, b_bs=0,
              c_bs=0, bias1=None, bias2=None, kshift_T=0, kshift=0, kstep=0, drop_seed=None,
              out_f16=False, out_bf16=False, beta=0.0):
        """bf16 256² LDS-DMA GEMM (mlvae_gemm_bf16) over bf16 operands: the step's big products.
        out_f16: C is fp16 (the wide recurrence's gate buffer); out_bf16: C is bf16 (dY)."""
        ws = w.gws_side if self._on_side else w.gws
        epi, p = (EPI_DROPOUT, self.cfg.dropout) if drop_seed is not None else (EPI_NONE, 0.0)
        if out_f16:
            epi |= EPI_OUT_F16
        if out_bf16:
            epi |= EPI_OUT_BF16
        check(lib().mlvae_gemm_bf16(ta, tb, M, N, K, batch, A_bf, lda, a_bs, B_bf, ldb, b_bs, C, ldc,
                                    c_bs, beta, bias1, bias2, epi, None, 0, kshift_T, kshift, kstep,
                                    drop_seed or 0, self._drop_off, p, _p(ws), w.gws_bytes,
                                    self._stream()),
              "mlvae_gemm_bf16")

    def _colsum(self, w, N, Cn, src, ld, out, out2=None):
        ws = w.gws_side if self._on_side else w.gws
        check(lib().mlvae_colsum(N, Cn, src, ld, out, out2, 0.0, _p(ws), w.gws_bytes,
                                 self._stream()), "mlvae_colsum")

    def _side(self, fn, ev=None):
        """Run fn's launches on the side stream once everything queued on the main stream up
        to event ev (default: now) is done (weight gradients overlap the next BPTT)."""
        if not self.overlap:
            return fn()
        if ev is None:
            ev = self._mark()
        self.side_stream.wait_event(ev)
        self._on_side = True
        try:
            fn()
        finally:
            self._on_side = False

    def _mark(self):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _defer_side(self, pending, fn):
        """Queue fn for the side stream behind the main stream's current position, but issue
        its launches only at the next _flush_side, so the critical-path launch is enqueued
        first.  (Measured neutral at c2, where the host enqueues a whole step in 0.38 ms of
        the GPU's 5.8 -- tools/host_rate.py -- and runs far ahead; it matters only when the
        host falls behind.)"""
        if not self.overlap:
            return fn()
        pending.append((fn, self._mark()))

    def _flush_side(self, pending):
        for fn, ev in pending:
            self._side(fn, ev)
        pending.clear()

    def _timed(self, name):
        """HIP events around one launch on the main stream (bench.py's roofline timing; launches
        issued to the side stream are not bracketed and are skipped)."""
        eng = self

        class _T:
            def __enter__(self_):
                self_.on = eng.kernel_timers is not None and not eng._on_side
                if self_.on:
                    self_.a = torch.cuda.Event(enable_timing=True)
                    self_.a.record(torch.cuda.current_stream(eng.device))

            def __exit__(self_, *exc):
                if self_.on:
                    b = torch.cuda.Event(enable_timing=True)
                    b.record(torch.cuda.current_stream(eng.device))
                    eng.kernel_timers.setdefault(name, []).append((self_.a, b))
        return _T()

    def _join_side(self):
        if self.overlap:
            ev = torch.cuda.Event()
            ev.record(self.side_stream)
            torch.cuda.current_stream(self.device).wait_event(ev)

    # ------------------------------------------------------------------ forward
    def forward(self, x, lens, eps=None, train=False, dropout_masks=None, need_grad_inputs=False):
        """compute_forward + compute_objectives.  x [B,T,F] fp32 (normalised features),
        lens [B] relative lengths.  Returns the workspace (outputs stay on device)."""
        cfg = self.cfg
        B, T, Fdim = x.shape
        if Fdim != cfg.F:
            raise ValueError(f"feature dim {Fdim} != input_size {cfg.F}")
        x = x.contiguous()
        if x.data_ptr() % 16:  # the fused kernels read 16-byte rows
            x = x.clone()
        lens = lens.to(device=self.device, dtype=torch.float32).contiguous()
        w = self.work(B, T)
        w.x, w.lens = x, lens
        self._T = T
        if self.world > 1:  # every rank holds B utterances of the global batch: shard r starts at r * B
            self.global_offset = self.rank * B
        N, E, Z, H, C, Fd = w.N, cfg.E, cfg.Z, cfg.H, cfg.C, cfg.F
        l, s = lib(), self._stream()
        X = _p(x)
        prep_ev = None
        if self.flat_bf is not None:  # this step's weights as bf16 GEMM operands
            check(l.mlvae_cast_bf16(self.layout.total, _p(self.flat), _pb(self.flat_bf), s), "cast_bf16")
            # the transposed / fp8 weight copies the layer-1 projection, the heads and the backward
            # read: beside the encoder and the layer-0 forward recurrence on the side stream when
            # that recurrence leaves CUs free (off the critical path), else in line
            if self.side_prep and not self._full_chip(B):
                self._on_side = True
                self.side_stream.wait_event(self._mark())
                try:
                    self._weight_prep(train)
                finally:
                    self._on_side = False
                prep_ev = torch.cuda.Event()
                prep_ev.record(self.side_stream)
            else:
                self._weight_prep(train)
        wb = self._wb
        count = None
        if self.world > 1:
            count = self._global_count(w)
        eps_off = self._eps_offset(T) + self.rng_step * (1 << 40)
        eps_t = None if eps is None else eps.to(self.device, torch.float32).contiguous().view(N, Z)
        w.eps_used = w.eps if eps_t is None else eps_t
        if w.enc_fused:
            # ---- encoder + reparameterisation noise + z + KL partial sums, one launch
            # (encoder.hip; ref:src/modules/vanilla_vae.py:21-45)
            ep = lambda n: self._ptr(f"encoder.{n}")
            with self._timed("encoder_fwd"):
                check(l.mlvae_encoder_fwd_ex(B, T, Fd, E, Z, X, ep("fc.0.blocks.0.weight"), ep("fc.0.blocks.0.bias"),
                                           ep("fc.0.blocks.2.weight"), ep("fc.0.blocks.2.bias"),
                                           ep("mean_fc.weight"), ep("mean_fc.bias"),
                                           None if eps_t is None else _p(eps_t), self.seed, eps_off, _p(lens),
                                           _pb(w.E1b), _pb(w.E2b), _p(w.ML), _p(w.Zs), _pb(w.Zb), w.ZA,
                                           _p(w.eps) if eps_t is None else None, _p(w.pke), int(self.split_fwd),
                                           s), "encoder_fwd")
            w.kl_parts = (w.pke, w.nke)
        else:
            # ---- reparameterisation noise
            if eps_t is None:
                check(l.mlvae_randn(N * Z, self.seed, eps_off, _p(w.eps), s), "mlvae_randn")
            # ---- encoder (ref:src/modules/vanilla_vae.py:21-28)
            ep = cfg.enc_prefix
            if cfg.enc_conv:  # Conv1d variant (modules/conv_vae.py, csrc/conv.hip)
                K = cfg.enc_conv
                with self._timed("conv_fwd"):
                    check(l.mlvae_conv1d_fwd(B, T, Fd, E, K, X, Fd, self._ptr(f"{ep}.0.weight"),
                                             self._ptr(f"{ep}.0.bias"), 1, _p(w.E1), E, s), "conv1d_fwd")
                    check(l.mlvae_conv1d_fwd(B, T, E, E, K, _p(w.E1), E, self._ptr(f"{ep}.2.weight"),
                                             self._ptr(f"{ep}.2.bias"), 1, _p(w.E2), E, s), "conv1d_fwd")
            else:
                self._mm(w, 0, 1, N, E, Fd, X, Fd, self._ptr(f"{ep}.0.weight"), Fd,
                         _p(w.E1), E, B_bf=wb(f"{ep}.0.weight"),
                         bias1=self._ptr(f"{ep}.0.bias"), epi=EPI_LRELU)
                self._mm(w, 0, 1, N, E, E, _p(w.E1), E, self._ptr(f"{ep}.2.weight"), E,
                         _p(w.E2), E, B_bf=wb(f"{ep}.2.weight"),
                         bias1=self._ptr(f"{ep}.2.bias"), epi=EPI_LRELU)
            self._mm(w, 0, 1, N, 2 * Z, E, _p(w.E2), E, self._ptr("encoder.mean_fc.weight"), E,
                     _p(w.ML), 2 * Z, B_bf=wb("encoder.mean_fc.weight"), bias1=self._ptr("encoder.mean_fc.bias"))
            check(l.mlvae_reparam_kl_fwd(B, T, Z, _p(w.ML), 2 * Z, _p(w.eps_used), _p(lens), _p(w.Zs),
                                         None, _p(w.pk), s), "reparam_kl_fwd")
            if w.bf:
                check(l.mlvae_cast_bf16(N * Z, _p(w.Zs), _pb(w.Zb), s), "cast_bf16")
            w.kl_parts = (w.pk, w.nk)
        # ---- decoder BiLSTM (ref:src/modules/decoder.py:22)
        # layer input as (fp32 tensor or None, bf16 tensor or None, width, bf16 row stride)
        xin, xin_bf, din, ldx = w.Zs, (w.Zb if w.bf else None), Z, w.ZA
        w.layer_in = []
        for li in range(cfg.L):
            if li == 1 and prep_ev is not None:  # the layer-1 weight copies (side stream) are done
                torch.cuda.current_stream(self.device).wait_event(prep_ev)
                prep_ev = None
            w.layer_in.append((xin, xin_bf, din, ldx))
            # layer 0 on the 32-wide latent: the projection inside the recurrence (below)
            zproj = bool(li == 0 and self.zproj and w.bf and w.g16 and din == 32 and ldx % 8 == 0 and
                         xin_bf is not None)
            if zproj:
                pass
            elif w.bf and din <= 32 and din % 8 == 0 and self.skinny_proj:
                # K = latent width: the write-bound skinny projection kernel (skinny.hip)
                check(l.mlvae_skinny_proj_ex(N, 8 * H, din, _pb(xin_bf), ldx,
                                             wb(f"decoder.rnn.weight_ih_l{li}"), din,
                                             self._ptr(f"decoder.rnn.bias_ih_l{li}"),
                                             self._ptr(f"decoder.rnn.bias_hh_l{li}"), _p(w.G[li]), 8 * H,
                                             int(w.g16), s), "skinny_proj")
            elif w.bf and cfg.fp8 and li > 0 and din % 16 == 0 and ldx == din:
                # configs[4]: fp8 e4m3 operands, per-tensor scales (x: the fixed 2^8, |x| <= 1/(1-p);
                # W_ih: 448 / max|W_ih|), block-scaled MFMA, alpha = 1 / (2^8 q_w) (fp8.hip)
                xs = x8_scale(cfg.dropout)
                with self._timed(f"proj_l{li}"):
                    # (W_ih's e4m3 copies and scale: _weight_prep)
                    if not w.__dict__.get("x8_fused", {}).get(li):  # else the recurrence wrote it
                        check(l.mlvae_cast_fp8(N * din, _pb(xin_bf), 1, None, xs, w.X8[li].data_ptr(), s), "cast_fp8")
                    check(l.mlvae_gemm_fp8(N, 8 * H, din, w.X8[li].data_ptr(), din, self.w8[li].data_ptr(), din,
                                           _p(w.G[li]), 8 * H, _p(self.w8s[li], 1),
                                           self._ptr(f"decoder.rnn.bias_ih_l{li}"),
                                           self._ptr(f"decoder.rnn.bias_hh_l{li}"),
                                           EPI_OUT_F16 if w.g16 else EPI_NONE, s), "gemm_fp8")
            elif w.bf and din % 8 == 0:  # input projection on the 256² GEMM
                with self._timed(f"proj_l{li}"):
                    self._fast(w, 0, 1, N, 8 * H, din, _pb(xin_bf), ldx, wb(f"decoder.rnn.weight_ih_l{li}"),
                               din, _p(w.G[li]), 8 * H, bias1=self._ptr(f"decoder.rnn.bias_ih_l{li}"),
                               bias2=self._ptr(f"decoder.rnn.bias_hh_l{li}"), out_f16=w.g16)
            else:
                if w.g16:
                    raise RuntimeError("fp16 gate buffer needs a bf16 layer input with din % 8 == 0")
                self._mm(w, 0, 1, N, 8 * H, din, _p(xin) if xin is not None else None, din,
                         self._ptr(f"decoder.rnn.weight_ih_l{li}"), din, _p(w.G[li]), 8 * H,
                         A_bf=_pb(xin_bf) if xin_bf is not None else None,
                         B_bf=wb(f"decoder.rnn.weight_ih_l{li}"),
                         bias1=self._ptr(f"decoder.rnn.bias_ih_l{li}"),
                         bias2=self._ptr(f"decoder.rnn.bias_hh_l{li}"))
            drop = li < cfg.L - 1 and train and cfg.dropout > 0
            # the wide kernels also write the next layer's dropout(h) (same Philox masks as
            # mlvae_dropout_ex) and skip the fp32 h nothing reads
            fuse_drop = w.g16 and drop and dropout_masks is None and self._fuse_drop
            need_y = (not w.g16 or (drop and not fuse_drop) or
                      (li == cfg.L - 1 and not (self.fused_heads and w.bf)))
            seed = self._drop_seed(li) if fuse_drop else 0
            # fp8 mode: the recurrence also writes the next layer's e4m3 input (no cast pass)
            x8_fused = (cfg.fp8 and fuse_drop and not need_y and w.X8 is not None and (li + 1) in w.X8
                        and 2 * H % 16 == 0)
            x8_ptr = w.X8[li + 1].data_ptr() if x8_fused else None
            w.__dict__.setdefault("x8_fused", {})[li + 1] = x8_fused
            # fp8 steady state: layer li+1's dgrad and weight gradient both run on e4m3 (the
            # backward's f8w), so the bf16 dropout(h) has no reader and is not written
            skip_ydb = bool(x8_fused and self.g8_ready and self.fp8_wgrad and getattr(self, "fp8_skip_ydb", False)
                            and (li + 1) in self.g8
                            and l.mlvae_gemm_fp8_tn_workspace_size(8 * H, 2 * H, N) <= w.gws_bytes)
            w.__dict__.setdefault("ydb_skipped", {})[li + 1] = skip_ydb
            ydb_arg = None if skip_ydb else (_pb(w.Ydb[li]) if fuse_drop else None)
            # the bf16 h of a layer below a fused dropout has one reader, its own dW_hh: the
            # recurrence writes it pre-shifted (row t = the h entering step t) and the weight
            # gradient runs unshifted (the m/n-contiguous eight-phase GEMM loop)
            yb_prev = bool(zproj and fuse_drop and getattr(self, "yb_prev", True))
            w.__dict__.setdefault("yb_prev", {})[li] = yb_prev
            with self._timed("lstm_fwd"):
                if zproj:
                    rp = lambda n: self._ptr(f"decoder.rnn.{n}")
                    check(l.mlvae_lstm_fwd_z2(B, T, H, rp("weight_hh_l0"), rp("weight_hh_l0_reverse"), _pb(xin_bf),
                                              ldx, din, rp("weight_ih_l0"), rp("weight_ih_l0_reverse"),
                                              rp("bias_ih_l0"), rp("bias_hh_l0"), rp("bias_ih_l0_reverse"),
                                              rp("bias_hh_l0_reverse"), _p(w.G[li]), _p(w.Cs[li]),
                                              _p(w.Y[li]) if need_y else None, _pb(w.Yb[li]), int(yb_prev),
                                              ydb_arg,
                                             x8_ptr,
                                              x8_scale(cfg.dropout) if x8_fused else 0.0, seed, self._drop_off,
                                              cfg.dropout if fuse_drop else 0.0, _p(w.xbuf), w.xbuf.numel(),
                                              _p(self.err), s), "lstm_fwd_z2")
                elif x8_fused:
                    check(l.mlvae_lstm_fwd_fp8(B, T, H, self._ptr(f"decoder.rnn.weight_hh_l{li}"),
                                               self._ptr(f"decoder.rnn.weight_hh_l{li}_reverse"), _p(w.G[li]),
                                               _p(w.Cs[li]), _pb(w.Yb[li]), ydb_arg, x8_ptr,
                                               x8_scale(cfg.dropout), seed, self._drop_off, cfg.dropout,
                                               _p(w.xbuf), w.xbuf.numel(), _p(self.err), s), "lstm_fwd_fp8")
                else:
                    check(l.mlvae_lstm_fwd_ex2(PREC[cfg.prec], B, T, H, self._ptr(f"decoder.rnn.weight_hh_l{li}"),
                                               self._ptr(f"decoder.rnn.weight_hh_l{li}_reverse"), _p(w.G[li]),
                                               int(w.g16), _p(w.Cs[li]), _p(w.Y[li]) if need_y else None,
                                               _pb(w.Yb[li]) if w.bf else None,
                                               _pb(w.Ydb[li]) if fuse_drop else None, seed, self._drop_off,
                                               cfg.dropout if fuse_drop else 0.0,
                                               _p(w.xbuf), w.xbuf.numel(), _p(self.err), s), "lstm_fwd")
            xin, xin_bf, din, ldx = w.Y[li], (w.Yb[li] if w.bf else None), 2 * H, 2 * H
            if drop:
                xin, xin_bf = w.Yd[li], (w.Ydb[li] if w.bf else None)
                if fuse_drop:
                    w.__dict__.setdefault("_drop_seed", {})[li] = (seed, None)
                else:
                    self._dropout(w, li, w.Y[li], xin, dropout_masks)
        if prep_ev is not None:
            torch.cuda.current_stream(self.device).wait_event(prep_ev)
        w.rnn_out = w.Y[cfg.L - 1]
        w.rnn_out_bf = w.Yb[cfg.L - 1] if w.bf else None
        # ---- heads (ref:src/modules/decoder.py:24-25, FCBlock ref:src/modules/fc_block.py:9-16)
        lt = LOSS[cfg.loss_type]
        w_kl, w_rec = self.loss_weights()
        w.heads_fused = self.fused_heads and w.bf
        if w.heads_fused:
            # both heads forward + recon loss (+ gradient) + heads backward + dY in one launch
            hp = lambda name: self._ptr(f"decoder.{name}")
            hg = lambda name: self._ptr(f"decoder.{name}", self.grad)
            tr = 1 if train else 0
            # train: the heads' five bias gradients come from in-kernel column sums (the backward
            # skips their colsum passes), and the intermediates the weight-gradient GEMMs read
            # (P1, P2, dOUT, dP2, dP1) are saved as bf16 -- their operand precision -- in the
            # fp32 buffers' memory (packed rows)
            w.heads_bias = bool(train) and w.heads_bws is not None and self.heads_bias_sums
            # bf16 dY from the heads' split form, read by the wide BPTT (per-layer flags)
            w.dy_bf16 = {li: False for li in range(cfg.L)}
            w.dy_bf16[cfg.L - 1] = bool(self.dy_bf16 and w.heads_bias and w.g16)
            bias_args = (_p(w.heads_bws), w.heads_bws.numel() * 4, hg("mean_fc.blocks.4.bias"),
                         hg("log_var_fc.blocks.4.bias"), hg("mean_fc.blocks.2.bias"),
                         hg("log_var_fc.blocks.2.bias"), hg("mean_fc.blocks.0.bias")) \
                if w.heads_bias else (None, 0, None, None, None, None, None)
            # the heads' dW3 / dW2 (both heads) inside the heads kernel: the backward skips their
            # four split-K GEMMs (and the kernel skips saving P2 / dOUT / dP2, read by nothing else)
            w.heads_wgrad = bool(w.heads_bias and self.heads_wgrad and w.heads_wgws is not None)
            mse_h = lt == 1
            wg_args = (_p(w.heads_wgws), w.heads_wgws.numel() * 4, hg("mean_fc.blocks.4.weight"),
                       None if mse_h else hg("log_var_fc.blocks.4.weight"), hg("mean_fc.blocks.2.weight"),
                       None if mse_h else hg("log_var_fc.blocks.2.weight")) \
                if w.heads_wgrad else (None, 0, None, None, None, None)
            # split-bf16 forward (split form only): P1 on W1 hi + lo, stages 2-3 on split W2 / W3 / P2
            w1s = self.split_fwd and w.heads_bias and self.w1_split is not None
            if w1s:
                check(l.mlvae_bf16_split_rows(hp("mean_fc.blocks.0.weight"), 2 * C, 2 * H, 64, _pb(self.w1_split), s),
                      "bf16_split_rows")
            with self._timed("heads"):
                check(l.mlvae_heads_fused_ex3(
                  B, T, Fd, C, 2 * H, lt, tr, _pb(w.rnn_out_bf), wb("decoder.mean_fc.blocks.0.weight"),
                  _pb(self.w1_t) if train else None, hp("mean_fc.blocks.0.bias"),
                  hp("mean_fc.blocks.2.weight"), hp("mean_fc.blocks.2.bias"),
                  hp("mean_fc.blocks.4.weight"), hp("mean_fc.blocks.4.bias"),
                  hp("log_var_fc.blocks.2.weight"), hp("log_var_fc.blocks.2.bias"),
                  hp("log_var_fc.blocks.4.weight"), hp("log_var_fc.blocks.4.bias"),
                  X, _p(lens), count, w_rec, _p(w.P1), _p(w.P2m), _p(w.P2v), _p(w.MUX), _p(w.LVX),
                  _p(w.dMUX) if train else None, _p(w.dLVX) if (train and lt == 0) else None,
                  _p(w.dP2m) if train else None, _p(w.dP2v) if train else None,
                  _p(w.dP1) if train else None, _p(w.dY[cfg.L - 1]) if train else None,
                  _p(w.ph), *bias_args, (3 if w.dy_bf16[cfg.L - 1] else 1) if w.heads_bias else 0,
                  *wg_args, _pb(self.w1_split) if w1s else None, s), "heads_fused")
            check(l.mlvae_elbo_finalize(_p(w.kl_parts[0]), w.kl_parts[1], _p(w.ph), w.nh, _p(lens), count, B, T, Z, Fd,
                                        w_kl, w_rec, _p(w.loss), s), "elbo_finalize")
            return w
        R = _p(w.rnn_out)
        self._mm(w, 0, 1, N, 2 * C, 2 * H, R, 2 * H, self._ptr("decoder.mean_fc.blocks.0.weight"),
                 2 * H, _p(w.P1), 2 * C, A_bf=_pb(w.rnn_out_bf) if w.bf else None,
                 B_bf=wb("decoder.mean_fc.blocks.0.weight"),
                 bias1=self._ptr("decoder.mean_fc.blocks.0.bias"), epi=EPI_LRELU)
        for hd, P2, out in (("mean_fc", w.P2m, w.MUX), ("log_var_fc", w.P2v, w.LVX)):
            off = 0 if hd == "mean_fc" else C
            self._mm(w, 0, 1, N, C, C, _p(w.P1, off), 2 * C,
                     self._ptr(f"decoder.{hd}.blocks.2.weight"), C, _p(P2), C,
                     B_bf=wb(f"decoder.{hd}.blocks.2.weight"),
                     bias1=self._ptr(f"decoder.{hd}.blocks.2.bias"), epi=EPI_LRELU)
            self._mm(w, 0, 1, N, Fd, C, _p(P2), C, self._ptr(f"decoder.{hd}.blocks.4.weight"), C,
                     _p(out), Fd, B_bf=wb(f"decoder.{hd}.blocks.4.weight"),
                     bias1=self._ptr(f"decoder.{hd}.blocks.4.bias"))
        # ---- ELBO part 2 (+ its gradient when training)
        dmux = _p(w.dMUX) if train else None
        dlvx = _p(w.dLVX) if (train and lt == 0) else None
        check(l.mlvae_recon(B, T, Fd, lt, _p(w.MUX), Fd, _p(w.LVX), Fd, X, Fd, _p(lens), count,
                            None, _p(w.pr), None, w_rec, dmux, dlvx, s), "recon")
        check(l.mlvae_elbo_finalize(_p(w.kl_parts[0]), w.kl_parts[1], _p(w.pr), w.nr, _p(lens), count, B, T, Z, Fd,
                                    w_kl, w_rec, _p(w.loss), s), "elbo_finalize")
        return w

    def _weight_prep(self, train):
        """This step's derived weight copies (after cast_bf16 of the flat buffer): the k-contiguous
        transposes the heads' split form and the dgrads read (train), and in fp8 mode W_ih_l{>=1}
        as e4m3 with its per-tensor scale (448 / max|W_ih|) and, for the fp8 dgrad, its
        transpose with the same scale (fp8.hip)."""
        cfg, l, s = self.cfg, lib(), self._stream()
        if train and self.w1_t is not None:
            check(l.mlvae_cast_bf16_t(2 * cfg.C, 2 * cfg.H, self._ptr("decoder.mean_fc.blocks.0.weight"),
                                      _pb(self.w1_t), s), "cast_bf16_t")
        if train:
            for li, dst in self.wih_t.items():
                check(l.mlvae_cast_bf16_t(8 * cfg.H, cfg.Z if li == 0 else 2 * cfg.H,
                                          self._ptr(f"decoder.rnn.weight_ih_l{li}"), _pb(dst), s), "cast_bf16_t")
        if cfg.fp8 and cfg.prec == "bf16":
            n = 8 * cfg.H * 2 * cfg.H
            for li in self.w8:
                wih = self._ptr(f"decoder.rnn.weight_ih_l{li}")
                check(l.mlvae_fp8_scale(n, wih, x8_scale(cfg.dropout), _p(self.w8s[li]), _p(self.f8ws),
                                        self.f8ws.numel() * 4, s), "fp8_scale")
                check(l.mlvae_cast_fp8(n, wih, 0, _p(self.w8s[li]), 0.0, self.w8[li].data_ptr(), s), "cast_fp8")
                if train and li in self.wih_t:  # the fp8 dgrad's W_ih^T, same scale
                    check(l.mlvae_cast_fp8(n, _pb(self.wih_t[li]), 1, _p(self.w8s[li]), 0.0,
                                           self.w8t[li].data_ptr(), s), "cast_fp8")

    def loss_weights(self):
        return float(self.cfg.kld_weight), float(self.cfg.recon_weight)

    def _eps_offset(self, T):
        return self.global_offset * T * self.cfg.Z

    @property
    def _drop_off(self):
        """Philox element offset of this shard's inter-layer dropout masks: the global index of
        its first element of the [B*T, 2H] layer output, so a data-parallel run draws exactly
        the masks of the single-GPU run on the global batch."""
        return self.global_offset * self._T * 2 * self.cfg.H

    def _drop_seed(self, li):
        """Philox key of the dropout after layer li in this step."""
        return (self.seed * 1000003 + self.rng_step * 131 + li) & ((1 << 63) - 1)

    def _dropout(self, w, li, src, dst, masks):
        mask_ptr = None
        if masks is not None:
            m = masks[li].to(self.device, torch.float32).contiguous()
            w.__dict__.setdefault("_masks", {})[li] = m
            mask_ptr = _p(m)
        seed = self._drop_seed(li)
        dst_bf = w.Ydb[li] if w.bf else None
        check(lib().mlvae_dropout_ex(src.numel(), _p(src), _p(dst) if dst is not None else None,
                                     _pb(dst_bf) if dst_bf is not None else None, mask_ptr, seed,
                                     self._drop_off, self.cfg.dropout, self._stream()), "dropout")
        w.__dict__.setdefault("_drop_seed", {})[li] = (seed, mask_ptr)

    def _global_count(self, w):
        from . import dist as mdist
        check(lib().mlvae_count_frames(_p(w.lens), w.B, w.T, _p(w.count), self._stream()), "count")
        mdist.allreduce_count(w.count, self.process_group)
        return _p(w.count)

    # ------------------------------------------------------------------ backward
    def _full_chip(self, B):
        """True when this batch's BPTT launch fills (>= 3/4 of) the chip: a side-stream GEMM
        would then only hold CUs the recurrence's co-resident workgroups wait for (measured at
        B = 256: 17.7 ms/step overlapped vs 15.3 serialised with whole-chip split-K plans)."""
        if self.force_overlap is not None:
            return not self.force_overlap
        wgs = lib().mlvae_lstm_launch_workgroups(B, self.cfg.H, PREC[self.cfg.prec], 0)
        return wgs >= 0.75 * _lib.device_cus()

    def backward(self, w):
        cfg = self.cfg
        B, T, N = w.B, w.T, w.N
        full = self._full_chip(B)
        self.overlap = not full
        dzw_done = False   # dW_ih_l0 already produced by the layer-0 skinny_dzw pass
        # the side-stream weight gradients' workgroup target scales with their work against the
        # BPTT they overlap (fixed length): proportional to the batch, halved on e4m3 operands
        # (twice the MFMA rate). split_overlap is the target at B = 64 in bf16; same process
        # (profiles/ab/r06_split_overlap.txt): B = 32 bf16 and B = 64 fp8 run best at 64, B = 64 bf16 at 128
        so = int(round(self.split_overlap * B / 64 * (0.5 if (cfg.fp8 and self.g8_ready) else 1.0)))
        split_overlap, split_tail = (256, 256) if full else (min(256, max(32, so)), self.split_tail)
        E, Z, H, C, Fd = cfg.E, cfg.Z, cfg.H, cfg.C, cfg.F
        l, s = lib(), self._stream()
        g = self.grad
        gp = lambda name: self._ptr(name, g)
        mse = cfg.loss_type == "mse"
        count = _p(w.count) if self.world > 1 else None
        # ---- heads tail: dgrad chain on the main stream (already done inside the fused heads
        # kernel when it ran), wgrads on the side stream
        fused = getattr(w, "heads_fused", False)
        pending = []  # side-stream work issued right after the next critical-path launch
        side = (lambda fn: self._defer_side(pending, fn)) if fused else self._side
        heads = [("mean_fc", w.P2m, w.dMUX, w.dP2m, 0)]
        if not mse:
            heads.append(("log_var_fc", w.P2v, w.dLVX, w.dP2v, C))
        wb = self._wb
        for hd, P2, dOut, dP2, off in heads:
            W3, W2 = self._ptr(f"decoder.{hd}.blocks.4.weight"), self._ptr(f"decoder.{hd}.blocks.2.weight")

            hb = getattr(w, "heads_bias", False)  # bias gradients already summed by the heads kernel

            def wg3(hd=hd, dOut=dOut, P2=P2, hb=hb):
                if hb:  # bf16 saved intermediates (the heads kernel's saved_bf16)
                    self._mm(w, 1, 0, Fd, C, N, None, Fd, None, C, gp(f"decoder.{hd}.blocks.4.weight"), C,
                             A_bf=_p(dOut), B_bf=_p(P2))
                else:
                    self._mm(w, 1, 0, Fd, C, N, _p(dOut), Fd, _p(P2), C, gp(f"decoder.{hd}.blocks.4.weight"), C)
                if not hb:
                    self._colsum(w, N, Fd, _p(dOut), Fd, gp(f"decoder.{hd}.blocks.4.bias"))
            if not getattr(w, "heads_wgrad", False):
                side(wg3)
            if not fused:
                self._mm(w, 0, 0, N, C, Fd, _p(dOut), Fd, W3, C, _p(dP2), C,
                         B_bf=wb(f"decoder.{hd}.blocks.4.weight"), epi=EPI_DLRELU, aux=_p(P2), ldaux=C)

            def wg2(hd=hd, dP2=dP2, off=off, hb=hb):
                if hb:  # bf16 rows: the head's P1 half starts off elements in
                    self._mm(w, 1, 0, C, C, N, None, C, None, 2 * C, gp(f"decoder.{hd}.blocks.2.weight"), C,
                             A_bf=_p(dP2), B_bf=_pb(w.P1, off))
                else:
                    self._mm(w, 1, 0, C, C, N, _p(dP2), C, _p(w.P1, off), 2 * C,
                             gp(f"decoder.{hd}.blocks.2.weight"), C)
                if not hb:
                    self._colsum(w, N, C, _p(dP2), C, gp(f"decoder.{hd}.blocks.2.bias"))
            if not getattr(w, "heads_wgrad", False):
                side(wg2)
            if not fused:
                self._mm(w, 0, 0, N, C, C, _p(dP2), C, W2, C, _p(w.dP1, off), 2 * C,
                         B_bf=wb(f"decoder.{hd}.blocks.2.weight"), epi=EPI_DLRELU,
                         aux=_p(w.P1, off), ldaux=2 * C)
        K1 = C if mse else 2 * C  # mse: the log_var head gets no gradient (torch: grad None)
        R = _p(w.rnn_out)
        R_bf = _pb(w.rnn_out_bf) if w.bf else None

        def wg1():
            if getattr(w, "heads_bias", False) and R_bf is not None:
                # bf16 dP1 [N, 2C] and rnn_out: the 256² kernel (m/n-contiguous, split-K)
                self._fast(w, 1, 0, K1, 2 * H, N, _p(w.dP1), 2 * C, R_bf, 2 * H,
                           gp("decoder.mean_fc.blocks.0.weight"), 2 * H)
                return
            self._mm(w, 1, 0, K1, 2 * H, N, _p(w.dP1), 2 * C, R, 2 * H,
                     gp("decoder.mean_fc.blocks.0.weight"), 2 * H, B_bf=R_bf)
            if not getattr(w, "heads_bias", False):
                self._colsum(w, N, K1, _p(w.dP1), 2 * C, gp("decoder.mean_fc.blocks.0.bias"))
        side(wg1)
        if not fused:
            self._mm(w, 0, 0, N, 2 * H, K1, _p(w.dP1), 2 * C, self._ptr("decoder.mean_fc.blocks.0.weight"),
                     2 * H, _p(w.dY[cfg.L - 1]), 2 * H, B_bf=wb("decoder.mean_fc.blocks.0.weight"))
        # ---- BiLSTM layers, top to bottom
        ran_f8 = False   # an fp8 BPTT recorded this step's amax (a batch too small for the wide
        for li in range(cfg.L - 1, -1, -1):   # kernels runs none: the amax parity must not flip)
            xin, xin_bf, din, ldx = w.layer_in[li]
            Gl = w.G[li]
            dGb = w.dGb[li] if w.bf else None
            # fp8 mode: the layer's BPTT also writes dG as e4m3 under delayed scaling (the scale
            # from the previous step's amax, this step's amax for the next) for the fp8 dgrad;
            # the first step has no amax yet and keeps the bf16 dgrad
            f8 = bool(cfg.fp8 and w.g16 and w.dG8 is not None and li in w.dG8 and li in getattr(self, "g8", {}))
            f8_dgrad = f8 and self.g8_ready
            # configs[4]: dW_ih of an fp8 layer on the e4m3 dG (this step's BPTT) and e4m3 input
            f8w = bool(f8_dgrad and self.fp8_wgrad and w.X8 is not None and li in w.X8 and ldx == din and din % 16 == 0
                       and l.mlvae_gemm_fp8_tn_workspace_size(8 * H, din, N) <= w.gws_bytes)
            # ... and both directions' dW_hh on the e4m3 dG and h: then no reader is left for a
            # bf16 dG and the BPTT writes the e4m3 copy alone
            f8hh = bool(f8w and getattr(self, "fp8_whh", False) and w.H8 is not None and li in w.H8
                        and H % 16 == 0 and l.mlvae_gemm_fp8_tn_ex_workspace_size(4 * H, H, N, 2) <= w.gws_bytes)
            # layer 0 (fused encoder, w.dG8 holds it only where _f8_layer0): dZ, dW_ih_l0 | biases and
            # dW_hh_l0 all on the e4m3 dG
            f8l0 = bool(li == 0 and f8_dgrad and w.enc_fused and w.H8 is not None and 0 in w.H8
                        and l.mlvae_gemm_fp8_tn_ex_workspace_size(4 * H, H, N, 2) <= w.gws_bytes
                        and l.mlvae_skinny_tn_workspace_size(8 * H, w.ZA, N) <= w.gws_bytes)
            if li == 0:
                f8hh = f8l0
            w.__dict__.setdefault("f8hh", {})[li] = f8hh
            with self._timed("lstm_bwd"):
                # the layer-0 biases come with dW_ih_l0 from skinny_tn when the encoder is fused
                rows = w.dbias_rows[li] if (w.g16 and not (li == 0 and w.enc_fused)) else None
                if f8:
                    ran_f8 = True
                    par = self.g8_par   # this step's amax word; the other holds the last step's
                    am = self.g8_amax[li].data_ptr()
                    if f8_dgrad and self.fp8_wgrad:  # [q_dG, 1 / (q_dG x-scale)] of the fp8 weight gradient
                        check(l.mlvae_fp8_delayed_scale(am + 4 * (1 - par), None, _p(self.x8s), G8_MARGIN,
                                                        _p(self.g8w[li]), s), "fp8_delayed_scale")
                    # [q_dG, alpha]: the fp8 dgrad's 1 / (q_dG q_W); layer 0's skinny products' 1 / q_dG
                    other = self.one1 if li == 0 else self.w8s[li]
                    check(l.mlvae_fp8_delayed_scale(am + 4 * (1 - par), am + 4 * par, _p(other), G8_MARGIN,
                                                    _p(self.g8[li]), s), "fp8_delayed_scale")
                    dyb = bool(getattr(w, "dy_bf16", {}).get(li, False))
                    check(l.mlvae_lstm_bwd_fp8_ex(B, T, H, self._ptr(f"decoder.rnn.weight_hh_l{li}"),
                                               self._ptr(f"decoder.rnn.weight_hh_l{li}_reverse"), _p(Gl),
                                               _p(w.Cs[li]), _p(w.dY[li]), int(dyb), None if f8hh else _pb(dGb),
                                               _p(rows) if rows is not None else None,
                                               w.dG8[li].data_ptr() if f8_dgrad else None, _p(self.g8[li]),
                                               am + 4 * par, _p(w.xbuf), w.xbuf.numel(), _p(self.err), s),
                          "lstm_bwd_fp8")
                else:
                    dyb = bool(getattr(w, "dy_bf16", {}).get(li, False))
                    check(l.mlvae_lstm_bwd_ex3(PREC[cfg.prec], B, T, H, self._ptr(f"decoder.rnn.weight_hh_l{li}"),
                                               self._ptr(f"decoder.rnn.weight_hh_l{li}_reverse"), _p(Gl),
                                               int(w.g16), _p(w.Cs[li]), _p(w.dY[li]), int(dyb),
                                               _pb(dGb) if dGb is not None else None,
                                               _p(rows) if rows is not None else None,
                                               _p(w.xbuf), w.xbuf.numel(), _p(self.err), s), "lstm_bwd")
            self._flush_side(pending)
            # dG: fp32 in G (fp32 mode) or bf16 in dGb (bf16 mode)
            dG, dG_bf = (None, dGb) if dGb is not None else (Gl, None)
            pg = lambda t, off=0: None if t is None else _p(t, off)
            pgb = lambda t, off=0: None if t is None else _pb(t, off)
            Ybl = w.Yb[li] if w.bf else None

            if w.__dict__.get("ydb_skipped", {}).get(li) and not f8w:
                raise RuntimeError(f"layer {li}: the forward skipped the bf16 dropout(h) the bf16 weight gradient reads")

            def wgl_body(li=li, dG=dG, dG_bf=dG_bf, xin=xin, xin_bf=xin_bf, din=din, ldx=ldx,
                         Ybl=Ybl, f8w=f8w, f8hh=f8hh):
                if li == 0 and w.enc_fused:
                    # both directions' dW_hh_l0 in one batched 256² launch; dW_ih_l0 and the
                    # biases follow the encoder backward on the main stream (skinny_tn below)
                    pre = bool(w.__dict__.get("yb_prev", {}).get(0))  # Yb rows already shifted
                    with self._timed("wgrad_hh_l0"):
                        if f8hh:
                            self._fp8_whh(w, 0, N, T, gp, shifted=pre)
                        elif pre:
                            self._fast(w, 1, 0, 4 * H, H, N, _pb(dG_bf), 8 * H, _pb(Ybl), 2 * H,
                                       gp("decoder.rnn.weight_hh_l0"), H, batch=2, a_bs=4 * H, b_bs=H,
                                       c_bs=4 * H * H)
                        else:
                            self._whh_bf16(w, 0, N, T, dG_bf, Ybl, gp)
                    return
                if dG_bf is not None and xin_bf is not None and din % 8 == 0 and H % 8 == 0:
                    # 256² GEMMs: dW_ih = dG^T X, and both directions' dW_hh = sum_t dG_t^T h_{t-/+1}
                    # in one batched launch (the two weights are adjacent in the flat gradient);
                    # HIP-event timed when they run on the main stream (the full-chip case)
                    with self._timed(f"wgrad_ih_l{li}"):
                        if f8w:
                            ws = w.gws_side if self._on_side else w.gws
                            check(lib().mlvae_gemm_fp8_tn(8 * H, din, N, w.dG8[li].data_ptr(), 8 * H, w.X8[li].data_ptr(),
                                                          din, gp(f"decoder.rnn.weight_ih_l{li}"), din,
                                                          _p(self.g8w[li], 1), _p(ws), w.gws_bytes, self._stream()),
                                  "gemm_fp8_tn")
                        else:
                            self._fast(w, 1, 0, 8 * H, din, N, _pb(dG_bf), 8 * H, _pb(xin_bf), ldx,
                                       gp(f"decoder.rnn.weight_ih_l{li}"), din)
                    with self._timed(f"wgrad_hh_l{li}"):
                        # (layer 0 of the Conv1d-encoder configs also writes its h pre-shifted)
                        pre = bool(w.__dict__.get("yb_prev", {}).get(li))
                        if f8hh:
                            self._fp8_whh(w, li, N, T, gp, shifted=pre)
                        elif pre:
                            self._fast(w, 1, 0, 4 * H, H, N, _pb(dG_bf), 8 * H, _pb(Ybl), 2 * H,
                                       gp(f"decoder.rnn.weight_hh_l{li}"), H, batch=2, a_bs=4 * H, b_bs=H,
                                       c_bs=4 * H * H)
                        else:
                            self._whh_bf16(w, li, N, T, dG_bf, Ybl, gp)
                else:
                    self._mm(w, 1, 0, 8 * H, din, N, pg(dG), 8 * H, pg(xin), din,
                             gp(f"decoder.rnn.weight_ih_l{li}"), din, A_bf=pgb(dG_bf), B_bf=pgb(xin_bf))
                    self._mm(w, 1, 0, 4 * H, H, N, pg(dG), 8 * H, _p(w.Y[li]), 2 * H,
                             gp(f"decoder.rnn.weight_hh_l{li}"), H, A_bf=pgb(dG_bf), B_bf=pgb(Ybl),
                             kshift_T=T, kshift=-1)
                    self._mm(w, 1, 0, 4 * H, H, N, pg(dG, 4 * H), 8 * H, _p(w.Y[li], H), 2 * H,
                             gp(f"decoder.rnn.weight_hh_l{li}_reverse"), H, A_bf=pgb(dG_bf, 4 * H),
                             B_bf=pgb(Ybl, H), kshift_T=T, kshift=1)
                if w.g16:  # the BPTT summed dG per batch group: sum the groups' rows
                    self._colsum(w, w.NBG, 8 * H, _p(w.dbias_rows[li]), 8 * H,
                                 gp(f"decoder.rnn.bias_ih_l{li}"), gp(f"decoder.rnn.bias_hh_l{li}"))
                elif dG_bf is not None:
                    ws = w.gws_side if self._on_side else w.gws
                    check(lib().mlvae_colsum_ex(N, 8 * H, _pb(dG_bf), 1, 8 * H, gp(f"decoder.rnn.bias_ih_l{li}"),
                                                gp(f"decoder.rnn.bias_hh_l{li}"), 0.0, _p(ws), w.gws_bytes,
                                                self._stream()), "colsum")
                else:
                    self._colsum(w, N, 8 * H, _p(dG), 8 * H, gp(f"decoder.rnn.bias_ih_l{li}"),
                                 gp(f"decoder.rnn.bias_hh_l{li}"))
            def wgl(li=li, body=wgl_body):
                # split-K target: the upper layers' weight gradients overlap the next BPTT, so
                # they take half the CUs; the bottom layer's run in the step's tail, on 160 of
                # the 256 CUs so the encoder backward beside them is not held off the chip
                # (alone 26 us, behind a whole-chip GEMM 112 us; c2 5.85 -> 5.80 ms/step).
                # (body bound here: a call issued after a later layer's loop iteration must
                # not pick up that iteration's wgl_body)
                prev = l.mlvae_gemm_bf16_set_split_target(split_tail if li == 0 else split_overlap)
                try:
                    body(li=li)
                finally:
                    l.mlvae_gemm_bf16_set_split_target(prev)

            # The dgrad (+ dropout backward) is the critical path into the next BPTT; the
            # weight gradients go to the side stream after it (so they overlap that BPTT, not
            # this GEMM).  Below the bottom layer nothing waits on the dgrad: its weight
            # gradients, the step's longest tail, go first.
            if li == 0:
                self._defer_side(pending, wgl)
            dx = w.dZs if li == 0 else w.dY[li - 1]
            drop = li > 0 and xin is not w.Y[li - 1]  # dropout between layers li-1 and li
            seed, mask_ptr = w._drop_seed[li - 1] if drop else (None, None)
            if li == 0 and w.enc_fused:
                if self._dzw_path(N) and w.ZA >= 48:
                    # dZ = dG W_ih_l0 and dW_ih_l0 | db = dG^T [z | 1] from one pass over dG
                    # (skinny.hip skinny_dzw: the skinny NT and TN kernels each read all of it).
                    # Same box, alternating: c3 10.70 -> 10.49 ms/step; at c2's 16,000 frames its
                    # 32 workgroups and 786 KB weight slab per workgroup lose (4.36 -> 4.43), so
                    # smaller batches keep the pair (profiles/ab/r04_dzw.txt)
                    check(l.mlvae_skinny_dzw(N, 8 * H, _pb(dG_bf), 8 * H, _pb(self.wih_t[0]), 8 * H, _pb(w.Zb),
                                             w.ZA, Z, _p(w.dZs), Z, gp("decoder.rnn.weight_ih_l0"),
                                             gp("decoder.rnn.bias_ih_l0"), gp("decoder.rnn.bias_hh_l0"),
                                             _p(w.gws), w.gws_bytes, s), "skinny_dzw")
                    dzw_done = True
                elif f8hh:  # fp8 mode: on the e4m3 dG, alpha = 1 / q_dG
                    check(l.mlvae_skinny_nt_fp8(N, Z, 8 * H, w.dG8[0].data_ptr(), 8 * H, _pb(self.wih_t[0]), 8 * H,
                                                _p(w.dZs), Z, _p(self.g8[0], 1), s), "skinny_nt_fp8")
                else:
                    # dZ = dG W_ih_l0: [N, 8H] x [8H, Z] on the skinny NT kernel
                    check(l.mlvae_skinny_nt(N, Z, 8 * H, _pb(dG_bf), 8 * H, _pb(self.wih_t[0]), 8 * H,
                                            _p(w.dZs), Z, s), "skinny_nt")
                self._flush_side(pending)
                fused = False
            elif f8_dgrad:
                # configs[4]: dX = dG W_ih on e4m3 operands (dG from the BPTT, W_ih^T cast with the
                # forward's scale), alpha = 1 / (q_dG q_W), the dropout backward in the epilogue
                epi8 = EPI_DROPOUT if (drop and mask_ptr is None) else EPI_NONE
                # dY of the layer below in bf16 when the wide BPTT reads it (as the bf16 dgrad)
                dyb = bool(self.dy_bf16 and w.g16 and (epi8 == EPI_DROPOUT or not drop)
                           and getattr(w, "dy_bf16", None) is not None)
                if dyb:
                    w.dy_bf16[li - 1] = True
                with self._timed(f"dgrad_l{li}"):
                    check(l.mlvae_gemm_fp8_ex(N, din, 8 * H, w.dG8[li].data_ptr(), 8 * H, self.w8t[li].data_ptr(),
                                              8 * H, _p(dx), din, _p(self.g8[li], 1), None, None,
                                              epi8 | (EPI_OUT_BF16 if dyb else 0),
                                              (seed or 0) if epi8 else 0, self._drop_off, cfg.dropout, s),
                          "gemm_fp8_ex")
                fused = epi8 == EPI_DROPOUT
            elif dG_bf is not None and li in self.wih_t and din >= 256:
                # dX = dG W_ih as an NT product over the k-contiguous W_ih^T copy; dY of the layer
                # below in bf16 when the wide BPTT reads it (the dropout backward fused)
                fused = drop and mask_ptr is None
                dyb = bool(self.dy_bf16 and w.g16 and (fused or not drop) and getattr(w, "dy_bf16", None) is not None)
                if dyb:
                    w.dy_bf16[li - 1] = True
                with self._timed(f"dgrad_l{li}"):
                    self._fast(w, 0, 1, N, din, 8 * H, _pb(dG_bf), 8 * H, _pb(self.wih_t[li]), 8 * H,
                               _p(dx), din, drop_seed=seed if fused else None, out_bf16=dyb)
            else:
                fused = self._mm(w, 0, 0, N, din, 8 * H, pg(dG), 8 * H,
                                 self._ptr(f"decoder.rnn.weight_ih_l{li}"), din, _p(dx), din,
                                 A_bf=pgb(dG_bf), B_bf=wb(f"decoder.rnn.weight_ih_l{li}"),
                                 drop_seed=seed if (drop and mask_ptr is None) else None)
            if drop and not fused:
                check(l.mlvae_dropout_ex(dx.numel(), _p(dx), _p(dx), None, mask_ptr, seed, self._drop_off,
                                         cfg.dropout, s),
                      "dropout_bwd")
            self._flush_side(pending)  # li == 0 without the fused encoder
            if li > 0:
                self._defer_side(pending, wgl)  # issued right after the next BPTT launch
            # (not beside a whole-chip BPTT: the collective's kernel would hold CUs the
            # recurrence's co-resident workgroups wait for; all of it then goes in optimizer_step)
            if li == cfg.L - 1 and self.world > 1 and self.bucket_allreduce and not full:
                self._flush_side(pending)  # the bucket waits on the side stream: issue it all
                self._start_suffix_allreduce()
        if ran_f8:
            self.g8_ready = True   # this step's BPTT recorded the amax the next step scales by
            self.g8_par ^= 1
        # ---- encoder
        w_kl, _ = self.loss_weights()
        if w.enc_fused:
            # reparam/KL gradient, both LReLU dgrads and the six encoder gradients (encoder.hip)
            ep = lambda n: self._ptr(f"encoder.{n}")
            ge = lambda n: gp(f"encoder.{n}")
            with self._timed("encoder_bwd"):
                check(l.mlvae_encoder_bwd(B, T, Fd, E, Z, _p(w.dZs), _p(w.ML), _p(w.eps_used), _pb(w.E1b),
                                        _pb(w.E2b), _p(w.x), ep("mean_fc.weight"), ep("fc.0.blocks.2.weight"),
                                        _p(w.lens), count, w_kl, ge("mean_fc.weight"), ge("mean_fc.bias"),
                                        ge("fc.0.blocks.2.weight"), ge("fc.0.blocks.2.bias"),
                                        ge("fc.0.blocks.0.weight"), ge("fc.0.blocks.0.bias"), _p(w.enc_ws),
                                        w.enc_ws.numel() * 4, s), "encoder_bwd")
            # dW_ih_l0 | db_ih_l0 = db_hh_l0 = dG^T [z | 1] (skinny.hip), on the main stream
            # while the side stream finishes dW_hh_l0 (the step's two tails run side by side)
            if w.f8hh.get(0):  # fp8 mode: on layer 0's e4m3 dG, alpha = 1 / q_dG
                check(l.mlvae_skinny_tn_fp8(8 * H, w.ZA, N, w.dG8[0].data_ptr(), 8 * H, _pb(w.Zb), w.ZA, Z,
                                            gp("decoder.rnn.weight_ih_l0"), gp("decoder.rnn.bias_ih_l0"),
                                            gp("decoder.rnn.bias_hh_l0"), _p(self.g8[0], 1), _p(w.gws), w.gws_bytes,
                                            s), "skinny_tn_fp8")
            elif not dzw_done:
                check(l.mlvae_skinny_tn(8 * H, w.ZA, N, _pb(w.dGb[0]), 8 * H, _pb(w.Zb), w.ZA, Z,
                                        gp("decoder.rnn.weight_ih_l0"), gp("decoder.rnn.bias_ih_l0"),
                                        gp("decoder.rnn.bias_hh_l0"), _p(w.gws), w.gws_bytes, s), "skinny_tn")
            self._join_side()
            return
        check(l.mlvae_reparam_kl_bwd(B, T, Z, _p(w.ML), 2 * Z, _p(w.eps_used), _p(w.lens), count,
                                     _p(w.dZs), None, w_kl, _p(w.dML), 2 * Z, s), "reparam_kl_bwd")

        def wge2():
            self._mm(w, 1, 0, 2 * Z, E, N, _p(w.dML), 2 * Z, _p(w.E2), E, gp("encoder.mean_fc.weight"), E)
            self._colsum(w, N, 2 * Z, _p(w.dML), 2 * Z, gp("encoder.mean_fc.bias"))
        self._side(wge2)
        self._mm(w, 0, 0, N, E, 2 * Z, _p(w.dML), 2 * Z, self._ptr("encoder.mean_fc.weight"), E,
                 _p(w.dE2), E, B_bf=wb("encoder.mean_fc.weight"), epi=EPI_DLRELU, aux=_p(w.E2), ldaux=E)

        ep = cfg.enc_prefix
        if cfg.enc_conv:  # Conv1d variant: weight gradients + the input gradient (csrc/conv.hip)
            K = cfg.enc_conv

            def wgc(cin, dy, xin, name, ws):
                check(l.mlvae_conv1d_wgrad(B, T, cin, E, K, _p(dy), E, xin, cin, gp(f"{ep}.{name}.weight"),
                                           gp(f"{ep}.{name}.bias"), _p(ws), ws.numel() * 4, self._stream()),
                      "conv1d_wgrad")
            self._side(lambda: wgc(E, w.dE2, _p(w.E1), 2, w.conv_ws[1]))
            with self._timed("conv_bwd"):
                check(l.mlvae_conv1d_dgrad(B, T, E, E, K, _p(w.dE2), E, self._ptr(f"{ep}.2.weight"), _p(w.E1),
                                           E, _p(w.dE1), E, s), "conv1d_dgrad")
                wgc(Fd, w.dE1, _p(w.x), 0, w.conv_ws[0])
            self._join_side()
            return

        def wge1():
            self._mm(w, 1, 0, E, E, N, _p(w.dE2), E, _p(w.E1), E, gp(f"{ep}.2.weight"), E)
            self._colsum(w, N, E, _p(w.dE2), E, gp(f"{ep}.2.bias"))
        self._side(wge1)
        self._mm(w, 0, 0, N, E, E, _p(w.dE2), E, self._ptr(f"{ep}.2.weight"), E,
                 _p(w.dE1), E, B_bf=wb(f"{ep}.2.weight"), epi=EPI_DLRELU,
                 aux=_p(w.E1), ldaux=E)
        self._mm(w, 1, 0, E, Fd, N, _p(w.dE1), E, _p(w.x), Fd, gp(f"{ep}.0.weight"), Fd)
        self._colsum(w, N, E, _p(w.dE1), E, gp(f"{ep}.0.bias"))
        self._join_side()

    # ------------------------------------------------------------------ optimizer
    def optimizer_step(self, w):
        """check_gradients (non-finite loss -> skip; clip_grad_norm_ 5.0) + Adam, on device."""
        cfg, l, s = self.cfg, lib(), self._stream()
        if self.world > 1:
            self._allreduce_grads(w)
        check(l.mlvae_grad_sumsq(_p(self.grad), self.layout.total, self.sq_parts.data_ptr(), s), "sumsq")
        b1, b2 = cfg.betas
        check(l.mlvae_adam_step_ex(_p(self.flat), _p(self.exp_avg), _p(self.exp_avg_sq), _p(self.grad),
                                   self.layout.total, self.sq_parts.data_ptr(), self.nparts,
                                   _p(w.loss, 2), self.step_ctr.data_ptr(), self.nonfinite_ctr.data_ptr(),
                                   self.err.data_ptr(), self.err_skips.data_ptr(),
                                   cfg.lr, b1, b2, cfg.adam_eps, cfg.max_grad_norm,
                                   _p(self.grad_norm), _p(self.hyp), 1, s), "adam")

    def _start_suffix_allreduce(self):
        """Everything the top LSTM layer's and the heads' gradients depend on is queued (the
        side stream holds their weight-gradient GEMMs): sum that contiguous suffix of the flat
        gradient over ranks on a communication stream, overlapping the lower layers' BPTT."""
        from . import dist as mdist
        if self.comm_stream is None:
            self.comm_stream = torch.cuda.Stream(self.device)
        self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
        if self.overlap:
            self.comm_stream.wait_stream(self.side_stream)
        with torch.cuda.stream(self.comm_stream):
            mdist.allreduce_grad_bucket(self.grad[self.ar_split:], self.process_group)
        self._ar_pending = True

    def _allreduce_grads(self, w):
        """The last gradient bucket (the prefix, or the whole buffer) with the step's scalars in
        its header: loss3 summed, and the skip-on-timeout decision made global -- a rank whose
        recurrence timed out contributed an undefined share to the summed gradient, so every rank
        skips that update.  Per step a rank issues three collectives: the frame count (forward),
        the suffix bucket (during the lower layers' BPTT) and this one."""
        from . import dist as mdist
        l, s = lib(), self._stream()
        hdr = self._grad_ext
        check(l.mlvae_dp_scalars(1, _p(hdr), _p(w.loss), self.err.data_ptr(), s), "dp_scalars")
        if self._ar_pending:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
            mdist.allreduce_grad_bucket(hdr[:4 + self.ar_split], self.process_group)
            self._ar_pending = False
        else:
            mdist.allreduce_grad_bucket(hdr, self.process_group)
        check(l.mlvae_dp_scalars(0, _p(hdr), _p(w.loss), self.err.data_ptr(), s), "dp_scalars")

    def _main(self):
        """Context: run on the high-priority main stream, ordered after (and before) the
        caller's current stream."""
        eng = self

        class _M:
            def __enter__(self_):
                if not eng.prioritize:
                    return
                self_.caller = torch.cuda.current_stream(eng.device)
                eng.main_stream.wait_stream(self_.caller)
                self_.ctx = torch.cuda.stream(eng.main_stream)
                self_.ctx.__enter__()

            def __exit__(self_, *exc):
                if not eng.prioritize:
                    return
                self_.ctx.__exit__(*exc)
                self_.caller.wait_stream(eng.main_stream)
        return _M()

    # ------------------------------------------------------------------ input normalisation
    def normalise(self, x, lens, norm, epoch=0):
        """The recipe's InputNormalization(norm_type='global') (SpeechBrain, un-vendored; built at
        ref:src/models/test_vanilla_vae/model.yaml:14-15, called at
        ref:src/models/test_vanilla_vae/model.py:24-25) on the device, as the first launches of
        the step (csrc/norm.hip): per-utterance statistics, the global running statistics
        updated in place in `norm` (a brain.features.InputNormalization: its glob_mean /
        glob_std buffers and host-side count, with that module's semantics), then
        (x - mean) / std into an engine buffer.  Under data parallelism the batch statistics
        are all-reduced in training, as the module does.  Returns the normalised [B, T, F]."""
        B, T, F = x.shape
        l, s = lib(), self._stream()
        if not l.mlvae_norm_supported(F):
            raise ValueError(f"input normalisation kernels need F % 4 == 0 (F={F})")
        x = x.contiguous()
        if x.data_ptr() % 16:
            x = x.clone()
        lens = lens.to(device=self.device, dtype=torch.float32).contiguous()
        utt = self._pool("norm_utt", (B, 2 * F))
        sums = self._pool("norm_sums", (2 * F + 4,))
        out = self._pool("norm_x", (B, T, F))
        with self._timed("norm"):
            check(l.mlvae_norm_stats(B, T, F, _p(x), _p(lens), _p(utt), _p(sums), float(norm.eps), s),
                  "norm_stats")
            if norm.training and self.world > 1:
                from . import dist as mdist
                mdist.allreduce_loss(sums[:2 * F + 1], self.process_group)   # sum over ranks
            gm, gs = norm.glob_mean, norm.glob_std
            fresh = gm.numel() == 0
            if fresh:
                gm = torch.zeros(F, device=self.device)
                gs = torch.zeros(F, device=self.device)
            elif gm.device != self.device or gm.dtype != torch.float32 or not gm.is_contiguous() \
                    or gm.data_ptr() % 16 or gs.data_ptr() % 16:
                gm = gm.to(self.device, torch.float32).contiguous().clone()
                gs = gs.to(self.device, torch.float32).contiguous().clone()
            norm.glob_mean, norm.glob_std = gm, gs
            mode, w_old, w_new = (1 if fresh else 0), 0.0, 0.0
            if norm.training:
                if norm.count == 0:
                    mode = 1
                elif epoch < norm.update_until_epoch:
                    wt = norm.avg_factor if norm.avg_factor is not None else 1.0 / (norm.count + 1)
                    mode, w_old, w_new = 2, 1 - wt, wt
                norm.count += 1
            check(l.mlvae_norm_update(F, _p(sums), _p(gm), _p(gs), mode, w_old, w_new, s), "norm_update")
            check(l.mlvae_norm_apply(B * T, F, _p(x), _p(gm), _p(gs), _p(out), s), "norm_apply")
        return out

    def train_step(self, x, lens, eps=None, dropout_masks=None, normalizer=None, epoch=0):
        """One fit_batch: [input normalisation,] forward, backward, clip + Adam.  Returns the
        device tensor [kld_loss, recon_loss, loss] (no host synchronisation).  normalizer: the
        recipe's InputNormalization (brain.features), run on the device inside the step."""
        with self._main():
            if normalizer is not None:
                x = self.normalise(x, lens, normalizer, epoch)
            w = self.forward(x, lens, eps=eps, train=True, dropout_masks=dropout_masks)
            self.backward(w)
            self.optimizer_step(w)
        self.rng_step += 1
        return w.loss

    def eval_step(self, x, lens, eps=None, normalizer=None, epoch=0):
        """Forward only; under data parallelism the returned [kld, recon, loss] is the global
        batch's (each rank's share uses the all-reduced frame count; the shares are summed)."""
        with self._main():
            if normalizer is not None:
                x = self.normalise(x, lens, normalizer, epoch)
            w = self.forward(x, lens, eps=eps, train=False)
            if self.world > 1:
                from . import dist as mdist
                mdist.allreduce_loss(w.loss, self.process_group)
        self.rng_step += 1
        return w.loss

    def check_errors(self):
        """Host-synchronising check of the persistent kernels' spin-timeout word.  The steps
        since the timeout were skipped by the fused Adam (err_skips), so the weights and the
        Adam state are those from before it."""
        if int(self.err.item()) != 0:
            raise RuntimeError("LSTM recurrence hand-off timed out (err word set): the outputs "
                               "of the affected steps are undefined; their optimizer updates were "
                               f"skipped ({int(self.err_skips.item())} steps)")

    def check_health(self, nonfinite_patience=3, where=""):
        """Once-per-stage host check (Brain.fit calls it at every stage end): the recurrence
        err word, and SpeechBrain's non-finite patience (check_gradients semantics,
        ref:src/models/md_model.py:82) on the device counter of skipped steps -- more than
        `nonfinite_patience` non-finite losses since the last check raises ValueError."""
        self.check_errors()
        ctr = int(self.nonfinite_ctr.item())
        new = ctr - self._nonfinite_seen
        self._nonfinite_seen = ctr
        if new > nonfinite_patience:
            raise ValueError(f"Loss is not finite and patience is exhausted ({new} non-finite "
                             f"steps skipped{where}, patience {nonfinite_patience})")
        return new
