"""torch.autograd.Functions over libmlvae.so: the operator layer under the drop-in
nn.Modules (modules/fc_block.py, modules/vanilla_vae.py, modules/decoder.py).

Every forward and backward below is a libmlvae.so launch on the current HIP stream; torch
only allocates the output tensors.  Inputs must be fp32 CUDA tensors (row-major [B, T, C]).
The fused training step (mlvae_hip/engine.py) uses the same kernels without autograd.
"""
import ctypes

import torch

from ._lib import SZ, check, lib

PREC = {"fp32": 0, "bf16": 1}
_state = {"prec": "fp32"}
_ws = {}


def set_precision(prec):
    """Operand precision of the matrix products: "fp32" (exact f32 MFMA) or "bf16"."""
    if prec not in PREC:
        raise ValueError(f"precision must be one of {list(PREC)}")
    _state["prec"] = prec


def get_precision():
    return _state["prec"]


class precision:
    """Context: matrix-product operand precision inside the block (the mixed-precision region of
    MDModel.fit_batch's auto_mix_prec branch; backward runs inside it too, since the HIP ops read
    the precision when they launch)."""

    def __init__(self, prec):
        self.prec = prec

    def __enter__(self):
        self.prev = get_precision()
        set_precision(self.prec)
        return self

    def __exit__(self, *exc):
        set_precision(self.prev)


def _prec():
    return PREC[_state["prec"]]


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t, off=0):
    return t.data_ptr() + 4 * off


def _need(t, name):
    if not (t.is_cuda and t.dtype == torch.float32):
        raise TypeError(f"{name}: expected a float32 HIP tensor, got {t.dtype} on {t.device} "
                        "(the HIP path has no CPU fallback)")
    return t.contiguous()


def _workspace(nbytes, key="gemm"):
    dev = torch.cuda.current_device()
    w = _ws.get((dev, key))
    if w is None or w.numel() * 4 < nbytes:
        w = torch.empty(max(nbytes // 4 + 1, 1024), device="cuda", dtype=torch.float32)
        _ws[(dev, key)] = w
    return w


def gemm(ta, tb, M, N, K, A, lda, B, ldb, C, ldc, bias1=None, bias2=None, epi=0, aux=None,
         ldaux=0, beta=0.0, kshift_T=0, kshift=0):
    """C = epi(op(A) op(B) + bias1 + bias2 + beta*C) on raw device pointers (ints)."""
    l = lib()
    ws = _workspace(l.mlvae_gemm_workspace_size(M, N, K))
    check(l.mlvae_gemm(_prec(), ta, tb, M, N, K, 1.0, A, lda, B, ldb, beta, C, ldc, bias1, bias2,
                       epi, aux, ldaux, kshift_T, kshift, _p(ws), ws.numel() * 4, _stream()),
          "mlvae_gemm")


def colsum(N, Cn, src, ld, out, out2=None, beta=0.0):
    l = lib()
    ws = _workspace(l.mlvae_colsum_workspace_size(N, Cn), "colsum")
    check(l.mlvae_colsum(N, Cn, src, ld, out, out2, beta, _p(ws), ws.numel() * 4, _stream()),
          "mlvae_colsum")


def _rows(x):
    return x.numel() // x.shape[-1]


# --------------------------------------------------------------------------- Linear (+LReLU)
class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b), act = LeakyReLU(0.01) or identity (ref:src/modules/fc_block.py:10-16)."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        x, w = _need(x, "linear x"), _need(w, "linear weight")
        b = _need(b, "linear bias") if b is not None else None
        M, K = _rows(x), x.shape[-1]
        N = w.shape[0]
        y = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
        gemm(0, 1, M, N, K, _p(x), K, _p(w), K, _p(y), N, bias1=_p(b) if b is not None else None,
             epi=1 if act else 0)
        ctx.save_for_backward(x, w, y)
        ctx.act, ctx.has_b = act, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = _need(dy, "linear grad")
        M, K, N = _rows(x), x.shape[-1], w.shape[0]
        if ctx.act:  # dpre = dy * lrelu'(y)
            dpre = torch.empty_like(dy)
            check(lib().mlvae_lrelu_bwd(dy.numel(), _p(dy), _p(y), _p(dpre), _stream()), "lrelu_bwd")
        else:
            dpre = dy
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            gemm(0, 0, M, K, N, _p(dpre), N, _p(w), K, _p(dx), K)
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            gemm(1, 0, N, K, M, _p(dpre), N, _p(x), K, _p(dw), K)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = torch.empty(N, device=dy.device, dtype=torch.float32)
            colsum(M, N, _p(dpre), N, _p(db))
        return dx, dw, db, None


def linear(x, w, b=None, act=False):
    return LinearFn.apply(x, w, b, act)


# --------------------------------------------------------------------------- Conv1d encoder
def _conv_ws(nbytes):
    return _workspace(max(int(nbytes), 16), key="conv_wgrad")


class Conv1dFn(torch.autograd.Function):
    """y = act(conv1d(x) + b) over the time axis of batch-first frames x [B, T, Cin]; w
    [Cout, Cin, K] (torch.nn.Conv1d layout, padding (K-1)/2 at each utterance's ends).
    BASELINE.json configs[3]'s Conv1d encoder (csrc/conv.hip); bf16 operands, fp32 accumulate."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        x, w = _need(x, "conv1d x"), _need(w, "conv1d weight")
        b = _need(b, "conv1d bias") if b is not None else None
        if x.dim() != 3:
            raise ValueError("conv1d: x must be [B, T, C]")
        if _prec() != 1:
            raise RuntimeError("the Conv1d encoder kernels use bf16 operands: set precision bf16")
        B, T, Cin = x.shape
        Cout, _, K = w.shape
        y = torch.empty(B, T, Cout, device=x.device, dtype=torch.float32)
        check(lib().mlvae_conv1d_fwd(B, T, Cin, Cout, K, _p(x), Cin, _p(w), _p(b) if b is not None else None,
                                     1 if act else 0, _p(y), Cout, _stream()), "conv1d_fwd")
        ctx.save_for_backward(x, w, y)
        ctx.act, ctx.has_b = act, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = _need(dy, "conv1d grad")
        B, T, Cin = x.shape
        Cout, _, K = w.shape
        if ctx.act:  # dpre = dy * lrelu'(y)
            dpre = torch.empty_like(dy)
            check(lib().mlvae_lrelu_bwd(dy.numel(), _p(dy), _p(y), _p(dpre), _stream()), "lrelu_bwd")
        else:
            dpre = dy
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            check(lib().mlvae_conv1d_dgrad(B, T, Cin, Cout, K, _p(dpre), Cout, _p(w), None, 0, _p(dx), Cin,
                                           _stream()), "conv1d_dgrad")
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            dw = torch.empty_like(w)
            db = torch.empty(Cout, device=dy.device, dtype=torch.float32)
            nb = lib().mlvae_conv1d_wgrad_workspace_size(B, T, Cin, Cout, K)
            ws = _conv_ws(nb)
            check(lib().mlvae_conv1d_wgrad(B, T, Cin, Cout, K, _p(dpre), Cout, _p(x), Cin, _p(dw), _p(db),
                                           _p(ws), ws.numel() * ws.element_size(), _stream()), "conv1d_wgrad")
            if not ctx.has_b:
                db = None
        return dx, dw, db, None


def conv1d(x, w, b=None, act=False):
    return Conv1dFn.apply(x, w, b, act)


# --------------------------------------------------------------------------- ELBO part 1
class ReparamKLFn(torch.autograd.Function):
    """z = eps*exp(lv/2) + mu and per-element KL (ref:src/modules/vanilla_vae.py:37-45);
    ml = [mu | log_var] along the last dim."""

    @staticmethod
    def forward(ctx, ml, eps):
        ml, eps = _need(ml, "ml"), _need(eps, "eps")
        Z = ml.shape[-1] // 2
        N = _rows(ml)
        z = torch.empty(*ml.shape[:-1], Z, device=ml.device, dtype=torch.float32)
        kl = torch.empty_like(z)
        # rows are independent: pass them as B=N utterances of T=1 frame (mask all-valid)
        ones = _ones(N)
        check(lib().mlvae_reparam_kl_fwd(N, 1, Z, _p(ml), 2 * Z, _p(eps), _p(ones), _p(z), _p(kl),
                                         None, _stream()), "reparam_kl_fwd")
        ctx.save_for_backward(ml, eps)
        return z, kl

    @staticmethod
    def backward(ctx, dz, dkl):
        ml, eps = ctx.saved_tensors
        Z = ml.shape[-1] // 2
        N = _rows(ml)
        dz = _need(dz, "dz") if dz is not None else torch.zeros(*ml.shape[:-1], Z, device=ml.device)
        dkl = _need(dkl, "dkl") if dkl is not None else torch.zeros_like(dz)
        dml = torch.empty_like(ml)
        check(lib().mlvae_reparam_kl_bwd(N, 1, Z, _p(ml), 2 * Z, _p(eps), _p(_ones(N)), None,
                                         _p(dz), _p(dkl), 0.0, _p(dml), 2 * Z, _stream()),
              "reparam_kl_bwd")
        return dml, None


def _ones(n):
    dev = torch.cuda.current_device()
    o = _ws.get((dev, "ones"))
    if o is None or o.numel() < n:
        o = torch.ones(max(n, 1024), device="cuda", dtype=torch.float32)
        _ws[(dev, "ones")] = o
    return o


def randn(shape, generator=None):
    """N(0,1) from the library's Philox stream; the seed is drawn from torch's (CPU) RNG so
    torch.manual_seed (ref:src/config/run.yaml:2-3) makes it reproducible."""
    seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator).item())
    out = torch.empty(*shape, device="cuda", dtype=torch.float32)
    check(lib().mlvae_randn(out.numel(), seed, 0, _p(out), _stream()), "randn")
    return out


# --------------------------------------------------------------------------- ELBO part 2
LOSS = {"likelihood": 0, "mse": 1}


class ReconFn(torch.autograd.Function):
    """Per-element reconstruction loss (ref:src/modules/decoder.py:37-53)."""

    @staticmethod
    def forward(ctx, mux, lvx, x, loss_type):
        mux, x = _need(mux, "mean"), _need(x, "target")
        lt = LOSS[loss_type]
        lvx = _need(lvx, "log_var") if lt == 0 else mux
        F = mux.shape[-1]
        N = _rows(mux)
        rec = torch.empty_like(mux)
        check(lib().mlvae_recon(N, 1, F, lt, _p(mux), F, _p(lvx), F, _p(x), F, _p(_ones(N)), None,
                                _p(rec), None, None, 0.0, None, None, _stream()), "recon")
        ctx.save_for_backward(mux, lvx, x)
        ctx.lt = lt
        return rec

    @staticmethod
    def backward(ctx, drec):
        mux, lvx, x = ctx.saved_tensors
        drec = _need(drec, "recon grad")
        F, N = mux.shape[-1], _rows(mux)
        dmux = torch.empty_like(mux)
        dlvx = torch.empty_like(mux) if ctx.lt == 0 else None
        check(lib().mlvae_recon(N, 1, F, ctx.lt, _p(mux), F, _p(lvx), F, _p(x), F, _p(_ones(N)),
                                None, None, None, _p(drec), 0.0, _p(dmux),
                                _p(dlvx) if dlvx is not None else None, _stream()), "recon_bwd")
        return dmux, dlvx, None, None


def recon_loss(mean, log_var, target, loss_type):
    if loss_type not in LOSS:
        raise ValueError(f"Invalid loss type: {loss_type}")  # ref:src/modules/decoder.py:50-51
    return ReconFn.apply(mean, log_var if loss_type == "likelihood" else mean, target, loss_type)


# --------------------------------------------------------------------------- masked mean
RED = {"mean": 0, "batchmean": 1, "batch": 2}


class MaskedMeanFn(torch.autograd.Function):
    """apply_lens_to_loss (ref:src/utils/data_utils.py:67-104)."""

    @staticmethod
    def forward(ctx, loss, lens, reduction):
        loss = _need(loss, "loss")
        lens = _need(lens.to(loss.device, torch.float32), "lens")
        B, T = loss.shape[0], loss.shape[1]
        C = loss.numel() // (B * T) if B * T else 1
        out = torch.empty(2 * B if B else 2, device=loss.device, dtype=torch.float32)
        check(lib().mlvae_masked_mean(B, T, C, _p(loss), _p(lens), RED[reduction], _p(out),
                                      _stream()), "masked_mean")
        ctx.save_for_backward(lens)
        ctx.shape, ctx.red = loss.shape, RED[reduction]
        return out[:B].clone() if reduction == "batch" else out[0].clone()

    @staticmethod
    def backward(ctx, g):
        (lens,) = ctx.saved_tensors
        B, T = ctx.shape[0], ctx.shape[1]
        C = 1
        for d in ctx.shape[2:]:
            C *= d
        g = _need(g.reshape(-1), "grad")
        dloss = torch.empty(ctx.shape, device=g.device, dtype=torch.float32)
        check(lib().mlvae_masked_mean_bwd(B, T, C, _p(lens), ctx.red, _p(g), _p(dloss), _stream()),
              "masked_mean_bwd")
        return dloss, None, None


def masked_mean(loss, lens, reduction="mean"):
    if reduction not in RED:
        raise ValueError(f"unknown reduction {reduction}")
    return MaskedMeanFn.apply(loss, lens, reduction)


# --------------------------------------------------------------------------- BiLSTM
def _lstm_ws(B, H):
    xb = SZ()
    check(lib().mlvae_lstm_workspace_size(B, H, _prec(), ctypes.byref(xb)), "lstm_workspace_size")
    x = _workspace(xb.value, "lstm_x")
    err = _ws.get((torch.cuda.current_device(), "lstm_err"))
    if err is None:
        err = torch.zeros(1, device="cuda", dtype=torch.int32)
        _ws[(torch.cuda.current_device(), "lstm_err")] = err
    return x, err


def _dropout(src, dst, seed, p):
    check(lib().mlvae_dropout(src.numel(), _p(src), _p(dst), None, seed, p, _stream()), "dropout")


class LSTMFn(torch.autograd.Function):
    """nn.LSTM(batch_first=True) on libmlvae, bidirectional (ndir 2: ref:src/modules/decoder.py:14-15,22)
    or not (ndir 1: ref:src/modules/phoneme_recognizer.py:13, boundary_detector.py:19): per layer
    an input-projection GEMM per direction + the persistent recurrence; inter-layer dropout
    (Philox, recomputed in backward) in train mode.  weights = the layer-major list
    [w_ih, w_hh, b_ih, b_hh] (+ [w_ih_r, w_hh_r, b_ih_r, b_hh_r] when bidirectional) * L."""

    @staticmethod
    def forward(ctx, x, H, L, ndir, dropout, seed, *weights):
        x = _need(x, "lstm input")
        B, T, _ = x.shape
        N = B * T
        l = lib()
        xbuf, err = _lstm_ws(B, H)
        nw = 4 * ndir
        saved, inputs, seeds = [], [], []
        h = x
        for li in range(L):
            w = [_need(t, "lstm weight") for t in weights[nw * li:nw * li + nw]]
            din = h.shape[-1]
            G = torch.empty(N, 4 * H * ndir, device=x.device, dtype=torch.float32)
            for d in range(ndir):
                wi, _, bi, bh = w[4 * d:4 * d + 4]
                gemm(0, 1, N, 4 * H, din, _p(h), din, _p(wi), din, _p(G, 4 * H * d), 4 * H * ndir,
                     bias1=_p(bi), bias2=_p(bh))
            Cs = torch.empty(N, H * ndir, device=x.device, dtype=torch.float32)
            Y = torch.empty(B, T, H * ndir, device=x.device, dtype=torch.float32)
            if ndir == 2:
                check(l.mlvae_lstm_fwd(_prec(), B, T, H, _p(w[1]), _p(w[5]), _p(G), _p(Cs), _p(Y),
                                       _p(xbuf), xbuf.numel() * 4, _p(err), _stream()), "lstm_fwd")
            else:
                check(l.mlvae_lstm1_fwd(_prec(), B, T, H, _p(w[1]), _p(G), _p(Cs), _p(Y), None,
                                        _p(xbuf), xbuf.numel() * 4, _p(err), _stream()), "lstm1_fwd")
            inputs.append(h)
            saved += [G, Cs, Y]
            h = Y
            if li < L - 1 and dropout > 0:
                s = (seed * 1000003 + li) & ((1 << 63) - 1)
                hd = torch.empty_like(Y)
                _dropout(Y, hd, s, dropout)
                seeds.append(s)
                h = hd
            else:
                seeds.append(None)
        ctx.save_for_backward(*inputs, *saved, *weights)
        ctx.H, ctx.L, ctx.ndir, ctx.dropout, ctx.seeds = H, L, ndir, dropout, seeds
        # nn.LSTM's (h_n, c_n) [L*ndir, B, H]: every layer's state after its last step (t = T-1
        # forward, t = 0 reverse; no packing, as nn.LSTM on a padded batch)
        hn = torch.empty(L * ndir, B, H, device=x.device, dtype=torch.float32)
        cn = torch.empty_like(hn)
        for li in range(L):
            G_, Cs_, Y_ = saved[3 * li:3 * li + 3]
            Cv = Cs_.view(B, T, H * ndir)
            for d in range(ndir):
                t_last = 0 if d else T - 1
                hn[li * ndir + d] = Y_[:, t_last, d * H:(d + 1) * H]
                cn[li * ndir + d] = Cv[:, t_last, d * H:(d + 1) * H]
        # h_n is differentiable (its gradient joins the layer output's at the last step); c_n's
        # gradient would need an initial cell gradient the BPTT kernels do not take: refused
        # loudly in backward.  Unused outputs arrive as None (no materialised zero tensors).
        ctx.set_materialize_grads(False)
        ctx.out_shape = h.shape
        return h, hn, cn

    @staticmethod
    def backward(ctx, dy, dhn=None, dcn=None):
        H, L, ndir = ctx.H, ctx.L, ctx.ndir
        nw, GL = 4 * ndir, 4 * H * ndir
        t = ctx.saved_tensors
        inputs, saved, weights = t[:L], t[L:4 * L], t[4 * L:]
        if dcn is not None and bool(dcn.ne(0).any()):
            raise NotImplementedError("gradient through c_n of the HIP LSTM is not supported "
                                      "(the BPTT starts from a zero cell gradient)")
        if dy is None:
            dy = torch.zeros(ctx.out_shape, device=t[0].device, dtype=torch.float32)
        dy = _need(dy, "lstm grad").clone()
        B, T = dy.shape[0], dy.shape[1]
        N = B * T
        l = lib()
        xbuf, err = _lstm_ws(B, H)
        dW = [None] * len(weights)
        dx = None
        for li in range(L - 1, -1, -1):
            G, Cs, Y = saved[3 * li:3 * li + 3]
            w = weights[nw * li:nw * li + nw]
            xin = inputs[li]
            din = xin.shape[-1]
            if dhn is not None:  # h_n[li, d] is Y_li at t = T-1 (forward) / t = 0 (reverse)
                for d in range(ndir):
                    dy[:, 0 if d else T - 1, d * H:(d + 1) * H] += dhn[li * ndir + d]
            if ndir == 2:
                check(l.mlvae_lstm_bwd(_prec(), B, T, H, _p(w[1]), _p(w[5]), _p(G), _p(Cs), _p(dy),
                                       _p(xbuf), xbuf.numel() * 4, _p(err), _stream()), "lstm_bwd")
            else:
                check(l.mlvae_lstm1_bwd(_prec(), B, T, H, _p(w[1]), _p(G), _p(Cs), _p(dy), None,
                                        _p(xbuf), xbuf.numel() * 4, _p(err), _stream()), "lstm1_bwd")
            dx = torch.empty(B, T, din, device=dy.device, dtype=torch.float32)
            for d in range(ndir):
                wi = w[4 * d]
                gemm(0, 0, N, din, 4 * H, _p(G, 4 * H * d), GL, _p(wi), din, _p(dx), din,
                     beta=1.0 if d else 0.0)
                gwi = torch.empty_like(wi)
                gemm(1, 0, 4 * H, din, N, _p(G, 4 * H * d), GL, _p(xin), din, _p(gwi), din)
                gwh = torch.empty_like(w[4 * d + 1])
                # dW_hh = sum_t dG_t^T h_{t-1} (forward) / h_{t+1} (reverse): time-shifted B rows
                gemm(1, 0, 4 * H, H, N, _p(G, 4 * H * d), GL, _p(Y, H * d), H * ndir, _p(gwh), H,
                     kshift_T=T, kshift=1 if d else -1)
                gbi = torch.empty_like(w[4 * d + 2])
                gbh = torch.empty_like(w[4 * d + 3])
                colsum(N, 4 * H, _p(G, 4 * H * d), GL, _p(gbi), _p(gbh))
                base = nw * li + 4 * d
                dW[base:base + 4] = [gwi, gwh, gbi, gbh]
            if li > 0 and ctx.seeds[li - 1] is not None:
                _dropout(dx, dx, ctx.seeds[li - 1], ctx.dropout)
            dy = dx
        if int(err.item()) != 0:
            raise RuntimeError("LSTM recurrence hand-off timed out")
        return (dx, None, None, None, None, None, *dW)


def lstm(x, lstm_module, train):
    """Run an nn.LSTM's parameters (batch_first, uni- or bidirectional) through the HIP
    recurrence; its own forward is not used."""
    if not lstm_module.batch_first:
        raise ValueError("the HIP LSTM path is batch_first only (as every reference LSTM)")
    H, L = lstm_module.hidden_size, lstm_module.num_layers
    ndir = 2 if lstm_module.bidirectional else 1
    weights = []
    for li in range(L):
        for sfx in ("", "_reverse")[:ndir]:
            for kind in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                weights.append(getattr(lstm_module, f"{kind}_l{li}{sfx}"))
    p = float(lstm_module.dropout) if train else 0.0
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
    return LSTMFn.apply(x, H, L, ndir, p, seed, *weights)[0]


def lstm_full(x, lstm_module, train, seed=None):
    """nn.LSTM's whole forward on the HIP recurrence: (output, (h_n, c_n)).  seed: the
    inter-layer dropout's Philox key (drawn from torch's generator when None)."""
    if not lstm_module.batch_first:
        raise ValueError("the HIP LSTM path is batch_first only (as every reference LSTM)")
    H, L = lstm_module.hidden_size, lstm_module.num_layers
    ndir = 2 if lstm_module.bidirectional else 1
    weights = [getattr(lstm_module, f"{kind}_l{li}{sfx}") for li in range(L)
               for sfx in ("", "_reverse")[:ndir] for kind in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    p = float(lstm_module.dropout) if train else 0.0
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
    out, hn, cn = LSTMFn.apply(x, H, L, ndir, p, seed, *weights)
    return out, (hn, cn)


def bilstm(x, lstm_module, train):
    """The decoder's bidirectional nn.LSTM (ref:src/modules/decoder.py:22)."""
    return lstm(x, lstm_module, train)


# --------------------------------------------------------------------------- MD-VAE upstream losses
def _md_err():
    dev = torch.cuda.current_device()
    e = _ws.get((dev, "md_err"))
    if e is None:
        e = torch.zeros(1, device="cuda", dtype=torch.int32)
        _ws[(dev, "md_err")] = e
    return e


def _raise_md(err):
    code = int(err.item())
    if code:
        err.zero_()
        raise AssertionError(
            "phoneme-recogniser targets: " +
            ("boundaries do not give one segment per phoneme from frame 0 " if code & 2 else "") +
            ("phoneme id outside [0, n_phonemes + 2)" if code & 4 else "") +
            " (ref:src/modules/phoneme_recognizer.py:65-67)")


class PhnBceFn(torch.autograd.Function):
    """PhonemeRecognizer.compute_losses on libmlvae (ref:src/modules/phoneme_recognizer.py:35-81):
    [B,T,C] BCE-with-logits against the boundary-expanded canonical phoneme sequence."""

    @staticmethod
    def forward(ctx, out, feat_lens, phn, phn_lens, boundary):
        out = _need(out, "recogniser output")
        B, T, C = out.shape
        fl = _need(feat_lens.to(out.device, torch.float32), "feat_lens")
        pl = _need(phn_lens.to(out.device, torch.float32), "phn_lens")
        bnd = _need(boundary.to(out.device, torch.float32), "boundary_seqs")
        ids = phn.to(out.device, torch.int64).contiguous()
        loss = torch.empty_like(out)
        err = _md_err()
        check(lib().mlvae_phn_bce(B, T, C, _p(out), C, _p(fl), ids.data_ptr(), ids.shape[1], _p(pl),
                                  _p(bnd), _p(loss), None, None, _p(err), _stream()), "phn_bce")
        _raise_md(err)  # the reference asserts on the host too (one sync per batch, not per utterance)
        ctx.save_for_backward(out, fl, ids, pl, bnd)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        out, fl, ids, pl, bnd = ctx.saved_tensors
        B, T, C = out.shape
        dloss = _need(dloss, "grad")
        dout = torch.empty_like(out)
        err = _md_err()
        check(lib().mlvae_phn_bce(B, T, C, _p(out), C, _p(fl), ids.data_ptr(), ids.shape[1], _p(pl),
                                  _p(bnd), None, _p(dloss), _p(dout), _p(err), _stream()), "phn_bce_bwd")
        return dout, None, None, None, None


def phn_bce(out, feat_lens, phn, phn_lens, boundary):
    return PhnBceFn.apply(out, feat_lens, phn, phn_lens, boundary)


class BoundaryHeadsFn(torch.autograd.Function):
    """BoundaryDetector after its FC heads (ref:src/modules/boundary_detector.py:42-97): Softplus
    + 1e-5, Beta(1, 9) KL, ten Kumaraswamy draws; returns (boundary_v, bce, kld).  u = the ten
    U(0,1) draws [10, B, T] (None: Philox keyed by seed and element index)."""

    @staticmethod
    def forward(ctx, za, zb, y, u, seed):
        za, zb = _need(za, "alpha head"), _need(zb, "beta head")
        y = _need(y.to(za.device, torch.float32), "boundary_seqs")
        u = _need(u, "uniforms") if u is not None else None
        v, bce, kld = torch.empty_like(za), torch.empty_like(za), torch.empty_like(za)
        check(lib().mlvae_boundary_fwd(za.numel(), _p(za), _p(zb), _p(y), _p(u) if u is not None else None,
                                       seed, 0, _p(v), _p(bce), _p(kld), _stream()), "boundary_fwd")
        ctx.save_for_backward(za, zb, y, *([u] if u is not None else []))
        ctx.seed, ctx.has_u = seed, u is not None
        return v, bce, kld

    @staticmethod
    def backward(ctx, dv, dbce, dkld):
        t = ctx.saved_tensors
        za, zb, y = t[:3]
        u = t[3] if ctx.has_u else None
        grads = [None if g is None else _need(g, "grad") for g in (dv, dbce, dkld)]
        dza, dzb = torch.empty_like(za), torch.empty_like(zb)
        check(lib().mlvae_boundary_bwd(za.numel(), _p(za), _p(zb), _p(y), _p(u) if u is not None else None,
                                       ctx.seed, 0, *[(_p(g) if g is not None else None) for g in grads],
                                       _p(dza), _p(dzb), _stream()), "boundary_bwd")
        return dza, dzb, None, None, None


def boundary_heads(za, zb, boundary, u=None):
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if u is None else 0
    return BoundaryHeadsFn.apply(za, zb, boundary, u, seed)


# --------------------------------------------------------------------------- GMM-VAE / H-VAE
class GmmLatentFn(torch.autograd.Function):
    """GMM-VAE latent block on the stacked head output P = [pm | plv | m | lv | logits]
    (ref:src/modules/gmm_vae.py:24-67): returns z, per-element KL and the straight-through
    hard Gumbel-softmax weights.  expo = the Exp(1) draws [.., N] (None: library Philox)."""

    @staticmethod
    def forward(ctx, P, eps, expo, N, Z, tau, seed):
        P, eps = _need(P, "gmm heads"), _need(eps, "eps")
        expo = _need(expo, "expo") if expo is not None else None
        rows = _rows(P)
        z = torch.empty(*P.shape[:-1], N * Z, device=P.device, dtype=torch.float32)
        kl = torch.empty_like(z)
        w = torch.empty(*P.shape[:-1], N, device=P.device, dtype=torch.float32)
        ysoft = torch.empty_like(w)
        check(lib().mlvae_gmm_latent_fwd(rows, N, Z, _p(P), P.shape[-1], _p(eps),
                                         _p(expo) if expo is not None else None, seed, 0, tau,
                                         _p(z), _p(kl), _p(w), _p(ysoft), _stream()),
              "gmm_latent_fwd")
        ctx.save_for_backward(P, eps, ysoft)
        ctx.shape = (N, Z, tau)
        return z, kl, w

    @staticmethod
    def backward(ctx, dz, dkl, dw):
        P, eps, ysoft = ctx.saved_tensors
        N, Z, tau = ctx.shape
        opt = lambda t, n: _need(t, n) if t is not None else None
        dz, dkl, dw = opt(dz, "dz"), opt(dkl, "dkl"), opt(dw, "dw")
        dP = torch.empty_like(P)
        nz = lambda t: _p(t) if t is not None else None
        check(lib().mlvae_gmm_latent_bwd(_rows(P), N, Z, _p(P), P.shape[-1], _p(eps), _p(ysoft),
                                         tau, nz(dz), nz(dkl), nz(dw), _p(dP), P.shape[-1],
                                         _stream()), "gmm_latent_bwd")
        return dP, None, None, None, None, None, None


class ApplyWeightFn(torch.autograd.Function):
    """y[.., c] = sum_n w[.., n] x[.., n*C + c] (ref:src/utils/data_utils.py:32-64)."""

    @staticmethod
    def forward(ctx, x, w):
        x, w = _need(x, "apply_weight x"), _need(w, "apply_weight weight")
        N = w.shape[-1]
        C = x.shape[-1] // N
        rows = _rows(w)
        if x.numel() != rows * N * C:
            raise ValueError(f"apply_weight: x {tuple(x.shape)} does not match weight {tuple(w.shape)}")
        y = torch.empty(*w.shape[:-1], C, device=x.device, dtype=torch.float32)
        check(lib().mlvae_apply_weight_fwd(rows, N, C, _p(x), N * C, _p(w), _p(y), C, _stream()),
              "apply_weight_fwd")
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = _need(dy, "apply_weight grad")
        N = w.shape[-1]
        C = x.shape[-1] // N
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        check(lib().mlvae_apply_weight_bwd(_rows(w), N, C, _p(x), N * C, _p(w), _p(dy), C,
                                           _p(dx) if dx is not None else None, N * C,
                                           _p(dw) if dw is not None else None, _stream()),
              "apply_weight_bwd")
        return dx, dw


def apply_weight(x, weight):
    """(B,T,N*C) or (B,T,N,C) weighted by (B,T,N) -> (B,T,C)."""
    B, T, N = weight.shape
    return ApplyWeightFn.apply(x.reshape(B, T, -1), weight)
