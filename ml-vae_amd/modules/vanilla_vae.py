"""VanillaVAE encoder on libmlvae (replaces ref:src/modules/vanilla_vae.py:9-45).

fc = Sequential(FCBlock(fc_sizes), LeakyReLU) -> mean_fc / log_var_fc (Linear) ->
reparameterise (z = eps * exp(log_var / 2) + mean) + per-element KL
-0.5 (1 + log_var - mean^2 - exp(log_var)), fused in one kernel.  eps is drawn from the
library's Philox stream seeded from torch's RNG, in eval mode too (as the reference).
"""
import torch
from torch import nn

from mlvae_hip import ops
from modules.fc_block import FCBlock


class VanillaVAE(nn.Module):
    def __init__(self, fc_sizes, latent_size):
        super().__init__()
        self.fc = nn.Sequential(FCBlock(fc_sizes), nn.LeakyReLU())
        self.mean_fc = nn.Linear(fc_sizes[-1], latent_size)
        self.log_var_fc = nn.Linear(fc_sizes[-1], latent_size)
        self.latent_size = latent_size

    def forward(self, feats, eps=None):  # feats (B, T, C)
        h = feats
        plan = self.fc[0].linear_plan()
        for i, (lin, act) in enumerate(plan):
            # the outer LeakyReLU (self.fc[1]) folds into the last FCBlock layer's epilogue
            h = ops.linear(h, lin.weight, lin.bias, act or i == len(plan) - 1)
        ml = _mean_logvar(h, self.mean_fc, self.log_var_fc)  # [.., 2Z] = [mean | log_var]
        if eps is None:
            eps = ops.randn(ml.shape[:-1] + (self.latent_size,))
        z, kl = ops.ReparamKLFn.apply(ml, eps)
        Z = self.latent_size
        return {"mean": ml[..., :Z], "log_var": ml[..., Z:], "sampled_h": z, "loss": kl}

    def reparameterize(self, mean, log_var, eps=None):
        ml = torch.cat([mean, log_var], -1)
        if eps is None:
            eps = ops.randn(mean.shape)
        return ops.ReparamKLFn.apply(ml, eps)[0]

    def compute_kld_loss(self, mean, log_var):
        ml = torch.cat([mean, log_var], -1)
        return ops.ReparamKLFn.apply(ml, torch.zeros_like(mean))[1]


class _MeanLogVar(torch.autograd.Function):
    """[mean | log_var] = h @ [Wm; Wv]^T + [bm; bv] as two GEMMs into one buffer."""

    @staticmethod
    def forward(ctx, h, wm, bm, wv, bv):
        h = ops._need(h, "encoder hidden")
        M, K = ops._rows(h), h.shape[-1]
        Z = wm.shape[0]
        ml = torch.empty(*h.shape[:-1], 2 * Z, device=h.device, dtype=torch.float32)
        ops.gemm(0, 1, M, Z, K, ops._p(h), K, ops._p(wm), K, ops._p(ml), 2 * Z, bias1=ops._p(bm))
        ops.gemm(0, 1, M, Z, K, ops._p(h), K, ops._p(wv), K, ops._p(ml, Z), 2 * Z, bias1=ops._p(bv))
        ctx.save_for_backward(h, wm, wv)
        return ml

    @staticmethod
    def backward(ctx, dml):
        h, wm, wv = ctx.saved_tensors
        dml = ops._need(dml, "grad")
        M, K, Z = ops._rows(h), h.shape[-1], wm.shape[0]
        dh = torch.empty_like(h)
        ops.gemm(0, 0, M, K, Z, ops._p(dml), 2 * Z, ops._p(wm), K, ops._p(dh), K)
        ops.gemm(0, 0, M, K, Z, ops._p(dml, Z), 2 * Z, ops._p(wv), K, ops._p(dh), K, beta=1.0)
        out = []
        for off, w in ((0, wm), (Z, wv)):
            dw = torch.empty_like(w)
            ops.gemm(1, 0, Z, K, M, ops._p(dml, off), 2 * Z, ops._p(h), K, ops._p(dw), K)
            db = torch.empty(Z, device=dml.device, dtype=torch.float32)
            ops.colsum(M, Z, ops._p(dml, off), 2 * Z, ops._p(db))
            out += [dw, db]
        return (dh, *out)


def _mean_logvar(h, mean_fc, log_var_fc):
    return _MeanLogVar.apply(h, mean_fc.weight, mean_fc.bias, log_var_fc.weight, log_var_fc.bias)
