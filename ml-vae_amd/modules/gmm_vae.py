"""GMMVAE encoder on libmlvae (replaces ref:src/modules/gmm_vae.py:8-67).

fc = Sequential(FCBlock(fc_sizes), LeakyReLU); the five heads (prior_mean_fc, prior_log_var_fc,
mean_fc, log_var_fc, gmm_weight_fc) run as ONE stacked GEMM whose output rows are
[prior_mean | prior_log_var | mean | log_var | gmm logits]; one fused kernel then draws the hard
Gumbel-softmax mixture weights (tau 0.1, straight-through), reparameterises every component and
evaluates the per-element GMM KL.  eps and the Gumbel draws come from the library's Philox
stream seeded from torch's RNG; tests inject them (eps=, expo=) to replay the reference.
"""
import torch
from torch import nn

from mlvae_hip import ops
from modules.fc_block import FCBlock

TAU = 0.1  # ref:src/modules/gmm_vae.py:31


class GMMVAE(nn.Module):
    def __init__(self, fc_sizes, latent_size, num_components):
        super().__init__()
        self.fc = nn.Sequential(FCBlock(fc_sizes), nn.LeakyReLU())
        E, NZ = fc_sizes[-1], latent_size * num_components
        self.prior_mean_fc = nn.Linear(E, NZ)
        self.prior_log_var_fc = nn.Linear(E, NZ)
        self.mean_fc = nn.Linear(E, NZ)
        self.log_var_fc = nn.Linear(E, NZ)
        self.gmm_weight_fc = nn.Linear(E, num_components)
        self.latent_size, self.num_components = latent_size, num_components

    def _heads(self):
        return (self.prior_mean_fc, self.prior_log_var_fc, self.mean_fc, self.log_var_fc,
                self.gmm_weight_fc)

    def forward(self, feats, eps=None, expo=None):  # feats (B, T, C)
        h = feats
        plan = self.fc[0].linear_plan()
        for i, (lin, act) in enumerate(plan):
            h = ops.linear(h, lin.weight, lin.bias, act or i == len(plan) - 1)
        heads = self._heads()
        W = torch.cat([m.weight for m in heads], 0)
        b = torch.cat([m.bias for m in heads], 0)
        P = ops.linear(h, W, b)  # (B, T, 4NZ + N)
        N, Z = self.num_components, self.latent_size
        NZ = N * Z
        if eps is None:
            eps = ops.randn(P.shape[:-1] + (NZ,))
        seed = 0 if expo is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
        z, kl, w = ops.GmmLatentFn.apply(P, eps, expo, N, Z, TAU, seed)
        return {
            "prior_mean": P[..., :NZ],
            "prior_log_var": P[..., NZ:2 * NZ],
            "mean": P[..., 2 * NZ:3 * NZ],
            "log_var": P[..., 3 * NZ:4 * NZ],
            "sampled_h": z,
            "gmm_weight": w,
            "loss": kl,
        }
