"""HierarchicalVAE on libmlvae (replaces ref:src/modules/h_vae.py:12-72).

A VanillaVAE (correct pronunciation) and a GMMVAE (mispronunciation) read the same frames; the
GMM outputs are collapsed over components with their hard mixture weights, both branches are
stacked on a new axis and mixed by pi (B, T, 2).  Every weighting is the apply_weight kernel.
"""
import torch
from torch import nn

from modules.gmm_vae import GMMVAE
from modules.vanilla_vae import VanillaVAE
from utils.data_utils import apply_weight


class HierarchicalVAE(nn.Module):
    def __init__(self, fc_sizes, latent_size, num_components):
        super().__init__()
        self.vanilla_vae = VanillaVAE(fc_sizes, latent_size)
        self.gmm_vae = GMMVAE(fc_sizes, latent_size, num_components)

    def forward(self, feats, pi, eps_v=None, eps_g=None, expo=None):
        v = self.vanilla_vae(feats, eps=eps_v)
        g = self.gmm_vae(feats, eps=eps_g, expo=expo)
        w = g["gmm_weight"]  # (B, T, N)
        out = {}
        for key in ("mean", "log_var", "sampled_h", "loss"):
            pair = torch.stack([v[key], apply_weight(g[key], w)], dim=2)  # (B, T, 2, C)
            out[key] = apply_weight(pair, pi)  # (B, T, C)
        return {
            "gmm_weight": w,
            "mean": out["mean"],
            "log_var": out["log_var"],
            "sampled_h": out["sampled_h"],
            "losses": {"vae_kld_loss": out["loss"]},
        }
