"""CPU restatement of the GMM-VAE and Hierarchical-VAE encoders.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product path.
Pinned by tests/test_oracle_hvae_golden.py against fixtures made from the reference modules
(tests/golden/make_golden_hvae.py).  Randomness is explicit: eps for the reparameterisation
and Exp(1) samples for the Gumbel draw (gumbels = -log(E), as torch's F.gumbel_softmax).

Parameters are a dict keyed by the reference's own parameter names.
"""
import torch
import torch.nn.functional as Fn

TAU = 0.1  # ref:src/modules/gmm_vae.py:31


def _lin(p, name, x):
    return x @ p[name + ".weight"].t() + p[name + ".bias"]


def fc_trunk(p, prefix, x):
    """Sequential(FCBlock([F,E,E]), LeakyReLU): ref:src/modules/gmm_vae.py:12-15,
    ref:src/modules/fc_block.py:4-21 (LeakyReLU(0.01) between layers, none at the end)."""
    h = Fn.leaky_relu(_lin(p, prefix + "fc.0.blocks.0", x), 0.01)
    h = _lin(p, prefix + "fc.0.blocks.2", h)
    return Fn.leaky_relu(h, 0.01)


def gumbel_softmax_hard(logits, expo, tau=TAU):
    """F.gumbel_softmax(logits, tau, hard=True) with the Exp(1) draw given
    (straight-through: y_hard - y_soft.detach() + y_soft)."""
    gumbels = -expo.log()
    y_soft = ((logits + gumbels) / tau).softmax(-1)
    index = y_soft.max(-1, keepdim=True)[1]
    y_hard = torch.zeros_like(logits).scatter_(-1, index, 1.0)
    return y_hard - y_soft.detach() + y_soft


def gmm_kld(prior_mean, prior_log_var, mean, log_var):
    """ref:src/modules/gmm_vae.py:58-67 (eps 1e-5 on the prior variance)."""
    return -0.5 * (1 + log_var - prior_log_var
                   - (log_var.exp() + (mean - prior_mean) ** 2) / (prior_log_var.exp() + 1e-5))


def gmm_vae_forward(p, x, eps, expo, prefix=""):
    """GMMVAE.forward, ref:src/modules/gmm_vae.py:24-48."""
    h = fc_trunk(p, prefix, x)
    pm = _lin(p, prefix + "prior_mean_fc", h)
    plv = _lin(p, prefix + "prior_log_var_fc", h)
    m = _lin(p, prefix + "mean_fc", h)
    lv = _lin(p, prefix + "log_var_fc", h)
    w = gumbel_softmax_hard(_lin(p, prefix + "gmm_weight_fc", h), expo)
    z = eps * torch.exp(0.5 * lv) + m  # ref:src/modules/gmm_vae.py:50-55
    return {"prior_mean": pm, "prior_log_var": plv, "mean": m, "log_var": lv, "sampled_h": z,
            "gmm_weight": w, "loss": gmm_kld(pm, plv, m, lv)}


def vanilla_forward(p, x, eps, prefix=""):
    """VanillaVAE.forward, ref:src/modules/vanilla_vae.py:24-45."""
    h = fc_trunk(p, prefix, x)
    m = _lin(p, prefix + "mean_fc", h)
    lv = _lin(p, prefix + "log_var_fc", h)
    z = eps * torch.exp(0.5 * lv) + m
    kl = -0.5 * (1 + lv - m ** 2 - lv.exp())
    return {"mean": m, "log_var": lv, "sampled_h": z, "loss": kl}


def apply_weight(x, w):
    """ref:src/utils/data_utils.py:32-64: sum_n w[..., n] * x[..., n, :] ((B,T,N*C) or (B,T,N,C))."""
    B, T, N = w.shape
    x = x.reshape(B, T, N, -1)
    return (w.unsqueeze(-1) * x).sum(2)


def hvae_forward(p, x, pi, eps_v, eps_g, expo):
    """HierarchicalVAE.forward, ref:src/modules/h_vae.py:22-72."""
    v = vanilla_forward(p, x, eps_v, "vanilla_vae.")
    g = gmm_vae_forward(p, x, eps_g, expo, "gmm_vae.")
    w = g["gmm_weight"]
    pair = {k: torch.stack([v[k], apply_weight(g[k], w)], 2)
            for k in ("mean", "log_var", "sampled_h", "loss")}
    out = {k: apply_weight(pair[k], pi) for k in ("mean", "log_var", "sampled_h")}
    return {"gmm_weight": w, **out, "vae_kld_loss": apply_weight(pair["loss"], pi)}
