"""Conv1d variant of the VanillaVAE encoder (BASELINE.json configs[3]: "Conv1d encoder variant,
long utterances T=2000, B=64").

The reference has no Conv1d anywhere; this module is VanillaVAE
(ref:src/modules/vanilla_vae.py:9-45) with its FCBlock (ref:src/modules/fc_block.py:4-21)
replaced by a stack of temporal convolutions, everything else identical:

  conv = Seq(ConvBlock([F, E, E], K), LeakyReLU)   Conv1d(F, E, K) LReLU Conv1d(E, E, K), LReLU
  mean_fc / log_var_fc = Linear(E, Z)              per frame
  z = eps * exp(log_var / 2) + mean; KL -0.5 (1 + log_var - mean^2 - exp(log_var))

Each Conv1d runs over the time axis of the batch-first frames [B, T, C] with padding (K-1)/2
(torch.nn.Conv1d on the [B, C, T] transpose): csrc/conv.hip through ops.conv1d.  Parameter
names: ``conv.0.blocks.{0,2}.weight`` [E, Cin, K] / ``.bias``, ``mean_fc.*``, ``log_var_fc.*``;
the fused engine (mlvae_hip/engine.py, ``VAEConfig.enc_conv``) uses the same names.
"""
from torch import nn

from mlvae_hip import ops
from modules.vanilla_vae import _mean_logvar


class ConvBlock(nn.Module):
    """Conv1d / LeakyReLU pairs over channel sizes, the last Conv1d without activation (the
    layout of FCBlock, ref:src/modules/fc_block.py:4-21)."""

    def __init__(self, channels, kernel_size=5):
        super().__init__()
        if kernel_size % 2 != 1:
            raise ValueError("kernel_size must be odd ('same' padding)")
        layers = []
        for i in range(len(channels) - 1):
            layers.append(nn.Conv1d(channels[i], channels[i + 1], kernel_size, padding=kernel_size // 2))
            if i < len(channels) - 2:
                layers.append(nn.LeakyReLU())
        self.blocks = nn.Sequential(*layers)

    def conv_plan(self):
        """[(nn.Conv1d, fused_leaky_relu)] in order."""
        mods = list(self.blocks)
        return [(m, i + 1 < len(mods) and isinstance(mods[i + 1], nn.LeakyReLU))
                for i, m in enumerate(mods) if isinstance(m, nn.Conv1d)]

    def forward(self, x):  # x [B, T, C]
        for conv, act in self.conv_plan():
            x = ops.conv1d(x, conv.weight, conv.bias, act)
        return x


class ConvVAE(nn.Module):
    def __init__(self, conv_sizes, latent_size, kernel_size=5):
        super().__init__()
        self.conv = nn.Sequential(ConvBlock(conv_sizes, kernel_size), nn.LeakyReLU())
        self.mean_fc = nn.Linear(conv_sizes[-1], latent_size)
        self.log_var_fc = nn.Linear(conv_sizes[-1], latent_size)
        self.latent_size = latent_size
        self.kernel_size = kernel_size

    def forward(self, feats, eps=None):  # feats (B, T, C)
        plan = self.conv[0].conv_plan()
        h = feats
        for i, (conv, act) in enumerate(plan):
            # the outer LeakyReLU (self.conv[1]) folds into the last layer's epilogue
            h = ops.conv1d(h, conv.weight, conv.bias, act or i == len(plan) - 1)
        ml = _mean_logvar(h, self.mean_fc, self.log_var_fc)
        if eps is None:
            eps = ops.randn(ml.shape[:-1] + (self.latent_size,))
        z, kl = ops.ReparamKLFn.apply(ml, eps)
        Z = self.latent_size
        return {"mean": ml[..., :Z], "log_var": ml[..., Z:], "sampled_h": z, "loss": kl}
