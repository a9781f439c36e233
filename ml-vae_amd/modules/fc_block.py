"""FCBlock on the HIP GEMM (replaces ref:src/modules/fc_block.py:4-21).

Layer layout matches the reference so state_dict keys line up: ``blocks`` is an
nn.Sequential of Linear / LeakyReLU(0.01) pairs, the last Linear without activation unless
``end_activation``.  ``dropout`` is accepted and unused, as in the reference (fc_block.py:5).
The LeakyReLU of each pair is fused into the GEMM epilogue.
"""
from torch import nn

from mlvae_hip import ops


class FCBlock(nn.Module):
    def __init__(self, fc_sizes, dropout=0.15, end_activation=False):
        super().__init__()
        sizes = list(fc_sizes)
        if len(sizes) < 2:
            raise ValueError("FCBlock needs at least an input and an output size")
        layers = []
        n_lin = len(sizes) - 1
        for i, (fan_in, fan_out) in enumerate(zip(sizes[:-1], sizes[1:])):
            layers.append(nn.Linear(fan_in, fan_out))
            if i < n_lin - 1 or end_activation:
                layers.append(nn.LeakyReLU())
        self.blocks = nn.Sequential(*layers)
        self.dropout = dropout
        self.end_activation = end_activation

    def linear_plan(self):
        """[(nn.Linear, fused_leaky_relu)] in order."""
        mods = list(self.blocks)
        plan = []
        for i, m in enumerate(mods):
            if isinstance(m, nn.Linear):
                act = i + 1 < len(mods) and isinstance(mods[i + 1], nn.LeakyReLU)
                plan.append((m, act))
        return plan

    def forward(self, x):
        for lin, act in self.linear_plan():
            x = ops.linear(x, lin.weight, lin.bias, act)
        return x
