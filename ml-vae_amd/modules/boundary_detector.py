"""BoundaryDetector on libmlvae (replaces ref:src/modules/boundary_detector.py:15-103).

rnn: a unidirectional nn.LSTM on the persistent HIP kernels (mlvae_hip.ops.LSTMFn).
fc_alpha / fc_beta: nn.Sequential(FCBlock, Softplus) as in the reference (same state_dict keys);
the Softplus, the +1e-5, the Beta(1, 9) KL and the ten Kumaraswamy draws with their BCE run in one
fused kernel over [B, T] (csrc/md.hip) on the FCBlock outputs.  The draws are Philox-keyed by
element index (the reference: torch.rand_like); ``forward(..., uniform_u=[10, B, T])`` injects
them instead (parity tests).
"""
import torch
from torch import nn

from mlvae_hip import ops
from modules.fc_block import FCBlock


class BoundaryDetector(nn.Module):
    def __init__(self, input_size, rnn_hidden_size, rnn_num_layers, fc_sizes):
        super().__init__()
        self.rnn = nn.LSTM(input_size, rnn_hidden_size, rnn_num_layers, batch_first=True)
        self.fc_alpha = nn.Sequential(FCBlock(fc_sizes), nn.Softplus())
        self.fc_beta = nn.Sequential(FCBlock(fc_sizes), nn.Softplus())

    def forward(self, x, feat_lens, boundary_seqs, uniform_u=None):
        rnn_out = ops.lstm(x, self.rnn, self.training)
        za = torch.squeeze(self.fc_alpha[0](rnn_out), dim=-1)  # pre-Softplus heads, (B, T)
        zb = torch.squeeze(self.fc_beta[0](rnn_out), dim=-1)
        v, bce, kld = ops.boundary_heads(za.contiguous(), zb.contiguous(), boundary_seqs, uniform_u)
        return {"boundary_v": v, "losses": {"boundary_bce_loss": bce, "boundary_kld_loss": kld}}

    def compute_kld_loss(self, alpha, beta):
        """KL(Beta(alpha, beta) || Beta(1, 9)) of already-activated parameters (reference API)."""
        return torch.distributions.kl.kl_divergence(
            torch.distributions.Beta(alpha, beta),
            torch.distributions.Beta(torch.tensor(1.0, device=alpha.device), torch.tensor(9.0, device=alpha.device)))
