"""Decoder on libmlvae (replaces ref:src/modules/decoder.py:10-53).

rnn: a bidirectional L-layer LSTM.  An nn.LSTM instance is kept as the parameter holder so
initialisation and state_dict keys (rnn.weight_ih_l0, ...) match the reference; its forward is
not used -- the recurrence runs in the persistent HIP kernels (mlvae_hip.ops.LSTMFn).
mean_fc / log_var_fc: FCBlock heads.  compute_recon_loss: Gaussian NLL ('likelihood', the
default) or MSE, per element; anything else raises ValueError('Invalid loss type: ...').
"""
from torch import nn

from mlvae_hip import ops
from modules.fc_block import FCBlock


class Decoder(nn.Module):
    def __init__(self, input_size, rnn_hidden_size, rnn_num_layers, rnn_dropout, fc_sizes,
                 loss_type='likelihood'):
        super().__init__()
        self.rnn = nn.LSTM(input_size, rnn_hidden_size, rnn_num_layers, dropout=rnn_dropout,
                           bidirectional=True, batch_first=True)
        self.mean_fc = FCBlock(fc_sizes)
        self.log_var_fc = FCBlock(fc_sizes)
        self.loss_type = loss_type

    def forward(self, sampled_h, target_feats):  # (B, T, C)
        rnn_out = ops.bilstm(sampled_h, self.rnn, self.training)
        mean = self.mean_fc(rnn_out)
        log_var = self.log_var_fc(rnn_out)
        loss = self.compute_recon_loss(mean, log_var, target_feats)
        return {"mean": mean, "log_var": log_var, "losses": {"recon_loss": loss}}

    def compute_recon_loss(self, mean, log_var, target):
        return ops.recon_loss(mean, log_var, target, self.loss_type)
