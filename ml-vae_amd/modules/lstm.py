"""torch.nn.LSTM drop-in on the HIP recurrence.

The MD-VAE recipes build their 2-layer unidirectional 512-unit sequence model directly as
``rnn: !new:torch.nn.LSTM`` (ref:src/models/MD_VAE/model.yaml:78-83; called at
ref:src/models/MD_VAE/model.py:116 as ``self.modules['rnn'](rnn_in)[0]``).  Pointing that yaml
entry at ``!new:modules.lstm.LSTM`` keeps the constructor, the parameters and their state_dict
keys (it IS an nn.LSTM), and runs forward / backward on libmlvae: per layer the input-projection
GEMM and the persistent recurrence (csrc/lstm.hip, uni- or bidirectional), inter-layer dropout in
train mode from a counter-based Philox stream.  Returns (output, (h_n, c_n)) as nn.LSTM does.
"""
import torch

from mlvae_hip import ops


class LSTM(torch.nn.LSTM):
    def forward(self, input, hx=None):
        if hx is not None:
            raise NotImplementedError("initial states: every reference LSTM starts from zeros")
        if not input.is_cuda:
            raise RuntimeError("modules.lstm.LSTM runs on the HIP device only (no CPU fallback)")
        if self.proj_size:
            raise NotImplementedError("proj_size is not used by the reference")
        return ops.lstm_full(input, self, self.training)
