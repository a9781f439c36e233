"""PhonemeRecognizer on libmlvae (replaces ref:src/modules/phoneme_recognizer.py:9-81).

rnn: a unidirectional L-layer nn.LSTM kept as the parameter holder (reference init and
state_dict keys rnn.weight_ih_l0, ...); the recurrence runs in the persistent HIP kernels
(mlvae_hip.ops.LSTMFn, one direction's workgroups).  fc: FCBlock.  compute_losses: the
per-frame BCE-with-logits against the canonical phoneme sequence expanded by the boundary
durations, one kernel over the batch (csrc/md.hip) instead of the reference's host loop; the
reference's asserts (boundary count != L_i) raise AssertionError likewise.
"""
from torch import nn

from mlvae_hip import ops
from modules.fc_block import FCBlock


class PhonemeRecognizer(nn.Module):
    def __init__(self, input_size, rnn_hidden_size, rnn_num_layers, fc_sizes, n_phonemes):
        super().__init__()
        self.rnn = nn.LSTM(input_size, rnn_hidden_size, rnn_num_layers, batch_first=True)
        self.fc = FCBlock(fc_sizes)
        self.n_phonemes = n_phonemes

    def forward(self, feats, feat_lens, plvl_cnnl_phn_seqs, plvl_cnnl_phn_seq_lens, boundary_seqs):
        out = ops.lstm(feats, self.rnn, self.training)
        out = self.fc(out)
        losses = self.compute_losses(out, feat_lens, plvl_cnnl_phn_seqs, plvl_cnnl_phn_seq_lens,
                                     boundary_seqs)
        return {"out": out, "losses": losses}

    def compute_losses(self, out, feat_lens, plvl_cnnl_phn_seqs, plvl_cnnl_phn_seq_lens, boundary_seqs):
        if out.shape[-1] != self.n_phonemes + 2:
            raise ValueError(f"recogniser output has {out.shape[-1]} classes, one-hot needs "
                             f"n_phonemes + 2 = {self.n_phonemes + 2}")
        loss = ops.phn_bce(out, feat_lens, plvl_cnnl_phn_seqs, plvl_cnnl_phn_seq_lens, boundary_seqs)
        return {"phn_recog_bce_loss": loss}
