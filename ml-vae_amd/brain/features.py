"""InputNormalization(norm_type='global') as used by the recipe
(ref:src/models/test_vanilla_vae/model.yaml:14-15, called at model.py:24-25).

SpeechBrain 0.5 semantics restated (parity unpinned): per-utterance mean/std over the first
round(len*T) frames, averaged over the batch; in train mode the global statistics are set on
the first batch and then running-averaged with weight 1/(count+1) while
epoch < update_until_epoch; x <- (x - mean) / std.  Host-side torch ops (outside the fused
train step, which takes already normalised features)."""
import torch


class InputNormalization(torch.nn.Module):
    def __init__(self, mean_norm=True, std_norm=True, norm_type="global", avg_factor=None,
                 requires_grad=False, update_until_epoch=3):
        super().__init__()
        if norm_type != "global":
            raise NotImplementedError("only norm_type='global' is used by the VAE recipe")
        self.mean_norm, self.std_norm = mean_norm, std_norm
        self.norm_type = norm_type
        self.avg_factor = avg_factor
        self.update_until_epoch = update_until_epoch
        self.eps = 1e-10
        self.count = 0
        self.register_buffer("glob_mean", torch.zeros(0))
        self.register_buffer("glob_std", torch.zeros(0))

    @torch.no_grad()
    def forward(self, x, lengths, spk_ids=None, epoch=0):
        means, stds = [], []
        for b in range(x.shape[0]):
            n = int(torch.round(lengths[b] * x.shape[1]).item())
            seg = x[b, :n]
            means.append(seg.mean(0))
            stds.append(torch.clamp(seg.std(0), min=self.eps))
        cur_mean = torch.stack(means).mean(0)
        cur_std = torch.stack(stds).mean(0)
        if self.training:
            if self.count == 0:
                self.glob_mean, self.glob_std = cur_mean, cur_std
            elif epoch < self.update_until_epoch:
                w = self.avg_factor if self.avg_factor is not None else 1.0 / (self.count + 1)
                self.glob_mean = (1 - w) * self.glob_mean + w * cur_mean
                self.glob_std = (1 - w) * self.glob_std + w * cur_std
            self.count += 1
        if self.glob_mean.numel() == 0:
            self.glob_mean, self.glob_std = cur_mean, cur_std
        out = x
        if self.mean_norm:
            out = out - self.glob_mean
        if self.std_norm:
            out = out / self.glob_std
        return out
