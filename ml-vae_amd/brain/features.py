"""InputNormalization(norm_type='global') as used by the recipe
(ref:src/models/test_vanilla_vae/model.yaml:14-15, called at model.py:24-25).

SpeechBrain 0.5 semantics restated (parity unpinned): per-utterance mean/std over the first
round(len*T) frames, averaged over the batch; in train mode the global statistics are set on
the first batch and then running-averaged with weight 1/(count+1) while
epoch < update_until_epoch; x <- (x - mean) / std.  Device-side torch ops with no host
synchronisation (outside the fused train step, which takes already normalised features)."""
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
        # per-utterance statistics over the first round(len*T) frames, as one masked device
        # reduction (no per-utterance host sync); std is the unbiased torch.std
        B, T = x.shape[0], x.shape[1]
        n = torch.round(lengths.to(x.device, torch.float32) * T)
        mask = (torch.arange(T, device=x.device, dtype=torch.float32).unsqueeze(0) < n.unsqueeze(1))
        mask = mask.to(x.dtype).reshape(B, T, *([1] * (x.dim() - 2)))
        nb = n.to(x.dtype).reshape(B, *([1] * (x.dim() - 2)))
        # zero-length utterances (the fillers of a short data-parallel evaluation slice) carry no
        # statistics: they are left out of the batch averages
        valid = (n > 0).to(x.dtype).reshape(B, *([1] * (x.dim() - 2)))
        nb = nb.clamp(min=1)
        means = (x * mask).sum(1) / nb
        var = (((x - means.unsqueeze(1)) * mask) ** 2).sum(1) / (nb - 1)
        stds = torch.clamp(var.sqrt(), min=self.eps)
        stds = torch.where(valid > 0, stds, torch.zeros_like(stds))  # 0/0 of an empty utterance
        nvalid = valid.sum(0).clamp(min=1)
        cur_mean = (means * valid).sum(0) / nvalid
        cur_std = (stds * valid).sum(0) / nvalid
        from brain.distributed import all_reduce_sum_, world_size
        if self.training and world_size() > 1:  # data parallel: the statistics of the global batch
            acc = torch.cat([(means * valid).sum(0).reshape(-1), (stds * valid).sum(0).reshape(-1),
                             valid.sum().reshape(1)])
            all_reduce_sum_(acc)
            k = cur_mean.numel()
            cur_mean = (acc[:k] / acc[-1]).reshape(cur_mean.shape)
            cur_std = (acc[k:2 * k] / acc[-1]).reshape(cur_std.shape)
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
