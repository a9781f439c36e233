"""Loss masking helpers (ref:src/utils/data_utils.py:67-104) on libmlvae."""
import torch

from mlvae_hip import ops


def length_to_mask(length, max_len=None, dtype=None, device=None):
    """SpeechBrain 0.5 semantics (un-vendored in the reference): arange(T) < length (fp32).
    Host-side helper for bookkeeping; the kernels apply the same rule on the device."""
    if max_len is None:
        max_len = int(length.max().long().item())
    mask = torch.arange(max_len, device=length.device, dtype=length.dtype).expand(
        len(length), max_len) < length.unsqueeze(1)
    return mask.to(dtype=dtype or length.dtype, device=device or length.device)


def apply_lens_to_loss(loss, lens, reduction='mean'):
    """sum(loss * mask) / sum(mask) ('mean'), / B ('batchmean') or per utterance ('batch'),
    mask = frames t < lens*T (relative lengths, fp32 compare as SpeechBrain's length_to_mask)."""
    return ops.masked_mean(loss, lens, reduction)


def apply_weight(x, weight):
    """Mixture weighting as one HIP launch (ref:src/utils/data_utils.py:32-64).

    x: (B, T, N, C) or (B, T, N * C); weight: (B, T, N) -> (B, T, C)."""
    return ops.apply_weight(x, weight)
