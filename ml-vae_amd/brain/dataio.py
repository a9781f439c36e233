"""Batches with relative lengths (SpeechBrain PaddedBatch semantics)."""
import torch


def length_to_mask(length, max_len=None, dtype=None, device=None):
    """arange(max_len) < length, compared in length's dtype (SpeechBrain 0.5)."""
    if max_len is None:
        max_len = int(length.max().long().item())
    mask = torch.arange(max_len, device=length.device, dtype=length.dtype).expand(
        len(length), max_len) < length.unsqueeze(1)
    return mask.to(dtype=dtype or length.dtype, device=device or length.device)


class PaddedBatch(dict):
    """dict of fields; tensor fields are (padded [B, Tmax, ...], relative lengths [B])."""

    def __init__(self, examples, key="feat"):
        feats = [e[key] for e in examples]
        tmax = max(f.shape[0] for f in feats)
        out = torch.zeros(len(feats), tmax, *feats[0].shape[1:], dtype=feats[0].dtype)
        for i, f in enumerate(feats):
            out[i, :f.shape[0]] = f
        lens = torch.tensor([f.shape[0] / tmax for f in feats], dtype=torch.float32)
        super().__init__()
        self[key] = (out, lens)
        self["id"] = [e.get("id", str(i)) for i, e in enumerate(examples)]

    def to(self, device):
        for k, v in self.items():
            if isinstance(v, tuple):
                self[k] = tuple(t.to(device, non_blocking=True) for t in v)
        return self
