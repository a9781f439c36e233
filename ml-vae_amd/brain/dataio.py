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
    """dict of fields; tensor fields (sequences: feat, phoneme / boundary sequences, ...) are
    (padded [B, Lmax, ...], relative lengths [B]); other fields are lists."""

    def __init__(self, examples, key="feat", pad_to=None):
        """pad_to: {field: length} -- pad those sequence fields to at least that many steps
        (data parallel: every rank pads to its global batch's longest utterance, so the
        relative lengths, the padded T and the counter-based random streams keyed by
        (utterance, frame) equal the single-process batch's)."""
        super().__init__()
        keys = [k for k in examples[0] if k != "id"]
        if key not in keys:
            keys.insert(0, key)
        for k in keys:
            vals = [e[k] for e in examples]
            if all(torch.is_tensor(v) and v.dim() >= 1 for v in vals):
                tmax = max(max(v.shape[0] for v in vals), (pad_to or {}).get(k, 0))
                out = torch.zeros(len(vals), tmax, *vals[0].shape[1:], dtype=vals[0].dtype)
                for i, v in enumerate(vals):
                    out[i, :v.shape[0]] = v
                lens = torch.tensor([v.shape[0] / tmax if tmax else 0.0 for v in vals],
                                    dtype=torch.float32)
                self[k] = (out, lens)
            else:
                self[k] = vals
        self["id"] = [e.get("id", str(i)) for i, e in enumerate(examples)]

    def to(self, device):
        for k, v in self.items():
            if isinstance(v, tuple):
                self[k] = tuple(t.to(device, non_blocking=True) for t in v)
        return self
