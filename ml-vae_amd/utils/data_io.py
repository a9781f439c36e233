"""Synthetic log-mel datasets standing in for the reference's pickle-cached corpora
(ref:src/utils/data_io.py:40-146; real corpora and Kaldi are out of scope).

Utterances: F-dim frames, lengths uniform in [min_frames, max_frames], values
log(1e-6 + |N(0,1)|^2) standardised (log-mel-like), seeded.  Batches follow SpeechBrain's
PaddedBatch: batch['feat'] = (padded [B, Tmax, F], relative lengths [B])."""
import torch

from brain.dataio import PaddedBatch


class SyntheticSet:
    def __init__(self, n_utts, feat_dim, min_frames, max_frames, seed, sorting="descending"):
        g = torch.Generator().manual_seed(seed)
        lens = torch.randint(min_frames, max_frames + 1, (n_utts,), generator=g)
        self.items = []
        for i, L in enumerate(lens.tolist()):
            x = torch.log(1e-6 + torch.randn(L, feat_dim, generator=g) ** 2)
            x = (x - x.mean()) / x.std()
            self.items.append({"id": f"utt{i:05d}", "feat": x})
        if sorting == "descending":
            self.items.sort(key=lambda e: -e["feat"].shape[0])
        elif sorting == "ascending":
            self.items.sort(key=lambda e: e["feat"].shape[0])

    def __len__(self):
        return len(self.items)

    def batches(self, stage=None, batch_size=8, **_):
        for i in range(0, len(self.items), batch_size):
            yield PaddedBatch(self.items[i:i + batch_size])


def prepare_datasets(hparams):
    d = hparams.get("synthetic", {})
    F = hparams["model"]["input_size"]
    sets = []
    for j, split in enumerate(("train", "valid", "test")):
        sets.append(SyntheticSet(d.get(f"n_{split}", 32), F, d.get("min_frames", 50),
                                 d.get("max_frames", 200), hparams.get("seed", 123456) + j,
                                 hparams.get("sorting", "descending")))
    return sets, None
