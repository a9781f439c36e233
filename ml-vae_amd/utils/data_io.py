"""Datasets of the recipe (ref:src/utils/data_io.py:24-146).

* ``PickledSet``: the reference's pre-computed corpora, ``<dataset_dir>/../computed_dataset/
  {train,valid,test}.pkl`` = {utt_id: {key: value}} over ``output_keys`` (written by the
  reference's prepare_datasets, ref:src/utils/data_io.py:40-104).  The Kaldi / librosa feature
  computation that produces them is out of scope; when the files exist they are read as is.
* ``SyntheticSet``: F-dim frames, lengths uniform in [min_frames, max_frames], values
  log(1e-6 + |N(0,1)|^2) standardised (log-mel-like), seeded.

Batches follow SpeechBrain's PaddedBatch: batch['feat'] = (padded [B, Tmax, F], relative lengths
[B]).  Under data parallelism rank r of W reads utterances [r*bs, (r+1)*bs) of every global batch
of W*bs (an incomplete last global batch is dropped, so every rank runs the same number of
steps)."""
import pickle
from pathlib import Path

import numpy as np
import torch

from brain.dataio import PaddedBatch

# the reference's keys (ref:src/utils/data_io.py:24-37)
output_keys = [
    'id', 'wav', 'aug_wav', 'duration', 'feat', 'aug_feat', 'kaldi_feat', 'aug_kaldi_feat',
    'gt_phn_seq', 'gt_cnncl_seq', 'flvl_gt_phn_seq', 'flvl_gt_cnncl_seq', 'aug_flvl_gt_cnncl_seq',
    'plvl_gt_md_lbl_seq', 'flvl_gt_md_lbl_seq', 'aug_flvl_gt_md_lbl_seq', 'gt_seg_seq',
    'gt_boundary_seq', 'gt_phn_end_seq', 'fa_seg_seq', 'fa_boundary_seq', 'fa_phn_end_seq', 'prior',
]


def _batched(items, batch_size, rank=0, world=1):
    if world <= 1:
        for i in range(0, len(items), batch_size):
            yield PaddedBatch(items[i:i + batch_size])
        return
    g = batch_size * world
    for i in range(0, len(items) - g + 1, g):
        yield PaddedBatch(items[i + rank * batch_size:i + (rank + 1) * batch_size])


def _sort(items, sorting):
    if sorting == "descending":
        items.sort(key=lambda e: -e["feat"].shape[0])
    elif sorting == "ascending":
        items.sort(key=lambda e: e["feat"].shape[0])
    return items


class PickledSet:
    """One split of the reference's computed dataset (a dict of per-utterance dicts)."""

    def __init__(self, pkl_path, sorting="descending"):
        with open(pkl_path, "rb") as f:
            data = pickle.load(f)  # the user's own corpus files, in the reference's format
        self.items = []
        for utt_id, d in data.items():
            e = {"id": utt_id}
            for k, v in d.items():
                if isinstance(v, np.ndarray):
                    v = torch.from_numpy(v)
                elif isinstance(v, list) and v and isinstance(v[0], (int, float)):
                    v = torch.tensor(v)
                if k == "feat" and torch.is_tensor(v):
                    v = v.float()
                e[k] = v
            self.items.append(e)
        _sort(self.items, sorting)

    def __len__(self):
        return len(self.items)

    def batches(self, stage=None, batch_size=8, rank=0, world=1, **_):
        return _batched(self.items, batch_size, rank, world)


class SyntheticSet:
    def __init__(self, n_utts, feat_dim, min_frames, max_frames, seed, sorting="descending"):
        g = torch.Generator().manual_seed(seed)
        lens = torch.randint(min_frames, max_frames + 1, (n_utts,), generator=g)
        self.items = []
        for i, L in enumerate(lens.tolist()):
            x = torch.log(1e-6 + torch.randn(L, feat_dim, generator=g) ** 2)
            x = (x - x.mean()) / x.std()
            self.items.append({"id": f"utt{i:05d}", "feat": x})
        _sort(self.items, sorting)

    def __len__(self):
        return len(self.items)

    def batches(self, stage=None, batch_size=8, rank=0, world=1, **_):
        return _batched(self.items, batch_size, rank, world)


def computed_dataset_dir(hparams):
    return Path(hparams["prepare"]["dataset_dir"]).parent / "computed_dataset"


def prepare_datasets(hparams):
    cdir = computed_dataset_dir(hparams)
    if hparams.get("dataset") != "synthetic" or all((cdir / f"{s}.pkl").exists() for s in ("train", "valid", "test")):
        missing = [s for s in ("train", "valid", "test") if not (cdir / f"{s}.pkl").exists()]
        if missing:
            raise FileNotFoundError(
                f"computed dataset {cdir}/{{{','.join(missing)}}}.pkl not found: the Kaldi / librosa "
                "feature preparation of ref:src/utils/data_io.py:56-93 is not part of this build; "
                "point prepare.dataset_dir at a corpus the reference has already computed")
        return [PickledSet(cdir / f"{s}.pkl", hparams.get("sorting", "descending"))
                for s in ("train", "valid", "test")], None
    d = hparams.get("synthetic", {})
    F = hparams["model"]["input_size"]
    sets = []
    for j, split in enumerate(("train", "valid", "test")):
        sets.append(SyntheticSet(d.get(f"n_{split}", 32), F, d.get("min_frames", 50),
                                 d.get("max_frames", 200), hparams.get("seed", 123456) + j,
                                 hparams.get("sorting", "descending")))
    return sets, None
