"""Datasets of the recipe (ref:src/utils/data_io.py:24-146).

* ``PickledSet``: the reference's pre-computed corpora, ``<dataset_dir>/../computed_dataset/
  {train,valid,test}.pkl`` = {utt_id: {key: value}} over ``output_keys`` (written by the
  reference's prepare_datasets, ref:src/utils/data_io.py:40-104).  The Kaldi / librosa feature
  computation that produces them is out of scope; when the files exist they are read as is.
* ``SyntheticSet``: F-dim frames, lengths uniform in [min_frames, max_frames], values
  log(1e-6 + |N(0,1)|^2) standardised (log-mel-like), seeded.

Batches follow SpeechBrain's PaddedBatch: batch['feat'] = (padded [B, Tmax, F], relative lengths
[B]).  Under data parallelism rank r of W reads utterances [r*bs, (r+1)*bs) of every global batch
of W*bs, padded to that global batch's longest utterance (so every rank sees the single-process
batch's T and relative lengths).  TRAIN drops an incomplete last global batch (every rank runs
the same number of optimizer steps); VALID / TEST keep it: ranks whose slice of the remainder is
short fill it with zero-length utterances, which every masked mean and frame count excludes."""
import io
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


def _seq_max(items):
    """{field: longest sequence} over the given utterances (tensor fields with a time axis)."""
    out = {}
    for e in items:
        for k, v in e.items():
            if torch.is_tensor(v) and v.dim() >= 1:
                out[k] = max(out.get(k, 0), v.shape[0])
    return out


def _empty_like(e):
    """A zero-length utterance with the fields of e (fills a short rank slice in evaluation)."""
    d = {"id": "__pad__"}
    for k, v in e.items():
        if k == "id":
            continue
        d[k] = v.new_zeros((0,) + tuple(v.shape[1:])) if torch.is_tensor(v) and v.dim() >= 1 else v
    return d


def _batched(items, batch_size, rank=0, world=1, stage=None, skip=0):
    """skip: the first `skip` batches are passed over at the index level (not collated)."""
    if world <= 1:
        for i in range(skip * batch_size, len(items), batch_size):
            yield PaddedBatch(items[i:i + batch_size])
        return
    g = batch_size * world
    train = stage is None or getattr(stage, "name", str(stage)).upper() == "TRAIN"
    end = len(items) - g + 1 if train else len(items)
    for i in range(skip * g, max(end, 0), g):
        glob = items[i:i + g]
        mine = glob[rank * batch_size:(rank + 1) * batch_size]
        mine = mine + [_empty_like(glob[0])] * (batch_size - len(mine))
        yield PaddedBatch(mine, pad_to=_seq_max(glob))


class BatchLoader:
    """The batches of one split, re-iterable: every pass (epoch) is a fresh walk over the items,
    as a DataLoader is (a bare generator would leave every epoch after the first empty).
    skip_next(n) makes the next pass start at batch n -- the resume point of an intra-epoch
    checkpoint -- without collating the batches it passes over.  `signature` is what must match
    for such a resume to skip the right utterances (batch size, world size, sorting, length)."""

    def __init__(self, items, batch_size, rank=0, world=1, stage=None, sorting=None):
        self.items, self.batch_size, self.rank, self.world = items, batch_size, rank, world
        self.stage, self.sorting = stage, sorting
        self._skip = 0

    def __len__(self):
        g = self.batch_size * self.world
        train = self.world > 1 and (self.stage is None or
                                    getattr(self.stage, "name", str(self.stage)).upper() == "TRAIN")
        return len(self.items) // g if train else (len(self.items) + g - 1) // g

    def skip_next(self, n):
        self._skip = int(n)

    def __iter__(self):
        skip, self._skip = self._skip, 0
        return _batched(self.items, self.batch_size, self.rank, self.world, self.stage, skip)

    def signature(self):
        return {"batch_size": self.batch_size, "world_size": self.world, "sorting": self.sorting,
                "n_batches": len(self)}


def _storage_from_bytes(b):
    """torch.storage._load_from_bytes without its weights_only=False: the tensor storages the
    reference's pickles hold load through torch's restricted (weights-only) unpickler."""
    return torch.load(io.BytesIO(b), weights_only=True)


class _CorpusUnpickler(pickle.Unpickler):
    """The reference's computed_dataset/*.pkl holds plain containers, numbers, strings, numpy
    arrays and torch tensors (SpeechBrain pipeline outputs); anything else (an arbitrary callable
    a crafted file could name) is refused."""
    _ALLOWED = {
        ("builtins", "dict"), ("builtins", "list"), ("builtins", "tuple"), ("builtins", "set"),
        ("builtins", "frozenset"), ("builtins", "int"), ("builtins", "float"), ("builtins", "str"),
        ("builtins", "bytes"), ("builtins", "bool"), ("builtins", "complex"),
        ("collections", "OrderedDict"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("torch._utils", "_rebuild_tensor_v2"),
        ("torch", "Size"), ("torch", "float32"), ("torch", "float64"), ("torch", "int64"),
    }

    def find_class(self, module, name):
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _storage_from_bytes
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"computed dataset pickle names {module}.{name}: refused "
                                     "(only containers, numbers, strings and numpy arrays load)")


def load_corpus_pickle(path):
    """Restricted load of a computed_dataset/*.pkl (no code from the file is executed)."""
    with open(path, "rb") as f:
        return _CorpusUnpickler(io.BytesIO(f.read())).load()


def _sort(items, sorting):
    if sorting == "descending":
        items.sort(key=lambda e: -e["feat"].shape[0])
    elif sorting == "ascending":
        items.sort(key=lambda e: e["feat"].shape[0])
    return items


class PickledSet:
    """One split of the reference's computed dataset (a dict of per-utterance dicts)."""

    def __init__(self, pkl_path, sorting="descending"):
        data = load_corpus_pickle(pkl_path)  # restricted: containers / numbers / numpy arrays
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
        self.sorting = sorting

    def __len__(self):
        return len(self.items)

    def batches(self, stage=None, batch_size=8, rank=0, world=1, **_):
        return BatchLoader(self.items, batch_size, rank, world, stage, self.sorting)


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
        self.sorting = sorting

    def __len__(self):
        return len(self.items)

    def batches(self, stage=None, batch_size=8, rank=0, world=1, **_):
        return BatchLoader(self.items, batch_size, rank, world, stage, self.sorting)


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
