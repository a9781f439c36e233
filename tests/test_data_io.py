"""Host logic of the recipe's data layer (utils/data_io.py, brain/dataio.py, brain/features.py):
data-parallel shards padded to the global batch, evaluation remainders kept, the restricted
corpus unpickler, the normaliser ignoring zero-length filler utterances."""
import os
import pickle

import numpy as np
import pytest
import torch

from brain import Stage
from brain.features import InputNormalization
from utils.data_io import SyntheticSet, _batched, load_corpus_pickle


def _items(lens, F=3):
    return [{"id": f"u{i}", "feat": torch.full((L, F), float(i))} for i, L in enumerate(lens)]


def test_dp_shards_padded_to_the_global_batch():
    items = _items([9, 7, 5, 4, 3, 2, 2, 1])
    single = list(_batched(items, 4))
    for r in range(2):
        shards = list(_batched(items, 2, rank=r, world=2, stage=Stage.TRAIN))
        assert len(shards) == 2
        for gi, sh in enumerate(shards):
            feats, lens = sh["feat"]
            g_feats, g_lens = single[gi]["feat"]
            assert feats.shape[1] == g_feats.shape[1]            # the single-process T
            assert torch.equal(lens, g_lens[2 * r:2 * r + 2])     # and relative lengths
            assert torch.equal(feats, g_feats[2 * r:2 * r + 2])


def test_dp_train_drops_eval_keeps_the_remainder():
    items = _items([9, 7, 5, 4, 3])        # 5 utterances, global batch 4
    assert len(list(_batched(items, 2, rank=1, world=2, stage=Stage.TRAIN))) == 1
    for stage in (Stage.VALID, Stage.TEST):
        got = [list(_batched(items, 2, rank=r, world=2, stage=stage)) for r in range(2)]
        assert len(got[0]) == len(got[1]) == 2                  # every rank takes the same steps
        last0, last1 = got[0][1], got[1][1]
        assert last0["id"] == ["u4", "__pad__"] and last1["id"] == ["__pad__", "__pad__"]
        assert last1["feat"][0].shape == (2, 3, 3)              # padded to the remainder's T
        assert torch.equal(last1["feat"][1], torch.zeros(2))     # masked out everywhere
        n_real = sum(int((b["feat"][1] > 0).sum()) for g in got for b in g)
        assert n_real == 5


def test_restricted_unpickler(tmp_path):
    d = {"u1": {"feat": torch.randn(4, 2), "prior": np.arange(3.0), "gt_phn_seq": [1, 2], "duration": 1.5}}
    p = tmp_path / "train.pkl"
    with open(p, "wb") as f:
        pickle.dump(d, f)
    r = load_corpus_pickle(p)
    assert torch.equal(r["u1"]["feat"], d["u1"]["feat"]) and r["u1"]["gt_phn_seq"] == [1, 2]

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    with open(p, "wb") as f:
        pickle.dump({"u": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_corpus_pickle(p)


def test_normaliser_ignores_zero_length_fillers():
    x = torch.randn(3, 10, 4)
    lens = torch.tensor([1.0, 0.5, 0.0])
    a, b = InputNormalization(), InputNormalization()
    ya = a(x, lens)
    b(x[:2], lens[:2])
    assert torch.isfinite(ya).all()
    assert torch.allclose(a.glob_mean, b.glob_mean) and torch.allclose(a.glob_std, b.glob_std)


def test_synthetic_set_batches_stage_argument():
    ds = SyntheticSet(10, 4, 5, 9, seed=1)
    assert sum(len(b["id"]) for b in ds.batches(stage=Stage.VALID, batch_size=4)) == 10
