"""The recipe's data-parallel pieces on CPU (brain/distributed.py, utils/data_io.py,
brain/features.py): sharded global batches, the reference's pickled computed datasets
(ref:src/utils/data_io.py:24-104), and the input normaliser's all-reduced statistics over two
gloo ranks."""
import pickle

import numpy as np
import pytest
import torch

from brain.features import InputNormalization
from utils.data_io import PickledSet, SyntheticSet


def test_rank_slices_partition_each_global_batch():
    ds = SyntheticSet(22, 8, 10, 30, seed=5)
    full = [b["id"] for b in ds.batches(batch_size=6)]
    shards = [[b["id"] for b in ds.batches(batch_size=3, rank=r, world=2)] for r in range(2)]
    assert len(shards[0]) == len(shards[1]) == 22 // 6  # incomplete last global batch dropped
    for step in range(len(shards[0])):
        assert shards[0][step] + shards[1][step] == full[step]


def test_pickled_computed_dataset_loads_and_pads(tmp_path):
    g = np.random.default_rng(0)
    data = {f"spk_{i}": {"feat": g.standard_normal((20 + i, 5)).astype(np.float32),
                         "gt_cnncl_seq": list(range(3 + i)), "duration": 1.5 + i}
            for i in range(5)}
    with open(tmp_path / "train.pkl", "wb") as f:
        pickle.dump(data, f)
    ds = PickledSet(tmp_path / "train.pkl")
    assert len(ds) == 5 and ds.items[0]["feat"].shape[0] == 24  # descending sort
    b = next(iter(ds.batches(batch_size=3)))
    feats, lens = b["feat"]
    assert feats.shape == (3, 24, 5) and torch.allclose(lens, torch.tensor([1.0, 23 / 24, 22 / 24]))
    seqs, slens = b["gt_cnncl_seq"]
    assert seqs.shape == (3, 7) and torch.equal(seqs[0], torch.arange(7))
    assert b["duration"] == [5.5, 4.5, 3.5] and b["id"] == ["spk_4", "spk_3", "spk_2"]


def _norm_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 12, 6, generator=g)
    lens = torch.tensor([1.0, 0.75, 0.5, 1.0])
    n = InputNormalization()
    n.train()
    for _ in range(2):
        n(x[2 * rank:2 * rank + 2], lens[2 * rank:2 * rank + 2])
    q.put((rank, n.glob_mean.numpy().copy(), n.glob_std.numpy().copy()))   # by value, not by fd
    dist.destroy_process_group()


def test_normaliser_statistics_are_global_under_data_parallel():
    import torch.multiprocessing as mp
    from test_dist_gloo import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_norm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 12, 6, generator=g)
    lens = torch.tensor([1.0, 0.75, 0.5, 1.0])
    ref = InputNormalization()
    ref.train()
    for _ in range(2):
        ref(x, lens)
    for _, m, s in res:
        m, s = torch.from_numpy(m), torch.from_numpy(s)
        assert torch.allclose(m, ref.glob_mean, atol=1e-6) and torch.allclose(s, ref.glob_std, atol=1e-6)
