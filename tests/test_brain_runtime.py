"""CPU tests of the recipe runtime around the fused step: SpeechBrain checkpoint layout,
device-side InputNormalization, the normaliser's call on the fused path, bench.py's process
model."""
import json
import os
import subprocess
import sys
import types
import warnings

import pytest
import torch
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ checkpoints
def test_checkpoint_layout_is_speechbrains(tmp_path):
    from brain import Checkpointer, EpochCounter
    lin = torch.nn.Linear(3, 2)
    ec = EpochCounter(5)
    next(ec), next(ec)
    ck = Checkpointer(tmp_path, {"encoder": lin, "epoch_counter": ec})
    d = ck.save_and_keep_only(meta={"loss": torch.tensor(1.25), "kld_loss.loss": 0.5},
                              min_keys=["loss"])
    name = os.path.basename(d)
    assert name.startswith("CKPT+") and len(name.split("+")) == 4   # CKPT+date+time+NN
    files = sorted(os.listdir(d))
    assert files == ["CKPT.yaml", "encoder.ckpt", "epoch_counter.ckpt"]
    text = open(os.path.join(d, "CKPT.yaml")).read()
    assert text.startswith("# yamllint disable\n")
    meta = yaml.safe_load(text)
    assert meta["loss"] == 1.25 and meta["end-of-epoch"] is True and "unixtime" in meta
    assert open(os.path.join(d, "epoch_counter.ckpt")).read() == "2"
    sd = torch.load(os.path.join(d, "encoder.ckpt"), weights_only=True)
    assert set(sd) == {"weight", "bias"} and torch.equal(sd["weight"], lin.weight.detach())


def test_recover_from_a_speechbrain_written_directory(tmp_path):
    """A directory laid out the way SpeechBrain's Checkpointer writes it (built by hand here)
    recovers, and min_key picks the lowest meta value."""
    from brain import Checkpointer, EpochCounter
    ref = {}
    for i, (loss, stamp) in enumerate(((2.0, "2024-01-01+10-00-00+00"), (0.5, "2024-01-01+11-00-00+00"),
                                       (1.0, "2024-01-01+12-00-00+00"))):
        d = tmp_path / f"CKPT+{stamp}"
        d.mkdir()
        (d / "CKPT.yaml").write_text("# yamllint disable\n" +
                                     yaml.safe_dump({"end-of-epoch": True, "loss": loss,
                                                     "unixtime": 1.7e9 + i}))
        w = {"weight": torch.full((2, 3), float(i)), "bias": torch.full((2,), float(i))}
        torch.save(w, d / "encoder.ckpt")
        (d / "epoch_counter.ckpt").write_text(str(10 + i))
        ref[loss] = w
    (tmp_path / "CKPT+broken").mkdir()  # no meta file: reported, not silently skipped
    lin, ec = torch.nn.Linear(3, 2), EpochCounter(50)
    ck = Checkpointer(tmp_path, {"encoder": lin, "epoch_counter": ec})
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        d = ck.recover_if_possible(min_key="loss")
    assert any("CKPT+broken" in str(r.message) for r in rec)
    assert d.endswith("11-00-00+00")
    assert torch.equal(lin.weight.detach(), ref[0.5]["weight"]) and ec.current == 11
    ck.recover_if_possible()  # most recent
    assert ec.current == 12
    assert ck.find_checkpoint(max_key="loss").endswith("10-00-00+00")


def test_mid_epoch_checkpoint_replays_the_epoch(tmp_path):
    from brain import Checkpointer, EpochCounter
    ec = EpochCounter(9)
    ec.current = 4
    ck = Checkpointer(tmp_path, {"epoch_counter": ec})
    ck.save_checkpoint(end_of_epoch=False)
    ec.current = 0
    ck.recover_if_possible()
    assert ec.current == 3


def test_ckpt_interval_minutes_saves_intra_epoch_checkpoints(tmp_path, monkeypatch):
    """--ckpt_interval_minutes (SpeechBrain Brain.fit): an end_of_epoch=False checkpoint on the
    host timer during TRAIN, each replacing the previous intra-epoch one only; the end-of-epoch
    save_and_keep_only (min_keys) then removes it and keeps the best epoch checkpoint."""
    import brain.core as core
    from brain import Checkpointer, EpochCounter
    from brain.core import INTRA_EPOCH_CKPT_FLAG, Brain, Stage

    clock = [1000.0]
    monkeypatch.setattr(core.time, "time", lambda: clock[0])

    class Toy(Brain):
        def compute_forward(self, batch, stage):
            return self.modules["lin"](batch)

        def compute_objectives(self, out, batch, stage):
            clock[0] += 40.0                     # every batch takes 40 "seconds"
            return out.pow(2).mean()

        def fit_batch(self, batch):               # CPU: no HIP clip
            loss = self.compute_objectives(self.compute_forward(batch, Stage.TRAIN), batch, Stage.TRAIN)
            return loss.detach()

        def on_stage_end(self, stage, loss, epoch=None):
            if stage == Stage.TRAIN:
                ck = self.checkpointer.list_checkpoints()
                self.seen = [(m["end_of_epoch"], INTRA_EPOCH_CKPT_FLAG in m["meta"]) for _, m in ck]
                clock[0] += 1.0
                self.checkpointer.save_and_keep_only(meta={"loss": loss}, min_keys=["loss"])

    lin = torch.nn.Linear(4, 2)
    ec = EpochCounter(1)
    ck = Checkpointer(tmp_path, {"lin": lin, "epoch_counter": ec})
    b = Toy(modules={"lin": lin}, opt_class=lambda p: torch.optim.SGD(p, lr=0.1),
            run_opts={"device": "cpu", "ckpt_interval_minutes": 1.0}, checkpointer=ck)
    b.fit(ec, [torch.randn(3, 4) for _ in range(6)])
    assert b.seen == [(False, True)]             # one intra-epoch checkpoint survived the epoch
    left = ck.list_checkpoints()
    assert len(left) == 1 and left[0][1]["end_of_epoch"] and "loss" in left[0][1]["meta"]


def test_optimizer_state_dict_is_torch_adam_layout():
    """EngineOptimizer's state_dict must load into torch.optim.Adam (and back)."""
    from mlvae_hip.engine import ParamLayout, VAEConfig
    from mlvae_hip.optim import EngineOptimizer
    cfg = VAEConfig(F=8, E=8, Z=4, H=8, L=2, C=8)
    lay = ParamLayout(cfg)

    class FakeEngine:  # host tensors standing in for the device buffers
        def __init__(self):
            self.cfg, self.layout = cfg, lay
            self.exp_avg = torch.randn(lay.total)
            self.exp_avg_sq = torch.rand(lay.total)
            self.step_ctr = torch.tensor([7], dtype=torch.int32)

        def view(self, name, buf):
            o = lay.offsets[name]
            return buf[o:o + lay.numel(name)].view(lay.shapes[name])
    e = FakeEngine()
    sd = EngineOptimizer(e).state_dict()
    params = [torch.nn.Parameter(torch.zeros(s)) for s in lay.shapes.values()]
    opt = torch.optim.Adam(params, lr=1e-3)
    opt.load_state_dict(sd)
    st = opt.state[params[5]]
    name5 = list(lay.shapes)[5]
    assert torch.equal(st["exp_avg"], e.view(name5, e.exp_avg)) and float(st["step"]) == 7.0
    e2 = FakeEngine()
    EngineOptimizer(e2).load_state_dict(opt.state_dict())
    for name in lay.shapes:
        assert torch.equal(e2.view(name, e2.exp_avg), e.view(name, e.exp_avg))
    assert int(e2.step_ctr) == 7


# ------------------------------------------------------------------ normaliser
def _norm_loop(x, lens, eps=1e-10):
    """Per-utterance loop (SpeechBrain 0.5 _compute_current_stats, restated)."""
    means, stds = [], []
    for b in range(x.shape[0]):
        n = int(torch.round(lens[b] * x.shape[1]).item())
        seg = x[b, :n]
        means.append(seg.mean(0))
        stds.append(torch.clamp(seg.std(0), min=eps))
    return torch.stack(means).mean(0), torch.stack(stds).mean(0)


def test_input_normalization_matches_per_utterance_loop():
    from brain import InputNormalization
    g = torch.Generator().manual_seed(0)
    norm = InputNormalization()
    state_mean = state_std = None
    for step in range(4):
        x = torch.randn(5, 37, 6, generator=g) * 3 + 1
        lens = torch.tensor([1.0, 0.6, 0.31, 0.9, 0.5])
        cm, cs = _norm_loop(x, lens)
        if step == 0:
            state_mean, state_std = cm, cs
        else:
            w = 1.0 / (step + 1)
            state_mean = (1 - w) * state_mean + w * cm
            state_std = (1 - w) * state_std + w * cs
        out = norm(x, lens, epoch=1)
        assert torch.allclose(norm.glob_mean, state_mean, rtol=1e-5, atol=1e-6)
        assert torch.allclose(norm.glob_std, state_std, rtol=1e-5, atol=1e-6)
        assert torch.allclose(out, (x - state_mean) / state_std, rtol=1e-5, atol=1e-5)
    assert norm.count == 4


def test_fused_path_calls_the_normaliser_like_compute_forward():
    """MDModel._normalised_feats (the fused path) must leave the normaliser in train mode on
    VALID batches, as the reference's SBModel.compute_forward does: after the same TRAIN and
    VALID batches, both routes hold the same global statistics and count."""
    from brain import InputNormalization, Stage
    from models.md_model import MDModel

    class Batch(dict):
        def to(self, device):
            return self
    g = torch.Generator().manual_seed(1)
    batches = [(Stage.TRAIN if i % 2 == 0 else Stage.VALID,
                Batch(feat=(torch.randn(3, 11, 4, generator=g), torch.tensor([1.0, 0.7, 0.5]))))
               for i in range(4)]
    n_fused, n_ref = InputNormalization(), InputNormalization()
    fake = types.SimpleNamespace(device="cpu", hparams=types.SimpleNamespace(
        normalizer=n_fused, epoch_counter=types.SimpleNamespace(current=1)))
    for stage, b in batches:
        MDModel._normalised_feats(fake, b, stage)
        feats, lens = b["feat"]
        n_ref(feats, lens, epoch=1)   # compute_forward: ref:src/models/test_vanilla_vae/model.py:24-25
    assert n_fused.count == n_ref.count == 4
    assert torch.equal(n_fused.glob_mean, n_ref.glob_mean)
    assert torch.equal(n_fused.glob_std, n_ref.glob_std)


# ------------------------------------------------------------------ bench process model
def test_bench_spawns_one_rank_per_gpu():
    """`bench.py --gpus 2` without torch.distributed.run starts two worker ranks itself
    (checked with the gloo dry run: no GPU touched)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["world"] == 2 and lines[0]["rank_sum"] == 3.0 and lines[0]["per_rank_batch"] == 128


# ------------------------------------------------------------------ loss weights
def test_weight_for_matches_reference_fixture():
    """MDModel._weight_for / compute_and_save_losses (the product's restatement of
    ref:src/models/md_model.py:189-213, incl. the '_kld' 2249/batch_size rule) against the
    totals the reference's own compute_and_save_losses produced (tests/golden/loss_weights.json)."""
    from models.md_model import MDModel
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "loss_weights.json")))
    for case in cases:
        fake = types.SimpleNamespace(hparams=types.SimpleNamespace(**case["hparams"]), stats_loggers={})
        fake._weight_for = types.MethodType(MDModel._weight_for, fake)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            total = MDModel.compute_and_save_losses(
                fake, {k: torch.tensor(v) for k, v in zip(case["keys"], case["values"])})
        assert abs(float(total) - case["total"]) <= 1e-6 * abs(case["total"]), case


def test_resume_from_intra_epoch_checkpoint_skips_trained_batches(tmp_path, monkeypatch):
    """resuming from an intra-epoch checkpoint re-runs that epoch (EpochCounter saved
    - 1) but must not train its first batches a second time: the checkpoint records how many
    batches of the epoch were done, and fit() skips them."""
    import brain.core as core
    from brain import Checkpointer, EpochCounter
    from brain.core import Brain, Stage

    clock = [1000.0]
    monkeypatch.setattr(core.time, "time", lambda: clock[0])
    data = [torch.full((3, 4), float(i)) for i in range(6)]

    class Toy(Brain):
        def compute_forward(self, batch, stage):
            return self.modules["lin"](batch)

        def compute_objectives(self, out, batch, stage):
            clock[0] += 40.0
            return out.pow(2).mean()

        def fit_batch(self, batch):
            self.trained.append(int(batch[0, 0].item()))
            if len(self.trained) == self.crash_after:
                raise KeyboardInterrupt   # the run dies after this batch
            return self.compute_objectives(self.compute_forward(batch, Stage.TRAIN), batch, Stage.TRAIN).detach()

    def make(crash_after):
        lin = torch.nn.Linear(4, 2)
        ec = EpochCounter(1)
        ck = Checkpointer(tmp_path, {"lin": lin, "epoch_counter": ec})
        b = Toy(modules={"lin": lin}, opt_class=lambda p: torch.optim.SGD(p, lr=0.1),
                run_opts={"device": "cpu", "ckpt_interval_minutes": 1.0}, checkpointer=ck)
        b.trained, b.crash_after = [], crash_after
        return b, ec

    b, ec = make(crash_after=5)
    try:
        b.fit(ec, data)
    except KeyboardInterrupt:
        pass
    # 40 s per batch, a checkpoint every 60 s: after batches 2 and 4 (the later one kept)
    assert b.trained == [0, 1, 2, 3, 4]
    b2, ec2 = make(crash_after=-1)
    b2.fit(ec2, data)
    assert b2.trained == [4, 5]   # batches 0-3 were in the checkpoint; 4 was lost with the crash


def _toy_brain(tmp_path, clock, epochs, bs_log):
    import brain.core as core
    from brain import Checkpointer, EpochCounter
    from brain.core import Brain, Stage

    class Toy(Brain):
        def compute_forward(self, batch, stage):
            return self.modules["lin"](batch["feat"][0])

        def compute_objectives(self, out, batch, stage):
            clock[0] += 40.0
            return out.pow(2).mean()

        def fit_batch(self, batch):
            bs_log.append(tuple(batch["id"]))
            if len(bs_log) == self.crash_after:
                raise KeyboardInterrupt
            return self.compute_objectives(self.compute_forward(batch, Stage.TRAIN), batch, Stage.TRAIN).detach()

    lin = torch.nn.Linear(4, 2)
    ec = EpochCounter(epochs)
    ck = Checkpointer(tmp_path, {"lin": lin, "epoch_counter": ec})
    b = Toy(modules={"lin": lin}, opt_class=lambda p: torch.optim.SGD(p, lr=0.1),
            run_opts={"device": "cpu", "ckpt_interval_minutes": 1.0}, checkpointer=ck)
    b.crash_after = -1
    del core
    return b, ec


def test_every_epoch_walks_the_dataset_and_a_resume_skips_by_index(tmp_path, monkeypatch):
    """The loaders are re-iterable (a bare generator left every epoch after the first empty), an
    intra-epoch resume skips the trained batches without collating them, and it is refused when
    the batch size differs from the saving run's (the count would skip the wrong
    utterances)."""
    import brain.core as core
    from utils.data_io import SyntheticSet
    clock = [1000.0]
    monkeypatch.setattr(core.time, "time", lambda: clock[0])
    ds = SyntheticSet(12, 4, 3, 6, seed=3)
    seen = []
    b, ec = _toy_brain(tmp_path / "a", clock, 2, seen)
    b.fit(ec, ds, train_loader_kwargs={"batch_size": 3})
    assert len(seen) == 8 and seen[:4] == seen[4:]          # both epochs saw all 4 batches
    # crash after 3 batches of a run, resume: batches 0-1 were checkpointed (40 s per batch,
    # one checkpoint a minute), so the resumed epoch starts at batch 2
    seen2 = []
    b2, ec2 = _toy_brain(tmp_path / "b", clock, 1, seen2)
    b2.crash_after = 3
    try:
        b2.fit(ec2, ds, train_loader_kwargs={"batch_size": 3})
    except KeyboardInterrupt:
        pass
    seen3 = []
    b3, ec3 = _toy_brain(tmp_path / "b", clock, 1, seen3)
    collated = []
    from brain import dataio
    real = dataio.PaddedBatch.__init__
    monkeypatch.setattr(dataio.PaddedBatch, "__init__",
                        lambda self, items, *a, **k: (collated.append(len(items)), real(self, items, *a, **k))[1])
    b3.fit(ec3, ds, train_loader_kwargs={"batch_size": 3})
    assert seen3 == seen[2:4] and len(collated) == 2       # only the two remaining batches built
    # the same checkpoint under another batch size: refused
    b4, ec4 = _toy_brain(tmp_path / "c", clock, 1, [])
    b4.crash_after = 3
    try:
        b4.fit(ec4, ds, train_loader_kwargs={"batch_size": 3})
    except KeyboardInterrupt:
        pass
    b5, ec5 = _toy_brain(tmp_path / "c", clock, 1, [])
    with pytest.raises(RuntimeError, match="batch_size"):
        b5.fit(ec5, ds, train_loader_kwargs={"batch_size": 4})
