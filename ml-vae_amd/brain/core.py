"""Brain: the epoch/batch loop around compute_forward / compute_objectives."""
import enum
import logging
import time
from types import SimpleNamespace

import torch

logger = logging.getLogger(__name__)


INTRA_EPOCH_CKPT_FLAG = "brain_intra_epoch_ckpt"   # SpeechBrain's meta key of intra-epoch saves


class Stage(enum.Enum):
    TRAIN = enum.auto()
    VALID = enum.auto()
    TEST = enum.auto()


DEFAULT_RUN_OPTS = {
    "debug": False,
    "debug_batches": 2,
    "debug_epochs": 2,
    "device": "cuda:0",
    "auto_mix_prec": False,
    "max_grad_norm": 5.0,
    "nonfinite_patience": 3,
    "noprogressbar": True,
    "ckpt_interval_minutes": 0,
    "distributed_launch": False,   # brain.distributed.init_from_env fills rank / world_size
    "distributed_backend": None,
    "rank": 0,
    "world_size": 1,
}


class Brain:
    """SpeechBrain-style training driver.  Subclasses implement compute_forward and
    compute_objectives; fit_batch may be overridden (the VAE recipe routes it to the fused
    HIP train step, mlvae_hip.engine)."""

    def __init__(self, modules=None, opt_class=None, hparams=None, run_opts=None,
                 checkpointer=None):
        self.opt_class = opt_class
        self.checkpointer = checkpointer
        opts = dict(DEFAULT_RUN_OPTS)
        opts.update(run_opts or {})
        for k, v in opts.items():
            setattr(self, k, v)
        self.run_opts = opts
        self.hparams = SimpleNamespace(**hparams) if hparams is not None else None
        self.modules = torch.nn.ModuleDict(modules or {}).to(self.device)
        self.step = 0
        self.optimizer_step = 0
        self.avg_train_loss = 0.0
        self.nonfinite_count = 0
        self._loss_sum = None  # device-side running loss (no per-batch host sync)

    # --------------------------------------------------------------- hooks
    def compute_forward(self, batch, stage):
        raise NotImplementedError

    def compute_objectives(self, predictions, batch, stage):
        raise NotImplementedError

    def on_fit_start(self):
        self.init_optimizers()
        self._resume_batches = 0
        if self.checkpointer is not None:
            self.checkpointer.recover_if_possible(device=torch.device(self.device))
            # an intra-epoch checkpoint (--ckpt_interval_minutes): the EpochCounter re-runs that
            # epoch, whose first `batches_done` batches were already trained -- they are skipped
            # (SpeechBrain resumes through its saveable dataloader's position; here the dataset's
            # batch order is reproducible per epoch, so skipping the same count is the same thing)
            meta = getattr(self.checkpointer, "recovered_meta", None) or {}
            if INTRA_EPOCH_CKPT_FLAG in meta:
                self._resume_batches = int(meta.get("batches_done", 0))
                self._resume_meta = meta

    def init_optimizers(self):
        if self.opt_class is not None:
            self.optimizer = self.opt_class(self.modules.parameters())
            if self.checkpointer is not None:
                self.checkpointer.add_recoverable("optimizer", self.optimizer)

    def on_stage_start(self, stage, epoch=None):
        pass

    def on_stage_end(self, stage, stage_loss, epoch=None):
        pass

    def on_evaluate_start(self, max_key=None, min_key=None):
        if self.checkpointer is not None:
            self.checkpointer.recover_if_possible(max_key=max_key, min_key=min_key,
                                                  device=torch.device(self.device))

    # --------------------------------------------------------------- batches
    def fit_batch(self, batch):
        outputs = self.compute_forward(batch, Stage.TRAIN)
        loss = self.compute_objectives(outputs, batch, Stage.TRAIN)
        loss.backward()
        if self.check_gradients(loss):
            self.optimizer.step()
        self.optimizer.zero_grad()
        self.optimizer_step += 1
        return loss.detach()

    def evaluate_batch(self, batch, stage):
        out = self.compute_forward(batch, stage=stage)
        loss = self.compute_objectives(out, batch, stage=stage)
        return loss.detach()

    def check_gradients(self, loss):
        """Skip non-finite losses (up to nonfinite_patience), else clip the global grad norm
        to max_grad_norm (SpeechBrain semantics)."""
        if not torch.isfinite(loss):
            self.nonfinite_count += 1
            logger.warning(f"Loss is {loss}.")
            if self.nonfinite_count > self.nonfinite_patience:
                raise ValueError("Loss is not finite and patience is exhausted. "
                                 "To debug, wrap `fit()` with autograd's `detect_anomaly()`")
            logger.warning("Patience not yet exhausted, ignoring this batch.")
            return False
        params = [p for p in self.modules.parameters() if p.grad is not None]
        if params:
            from mlvae_hip.optim import clip_grad_norm_
            clip_grad_norm_(params, self.max_grad_norm)
        return True

    def update_average(self, loss, avg_loss):
        """Running mean of the batch losses.  Kept on the device: the host reads it once per
        stage instead of once per batch (the reference syncs every batch)."""
        loss = loss.detach().reshape(())
        if self._loss_sum is None or self.step == 1:
            self._loss_sum = torch.zeros((), device=loss.device)
            self._loss_n = torch.zeros((), device=loss.device)
        fin = torch.isfinite(loss)
        self._loss_sum += torch.where(fin, loss, torch.zeros_like(loss))
        self._loss_n += fin.to(loss.dtype)
        return self._loss_sum, self._loss_n

    def _stage_loss(self, acc):
        if acc is None or isinstance(acc, float):
            return float(acc or 0.0)
        s, n = acc
        n = float(n.item())
        return float(s.item()) / n if n > 0 else float("nan")

    # --------------------------------------------------------------- loops
    def fit(self, epoch_counter, train_set, valid_set=None, progressbar=None,
            train_loader_kwargs=None, valid_loader_kwargs=None):
        train_set = self.make_dataloader(train_set, Stage.TRAIN, **(train_loader_kwargs or {}))
        if valid_set is not None:
            valid_set = self.make_dataloader(valid_set, Stage.VALID, **(valid_loader_kwargs or {}))
        self.on_fit_start()
        for epoch in epoch_counter:
            self.on_stage_start(Stage.TRAIN, epoch)
            self.modules.train()
            self.nonfinite_count = 0
            self.step = 0
            acc = None
            last_ckpt = time.time()
            skip, self._resume_batches = self._resume_batches, 0
            self._batches_skipped = skip
            if skip:
                self._check_resume_signature(train_set)
            if skip and hasattr(train_set, "skip_next"):
                train_set.skip_next(skip)   # index-level: the trained batches are not collated
                skip = 0
            for i, batch in enumerate(train_set):
                if i < skip:  # trained before the intra-epoch checkpoint this run resumed from
                    continue
                self.step += 1
                loss = self.fit_batch(batch)
                acc = self.update_average(loss, acc)
                if self.debug and self.step == self.debug_batches:
                    break
                # --ckpt_interval_minutes: an intra-epoch checkpoint on the host timer (SpeechBrain
                # Brain.fit); rank 0 writes it, replacing only the previous intra-epoch one
                if (self.checkpointer is not None and self.ckpt_interval_minutes > 0
                        and time.time() - last_ckpt >= self.ckpt_interval_minutes * 60.0):
                    if self.rank == 0:
                        self._save_intra_epoch_ckpt(train_set)
                    last_ckpt = time.time()
            self.avg_train_loss = self._stage_loss(acc)
            self.on_stage_end(Stage.TRAIN, self.avg_train_loss, epoch)
            self.avg_train_loss = 0.0
            self.step = 0
            if valid_set is not None:
                self.on_stage_start(Stage.VALID, epoch)
                self.modules.eval()
                acc = None
                with torch.no_grad():
                    for batch in valid_set:
                        self.step += 1
                        loss = self.evaluate_batch(batch, stage=Stage.VALID)
                        acc = self.update_average(loss, acc)
                        if self.debug and self.step == self.debug_batches:
                            break
                    self.step = 0
                    self.on_stage_end(Stage.VALID, self._stage_loss(acc), epoch)
            if self.debug and epoch == self.debug_epochs:
                break

    def _save_intra_epoch_ckpt(self, train_set=None):
        meta = {INTRA_EPOCH_CKPT_FLAG: True, "batches_done": self.step + self._batches_skipped}
        sig = getattr(train_set, "signature", None)
        if sig is not None:   # what a resume must match to skip the same utterances
            meta.update({"loader_" + k: v for k, v in sig().items()})
        self.checkpointer.save_and_keep_only(
            end_of_epoch=False, num_to_keep=1, meta=meta,
            ckpt_predicate=lambda meta: INTRA_EPOCH_CKPT_FLAG in meta)

    def _check_resume_signature(self, train_set):
        """An intra-epoch resume skips `batches_done` batches by count: refuse it when the batch
        size, world size, sorting or epoch length differ from the saving run's (the count would
        then skip the wrong utterances or retrain some)."""
        meta = getattr(self, "_resume_meta", None) or {}
        sig = getattr(train_set, "signature", None)
        if sig is None:
            return
        bad = {k: (meta["loader_" + k], v) for k, v in sig().items()
               if "loader_" + k in meta and meta["loader_" + k] != v}
        if bad:
            raise RuntimeError("intra-epoch checkpoint was saved with a different data layout "
                               + ", ".join(f"{k}: saved {a!r}, now {b!r}" for k, (a, b) in bad.items())
                               + "; resume with the same batch size / world size / sorting, or "
                               "start the epoch over from an end-of-epoch checkpoint")

    def evaluate(self, test_set, max_key=None, min_key=None, progressbar=None,
                 test_loader_kwargs=None):
        test_set = self.make_dataloader(test_set, Stage.TEST, **(test_loader_kwargs or {}))
        self.on_evaluate_start(max_key=max_key, min_key=min_key)
        self.on_stage_start(Stage.TEST, epoch=None)
        self.modules.eval()
        acc = None
        with torch.no_grad():
            for batch in test_set:
                self.step += 1
                loss = self.evaluate_batch(batch, stage=Stage.TEST)
                acc = self.update_average(loss, acc)
                if self.debug and self.step == self.debug_batches:
                    break
            self.step = 0
            avg = self._stage_loss(acc)
            self.on_stage_end(Stage.TEST, avg, None)
        return avg

    def make_dataloader(self, dataset, stage, **loader_kwargs):
        if hasattr(dataset, "batches"):
            if self.world_size > 1:  # this rank's slice of every global batch
                loader_kwargs = dict(loader_kwargs, rank=self.rank, world=self.world_size)
            return dataset.batches(stage=stage, **loader_kwargs)
        return dataset
