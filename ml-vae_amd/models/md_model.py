"""MDModel: the recipe-level Brain (semantics of ref:src/models/md_model.py:15-213).

Hooks kept: init_optimizers (single 'optimizer' partial, dict or list of 'optimizers';
'No optimizers defined.' otherwise), fit_batch, on_fit_start / on_stage_start /
on_stage_end (train_log.txt, checkpoint after VALID with min/max keys, test_output/ files),
compute_and_save_losses (weights '<key>_weight', default 1 with a warning; '_kld' weights
divided by 2249 / batch_size).

MI355X path: when the modules are the VAE recipe's (VanillaVAE encoder + Decoder) and the
optimizer is Adam, init_optimizers builds a mlvae_hip.VAEEngine over the modules'
parameters and fit_batch / evaluate_batch run the fused HIP step (forward, ELBO, backward,
clip, Adam: one stream of libmlvae launches, no host sync).  Anything else runs the
module-level HIP ops under autograd with mlvae_hip.optim.Adam.
"""
import functools
import logging
import warnings
from pathlib import Path

import torch

from brain import Brain, Stage
from brain.train_logger import FileTrainLogger
from utils.metric_stats.loss_metric_stats import LossMetricStats

logger = logging.getLogger(__name__)

N_SAMPLES_KLD = 2249  # the reference's hard-coded corpus size for '_kld' weights


class MDModel(Brain):
    def __init__(self, label_encoder=None, **kwargs):
        super().__init__(**kwargs)
        self.label_encoder = label_encoder
        self.engine = None
        self.stats_loggers = {}

    # ------------------------------------------------------------------ optimizers
    def _optimizer_infos(self):
        hp = self.hparams
        if hasattr(hp, "optimizers"):
            infos = hp.optimizers
            if isinstance(infos, list):
                infos = {f"optimizer_{i}": v for i, v in enumerate(infos)}
            return infos
        if hasattr(hp, "optimizer"):
            return {"optimizer": hp.optimizer}
        raise ValueError("No optimizers defined.")

    def _fused_candidate(self, infos):
        from modules.decoder import Decoder
        from modules.conv_vae import ConvVAE
        from modules.vanilla_vae import VanillaVAE
        from mlvae_hip import optim as hip_optim
        if set(self.modules.keys()) != {"encoder", "decoder"} or len(infos) != 1:
            return None
        if not (isinstance(self.modules["encoder"], (VanillaVAE, ConvVAE)) and
                isinstance(self.modules["decoder"], Decoder)):
            return None
        info = next(iter(infos.values()))
        if not isinstance(info, functools.partial):
            return None
        if info.func not in (torch.optim.Adam, hip_optim.Adam):
            return None
        if info.keywords.get("weight_decay", 0) or info.keywords.get("amsgrad", False):
            return None
        return info

    def init_optimizers(self):
        infos = self._optimizer_infos()
        fused = self._fused_candidate(infos) if getattr(self, "use_fused_step", True) else None
        if fused is not None:
            from mlvae_hip.engine import VAEEngine
            from mlvae_hip.optim import EngineOptimizer
            kw = fused.keywords
            prec = getattr(self.hparams, "precision", "fp32")
            fp8 = prec == "fp8"  # configs[4]: bf16 step with the fp8 layer-1 input projection
            if fp8:
                prec = "bf16"
            if self.auto_mix_prec and prec != "bf16":
                # --auto_mix_prec (the reference's fp16 autocast + GradScaler, ref:src/models/
                # md_model.py:60-76): the fused step's mixed-precision mode is bf16 operands with
                # fp32 accumulation / master weights; bf16 keeps fp32's exponent range, so the
                # loss needs no scaling
                logger.info("auto_mix_prec: fused step in bf16 operand mode")
                prec = "bf16"
            self.engine = VAEEngine.from_modules(
                self.modules["encoder"], self.modules["decoder"], device=self.device,
                prec=prec,
                kld_weight=self._weight_for("kld_loss"), recon_weight=self._weight_for("recon_loss"),
                lr=kw.get("lr", 1e-3), betas=kw.get("betas", (0.9, 0.999)), eps=kw.get("eps", 1e-8),
                max_grad_norm=self.max_grad_norm,
                seed=int(torch.randint(0, 2 ** 62, (1,)).item()), fp8=fp8)
            self.optimizers = {"optimizer": EngineOptimizer(self.engine)}
            if self.world_size > 1:  # data parallel: global offsets, broadcast weights, grad all-reduce
                from mlvae_hip import dist as mdist
                mdist.attach(self.engine, self.rank, self.world_size,
                             int(getattr(self.hparams, "batch_size", 8)))
        else:
            from mlvae_hip import ops
            from mlvae_hip import optim as hip_optim
            # module mode: the HIP ops' operand precision from the yaml's `precision` (fp8 has
            # no module-mode kernels: its bf16 step)
            prec = getattr(self.hparams, "precision", None)
            if prec is not None:
                ops.set_precision("bf16" if prec == "fp8" else prec)
            self.optimizers = {}
            for key, info in infos.items():
                if isinstance(info, dict):
                    if "modules" in info:
                        params = [p for m in info["modules"] for p in self.modules[m].parameters()]
                    else:
                        params = self.modules.parameters()
                    opt = info["opt_class"](params)
                else:
                    if isinstance(info, functools.partial) and info.func is torch.optim.Adam:
                        info = functools.partial(hip_optim.Adam, *info.args, **info.keywords)
                    opt = info(self.modules.parameters())
                self.optimizers[key] = opt
            if self.auto_mix_prec:
                # SpeechBrain builds the GradScaler with the Brain, before on_fit_start recovers:
                # registered here (init_optimizers runs right before recover_if_possible), a
                # resumed run restores its loss scale and growth tracker
                self._amp_scaler()
        if self.checkpointer is not None:
            for key, opt in self.optimizers.items():
                self.checkpointer.add_recoverable(key, opt)

    # ------------------------------------------------------------------ batches
    def fit_batch(self, batch):
        if self.engine is not None:
            feats, lens, norm = self._engine_inputs(batch)
            loss = self.engine.train_step(feats, lens, normalizer=norm,
                                          epoch=self.hparams.epoch_counter.current)
            self._log_losses(loss)
            self.optimizer_step += 1
            return loss[2].detach()
        opts = list(self.optimizers.values())
        if self.auto_mix_prec:
            # ref:src/models/md_model.py:60-76: zero_grad, autocast forward, scaled backward,
            # unscale, check_gradients, scaler.step, scaler.update.  The autocast region is the
            # HIP ops' bf16-operand mode (fp32 accumulation); the dynamic loss scale is kept.
            from mlvae_hip import ops
            scaler = self._amp_scaler()
            for opt in opts:
                opt.zero_grad()
            with ops.precision("bf16"):
                outputs = self.compute_forward(batch, Stage.TRAIN)
                loss = self.compute_objectives(outputs, batch, Stage.TRAIN)
                scaler.scale(loss).backward()
            self._dp_mean_grads()
            for opt in opts:
                scaler.unscale_(opt)
            if self.check_gradients(loss):
                for opt in opts:
                    scaler.step(opt)
            scaler.update()
            self.optimizer_step += 1
            return loss.detach()
        outputs = self.compute_forward(batch, Stage.TRAIN)
        loss = self.compute_objectives(outputs, batch, Stage.TRAIN)
        loss.backward()
        self._dp_mean_grads()
        if self.check_gradients(loss):
            for opt in opts:
                opt.step()
        for opt in opts:
            opt.zero_grad()
        self.optimizer_step += 1
        return loss.detach()

    def _dp_mean_grads(self):
        if self.world_size > 1:  # module mode under DP: DDP's mean of the ranks' gradients
            import torch.distributed as tdist
            for p_ in self.modules.parameters():
                if p_.grad is not None:
                    tdist.all_reduce(p_.grad)
                    p_.grad /= self.world_size

    def _amp_scaler(self):
        """SpeechBrain's GradScaler for auto_mix_prec (a checkpoint recoverable, 'scaler')."""
        if getattr(self, "scaler", None) is None:
            self.scaler = torch.amp.GradScaler("cuda")
            if self.checkpointer is not None:
                self.checkpointer.add_recoverable("scaler", self.scaler)
        return self.scaler

    def evaluate_batch(self, batch, stage):
        if self.engine is not None:
            feats, lens, norm = self._engine_inputs(batch)
            loss = self.engine.eval_step(feats, lens, normalizer=norm,
                                         epoch=self.hparams.epoch_counter.current)
            self._log_losses(loss)
            return loss[2].detach()
        return super().evaluate_batch(batch, stage)

    def _engine_inputs(self, batch):
        """(feats, lens, normaliser) for the fused step: the recipe's InputNormalization
        (brain.features) runs inside the step on the device (csrc/norm.hip) with the module's
        own state and semantics; any other normaliser object is applied here first."""
        from brain.features import InputNormalization
        from mlvae_hip._lib import lib
        batch = batch.to(self.device)
        feats, lens = batch["feat"]
        norm = getattr(self.hparams, "normalizer", None)
        # the device normaliser applies (x - mean) / std: a module with mean_norm or std_norm
        # off runs its own forward instead
        if isinstance(norm, InputNormalization) and norm.mean_norm and norm.std_norm \
                and lib().mlvae_norm_supported(feats.shape[-1]):
            return feats.contiguous(), lens, norm
        if norm is not None:
            feats = norm(feats, lens, epoch=self.hparams.epoch_counter.current)
        return feats.contiguous(), lens, None

    def _normalised_feats(self, batch, stage):
        batch = batch.to(self.device)
        feats, lens = batch["feat"]
        norm = getattr(self.hparams, "normalizer", None)
        if norm is not None:
            # called exactly as SBModel.compute_forward does (ref:src/models/test_vanilla_vae/
            # model.py:24-25): the normaliser is not one of the Brain's modules, so it stays in
            # train mode and its global statistics also update on VALID/TEST batches
            feats = norm(feats, lens, epoch=self.hparams.epoch_counter.current)
        return feats.contiguous(), lens

    def _log_losses(self, loss):
        for i, key in enumerate(("kld_loss", "recon_loss")):
            st = self.stats_loggers.get(key + "_stats")
            if st is not None:
                st.append(loss[i])

    # ------------------------------------------------------------------ losses
    def _weight_for(self, loss_key):
        weight_key = loss_key.replace("_loss", "_weight")
        weight = getattr(self.hparams, weight_key, "none")
        if weight == "none":
            warnings.warn(f"{weight_key} not found, use 1 as default")
            weight = 1
        if "_kld" in weight_key:
            weight /= (N_SAMPLES_KLD / self.hparams.batch_size)
        return weight

    def compute_and_save_losses(self, losses):
        total = 0
        for key, value in losses.items():
            total = total + self._weight_for(key) * value
            st = self.stats_loggers.get(key + "_stats")
            if st is not None:
                st.append(value)
            else:
                warnings.warn(f"loss stats logger {key}_stats not found")
        return total

    # ------------------------------------------------------------------ stage hooks
    def on_fit_start(self):
        super().on_fit_start()
        out = Path(self.hparams.output_dir)
        out.mkdir(parents=True, exist_ok=True)
        self.train_logger = FileTrainLogger(save_file=out / "train_log.txt")
        logger.info(str(self.modules))
        with open(out / "train_log.txt", "w") as f:
            f.write(str(self.modules) + "\n")

    def on_stage_start(self, stage, epoch=None):
        self.stats_loggers = {}
        for key in self.hparams.metric_keys:
            if key.endswith("_loss"):
                self.stats_loggers[key + "_stats"] = LossMetricStats(key)

    def _collect_metrics(self, stage_loss):
        log = {"loss": round(stage_loss, 3)}
        for metric_key in self.hparams.metric_keys:
            parts = metric_key.split(".")
            st = self.stats_loggers.get(f"{parts[0].lower()}_stats")
            if st is None:
                continue
            if len(parts) == 1:
                for k, v in st.summarize(None).items():
                    log[f"{metric_key}.{k}"] = round(v, 2)
            else:
                log[metric_key] = round(float(st.summarize(parts[1])), 2)
        return log

    def on_stage_end(self, stage, stage_loss, epoch=None):
        if self.engine is not None:
            # the fused step's device-side failure words, read once per stage (no per-step
            # sync): recurrence hand-off timeout -> RuntimeError; more than nonfinite_patience
            # skipped non-finite steps -> ValueError (SpeechBrain check_gradients semantics)
            self.engine.check_health(self.nonfinite_patience,
                                     where=f" in {stage.name} stage, epoch {epoch}")
        name = stage.name.lower()
        if epoch is None:
            epoch = self.hparams.epoch_counter.current
        log = self._collect_metrics(stage_loss)
        if stage in (Stage.TRAIN, Stage.VALID):
            if self.rank == 0:
                self.train_logger.log_stats(stats_meta={"stage": name, "epoch": epoch},
                                            **{f"{name}_stats": log})
            if stage == Stage.VALID:
                max_keys = [self.hparams.max_key] if getattr(self.hparams, "max_key", None) else []
                min_keys = [self.hparams.min_key] if getattr(self.hparams, "min_key", None) else []
                if not max_keys and not min_keys:
                    raise ValueError("no max_key or min_key provided")
                if self.checkpointer is not None and self.rank == 0:  # rank 0 writes
                    self.checkpointer.save_and_keep_only(meta=log, max_keys=max_keys,
                                                         min_keys=min_keys)
                from brain.distributed import barrier
                barrier()
        if stage == Stage.TEST and self.rank == 0:
            out = Path(self.hparams.output_dir) / "test_output"
            out.mkdir(parents=True, exist_ok=True)
            with open(out / "test_metrics.txt", "w") as f:
                f.write(f"Epoch: {epoch}\n")
                for k, v in log.items():
                    f.write(f"{k}: {v}\n")
                f.write(f"Epoch: {epoch}\t" + "\t".join(str(v) for v in log.values()) + "\n")
            for key, st in self.stats_loggers.items():
                with open(out / f"{key.replace('_stats', '')}.txt", "w") as f:
                    st.write_stats(f)
