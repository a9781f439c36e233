"""VanillaVAE + BiLSTM-decoder recipe (semantics of ref:src/models/test_vanilla_vae/model.py:12-55).

compute_forward: normalise (global InputNormalization) -> encoder -> decoder(sampled_h, feats).
compute_objectives: masked means of the KL and reconstruction terms, weighted and summed
by compute_and_save_losses.  With the fused engine active (the default for this recipe,
see models/md_model.py) fit_batch/evaluate_batch bypass these two hooks and run the same
computation as one stream of HIP launches.
"""
from models.md_model import MDModel
from utils.data_utils import apply_lens_to_loss
from utils.metric_stats.loss_metric_stats import LossMetricStats


class SBModel(MDModel):
    def on_stage_start(self, stage, epoch=None):
        super().on_stage_start(stage, epoch)
        self.stats_loggers["kld_loss_stats"] = LossMetricStats("kld_loss")
        self.stats_loggers["recon_loss_stats"] = LossMetricStats("recon_loss")

    def compute_forward(self, batch, stage):
        batch = batch.to(self.device)
        feats, lens = batch["feat"]
        feats = self.hparams.normalizer(feats, lens, epoch=self.hparams.epoch_counter.current)
        enc = self.modules["encoder"](feats.contiguous())
        dec = self.modules["decoder"](enc["sampled_h"], feats.contiguous())
        return {"encoder_out": enc, "decoder_out": dec}

    def compute_objectives(self, predictions, batch, stage):
        feats, lens = batch["feat"]
        losses = {
            "kld_loss": apply_lens_to_loss(predictions["encoder_out"]["loss"], lens),
            "recon_loss": apply_lens_to_loss(predictions["decoder_out"]["losses"]["recon_loss"], lens),
        }
        return self.compute_and_save_losses(losses)
