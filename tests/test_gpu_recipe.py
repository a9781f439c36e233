"""End to end through the drop-in surface: train.py-style experiment assembly (HyperPyYAML,
Brain loop, SBModel) on synthetic log-mel, fused HIP step, checkpoint + evaluate."""
import os
import subprocess
import sys

import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu


def _run(args, cwd):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    return subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True,
                          text=True, timeout=600)


def test_train_and_test_scripts(tmp_path):
    from gpu_utils import need_gpu
    need_gpu()
    common = ["config/run.yaml", "--model_class", "test_vanilla_vae", "--model_name", "vae_ci",
              "--model", "!include:../models/test_vanilla_vae/model.yaml",
              "--output_dir", str(tmp_path / "out"),
              "--extra_overrides", "{model: {n_epochs: 2, input_size: 80, dec_rnn_hidden_size: 64}}"]
    r = _run(["train.py"] + common, PKG)
    assert r.returncode == 0, r.stderr[-3000:]
    log = open(tmp_path / "out" / "train_log.txt").read()
    assert "epoch: 2" in log and "valid loss" in log, log[-2000:]
    ck = os.listdir(tmp_path / "out" / "checkpoints")
    assert len(ck) >= 1
    r = _run(["test.py"] + common, PKG)
    assert r.returncode == 0, r.stderr[-3000:]
    m = open(tmp_path / "out" / "test_output" / "test_metrics.txt").read()
    assert "kld_loss.loss" in m and "recon_loss.loss" in m


@pytest.mark.parametrize("model_class,precision", [("test_conv_vae", "bf16"), ("test_vanilla_vae", "fp8")])
def test_recipe_variants(tmp_path, model_class, precision):
    """configs[3]'s Conv1d-encoder recipe (models/test_conv_vae) and configs[4]'s fp8 mode
    (`precision: fp8`) through train.py on the fused engine."""
    from gpu_utils import need_gpu
    need_gpu()
    args = ["train.py", "config/run.yaml", "--model_class", model_class, "--model_name", f"vae_{precision}",
            "--model", f"!include:../models/{model_class}/model.yaml", "--output_dir", str(tmp_path / "out"),
            "--extra_overrides", "{model: {n_epochs: 1, input_size: 80, dec_rnn_hidden_size: 512, "
                                 "precision: " + precision + "}}"]
    r = _run(args, PKG)
    assert r.returncode == 0, r.stderr[-3000:]
    log = open(tmp_path / "out" / "train_log.txt").read()
    assert "epoch: 1" in log and "valid loss" in log, log[-2000:]
    assert ("ConvVAE" in log) == (model_class == "test_conv_vae")
