"""The recipe configs (ml-vae_amd/config/run.yaml + models/test_vanilla_vae/model.yaml)
resolve to the same hyper-parameters and module structure as the reference's own files did
when the fixture tests/golden/resolved_config.json was generated (make_golden.py)."""
import functools
import json
import os

import torch

from conftest import PKG
from hyperpyyaml import load_hyperpyyaml
from hyperpyyaml.core import recursive_update

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resolved_config.json")


def _load():
    extra = {"model": {"n_epochs": 1, "input_size": 80}}
    ov = ("dataset: synthetic\nmodel_class: test_vanilla_vae\nmodel_name: vae\n"
          "model: !include:../models/test_vanilla_vae/model.yaml\n")
    with open(os.path.join(PKG, "config", "run.yaml")) as f:
        hp = load_hyperpyyaml(f, [extra, ov])
    recursive_update(hp, extra)
    return hp


def test_recipe_matches_reference_resolution():
    ref = json.load(open(GOLD))
    hp = _load()
    m, rm = hp["model"], ref["model"]
    for k in ("n_epochs", "input_size", "latent_size", "enc_fc_size", "dec_rnn_hidden_size",
              "dec_rnn_num_layers", "dec_rnn_dropout", "dec_fc_size", "lr", "kld_weight",
              "metric_keys", "min_key", "batch_size", "model_name", "output_dir", "n_phonemes"):
        assert m[k] == rm[k], k
    # identical module structure (same repr) -> same parameter names and shapes
    assert repr(m["encoder"]) == rm["encoder"]["repr"]
    assert repr(m["decoder"]) == rm["decoder"]["repr"]
    assert isinstance(m["optimizer"], functools.partial)
    assert m["optimizer"].keywords["lr"] == rm["optimizer"]["keywords"]["lr"]
    assert m["modules"]["encoder"] is m["encoder"]
    assert m["checkpointer"].recoverables["decoder"] is m["decoder"]
    assert m["epoch_counter"].limit == 1
    assert hp["batch_size"] == ref["batch_size"] and hp["seed"] == ref["seed"]


def test_seed_gives_reference_init():
    """`__set_seed: !apply:torch.manual_seed` then the same constructor order: the modules'
    initial weights equal the reference's under the same seed (nn.Linear / nn.LSTM init)."""
    hp = _load()
    torch.manual_seed(123456)
    from modules.vanilla_vae import VanillaVAE
    a = VanillaVAE([80, 64, 64], 32)
    torch.manual_seed(123456)
    b = VanillaVAE([80, 64, 64], 32)
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)
    assert list(hp["model"]["encoder"].state_dict().keys()) == list(a.state_dict().keys())
