"""Experiment assembly (semantics of ref:src/prepare_experiment.py:10-60): CLI -> hparams
(HyperPyYAML, --extra_overrides applied before and after construction) -> experiment dir
-> datasets -> models.<model_class>.model.SBModel."""
import importlib

import yaml

import brain
from hyperpyyaml import load_hyperpyyaml
from hyperpyyaml.core import recursive_update
from utils.data_io import prepare_datasets


def prepare_experiment(args, prepare_exp_dir):
    hparams_file, run_opts, overrides = brain.parse_arguments(args)
    # data-parallel launch (torch.distributed.run): process group, rank's device (brain.distributed)
    from brain.distributed import init_from_env, is_main
    init_from_env(run_opts)
    parsed = yaml.safe_load(_strip_tags(overrides)) if overrides else None
    extra_overrides = {}
    if parsed and "extra_overrides" in parsed:
        extra_overrides = parsed["extra_overrides"] or {}
        if isinstance(extra_overrides, str):
            extra_overrides = yaml.safe_load(extra_overrides) or {}
        overrides = "\n".join(l for l in overrides.splitlines()
                              if not l.startswith("extra_overrides:"))
    with open(hparams_file) as fin:
        hparams = load_hyperpyyaml(fin, [extra_overrides, overrides])
    recursive_update(hparams, extra_overrides)

    if prepare_exp_dir and is_main():
        brain.create_experiment_directory(experiment_directory=hparams["output_dir"],
                                          hyperparams_to_save=hparams_file,
                                          overrides=[extra_overrides, overrides])
    prepared = {"hparams": hparams}
    try:
        prep = importlib.import_module(f"datasets.{hparams['dataset']}.prepare")
    except ModuleNotFoundError:
        prep = None  # a corpus the reference computed already: utils.data_io reads its pickles
    if prep is not None:
        prep.prepare(**hparams["prepare"])
    datasets, label_encoder = prepare_datasets(hparams)
    prepared["datasets"] = datasets
    if "model_class" in hparams:
        SBModel = importlib.import_module(f"models.{hparams['model_class']}.model").SBModel
        prepared["model"] = SBModel(label_encoder=label_encoder,
                                    modules=hparams["model"]["modules"],
                                    hparams=hparams["model"], run_opts=run_opts,
                                    checkpointer=hparams["model"]["checkpointer"])
    return prepared


def _strip_tags(text):
    # only used to find extra_overrides; tagged values (e.g. !include:) are irrelevant here
    import re
    return re.sub(r"!\S+", "", text)
