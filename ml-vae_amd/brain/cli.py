"""Command line: `train.py hparams.yaml [--run_opt value ...] [--yaml_key value ...]`
(SpeechBrain parse_arguments semantics: run options are consumed, every other
--key value pair becomes a yaml override string)."""
import argparse
import os
import shutil
import sys

RUN_OPTS = {
    "--device": str, "--debug": "flag", "--debug_batches": int, "--debug_epochs": int,
    "--auto_mix_prec": "flag", "--max_grad_norm": float, "--nonfinite_patience": int,
    "--noprogressbar": "flag", "--log_config": str, "--distributed_launch": "flag",
    "--distributed_backend": str, "--data_parallel_backend": "flag",
    "--ckpt_interval_minutes": float, "--precision": str,
}


def parse_arguments(arg_list=None):
    if arg_list is None:
        arg_list = sys.argv[1:]
    p = argparse.ArgumentParser(description="Run an ML-VAE recipe")
    p.add_argument("param_file", type=str)
    for name, kind in RUN_OPTS.items():
        if kind == "flag":
            p.add_argument(name, default=None, action="store_true")
        else:
            p.add_argument(name, type=kind, default=None)
    run_opts, overrides = p.parse_known_args(arg_list)
    run_opts = {k: v for k, v in vars(run_opts).items() if v is not None}
    param_file = run_opts.pop("param_file")
    # remaining "--key value" pairs -> yaml override text
    lines = []
    i = 0
    while i < len(overrides):
        tok = overrides[i]
        if not tok.startswith("--"):
            raise ValueError(f"unexpected argument {tok}")
        key = tok[2:]
        if "=" in key:
            key, val = key.split("=", 1)
            i += 1
        else:
            val = overrides[i + 1] if i + 1 < len(overrides) else ""
            i += 2
        lines.append(f"{key}: {val}")
    return param_file, run_opts, "\n".join(lines)


def create_experiment_directory(experiment_directory, hyperparams_to_save=None, overrides=None,
                                log_config=None, save_env_desc=True):
    os.makedirs(experiment_directory, exist_ok=True)
    if hyperparams_to_save is not None:
        shutil.copy(hyperparams_to_save, os.path.join(experiment_directory, "hyperparams.yaml"))
    with open(os.path.join(experiment_directory, "overrides.txt"), "w") as f:
        f.write(repr(overrides))
