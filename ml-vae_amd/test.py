"""Evaluate the best checkpoint on the test split (ref:src/test.py)."""
import sys

from prepare_experiment import prepare_experiment

if __name__ == "__main__":
    prepared = prepare_experiment(sys.argv[1:], prepare_exp_dir=False)
    hparams = prepared["hparams"]
    model = prepared["model"]
    model.init_optimizers()
    model.evaluate(prepared["datasets"][2], max_key=hparams["model"].get("max_key"),
                   min_key=hparams["model"].get("min_key"),
                   test_loader_kwargs=hparams["test_dataloader_opts"])
