"""python train.py config/run.yaml --model_class test_vanilla_vae --model_name vae \
       --model !include:../models/test_vanilla_vae/model.yaml [--extra_overrides "{...}"]
(same command line as ref:src/train.py).  Data parallel, one process per GPU:
python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 train.py ... (brain.distributed)."""
import sys

import torch

from prepare_experiment import prepare_experiment

torch.use_deterministic_algorithms(True, warn_only=True)

if __name__ == "__main__":
    prepared = prepare_experiment(sys.argv[1:], prepare_exp_dir=True)
    hparams = prepared["hparams"]
    train_set, valid_set, test_set = prepared["datasets"]
    model = prepared["model"]
    model.fit(hparams["model"]["epoch_counter"], train_set, valid_set,
              train_loader_kwargs=hparams["train_dataloader_opts"],
              valid_loader_kwargs=hparams["valid_dataloader_opts"])
    import torch.distributed as dist
    if dist.is_initialized():  # data-parallel launch (brain.distributed)
        dist.destroy_process_group()
