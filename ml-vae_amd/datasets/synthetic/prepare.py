"""Synthetic corpus "preparation": nothing to download or convert (no network, no corpora).
Kept so the reference's `datasets.<dataset>.prepare.prepare(**hparams['prepare'])` call
(ref:src/prepare_experiment.py:39-40) has a target."""


def prepare(**kwargs):
    return kwargs
