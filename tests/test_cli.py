from brain.cli import parse_arguments


def test_parse_arguments_splits_run_opts_and_overrides():
    f, opts, ov = parse_arguments(["config/run.yaml", "--device", "cuda:0", "--debug",
                                   "--model_class", "test_vanilla_vae",
                                   "--model", "!include:../models/test_vanilla_vae/model.yaml",
                                   "--extra_overrides", "{model: {n_epochs: 1}}"])
    assert f == "config/run.yaml"
    assert opts == {"device": "cuda:0", "debug": True}
    assert ov.splitlines() == ["model_class: test_vanilla_vae",
                               "model: !include:../models/test_vanilla_vae/model.yaml",
                               "extra_overrides: {model: {n_epochs: 1}}"]


def test_epoch_counter_and_checkpointer(tmp_path):
    import torch
    from brain import Checkpointer, EpochCounter
    ec = EpochCounter(3)
    assert list(ec) == [1, 2, 3]
    lin = torch.nn.Linear(2, 2)
    ck = Checkpointer(tmp_path / "ck", {"lin": lin, "ec": ec})
    ck.save_and_keep_only(meta={"loss": 2.0}, min_keys=["loss"])
    ck.save_and_keep_only(meta={"loss": 1.0}, min_keys=["loss"])
    ck.save_and_keep_only(meta={"loss": 3.0}, min_keys=["loss"])
    kept = [m["meta"]["loss"] for _, m in ck.list_checkpoints()]
    assert sorted(kept) == [1.0, 3.0]
    ec.current = 0
    ck.recover_if_possible(min_key="loss")
    assert ec.current == 3
