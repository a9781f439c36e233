"""Helpers to read the committed golden fixtures (tests/golden/*.npz)."""
import json
import os
from collections import OrderedDict

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tiny_likelihood", "tiny_mse", "tiny_dropout", "tiny_quirk_lens", "mid_likelihood",
         "one_layer"]


def load_case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(d["meta_json"]))
    t = lambda k: torch.from_numpy(np.array(d[k]))
    params = OrderedDict((k, t("init/" + k)) for k in meta["param_names"])
    steps = []
    for s in range(meta["n_steps"]):
        pre = f"step{s}/"
        st = {k[len(pre):]: t(k) for k in d.files if k.startswith(pre)}
        st["grads"] = OrderedDict((k, st.pop("grad/" + k)) for k in meta["param_names"])
        st["params"] = OrderedDict((k, st.pop("param/" + k)) for k in meta["param_names"])
        steps.append(st)
    return meta, t("x"), t("lens"), params, steps


def cfg_of(meta):
    return dict(L=meta["L"], loss_type=meta["loss_type"], kld_weight=meta["kld_weight"],
                batch_size=meta["B"], lr=meta["lr"])
