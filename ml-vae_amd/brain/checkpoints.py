"""Checkpointer in SpeechBrain 0.5's on-disk layout (the recipe's recoverables:
ref:src/models/test_vanilla_vae/model.yaml:7-12; optimizers added at
ref:src/models/md_model.py:50-52; save_and_keep_only after VALID at md_model.py:150-164).

    <checkpoints_dir>/CKPT+<YYYY-mm-dd+HH-MM-SS>+<NN>/
        CKPT.yaml          "# yamllint disable" + {unixtime, end-of-epoch, **meta}
        <recoverable>.ckpt torch.save(state_dict) for modules and optimizers;
                           the epoch counter as plain text (its SpeechBrain saver)

Recovery ranks checkpoints by meta[max_key], by -meta[min_key] (only checkpoints that carry the
key) or by recency (unixtime), as SpeechBrain's find_checkpoints does, and loads every file
with torch.load(weights_only=True).  Directories written by round 1 of this build (CKPT.json)
are still read; a CKPT+* directory that cannot be parsed is reported with a warning instead of
being skipped silently."""
import glob
import json
import logging
import os
import shutil
import time
import warnings

import torch
import yaml

logger = logging.getLogger(__name__)

CKPT_PREFIX = "CKPT"
METAFNAME = f"{CKPT_PREFIX}.yaml"
PARAMFILE_EXT = ".ckpt"


class Checkpointer:
    def __init__(self, checkpoints_dir, recoverables=None, allow_partial_load=False):
        self.checkpoints_dir = str(checkpoints_dir)
        self.recoverables = dict(recoverables or {})
        self.allow_partial_load = allow_partial_load

    def add_recoverable(self, name, obj):
        self.recoverables[name] = obj

    # ------------------------------------------------------------------ save
    @staticmethod
    def _save_obj(obj, path):
        if hasattr(obj, "ckpt_save"):  # custom saver (EpochCounter: plain text)
            obj.ckpt_save(path)
            return
        # clone to CPU: parameters may be views of one flat device buffer, and torch.save
        # would otherwise serialise the whole underlying storage for every view
        sd = obj.state_dict()
        torch.save(_to_cpu(sd), path)

    def _new_dir(self):
        stamp = time.strftime("%Y-%m-%d+%H-%M-%S", time.localtime())
        for n in range(100):
            d = os.path.join(self.checkpoints_dir, f"{CKPT_PREFIX}+{stamp}+{n:02d}")
            if not os.path.exists(d):
                return d
        raise RuntimeError("more than 100 checkpoints in one second")

    def save_checkpoint(self, meta=None, end_of_epoch=True, name=None):
        os.makedirs(self.checkpoints_dir, exist_ok=True)
        d = os.path.join(self.checkpoints_dir, f"{CKPT_PREFIX}+{name}") if name else self._new_dir()
        os.makedirs(d, exist_ok=True)
        for k, obj in self.recoverables.items():
            self._save_obj(obj, os.path.join(d, k + PARAMFILE_EXT))
        info = {"unixtime": time.time(), "end-of-epoch": bool(end_of_epoch)}
        info.update(_plain(meta or {}))
        with open(os.path.join(d, METAFNAME), "w") as f:
            f.write("# yamllint disable\n")
            f.write(yaml.safe_dump(info))
        return d

    # ------------------------------------------------------------------ find
    def list_checkpoints(self):
        """[(dir, {"meta": {...}, "unixtime": t, "end_of_epoch": b})] of every readable
        checkpoint (SpeechBrain CKPT.yaml, or this build's round-1 CKPT.json)."""
        out = []
        for d in sorted(glob.glob(os.path.join(self.checkpoints_dir, f"{CKPT_PREFIX}+*"))):
            if not os.path.isdir(d):
                continue
            meta = None
            try:
                if os.path.exists(os.path.join(d, METAFNAME)):
                    with open(os.path.join(d, METAFNAME)) as f:
                        raw = yaml.safe_load(f) or {}
                    t = float(raw.pop("unixtime", os.path.getmtime(d)))
                    eoe = bool(raw.pop("end-of-epoch", True))
                    meta = {"meta": raw, "unixtime": t, "end_of_epoch": eoe}
                elif os.path.exists(os.path.join(d, "CKPT.json")):
                    with open(os.path.join(d, "CKPT.json")) as f:
                        raw = json.load(f)
                    meta = {"meta": raw.get("meta", {}), "unixtime": float(raw.get("unixtime", 0)),
                            "end_of_epoch": True}
            except (OSError, ValueError, yaml.YAMLError) as e:
                warnings.warn(f"checkpoint directory {d} cannot be read ({e}); ignoring it")
                continue
            if meta is None:
                warnings.warn(f"checkpoint directory {d} has no {METAFNAME}; ignoring it")
                continue
            out.append((d, meta))
        return out

    def find_checkpoints(self, max_key=None, min_key=None, max_num_checkpoints=None, predicate=None):
        """Checkpoints ranked best first (SpeechBrain find_checkpoints); predicate(meta) filters."""
        if max_key is not None and min_key is not None:
            raise ValueError("give max_key or min_key, not both")
        ckpts = self.list_checkpoints()
        if predicate is not None:
            ckpts = [c for c in ckpts if predicate(c[1]["meta"])]
        if max_key is not None:
            ckpts = [c for c in ckpts if max_key in c[1]["meta"]]
            ckpts.sort(key=lambda c: c[1]["meta"][max_key], reverse=True)
        elif min_key is not None:
            ckpts = [c for c in ckpts if min_key in c[1]["meta"]]
            ckpts.sort(key=lambda c: c[1]["meta"][min_key])
        else:
            ckpts.sort(key=lambda c: c[1]["unixtime"], reverse=True)
        return ckpts[:max_num_checkpoints] if max_num_checkpoints else ckpts

    def find_checkpoint(self, max_key=None, min_key=None):
        ckpts = self.find_checkpoints(max_key=max_key, min_key=min_key, max_num_checkpoints=1)
        return ckpts[0][0] if ckpts else None

    def save_and_keep_only(self, meta=None, end_of_epoch=True, max_keys=None, min_keys=None,
                           num_to_keep=1, ckpt_predicate=None):
        """Save, then delete the checkpoints that are neither among the num_to_keep most recent
        nor the best by a max/min key.  ckpt_predicate(meta dict) limits both the ranking and
        the deletion to the checkpoints it accepts (SpeechBrain: the intra-epoch checkpoints
        replace only each other)."""
        d = self.save_checkpoint(meta, end_of_epoch=end_of_epoch)
        keep = {d}
        for c, _ in self.find_checkpoints(max_num_checkpoints=num_to_keep, predicate=ckpt_predicate):
            keep.add(c)
        for k in max_keys or []:
            for c, _ in self.find_checkpoints(max_key=k, max_num_checkpoints=num_to_keep, predicate=ckpt_predicate):
                keep.add(c)
        for k in min_keys or []:
            for c, _ in self.find_checkpoints(min_key=k, max_num_checkpoints=num_to_keep, predicate=ckpt_predicate):
                keep.add(c)
        for c, m in self.list_checkpoints():
            if c not in keep and (ckpt_predicate is None or ckpt_predicate(m["meta"])):
                shutil.rmtree(c, ignore_errors=True)
        return d

    # ------------------------------------------------------------------ recover
    def recover_if_possible(self, max_key=None, min_key=None, device=None):
        d = self.find_checkpoint(max_key=max_key, min_key=min_key)
        self.recovered_meta = None
        if d is None:
            logger.info("no checkpoint to recover in %s", self.checkpoints_dir)
            return None
        eoe = True
        for c, m in self.list_checkpoints():
            if c == d:
                eoe = m["end_of_epoch"]
                self.recovered_meta = dict(m["meta"], end_of_epoch=eoe)
        for k, obj in self.recoverables.items():
            path = os.path.join(d, k + PARAMFILE_EXT)
            if not os.path.exists(path):
                if self.allow_partial_load:
                    continue
                raise RuntimeError(f"checkpoint {d} has no {k}{PARAMFILE_EXT}")
            if hasattr(obj, "ckpt_recover"):
                obj.ckpt_recover(path, end_of_epoch=eoe)
                continue
            sd = torch.load(path, map_location=device or "cpu", weights_only=True)
            obj.load_state_dict(sd)
        logger.info("recovered %s", d)
        return d


def _to_cpu(v):
    if torch.is_tensor(v):
        return v.detach().to("cpu", copy=True)
    if isinstance(v, dict):
        return type(v)((k, _to_cpu(x)) for k, x in v.items())
    if isinstance(v, (list, tuple)):
        return type(v)(_to_cpu(x) for x in v)
    return v


def _plain(meta):
    """yaml.safe_dump-able copy of a meta dict (tensors / numpy scalars -> Python floats)."""
    out = {}
    for k, v in meta.items():
        if torch.is_tensor(v):
            v = v.item()
        elif hasattr(v, "item") and not isinstance(v, (list, dict, str)):
            v = v.item()
        out[str(k)] = v
    return out
