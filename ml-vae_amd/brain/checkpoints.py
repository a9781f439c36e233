"""Checkpointer: named recoverables saved per checkpoint directory, best-by-key recovery."""
import glob
import json
import os
import shutil
import time

import torch


class Checkpointer:
    def __init__(self, checkpoints_dir, recoverables=None, allow_partial_load=False):
        self.checkpoints_dir = str(checkpoints_dir)
        self.recoverables = dict(recoverables or {})
        self.allow_partial_load = allow_partial_load

    def add_recoverable(self, name, obj):
        self.recoverables[name] = obj

    def _save_obj(self, obj, path):
        # clone to CPU: parameters may be views of one flat device buffer, and torch.save
        # would otherwise serialise the whole underlying storage for every view
        sd = {k: (v.detach().to("cpu", copy=True) if torch.is_tensor(v) else v)
              for k, v in obj.state_dict().items()}
        torch.save(sd, path)

    def save_checkpoint(self, meta=None, name=None):
        os.makedirs(self.checkpoints_dir, exist_ok=True)
        name = name or time.strftime("CKPT+%Y-%m-%d+%H-%M-%S") + f"+{time.time_ns() % 100000:05d}"
        d = os.path.join(self.checkpoints_dir, name)
        os.makedirs(d, exist_ok=True)
        for k, obj in self.recoverables.items():
            self._save_obj(obj, os.path.join(d, f"{k}.ckpt"))
        with open(os.path.join(d, "CKPT.json"), "w") as f:
            json.dump({"meta": meta or {}, "unixtime": time.time()}, f)
        return d

    def list_checkpoints(self):
        out = []
        for d in sorted(glob.glob(os.path.join(self.checkpoints_dir, "CKPT+*"))):
            try:
                with open(os.path.join(d, "CKPT.json")) as f:
                    out.append((d, json.load(f)))
            except (OSError, ValueError):
                continue
        return out

    def find_checkpoint(self, max_key=None, min_key=None):
        ckpts = self.list_checkpoints()
        if not ckpts:
            return None
        if max_key is not None:
            ckpts = [c for c in ckpts if max_key in c[1]["meta"]]
            return max(ckpts, key=lambda c: c[1]["meta"][max_key])[0] if ckpts else None
        if min_key is not None:
            ckpts = [c for c in ckpts if min_key in c[1]["meta"]]
            return min(ckpts, key=lambda c: c[1]["meta"][min_key])[0] if ckpts else None
        return max(ckpts, key=lambda c: c[1]["unixtime"])[0]

    def save_and_keep_only(self, meta=None, max_keys=None, min_keys=None, num_to_keep=1):
        d = self.save_checkpoint(meta)
        keep = {d}
        for k in max_keys or []:
            c = self.find_checkpoint(max_key=k)
            if c:
                keep.add(c)
        for k in min_keys or []:
            c = self.find_checkpoint(min_key=k)
            if c:
                keep.add(c)
        for c, _ in self.list_checkpoints():
            if c not in keep:
                shutil.rmtree(c, ignore_errors=True)
        return d

    def recover_if_possible(self, max_key=None, min_key=None, device=None):
        d = self.find_checkpoint(max_key=max_key, min_key=min_key)
        if d is None:
            return None
        for k, obj in self.recoverables.items():
            path = os.path.join(d, f"{k}.ckpt")
            if not os.path.exists(path):
                if self.allow_partial_load:
                    continue
                raise RuntimeError(f"checkpoint {d} has no {k}")
            sd = torch.load(path, map_location=device or "cpu", weights_only=True)
            obj.load_state_dict(sd)
        return d
