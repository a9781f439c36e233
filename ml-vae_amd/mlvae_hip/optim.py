"""Optimizers on libmlvae.so.

* ``Adam`` -- torch.optim.Adam-compatible constructor (params, lr, betas, eps,
  weight_decay=0) for the module-level path: one fused update launch per tensor, bias
  corrections from a device step counter (ref:src/models/test_vanilla_vae/model.yaml:45-47).
* ``clip_grad_norm_`` -- SpeechBrain check_gradients' clip (max_grad_norm 5.0) on the device.
* The fused training step (mlvae_hip.engine) does sum-of-squares, clip and Adam over one flat
  buffer instead; ``EngineOptimizer`` exposes it with the optimizer interface.
"""
import math

import torch

from ._lib import check, lib


def _p(t):
    return t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _sumsq_partials(tensors):
    l = lib()
    counts = [l.mlvae_sumsq_partials_count(t.numel()) for t in tensors]
    buf = torch.zeros(max(sum(counts), 1), device=tensors[0].device, dtype=torch.float64)
    off = 0
    for t, c in zip(tensors, counts):
        check(l.mlvae_grad_sumsq(_p(t), t.numel(), _p(buf) + 8 * off, _stream()), "grad_sumsq")
        off += c
    return buf, off


def clip_grad_norm_(parameters, max_norm):
    """Scale all grads by min(max_norm / (||g||_2 + 1e-6), 1); returns the total norm tensor."""
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.zeros(())
    for g in grads:
        if not (g.is_cuda and g.is_contiguous() and g.dtype == torch.float32):
            raise TypeError("clip_grad_norm_: contiguous fp32 HIP grads required")
    buf, n = _sumsq_partials(grads)
    norm = torch.zeros(1, device=grads[0].device)
    for i, g in enumerate(grads):
        check(lib().mlvae_clip_scale(_p(g), g.numel(), _p(buf), n, float(max_norm),
                                     _p(norm) if i == 0 else None, _stream()), "clip_scale")
    return norm[0]


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam semantics on libmlvae (no weight decay, amsgrad off).  The step count
    lives in a device counter shared by every parameter (bias corrections without a host
    sync); each param group gets its own lr / step-size scratch, and state_dict() /
    load_state_dict() carry the count as torch does (a per-parameter "step")."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay:
            raise NotImplementedError("weight decay is not used by the VAE recipe")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._step_ctr = None
        self._zero = None
        self._hyp = {}

    def _device_state(self, dev):
        if self._step_ctr is None or self._step_ctr.device != dev:
            self._step_ctr = torch.zeros(1, device=dev, dtype=torch.int32)
            self._zero = torch.zeros(1, device=dev, dtype=torch.float64)
            # a recovered checkpoint carries the count in every parameter's "step"
            steps = [st["step"] for st in self.state.values() if "step" in st]
            if steps:
                self._step_ctr.fill_(int(max(float(torch.as_tensor(s).max()) for s in steps)))

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._step_ctr = None  # rebuilt from the loaded per-parameter "step" at the next step()
        for st in self.state.values():
            if "step" in st:
                st["step"] = torch.as_tensor(st["step"], dtype=torch.float32).reshape(()).clone()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        l = lib()
        work = []
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is None:
                    continue  # torch semantics: no grad -> untouched, no state
                st = self.state[p]
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                work.append((gi, group, p, st))
        if not work:
            return loss
        dev = work[0][2].device
        self._device_state(dev)
        first_of_group = set()
        seen = set()
        for i, (gi, _, _, _) in enumerate(work):
            if gi not in seen:
                seen.add(gi)
                first_of_group.add(i)
        for i, (gi, group, p, st) in enumerate(work):
            # advance: 1 = last tensor of the step (prologue + step counter), 0 = first tensor of
            # its group (prologue: this group's lr), -1 = reuse the group's prologue
            adv = 1 if i == len(work) - 1 else (0 if i in first_of_group else -1)
            hyp = self._hyp.get(gi)
            if hyp is None or hyp.device != dev:
                hyp = self._hyp[gi] = torch.zeros(4, device=dev, dtype=torch.float32)
            b1, b2 = group["betas"]
            # clipping already happened in check_gradients: max_norm = inf -> coef 1
            check(l.mlvae_adam_step(_p(p), _p(st["exp_avg"]), _p(st["exp_avg_sq"]), _p(p.grad),
                                    p.numel(), _p(self._zero), 1, None, _p(self._step_ctr), None,
                                    float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                    math.inf, None, _p(hyp), adv, _stream()), "adam_step")
            st["step"] = self._step_ctr
        return loss

    def state_dict(self):
        sd = super().state_dict()
        for st in sd["state"].values():  # torch.optim.Adam layout: a float scalar "step"
            if "step" in st:
                st["step"] = torch.as_tensor(st["step"]).to("cpu", torch.float32).reshape(()).clone()
        return sd

    def zero_grad(self, set_to_none=True):
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None


class EngineOptimizer:
    """Optimizer facade of a VAEEngine (the fused step already applied the update).

    state_dict() is torch.optim.Adam's layout over the modules' parameters in
    Brain.modules.parameters() order (per-parameter exp_avg / exp_avg_sq / step + one param
    group), so a checkpoint written on the fused path loads into the module path's Adam (or
    torch's) and vice versa."""

    def __init__(self, engine):
        self.engine = engine

    def step(self):
        pass

    def zero_grad(self, set_to_none=True):
        pass

    def _names(self):
        return list(self.engine.layout.shapes.keys())

    def state_dict(self):
        e, cfg = self.engine, self.engine.cfg
        step = torch.tensor(float(e.step_ctr.item()))
        state = {}
        for i, name in enumerate(self._names()):
            state[i] = {"step": step.clone(),
                        "exp_avg": e.view(name, e.exp_avg).detach().to("cpu", copy=True),
                        "exp_avg_sq": e.view(name, e.exp_avg_sq).detach().to("cpu", copy=True)}
        group = {"lr": cfg.lr, "betas": tuple(cfg.betas), "eps": cfg.adam_eps, "weight_decay": 0,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "params": list(range(len(state)))}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        e = self.engine
        with torch.no_grad():
            if "state" not in sd:  # round-1 flat layout
                e.exp_avg.copy_(sd["exp_avg"])
                e.exp_avg_sq.copy_(sd["exp_avg_sq"])
                e.step_ctr.copy_(torch.as_tensor(sd["step"]).reshape(1).to(torch.int32))
                return
            names = self._names()
            if len(sd["state"]) and max(int(k) for k in sd["state"]) >= len(names):
                raise KeyError("optimizer state has more parameters than the engine")
            steps = [0]
            for k, st in sd["state"].items():
                name = names[int(k)]
                e.view(name, e.exp_avg).copy_(st["exp_avg"])
                e.view(name, e.exp_avg_sq).copy_(st["exp_avg_sq"])
                steps.append(int(float(torch.as_tensor(st["step"]).max())))
            e.step_ctr.fill_(max(steps))
            if sd.get("param_groups"):
                g = sd["param_groups"][0]
                e.cfg.lr = float(g.get("lr", e.cfg.lr))
