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
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay:
            raise NotImplementedError("weight decay is not used by the VAE recipe")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._step_ctr = None
        self._zero = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        l = lib()
        work = []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue  # torch semantics: no grad -> untouched, no state
                st = self.state[p]
                if not st:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                work.append((group, p, st))
        if not work:
            return loss
        dev = work[0][1].device
        if self._step_ctr is None:
            self._step_ctr = torch.zeros(1, device=dev, dtype=torch.int32)
            self._zero = torch.zeros(1, device=dev, dtype=torch.float64)
            self._hyp = torch.zeros(4, device=dev, dtype=torch.float32)
        for i, (group, p, st) in enumerate(work):
            adv = 1 if i == len(work) - 1 else (0 if i == 0 else -1)
            if len(work) == 1:
                adv = 1
            b1, b2 = group["betas"]
            # clipping already happened in check_gradients: max_norm = inf -> coef 1
            check(l.mlvae_adam_step(_p(p), _p(st["exp_avg"]), _p(st["exp_avg_sq"]), _p(p.grad),
                                    p.numel(), _p(self._zero), 1, None, _p(self._step_ctr), None,
                                    float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                    math.inf, None, _p(self._hyp), adv, _stream()), "adam_step")
            st["step"] = self._step_ctr
        return loss

    def zero_grad(self, set_to_none=True):
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None


class EngineOptimizer:
    """Optimizer facade of a VAEEngine (the fused step already applied the update)."""

    def __init__(self, engine):
        self.engine = engine

    def step(self):
        pass

    def zero_grad(self, set_to_none=True):
        pass

    def state_dict(self):
        e = self.engine
        return {"exp_avg": e.exp_avg.cpu(), "exp_avg_sq": e.exp_avg_sq.cpu(),
                "step": e.step_ctr.cpu()}

    def load_state_dict(self, sd):
        e = self.engine
        e.exp_avg.copy_(sd["exp_avg"])
        e.exp_avg_sq.copy_(sd["exp_avg_sq"])
        e.step_ctr.copy_(sd["step"])
