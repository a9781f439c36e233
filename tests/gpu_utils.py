"""Shared helpers for the -m gpu tests (they call libmlvae.so through its C ABI)."""
import pytest
import torch

from mlvae_hip import _lib


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device in this container")
    rc, arch = _lib.device_check()
    assert rc == 0, f"device check failed: {arch} {_lib.last_error()}"


def P(t, off=0):
    return t.data_ptr() + 4 * off


def stream():
    return torch.cuda.current_stream().cuda_stream


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def norm_rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
