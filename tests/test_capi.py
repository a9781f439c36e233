"""The C-ABI library loads on a CPU-only host and exports every entry point that
include/mlvae.h declares (no compute calls here)."""
import ctypes
import os
import re

from conftest import ROOT
from mlvae_hip import _lib


def _declared():
    text = open(os.path.join(ROOT, "include", "mlvae.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mlvae_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    names = _declared()
    assert len(names) >= 20
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(_declared()) <= set(_lib.exported_symbols()) | {"mlvae_set_error"}


def test_abi_version_and_error_channel():
    l = _lib.lib()
    assert l.mlvae_abi_version() == 1
    rc = l.mlvae_gemm(7, 0, 0, 4, 4, 4, 1.0, None, 4, None, 4, 0.0, 1, 4, None, None, 0, None, 0,
                      0, 0, None, 0, None)
    assert rc == 1 and "prec" in _lib.last_error()


def test_lstm_workspace_covers_the_stepwise_fp32_bptt():
    """fp32 past H = 512: the stepwise BPTT keeps the cell gradient [2, B, H] in the workspace
    (host-side sizing only, no GPU call)."""
    import ctypes
    from mlvae_hip._lib import lib
    for B, H in ((5, 1024), (64, 2048)):
        xb = ctypes.c_size_t()
        assert lib().mlvae_lstm_workspace_size(B, H, 0, ctypes.byref(xb)) == 0
        assert xb.value >= 2 * B * H * 4
