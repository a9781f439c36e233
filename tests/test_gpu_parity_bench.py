"""Whole-step parity at the sizes bench.py measures, against the CPU oracle (tests/step_parity.py).

* c3 (the headline): B=256, T=500 -- the wide-batch recurrence instantiation the bench runs
  (lstm_{fwd,bwd}_wide_kernel<2,16>: 16 utterances x 64 units per workgroup, 256 workgroups);
* c4 (configs[3]): Conv1d K=5 encoder, B=64, T=2000;
* c5 (configs[4]): fp8 mode, per-GPU batch B=64 (512 over 8 GPUs), T=500.

Bounds (SURVEY.md 8(d) for bf16: loss 1e-3 relative, mu / log_var 1e-2 norm-relative) and the
update-direction check of step_parity.py: >= 99.5 % sign agreement of the Adam update with the
oracle's over the weights whose gradient is defined (|g| > 0.1 rms of its tensor), and the
update vector within 0.15 norm-relative there.  The measured values are printed."""
import numpy as np
import pytest
import torch

from gpu_utils import need_gpu
from step_parity import errors, report, run_second_step, run_step

pytestmark = pytest.mark.gpu

SIGN_MIN = 0.995
UPDATE_ERR = 0.15


def _check(e, grads, grad_max, grad_med, out_max=1e-2, update_max=UPDATE_ERR, rnn_max=None):
    assert e["loss"] <= 1e-3 and e["recon_loss"] <= 1e-3, e
    assert e["kld_loss"] <= 1e-2, e
    for k in ("mu", "log_var", "mu_x", "log_var_x"):
        assert e[k] <= out_max, (k, e[k])
    for k, v in grads.items():
        assert v <= grad_max, (k, v)
    assert float(np.median(list(grads.values()))) <= grad_med
    assert e["update_sign"] >= SIGN_MIN, e["update_sign"]
    assert e["update_err"] <= update_max, e["update_err"]
    if rnn_max is not None:  # the recurrent weights' gradients (a one-step time shift of h in dW_hh
        for k, v in grads.items():  # once passed the looser bounds at 3.9e-2: tools/gpu_c4chk.sh)
            if k.startswith("decoder.rnn."):
                assert v <= rnn_max, (k, v)


def test_c3_headline_B256_T500_matches_oracle():
    """The benchmarked step at the metric's batch: B=256, T=500, dropout 0.15, bf16."""
    need_gpu()
    from mlvae_hip._lib import lib
    from mlvae_hip.engine import VAEConfig
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16")
    B, T = 256, 500
    lens = torch.linspace(0.6, 1.0, B)
    lens[5], lens[9] = 127 / 500, 254 / 500
    wgs = lib().mlvae_lstm_launch_workgroups(B, 512, 1, 0)
    eng, w, rec, new_ref, params = run_step(cfg, B, T, 2718, lens)
    e, grads = errors(eng, w, rec, new_ref, params, B, T)
    report(f"c3 B=256 T=500 wide {wgs} WGs", e, grads)
    _check(e, grads, 4e-2, 1.5e-2, update_max=1.5e-2, rnn_max=1.5e-2)


def test_c4_conv_B64_T2000_matches_oracle():
    """configs[3] at its benchmarked size: Conv1d K=5 encoder, B=64, T=2000, dropout 0.15."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16", enc_conv=5)
    B, T = 64, 2000
    lens = torch.linspace(0.55, 1.0, B)
    eng, w, rec, new_ref, params = run_step(cfg, B, T, 4243, lens)
    e, grads = errors(eng, w, rec, new_ref, params, B, T)
    report("c4 conv K=5 B=64 T=2000", e, grads)
    _check(e, grads, 4e-2, 1.5e-2, update_max=1.5e-2, rnn_max=1.5e-2)


def test_c5_fp8_B64_T500_matches_oracle():
    """configs[4]'s per-GPU shard in fp8 mode at T=500 (the fp8 products' own bounds: e4m3 keeps
    3 mantissa bits)."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16", fp8=True)
    B, T = 64, 500
    lens = torch.linspace(0.6, 1.0, B)
    eng, w, rec, new_ref, params = run_step(cfg, B, T, 809, lens)
    e, grads = errors(eng, w, rec, new_ref, params, B, T)
    report("c5 fp8 B=64 T=500", e, grads)
    _check(e, grads, 0.12, 3e-2)


def test_c5_fp8_second_step_fp8_dgrad_matches_oracle():
    """configs[4] in its steady state: from the second step on the fp8 mode also runs the layer-1
    dgrad, dW_ih and dW_hh and layer 0's dZ, dW_ih | biases and dW_hh on e4m3 operands (dG written by the BPTT under delayed scaling from the first step's
    amax, W_ih^T with the forward's scale, the dropout backward in the epilogue) and the layer
    input arrives as e4m3 from the recurrence itself -- alone, without the bf16 copy no GEMM
    reads any more.  The oracle replays step 2 from the engine's
    state after step 1 (parameters, Adam moments)."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=2, C=64, dropout=0.15, prec="bf16", fp8=True)
    B, T = 64, 500
    lens = torch.linspace(0.6, 1.0, B)
    eng, w, rec, new_ref, params = run_second_step(cfg, B, T, 810, lens)
    assert eng.g8_ready and float(eng.g8[1][0].item()) != 1.0   # a real delayed scale was used
    assert w.ydb_skipped.get(1)   # layer 0 wrote the e4m3 dropout(h) alone (no bf16 reader)
    assert w.f8hh.get(1)          # dW_hh_l1 on e4m3 dG and h: the BPTT wrote no bf16 dG
    assert w.f8hh.get(0)          # layer 0 too: dZ, dW_ih_l0 | biases, dW_hh_l0 on its e4m3 dG
    e, grads = errors(eng, w, rec, new_ref, params, B, T)
    report("c5 fp8 step 2 (fp8 dgrad, dW_ih, dW_hh; layer-0 e4m3 dG) B=64 T=500", e, grads)
    print("  e4m3-operand gradients:", {k: f"{grads[k]:.2e}" for k in grads if "rnn" in k or "encoder" in k})
    _check(e, grads, 0.12, 3e-2)


def test_fp8_three_layers_second_step_matches_oracle():
    """fp8 mode with a 3-layer decoder: layers 1 and 2 both run their projection,
    dgrad and weight gradient on e4m3, and layer 2's weight gradient on the side stream reads its
    own e4m3 input and dG while layer 1's BPTT and dgrad run -- per-layer X8 / dG8 buffers.  Step 2
    (the fp8 dgrad / weight gradient are live from the second step on), B = 48 (ragged batch group
    of the wide recurrence), T = 120."""
    need_gpu()
    from mlvae_hip.engine import VAEConfig
    cfg = VAEConfig(F=80, E=64, Z=32, H=512, L=3, C=64, dropout=0.15, prec="bf16", fp8=True)
    B, T = 48, 120
    lens = torch.linspace(0.6, 1.0, B)
    eng, w, rec, new_ref, params = run_second_step(cfg, B, T, 811, lens)
    assert eng.g8_ready and all(float(eng.g8[li][0].item()) != 1.0 for li in (1, 2))
    assert w.ydb_skipped.get(1) and w.ydb_skipped.get(2)
    assert w.f8hh.get(1) and w.f8hh.get(2) and w.f8hh.get(0)
    e, grads = errors(eng, w, rec, new_ref, params, B, T)
    report("fp8 L=3 step 2 B=48 T=120", e, grads)
    _check(e, grads, 0.12, 3e-2)
