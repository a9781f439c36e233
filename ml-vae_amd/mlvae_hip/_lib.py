"""ctypes binding of libmlvae.so (C ABI declared in include/mlvae.h).

The library is the product: there is no CPU fallback.  ``lib()`` raises if the
in-tree ``libmlvae.so`` is missing or cannot be loaded, and ``check()`` turns a
non-zero status into a RuntimeError carrying ``mlvae_last_error()``.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MLVAE_LIB_PATH") or os.path.join(_HERE, "libmlvae.so")  # override: A/B timing

P = C.c_void_p
I = C.c_int
F = C.c_float
SZ = C.c_size_t
U64 = C.c_ulonglong

# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS = {
    "mlvae_last_error": [],
    "mlvae_abi_version": [],
    "mlvae_device_check": [C.c_char_p, I],
    "mlvae_gemm_workspace_size": [I, I, I],
    "mlvae_gemm": [I, I, I, I, I, I, F, P, I, P, I, F, P, I, P, P, I, P, I, I, I, P, SZ, P],
    "mlvae_gemm_ex_workspace_size": [I, I, I],
    "mlvae_gemm_ex": [I, I, I, I, I, F, P, I, I, P, I, I, F, P, I, P, P, I, P, I, I, I, P, SZ, P],
    "mlvae_gemm_ex_drop": [I, I, I, I, I, F, P, I, I, P, I, I, F, P, I, P, P, I, P, I, I, I, U64, U64,
                           F, P, SZ, P],
    "mlvae_cast_bf16": [SZ, P, P, P],
    "mlvae_cast_bf16_t": [I, I, P, P, P],
    "mlvae_gemm_bf16_workspace_size": [I, I, I, I],
    "mlvae_gemm_bf16_set_split_target": [I],
    "mlvae_gemm_bf16_set_variant": [I],
    "mlvae_gemm_bf16": [I, I, I, I, I, I, P, I, C.c_longlong, P, I, C.c_longlong, P, I, C.c_longlong,
                        F, P, P, I, P, I, I, I, I, U64, U64, F, P, SZ, P],
    "mlvae_lstm_workspace_size": [I, I, I, C.POINTER(SZ)],
    "mlvae_lstm_fwd": [I, I, I, I, P, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm_bwd": [I, I, I, I, P, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm_fwd_ex": [I, I, I, I, P, P, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm_bwd_ex": [I, I, I, I, P, P, P, P, P, P, P, SZ, P, P],
    "mlvae_viterbi_workspace_size": [I, I, I],
    "mlvae_viterbi_md": [I, I, I, I, P, I, P, P, P, P, P, P, F, P, SZ, P, P, P, P, P, P],
    "mlvae_phn_bce": [I, I, I, P, I, P, P, I, P, P, P, P, P, P, P],
    "mlvae_gemm_fp8": [I, I, I, P, I, P, I, P, I, P, P, P, I, P],
    "mlvae_fp8_scale_workspace_size": [],
    "mlvae_fp8_scale": [SZ, P, F, P, P, SZ, P],
    "mlvae_cast_fp8": [SZ, P, I, P, F, P, P],
    "mlvae_conv1d_supported": [I, I, I],
    "mlvae_conv1d_fwd": [I, I, I, I, I, P, I, P, P, I, P, I, P],
    "mlvae_conv1d_dgrad": [I, I, I, I, I, P, I, P, P, I, P, I, P],
    "mlvae_conv1d_wgrad_workspace_size": [I, I, I, I, I],
    "mlvae_conv1d_wgrad": [I, I, I, I, I, P, I, P, I, P, P, P, SZ, P],
    "mlvae_boundary_fwd": [SZ, P, P, P, P, U64, U64, P, P, P, P],
    "mlvae_boundary_bwd": [SZ, P, P, P, P, U64, U64, P, P, P, P, P, P],
    "mlvae_lstm1_fwd": [I, I, I, I, P, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm1_bwd": [I, I, I, I, P, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm_gates_fp16": [I, I, I],
    "mlvae_lstm_gates_fp16_t": [I, I, I, I],
    "mlvae_lstm_fwd_ex2": [I, I, I, I, P, P, P, I, P, P, P, P, U64, U64, F, P, SZ, P, P],
    "mlvae_lstm_bwd_ex2": [I, I, I, I, P, P, P, I, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm_bwd_ex3": [I, I, I, I, P, P, P, I, P, P, I, P, P, P, SZ, P, P],
    "mlvae_elbo_partials_count": [I, I, I],
    "mlvae_heads_partials_count": [I, I],
    "mlvae_heads_supported": [I, I, I],
    "mlvae_heads_fused": [I, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, F,
                          P, P, P, P, P, P, P, P, P, P, P, P, P],
    "mlvae_heads_bias_workspace_size": [I, I, I, I],
    "mlvae_heads_fused_ex": [I, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, F,
                             P, P, P, P, P, P, P, P, P, P, P, P, P, SZ, P, P, P, P, P, I, P],
    "mlvae_heads_fused_ex2": [I, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, F,
                              P, P, P, P, P, P, P, P, P, P, P, P, P, SZ, P, P, P, P, P, I,
                              P, SZ, P, P, P, P, P],
    "mlvae_heads_fused_ex3": [I, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, F,
                              P, P, P, P, P, P, P, P, P, P, P, P, P, SZ, P, P, P, P, P, I,
                              P, SZ, P, P, P, P, P, P],
    "mlvae_bf16_split_rows": [P, I, I, I, P, P],
    "mlvae_dp_scalars": [I, P, P, P, P],
    "mlvae_heads_wgrad_workspace_size": [I, I, I, I],
    "mlvae_heads_set_nt_mode": [I],
    "mlvae_skinny_proj": [I, I, I, P, I, P, I, P, P, P, I, P],
    "mlvae_skinny_proj_ex": [I, I, I, P, I, P, I, P, P, P, I, I, P],
    "mlvae_skinny_nt": [I, I, I, P, I, P, I, P, I, P],
    "mlvae_skinny_tn_workspace_size": [I, I, I],
    "mlvae_skinny_tn": [I, I, I, P, I, P, I, I, P, P, P, P, SZ, P],
    "mlvae_skinny_nt_fp8": [I, I, I, P, I, P, I, P, I, P, P],
    "mlvae_skinny_tn_fp8": [I, I, I, P, I, P, I, I, P, P, P, P, P, SZ, P],
    "mlvae_skinny_dzw": [I, I, P, I, P, I, P, I, I, P, I, P, P, P, P, SZ, P],
    "mlvae_skinny_dzw_workspace_size": [I, I],
    "mlvae_encoder_supported": [I, I, I],
    "mlvae_encoder_partials_count": [I, I],
    "mlvae_encoder_workspace_size": [I, I, I, I, I],
    "mlvae_encoder_fwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, U64, U64, P, P, P, P, P, P, I, P, P, P],
    "mlvae_encoder_fwd_ex": [I, I, I, I, I, P, P, P, P, P, P, P, P, U64, U64, P, P, P, P, P, P, I, P, P, I, P],
    "mlvae_encoder_bwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, F, P, P, P, P, P, P, P, SZ, P],
    "mlvae_reparam_kl_fwd": [I, I, I, P, I, P, P, P, P, P, P],
    "mlvae_reparam_kl_bwd": [I, I, I, P, I, P, P, P, P, P, F, P, I, P],
    "mlvae_recon": [I, I, I, I, P, I, P, I, P, I, P, P, P, P, P, F, P, P, P],
    "mlvae_elbo_finalize": [P, I, P, I, P, P, I, I, I, I, F, F, P, P],
    "mlvae_masked_mean": [I, I, I, P, P, I, P, P],
    "mlvae_count_frames": [P, I, I, P, P],
    "mlvae_randn": [SZ, U64, U64, P, P],
    "mlvae_sumsq_partials_count": [SZ],
    "mlvae_grad_sumsq": [P, SZ, P, P],
    "mlvae_adam_step": [P, P, P, P, SZ, P, I, P, P, P, F, F, F, F, F, P, P, I, P],
    "mlvae_adam_step_ex": [P, P, P, P, SZ, P, I, P, P, P, P, P, F, F, F, F, F, P, P, I, P],
    "mlvae_colsum_workspace_size": [I, I],
    "mlvae_colsum": [I, I, P, I, P, P, F, P, SZ, P],
    "mlvae_colsum_ex": [I, I, P, I, I, P, P, F, P, SZ, P],
    "mlvae_dropout": [SZ, P, P, P, U64, F, P],
    "mlvae_dropout_ex": [SZ, P, P, P, P, U64, U64, F, P],
    "mlvae_lrelu_bwd": [SZ, P, P, P, P],
    "mlvae_clip_scale": [P, SZ, P, I, F, P, P],
    "mlvae_masked_mean_bwd": [I, I, I, P, I, P, P, P],
    "mlvae_gmm_latent_fwd": [I, I, I, P, I, P, P, U64, U64, F, P, P, P, P, P],
    "mlvae_gmm_latent_bwd": [I, I, I, P, I, P, P, F, P, P, P, P, I, P],
    "mlvae_apply_weight_fwd": [I, I, I, P, I, P, P, I, P],
    "mlvae_apply_weight_bwd": [I, I, I, P, I, P, P, I, P, I, P, P],
    "mlvae_lstm_launch_workgroups": [I, I, I, I],
    "mlvae_lstm_set_debug": [P],
    "mlvae_lstm_set_debug_mode": [I],
    "mlvae_lstm_fwd_fp8": [I, I, I, P, P, P, P, P, P, P, F, U64, U64, F, P, SZ, P, P],
    "mlvae_lstm_fwd_z": [I, I, I, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, F, U64, U64, F, P, SZ, P, P],
    "mlvae_lstm_fwd_z2": [I, I, I, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, I, P, P, F, U64, U64, F, P, SZ, P, P],
    "mlvae_lstm_bwd_fp8": [I, I, I, P, P, P, P, P, P, P, P, P, P, P, SZ, P, P],
    "mlvae_lstm_bwd_fp8_ex": [I, I, I, P, P, P, P, P, I, P, P, P, P, P, P, SZ, P, P],
    "mlvae_fp8_delayed_scale": [P, P, P, F, P, P],
    "mlvae_gemm_fp8_ex": [I, I, I, P, I, P, I, P, I, P, P, P, I, U64, U64, F, P],
    "mlvae_gemm_fp8_tn_workspace_size": [I, I, I],
    "mlvae_gemm_fp8_tn": [I, I, I, P, I, P, I, P, I, P, P, SZ, P],
    "mlvae_gemm_fp8_tn_ex_workspace_size": [I, I, I, I],
    "mlvae_gemm_fp8_tn_ex": [I, I, I, I, P, I, C.c_longlong, P, I, C.c_longlong, P, I, C.c_longlong, P, I, I, I,
                             P, SZ, P],
    "mlvae_norm_supported": [I],
    "mlvae_norm_stats": [I, I, I, P, P, P, P, F, P],
    "mlvae_norm_update": [I, P, P, P, I, F, F, P],
    "mlvae_norm_apply": [SZ, I, P, P, P, P, P],
}
_RESTYPE = {
    "mlvae_last_error": C.c_char_p,
    "mlvae_conv1d_wgrad_workspace_size": SZ,
    "mlvae_skinny_dzw_workspace_size": SZ,
    "mlvae_fp8_scale_workspace_size": SZ,
    "mlvae_gemm_fp8_tn_workspace_size": SZ,
    "mlvae_gemm_fp8_tn_ex_workspace_size": SZ,
    "mlvae_gemm_workspace_size": SZ,
    "mlvae_gemm_ex_workspace_size": SZ,
    "mlvae_colsum_workspace_size": SZ,
    "mlvae_gemm_bf16_workspace_size": SZ,
    "mlvae_skinny_tn_workspace_size": SZ,
    "mlvae_encoder_workspace_size": SZ,
    "mlvae_viterbi_workspace_size": SZ,
    "mlvae_heads_bias_workspace_size": SZ,
    "mlvae_heads_wgrad_workspace_size": SZ,
}

_lib = None


class MlvaeError(RuntimeError):
    pass


def lib():
    """Load libmlvae.so (once).  Raises if it is absent: the HIP path has no fallback."""
    global _lib
    if _lib is None:
        # torch first: its bundled libamdhip64.so.7 then satisfies libmlvae.so's dependency,
        # so torch (allocations, streams) and the kernels share ONE HIP runtime; loading
        # libmlvae.so first would map /opt/rocm's runtime as a second, incompatible copy.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise MlvaeError(
                f"{LIB_PATH} is missing: build it with `python -m mlvae_hip.build` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        h = C.CDLL(LIB_PATH)
        # MLVAE_LIB_PATH (same-box A/B against an older build): entry points that build lacks
        # stay unbound (a call to one raises); the default library must export every one
        ab = "MLVAE_LIB_PATH" in os.environ
        for name, args in _SIGS.items():
            if ab and not hasattr(h, name):
                continue
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, I)
        _lib = h
        mode = os.environ.get("MLVAE_LSTM_DEBUG_MODE")
        if mode:  # diagnostics / A-B timing switches of the recurrence (lstm.hip)
            h.mlvae_lstm_set_debug_mode(int(mode))
    return _lib


def exported_symbols():
    return list(_SIGS.keys())


def last_error():
    return lib().mlvae_last_error().decode(errors="replace")


def check(rc, what=""):
    if rc != 0:
        raise MlvaeError(f"{what or 'mlvae'} failed (status {rc}): {last_error()}")
    return rc


def device_check():
    buf = C.create_string_buffer(64)
    rc = lib().mlvae_device_check(buf, 64)
    return rc, buf.value.decode()


_cus = None


def device_cus():
    """Compute units of the current HIP device (256 on MI355X)."""
    global _cus
    if _cus is None:
        import torch
        _cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return _cus
