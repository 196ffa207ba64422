"""ctypes binding of libendossl_hip.so -- the C-ABI declared in include/endossl.h.

This is the only way the Python host reaches the GPU compute path: there is no CPU fallback.
If the shared library is missing (not built, or built for another arch) every compute call
raises `EndosslLibraryError` -- loudly, never silently degrading to PyTorch ops.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ENDOSSL_LIB", os.path.join(_HERE, "lib", "libendossl_hip.so"))

V, I, L, F, Z = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_size_t
U64 = ctypes.c_ulonglong

# name -> (restype, argtypes).  Mirrors include/endossl.h one-to-one (tests/test_abi.py checks it).
SIGNATURES = {
    "es_abi_version": (I, []),
    "es_gemm_nt": (I, [I, V, I, V, I, V, V, I, V, V, I, I, I, I, I, V]),
    "es_gemm_nt_resid_ln": (I, [V, I, V, I, V, V, I, V, I, V, V, V, I, V, V, I, I, I, F, V]),
    "es_set_gemm_variant": (I, [I]),
    "es_set_gemm_small_tile": (I, [I]),
    "es_gemm_tn_workspace": (Z, [I, I, I]),
    "es_gemm_tn": (I, [V, I, V, I, I, I, I, I, V, V, I, V, V]),
    "es_gemm_tn_ex": (I, [V, I, V, I, I, I, I, I, V, V, I, V, I, V]),
    "es_set_tn_variant": (I, [I]),
    "es_set_attn_variant": (I, [I]),
    "es_set_attn_bwd_variant": (I, [I]),
    "es_set_attn_bwd_grid": (I, [I]),
    "es_set_ln_fwd_grid": (I, [I]),
    "es_set_attn_bwd_long": (I, [I]),
    "es_splitk_reduce": (I, [V, V, I, I, I, V]),
    "es_tn_problem_size": (Z, []),
    "es_gemm_tn_grouped_prepare": (I, [V, I]),
    "es_gemm_tn_grouped": (I, [V, I, I, V]),
    "es_set_stem_kernels": (I, [I]),
    "es_gemm_tn_big_grouped_table_bytes": (Z, [I]),
    "es_gemm_tn_big_grouped_workspace": (Z, [V, I, I]),
    "es_gemm_tn_big_grouped_prepare": (I, [V, I, I, V, Z, V, V]),
    "es_gemm_tn_big_grouped": (I, [V, I, V, V]),
    "es_gemm_tn_big_grouped_timed": (I, [V, I, V, V, V, V]),
    "es_event_create": (I, [V]),
    "es_event_elapsed": (I, [V, V, V]),
    "es_event_destroy": (I, [V]),
    "es_colsum": (I, [V, I, I, I, V, I, V, I, V]),
    "es_attn_fwd": (I, [V, I, V, I, V, I, I, I, F, V]),
    "es_attn_bwd": (I, [V, I, V, I, V, V, V, I, V, I, I, I, I, F, V]),
    "es_attn_cls_fwd": (I, [V, I, V, I, V, I, I, I, F, V]),
    "es_attn_cls_bwd": (I, [V, I, V, I, V, V, I, V, I, I, I, I, F, V]),
    "es_reduce_partials": (I, [V, V, I, I, I, V]),
    "es_layernorm_fwd": (I, [V, I, V, V, V, I, V, V, I, I, F, V]),
    "es_layernorm_bwd": (I, [V, I, V, I, V, V, V, V, I, V, I, V, I, V, V, V, I, I, I, I, V]),
    "es_layernorm_bwd_b16": (I, [V, I, V, I, V, V, V, V, I, V, I, V, I, V, V, V, I, I, I, I, V]),
    "es_layernorm_bwd_grid": (I, [I, I]),
    "es_ln_param_grads_entry_size": (I, []),
    "es_ln_param_grads_multi": (I, [V, I, V]),
    "es_gelu_fwd": (I, [V, V, L, V]),
    "es_gelu_bwd": (I, [V, V, V, L, V]),
    "es_patch_im2col": (I, [V, V, I, I, I, V]),
    "es_patch_im2col_u8": (I, [V, F, F, F, F, F, F, V, I, I, I, V]),
    "es_cls_init": (I, [V, I, V, V, I, I, I, V]),
    "es_embed_bwd": (I, [V, I, V, I, V, V, I, I, I, I, V]),
    "es_cls_head_fwd": (I, [V, I, I, V, V, V, V, V, I, V, V, I, I, I, F, V]),
    "es_cls_head_bwd": (I, [V, I, V, V, V, V, V, V, V, I, I, V, V, V, V, I, I, I, V]),
    "es_cls_head_bwd_ex": (I, [V, I, V, V, V, V, V, V, V, I, I, V, V, V, V, I, I, I, I, V]),
    "es_cls_ln_fwd": (I, [V, I, I, V, V, V, I, V, V, I, I, F, V]),
    "es_cls_ln_bwd": (I, [V, I, V, V, V, V, I, I, V, V, I, I, V]),
    "es_dense_fwd": (I, [V, I, V, V, V, I, I, I, I, I, F, V, F, V]),
    "es_dense_bwd_workspace": (Z, [I, I]),
    "es_dense_bwd": (I, [V, I, V, I, I, F, V, F, V, I, V, V, I, I, V, V, I, I, I, V, V]),
    "es_bn1d_fwd": (I, [V, I, V, V, V, V, V, F, F, I, V, I, V, V, I, I, V]),
    "es_bn1d_bwd": (I, [V, I, V, V, V, V, I, V, V, I, I, V]),
    "es_dropout_keep": (I, [V, L, F, U64, U64, V]),
    "es_bn1d_sums": (I, [V, I, I, I, V, F, V, V]),
    "es_bn1d_fwd_global": (I, [V, I, V, V, V, V, F, V, V, V, F, F, V, I, V, V, I, I, V]),
    "es_bn1d_bwd_sums": (I, [V, I, V, I, I, V, V]),
    "es_bn1d_bwd_global": (I, [V, I, V, V, V, V, V, F, V, I, V, V, I, I, V]),
    "es_l2norm_fwd": (I, [V, I, V, I, V, I, I, V]),
    "es_l2norm_bwd": (I, [V, I, V, I, V, V, I, I, I, V]),
    "es_comatch_pseudo_workspace": (Z, [I, I, I]),
    "es_comatch_pseudo": (I, [V, I, I, I, V, I, I, I, V, I, I, V, V, I, F, F, F, V, V, V, V, V, V]),
    "es_comatch_pseudo_ex": (I, [V, I, I, I, V, I, I, I, I, V, I, I, V, V, I, F, F, F, V, V, V, V, V, V]),
    "es_softmax_colmean": (I, [V, I, I, I, V, V]),
    "es_comatch_bank_write": (I, [V, I, I, V, I, I, I, V, V, I, V, V, I, I, V]),
    "es_comatch_contrastive_workspace": (Z, [I]),
    "es_comatch_contrastive_fwd_bwd": (I, [V, I, V, I, V, I, I, I, F, F, F, V, V, I, V, I, V, V]),
    "es_comatch_contrastive_ex_workspace": (Z, [I, I]),
    "es_comatch_contrastive_fwd_bwd_ex": (I, [V, I, V, I, V, V, I, I, I, I, I, F, F, F, F, V, V, I, V, I, V, V]),
    "es_comatch_focal_fwd_bwd": (I, [V, I, V, V, I, I, F, F, V, V, I, V, V]),
    "es_fm_consistency_fwd_bwd": (I, [V, I, V, I, I, I, F, F, V, V, V, V, I, V, V]),
    "es_poly_ce_fwd_bwd": (I, [V, I, V, V, I, I, F, F, V, I, V, V]),
    "es_conv2d_fwd": (I, [V, I, I, I, I, L, L, L, L, V, V, I, I, I, I, I, V, L, L, L, I, V]),
    "es_conv2d_bwd_data": (I, [V, L, L, L, V, I, I, I, I, I, I, I, I, I, V, L, L, L, L, I, V]),
    "es_conv2d_dw_tiles": (I, [I, I, I, I]),
    "es_conv2d_bwd_weight_workspace": (Z, [I, I, I, I, I]),
    "es_conv2d_bwd_weight": (I, [V, I, I, I, I, L, L, L, L, V, L, L, L, I, I, I, I, I, I, V, V, I, V]),
    "es_conv2d_bf16_eligible": (I, [I, I, I, I]),
    "es_set_conv_dw_target": (I, [I]),
    "es_conv2d_pack_bf16": (I, [V, I, I, I, I, V, V, V]),
    "es_conv_pack_entry_size": (I, []),
    "es_set_conv_ring": (I, [I]),
    "es_set_conv_dw_buf": (I, [I]),
    "es_set_conv_small": (I, [I]),
    "es_conv2d_pack_bf16_multi": (I, [V, I, L, V]),
    "es_conv2d_fwd_bf16": (I, [V, I, I, I, I, L, L, L, L, V, V, I, I, I, I, I, V, L, L, L, I, V]),
    "es_conv2d_bwd_data_bf16": (I, [V, L, L, L, V, I, I, I, I, I, I, I, I, I, V, L, L, L, L, I, V]),
    "es_conv2d_bnstats_size": (Z, [I, I]),
    "es_conv2d_fwd_bf16_bnstats": (I, [V, I, I, I, I, L, L, L, L, V, V, I, I, I, I, I, V, L, L, L, V, V]),
    "es_bn2d_fwd_partials": (I, [V, I, I, V, V, V, V, V, V, F, F, V, I, V, V, V, V]),
    "es_conv2d_bwd_weight_bf16_workspace": (Z, [I, I, I, I, I, I]),
    "es_conv2d_bwd_weight_bf16": (I, [V, I, I, I, I, L, L, L, L, V, L, L, L, I, I, I, I, I, I, V, V, I, V]),
    "es_chan_workspace": (Z, [I, I]),
    "es_chan_sum": (I, [V, I, I, L, L, I, V, V, I, V]),
    "es_bn2d_fwd": (I, [V, I, I, V, V, V, V, V, F, F, I, V, I, V, V, V, V, V]),
    "es_bn2d_bwd": (I, [V, V, V, I, I, I, V, V, V, I, V, F, V, V, V, V, I, V, V]),
    "es_bn2d_sums": (I, [V, I, I, I, V, I, V, V, V]),
    "es_bn2d_fwd_global": (I, [V, I, I, V, V, V, V, V, F, F, V, V, I, V, I, V, V, V, V]),
    "es_bn2d_bwd_sums": (I, [V, V, V, I, I, I, V, V, V, V, V]),
    "es_bn2d_bwd_global": (I, [V, V, V, I, I, I, V, V, V, V, V, I, V, V, V, V, I, V]),
    "es_maxpool2d_fwd": (I, [V, I, I, I, I, I, I, I, V, V, V]),
    "es_maxpool2d_bwd": (I, [V, V, I, I, I, I, I, I, I, V, V]),
    "es_avgpool2d_fwd": (I, [V, I, I, I, I, I, V, V]),
    "es_avgpool2d_bwd": (I, [V, I, I, I, I, I, V, I, V]),
    "es_upsample_add_fwd": (I, [V, V, I, I, I, I, I, V, V]),
    "es_upsample_bwd": (I, [V, I, I, I, I, I, V, V]),
    # bf16 activation / gradient maps (flags: bit 0 the input maps bf16, bit 1 the output map bf16)
    "es_conv2d_fwd_bf16_ex": (I, [V, I, I, I, I, L, L, L, L, V, V, I, I, I, I, I, V, L, L, L, I, V, I, V]),
    "es_conv2d_bwd_data_bf16_ex": (I, [V, L, L, L, V, I, I, I, I, I, I, I, I, I, V, L, L, L, L, I, I, V]),
    "es_conv2d_bwd_weight_bf16_ex": (I, [V, I, I, I, I, L, L, L, L, V, L, L, L, I, I, I, I, I, I, V, V, I, I, V]),
    "es_conv2d_fwd_bf16_bnin_ex": (I, [V, I, I, I, I, L, L, L, L, V, V, I, I, I, I, I, V, L, L, L, I, V, I, V, V, V, V, V]),
    "es_conv2d_bwd_weight_bf16_bnin_ex": (I, [V, I, I, I, I, L, L, L, L, V, L, L, L, I, I, I, I, I, I, V, V, I, I,
                                             V, V, V, V, V]),
    "es_chan_sum_ex": (I, [V, I, I, L, L, I, V, V, I, I, V]),
    "es_set_bn_cs": (I, [I]),
    "es_set_bn_sum8": (I, [I]),
    "es_bn2d_fwd_ex": (I, [V, I, I, V, V, V, V, V, F, F, I, V, I, V, V, V, V, I, V]),
    "es_bn2d_bwd_ex": (I, [V, V, V, I, I, I, V, V, V, I, V, F, V, V, V, V, I, V, I, V]),
    "es_bn2d_bwd_recompute_ex": (I, [V, V, I, I, V, V, V, V, V, V, V, I, V, I, V]),
    "es_bn2d_fwd_partials_ex": (I, [V, I, I, V, V, V, V, V, V, F, F, V, I, V, V, V, I, V]),
    "es_bn2d_sums_ex": (I, [V, I, I, I, V, I, V, V, I, V]),
    "es_bn2d_fwd_global_ex": (I, [V, I, I, V, V, V, V, V, F, F, V, V, I, V, I, V, V, V, I, V]),
    "es_bn2d_bwd_sums_ex": (I, [V, V, V, I, I, I, V, V, V, V, I, V]),
    "es_bn2d_bwd_global_ex": (I, [V, V, V, I, I, I, V, V, V, V, V, I, V, V, V, V, I, I, V]),
    "es_maxpool2d_fwd_ex": (I, [V, I, I, I, I, I, I, I, V, V, I, V]),
    "es_maxpool2d_bwd_ex": (I, [V, V, I, I, I, I, I, I, I, V, I, V]),
    "es_avgpool2d_fwd_ex": (I, [V, I, I, I, I, I, V, I, V]),
    "es_avgpool2d_bwd_ex": (I, [V, I, I, I, I, I, V, I, I, V]),
    "es_upsample_add_fwd_ex": (I, [V, V, I, I, I, I, I, V, I, V]),
    "es_upsample_bwd_ex": (I, [V, I, I, I, I, I, V, I, V]),
    "es_fcu_down_tokens_fwd": (I, [V, V, V, V, V, V, V, I, I, I, F, V]),
    "es_fcu_down_workspace": (Z, [I, I, I]),
    "es_fcu_down_tokens_bwd": (I, [V, V, V, V, V, V, V, V, V, V, I, I, I, I, V, V]),
    "es_fcu_down_tokens_bwd_ex": (I, [V, V, V, V, V, V, V, V, V, V, I, I, I, I, V, I, V]),
    "es_tokens_cls_set": (I, [V, I, I, I, V, V]),
    "es_ce_weighted_fwd_bwd": (I, [V, I, V, V, I, I, F, V, I, V, V]),
    "es_ce_weight_sum": (I, [V, V, I, I, V, V]),
    "es_ce_weighted_fwd_bwd_global": (I, [V, I, V, V, V, I, I, F, V, I, V, V]),
    "es_adam_ema_step": (I, [V, V, V, V, V, L, F, F, F, F, F, F, F, F, V]),
    "es_ema_entry_size": (I, []),
    "es_ema_update_multi": (I, [V, V, I, F, F, V]),
    "es_pack_entry_size": (I, []),
    "es_pack_weights": (I, [V, V, I, V]),
    "es_cast_f32_bf16": (I, [V, V, L, V]),
    "es_add_f32": (I, [V, V, L, V]),
    # fp32 parity mode (csrc/parity.hip): the bf16 entry points' signatures, fp32 storage
    "es_gemm_nt_f32": (I, [I, V, I, V, I, V, V, I, V, V, I, I, I, I, I, V]),
    "es_gemm_tn_f32_workspace": (Z, [I, I, I]),
    "es_gemm_tn_f32": (I, [V, I, V, I, I, I, I, I, V, V, I, V, V]),
    "es_attn_fwd_f32": (I, [V, I, V, I, V, I, I, I, F, V]),
    "es_attn_bwd_f32": (I, [V, I, V, I, V, V, V, I, V, I, I, I, I, F, V]),
    "es_attn_cls_fwd_f32": (I, [V, I, V, I, V, I, I, I, F, V]),
    "es_attn_cls_bwd_f32": (I, [V, I, V, I, V, V, I, V, I, I, I, I, F, V]),
    "es_layernorm_fwd_f32": (I, [V, I, V, V, V, I, V, V, I, I, F, V]),
    "es_layernorm_bwd_f32": (I, [V, I, V, I, V, V, V, V, I, V, I, V, I, V, V, V, I, I, I, I, V]),
    "es_patch_im2col_f32": (I, [V, V, I, I, I, V]),
    "es_patch_im2col_u8_f32": (I, [V, F, F, F, F, F, F, V, I, I, I, V]),
    "es_embed_bwd_f32": (I, [V, I, V, I, V, V, I, I, I, I, V]),
    "es_pack_weights_f32": (I, [V, V, I, V]),
    "es_copy_f32": (I, [V, V, L, V]),
}

ABI_VERSION = 1
_STATUS = {-1: "bad shape", -2: "bad argument", -3: "HIP error"}


class EndosslLibraryError(RuntimeError):
    pass


class EndosslCallError(RuntimeError):
    pass


_lib = None


def load(path=None):
    """Load (once) and type the shared library.  Raises EndosslLibraryError if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise EndosslLibraryError(
            f"endossl HIP library not found at {p}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (make -C endoscopy-image-classification_amd/csrc).  There is no CPU fallback.")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.es_abi_version() != ABI_VERSION:
        raise EndosslLibraryError(f"ABI mismatch: library {lib.es_abi_version()} != python {ABI_VERSION}")
    # kernel-family pins for A/B runs (scripts/): ENDOSSL_GEMM_VARIANT / ENDOSSL_TN_VARIANT (the other
    # es_set_* knobs are reached through the library handle)
    for env, fn in (("ENDOSSL_TN_VARIANT", "es_set_tn_variant"), ("ENDOSSL_GEMM_VARIANT", "es_set_gemm_variant")):
        if os.environ.get(env) and getattr(lib, fn)(int(os.environ[env])) == -2:
            raise EndosslLibraryError(f"{env}={os.environ[env]}: no such kernel family ({fn} returned ES_BAD_ARG)")
    if path is None:
        _lib = lib
    return lib


def call(name, *args):
    """Invoke an entry point and raise on a non-zero status."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise EndosslCallError(f"{name} failed: {_STATUS.get(rc, rc)}")
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Refuses CPU tensors: no CPU fallback exists."""
    if t is None:
        return None
    if not t.is_cuda:
        raise EndosslCallError("endossl kernels take device tensors only (got a CPU tensor)")
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


class KernelEvent:
    """A timing event for the library's *_timed launches (es_event_create): stamped by the kernel dispatch
    itself, so start.elapsed_time(stop) is the launches' execution time as a rocprofv3 kernel trace reports
    it.  Same interface as torch.cuda.Event.elapsed_time (ms; waits for `stop`)."""

    def __init__(self):
        self.handle = ctypes.c_void_p()
        rc = load().es_event_create(ctypes.byref(self.handle))
        if rc != 0:
            raise EndosslLibraryError(f"es_event_create: status {rc}")

    def elapsed_time(self, stop):
        ms = ctypes.c_float()
        rc = load().es_event_elapsed(self.handle, stop.handle, ctypes.byref(ms))
        if rc != 0:
            raise EndosslLibraryError(f"es_event_elapsed: status {rc}")
        return ms.value

    def __del__(self):
        try:
            if self.handle:
                load().es_event_destroy(self.handle)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass
