"""ctypes binding of the HIP C ABI (include/arcweld_amd.h).

The library is loaded AFTER ``import torch`` so that its ``libamdhip64.so.7`` dependency resolves (by SONAME) to
the HIP runtime torch already loaded: device pointers, streams and the caching allocator are then shared.
There is no fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the library load, see module docstring)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ARCWELD_LIB overrides the library path (A/B timing of two builds in one process tree: tools/ab_bench.sh)
LIB_PATH = os.environ.get("ARCWELD_LIB") or os.path.join(PKG_DIR, "lib", "libarcweld_amd.so")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "arcweld_amd.h")

AW_F32, AW_BF16 = 0, 1
AW_ACT_GELU_ERF, AW_ACT_GELU_TANH, AW_ACT_DERIV = 0, 1, 2
AW_STORE_NT, AW_STORE_WT = 0, 1   # aw_gemm_args.store_policy

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f = ctypes.c_float
c_p = ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("a_dtype", c_int),
        ("A", c_p), ("lda", c_i64), ("a_trans", c_int),
        ("B", c_p), ("ldb", c_i64), ("b_trans", c_int),
        ("conv_cin", c_int), ("conv_seg", c_int), ("conv_dir", c_int), ("conv_operand", c_int),
        ("alpha", c_f), ("beta", c_f),
        ("bias", c_p),
        ("act", c_int),
        ("pre", c_p), ("ld_pre", c_i64),
        ("resid", c_p), ("ld_resid", c_i64),
        ("drop_p", c_f), ("drop_seed", ctypes.c_uint64),
        ("C", c_p), ("ldc", c_i64), ("c_dtype", c_int),
        ("C2", c_p), ("ldc2", c_i64), ("c2_mode", c_int), ("c2_dtype", c_int),
        ("drop2_p", c_f), ("drop2_seed", ctypes.c_uint64),
        ("colstats", c_p), ("stats_mod", c_int),
        ("a_rowsum", c_p),
        ("bias_mod", c_int),
        ("accumulate", c_int), ("col_mod", c_int), ("col_mul", c_int), ("col_off", c_int),
        ("seed_ptr", c_p),
        ("pre_dtype", c_int),
        ("store_policy", c_int),
        ("resid_dtype", c_int),
    ]


class RelayoutJob(ctypes.Structure):
    """aw_relayout_job (include/arcweld_amd.h)."""
    _fields_ = [("W", c_p), ("out", c_p), ("O", c_int), ("I", c_int), ("k", c_int), ("tap", c_int),
                ("mode", c_int), ("ldo", c_i64)]


class OperandDesc(ctypes.Structure):
    """aw_operand_desc (include/arcweld_amd.h)."""
    _fields_ = [("out", c_p), ("O", c_int), ("I", c_int), ("k", c_int), ("tap", c_int), ("mode", c_int),
                ("dtype", c_int), ("ldo", c_i64)]


OPS_PER_SEG = 2     # AW_OPS_PER_SEG

RES_CHAIN_MAX = 16  # AW_RES_CHAIN_MAX
RES_PACK_MAX = 32   # AW_RES_PACK_MAX
_E = RES_CHAIN_MAX


class ResChainFwdArgs(ctypes.Structure):
    """aw_res_chain_fwd_args (include/arcweld_amd.h)."""
    _fields_ = [("N", c_i64), ("H", c_int), ("R", c_int), ("taps", c_int), ("seg", c_int), ("a0", c_p), ("x0", c_p),
                ("w1", c_p * _E), ("w2", c_p * _E), ("b1", c_p * _E), ("b2", c_p * _E),
                ("dgelu_h", c_p * _E), ("a1", c_p * _E), ("dgelu_x", c_p * _E), ("a", c_p * _E),
                ("drop_p", c_f), ("drop_seed", ctypes.c_uint64 * _E), ("seed_ptr", c_p), ("store_policy", c_int),
                ("drop_masks", c_p)]


class ResChainBwdArgs(ctypes.Structure):
    """aw_res_chain_bwd_args (include/arcweld_amd.h)."""
    _fields_ = [("N", c_i64), ("H", c_int), ("R", c_int), ("taps", c_int), ("seg", c_int), ("gx", c_p), ("gxo", c_p),
                ("x0", c_p), ("w1t", c_p * _E), ("w2t", c_p * _E), ("dgelu_h", c_p * _E), ("dgelu_x", c_p * _E),
                ("gh", c_p * _E), ("gxo_out", c_p * _E),
                ("drop_p", c_f), ("store_policy", c_int), ("drop_masks", c_p)]

# name -> argtypes (every entry returns int status except aw_last_error)
SIGNATURES = {
    "aw_version": [],
    "aw_gemm": [ctypes.POINTER(GemmArgs), c_p],
    "aw_gemm_ws": [ctypes.POINTER(GemmArgs), c_p, c_i64, c_p],
    "aw_gemm_workspace": [ctypes.POINTER(GemmArgs)],
    "aw_gemm_grouped": [ctypes.POINTER(GemmArgs), c_int, c_p],
    "aw_gemm_set_tile": [c_int],
    "aw_gemm_set_wgrad_policy": [c_int],
    "aw_wgrad_batch_workspace": [ctypes.POINTER(GemmArgs), c_int],
    "aw_wgrad_batch": [ctypes.POINTER(GemmArgs), c_int, c_p, c_i64, c_p],
    "aw_wgrad_set_spin_limit": [c_int],
    "aw_res_chain_fwd": [ctypes.POINTER(ResChainFwdArgs), c_p],
    "aw_res_chain_bwd": [ctypes.POINTER(ResChainBwdArgs), c_p],
    "aw_res_pack_weights": [ctypes.POINTER(c_p), ctypes.POINTER(c_p), ctypes.POINTER(c_p), c_int, c_int, c_p],
    "aw_res_dropout_masks_bytes": [c_i64, c_int],
    "aw_res_dropout_masks": [c_i64, c_int, c_f, ctypes.POINTER(ctypes.c_uint64), c_p, c_p, c_p],
    "aw_weight_relayout_batch": [ctypes.POINTER(RelayoutJob), c_int, c_int, c_p],
    "aw_vq_forward": [c_p, c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p],
    "aw_vq_forward_ex": [c_p, c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_int, c_p],
    "aw_vq_finalize": [c_p, c_p, c_i64, c_int, c_int, c_f, c_p, c_p, c_p],
    "aw_vq_forward_ex2": [c_p, c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_int, c_p, c_p, c_int, c_p],
    "aw_vq_finalize_ex": [c_p, c_int, c_p, c_i64, c_int, c_int, c_f, c_p, c_p, c_p],
    "aw_vq_backward": [c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_f, c_p, c_p, c_p],
    "aw_vq_backward_ex": [c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_f, c_p, c_p, c_p, c_int, c_p],
    "aw_vq_onehot": [c_p, c_i64, c_int, c_p, c_p],
    "aw_vq_gather": [c_p, c_p, c_i64, c_int, c_p, c_p],
    "aw_patchify": [c_p, c_i64, c_int, c_int, c_int, c_p, c_i64, c_int, c_p],
    "aw_weight_relayout": [c_p, c_int, c_int, c_int, c_int, c_int, c_p, c_i64, c_int, c_p],
    "aw_weight_grad_scatter": [c_p, c_int, c_int, c_int, c_int, c_int, c_i64, c_p, c_p],
    "aw_cast": [c_p, c_i64, c_p, c_int, c_p],
    "aw_unpatch_head_fwd": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p],
    "aw_bn_finalize": [c_p, c_i64, c_int, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_int, c_p, c_p],
    "aw_unpatch_head_bwd1": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "aw_unpatch_head_bwd2": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_int, c_p, c_int, c_p, c_p],
    "aw_unpatch_head_fwd_ex": [c_p, c_int, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p],
    "aw_unpatch_head_bwd1_ex": [c_p, c_int, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "aw_unpatch_head_fwd_bwd1": [c_p, c_int, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                 c_p, c_p, c_p, c_p],
    "aw_unpatch_head_bwd2_ex": [c_p, c_int, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_int, c_p, c_int, c_p, c_p],
    "aw_bn_group_stats": [c_p, c_i64, c_int, c_int, c_p, c_p],
    "aw_bn_group_finalize": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_int, c_p, c_p],
    "aw_bn_apply": [c_p, c_i64, c_int, c_int, c_p, c_int, c_p, c_f, ctypes.c_uint64, c_p, c_p, c_p, c_int, c_p],
    "aw_bn_bwd_reduce": [c_p, c_i64, c_int, c_int, c_p, c_p, c_f, ctypes.c_uint64, c_p, c_p, c_p],
    "aw_bn_bwd_apply": [c_p, c_i64, c_int, c_int, c_p, c_p, c_f, ctypes.c_uint64, c_p, c_p, c_i64, c_int, c_p, c_int,
                        c_p, c_p, c_p],
    "aw_mse_fwd": [c_p, c_p, c_i64, c_p, c_p],
    "aw_mse_bwd": [c_p, c_p, c_i64, c_p, c_p, c_p],
    "aw_scalar_add": [c_p, c_p, c_p, c_p],
    "aw_mse_finalize": [c_p, c_i64, c_p, c_p],
    "aw_mse_finalize_add": [c_p, c_i64, c_p, c_p, c_p, c_p],
    "aw_radam_step": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_i64, c_i64, c_f, c_f, c_f, c_f, c_p, c_p,
                      c_int, c_p],
    "aw_radam_step_ops": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_i64, c_i64, c_f, c_f, c_f, c_f, c_p, c_p,
                          c_p, c_int, c_p],
    "aw_counter_add": [c_p, c_i64, c_p],
    "aw_counter_add_snapshot": [c_p, c_i64, c_p, c_p],
    "aw_counter_add_snapshot_zero": [c_p, c_i64, c_p, c_p, c_i64, c_p],
    "aw_grad_norm_clip": [c_p, c_p, c_p, c_p, c_int, c_i64, c_f, c_p, c_p, c_p, c_p],
    "aw_scale": [c_p, c_i64, c_p, c_p],
    "aw_layernorm_fwd": [c_p, c_i64, c_int, c_p, c_p, c_f, c_p, c_int, c_p, c_p, c_p],
    "aw_layernorm_bwd": [c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_p, c_int, c_p, c_p, c_p, c_int, c_f,
                         ctypes.c_uint64, c_p, c_p],
    "aw_class_head_fwd": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "aw_class_head_bwd": [c_p, c_p, c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "aw_embed_fwd": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p],
    "aw_embed_ln_fwd": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_int, c_p, c_p, c_p],
    "aw_embed_bwd": [c_p, c_i64, c_int, c_int, c_p, c_p, c_p],
    "aw_embed_bwd_sorted": [c_p, c_i64, c_int, c_int, c_int, c_p, c_p, c_p, c_p],
    "aw_embed_sort": [c_p, c_i64, c_int, c_p, c_p],
    "aw_embed_bwd_segsum": [c_p, c_int, c_int, c_p, c_p, c_p],
    "aw_attn_fwd": [c_p, c_i64, c_int, c_int, c_int, c_int, c_p, c_p, c_p],
    "aw_attn_bwd": [c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_int, c_int, c_p, c_p, c_p],
    "aw_attn_fwd_dropout": [c_p, c_i64, c_int, c_int, c_int, c_int, c_p, c_p, c_f, ctypes.c_uint64, c_p, c_p],
    "aw_attn_bwd_dropout": [c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_int, c_int, c_p, c_p, c_f, ctypes.c_uint64,
                            c_p, c_p],
    "aw_attn_decode": [c_p, c_i64, c_int, c_int, c_int, c_int, c_int, c_p, c_int, c_p, c_p],
    "aw_ce_fwd": [c_p, c_i64, c_int, c_i64, c_p, c_int, c_p, c_p, c_p, c_p],
    "aw_ce_bwd": [c_p, c_i64, c_int, c_i64, c_p, c_int, c_p, c_p, c_p, c_p, c_i64, c_int, c_p],
    "aw_ce_finalize": [c_p, c_p, c_p, c_p],
    "aw_vq_cluster_sums": [c_p, c_p, c_i64, c_int, c_int, c_p, c_p],
    "aw_kmeans_update": [c_p, c_p, c_p, c_int, c_int, c_p, c_p],
    "aw_rvq_ema_update": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_f, c_f, c_f, ctypes.c_uint64, c_p, c_p,
                          c_p],
    "aw_rvq_residual": [c_p, c_p, c_i64, c_p, c_int, c_p, c_p],
    "aw_rvq_backward": [c_p, c_p, c_p, c_p, c_int, c_i64, c_int, c_f, c_p, c_p],
}

RET_I64 = {"aw_gemm_workspace", "aw_wgrad_batch_workspace", "aw_res_dropout_masks_bytes"}

_lib = None


class NativeError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library with typed entry points."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeError(f"HIP library not built: {path} is missing (run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` or `make -C vq-vae-transformer-arc-welding_amd/csrc`)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    lib.aw_last_error.restype = ctypes.c_char_p
    lib.aw_last_error.argtypes = []
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = c_i64 if name in RET_I64 else c_int
        fn.argtypes = argtypes
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    status = getattr(lib, name)(*args)
    if status != 0:
        raise NativeError(f"{name} failed ({status}): {lib.aw_last_error().decode(errors='replace')}")


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL).  CPU tensors are rejected: no host fallback exists."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeError("arcweld HIP kernels need device tensors (got a CPU tensor); there is no CPU fallback")
    return t.data_ptr()


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return AW_F32
    if dt == torch.bfloat16:
        return AW_BF16
    raise NativeError(f"unsupported operand dtype {dt}")
