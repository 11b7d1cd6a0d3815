"""ctypes binding of the C ABI in include/pcs.h (libpcs.so, built in-tree for gfx950).

There is no fallback: if the library is missing or fails to load, every GPU entry point
raises.  ``torch`` is imported first so that the HIP runtime torch ships (same SONAME
``libamdhip64.so.7``) is the one the library binds to -- one runtime per process.
"""
from __future__ import annotations

import ctypes as ct
import os

import torch  # noqa: F401  (loads torch's HIP runtime before libpcs.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "csrc", "libpcs.so")

F32, BF16, FP8 = 0, 1, 2
PRO_RAW, PRO_BNRELU, PRO_BWD, PRO_BWD_POOL, PRO_CAT = 0, 1, 2, 3, 4
EPI_FWD, EPI_DGRAD, EPI_RAW, EPI_BNRELU = 0, 1, 2, 3
HEAD_FWD, HEAD_CE, HEAD_BWD = 0, 1, 2

_vp = ct.c_void_p
_i64 = ct.c_int64
_i32 = ct.c_int32
_f = ct.c_float


class GemmArgs(ct.Structure):
    _fields_ = [
        ("num_scenes", _i64), ("scene_rows", _i64),
        ("K", _i32), ("Ncols", _i32), ("dtype", _i32), ("prologue", _i32), ("epilogue", _i32),
        ("chunks_per_scene", _i32),
        ("A", _vp), ("A2", _vp), ("pa", _vp), ("pb", _vp), ("pc", _vp), ("a_mask", _vp),
        ("a_keep_scale", _f),
        ("pool_idx", _vp), ("pool_coef", _vp),
        ("W", _vp), ("C", _vp), ("bias", _vp), ("scene_bias", _vp), ("addend", _vp),
        ("c_mask", _vp), ("c_keep_scale", _f),
        ("Yp", _vp), ("es", _vp), ("et", _vp), ("emean", _vp), ("erstd", _vp),
        ("stats", _vp), ("pool", _vp), ("flags", _i32),
        ("pool_w", _vp), ("pool_ldw", _i64), ("pool_c", _i32), ("w_scale", _vp),
        ("W2", _vp), ("K1", _i32), ("gram", _vp),
    ]


FLAG_GENERIC = 1
FLAG_NO_GLDS = 2
FLAG_AW_FP8 = 4
FLAG_C_FP8 = 8
FLAG_POOL_SIGNED_W = 16


class WgradArgs(ct.Structure):
    _fields_ = [
        ("num_scenes", _i64), ("scene_rows", _i64),
        ("Cout", _i32), ("Cin", _i32), ("dtype", _i32), ("splits_per_scene", _i32),
        ("dy_mode", _i32),
        ("dZ", _vp), ("Y", _vp), ("alpha", _vp), ("beta", _vp), ("gamma", _vp),
        ("pool_idx", _vp), ("pool_coef", _vp),
        ("x_mode", _i32),
        ("X", _vp), ("s", _vp), ("t", _vp), ("x_mask", _vp), ("x_keep_scale", _f),
        ("partial", _vp), ("dW", _vp), ("ldw", _i64), ("flags", _i32), ("dy_colsum", _vp),
    ]


class Seg12Args(ct.Structure):
    _fields_ = [
        ("num_scenes", _i64), ("scene_rows", _i64), ("chunks_per_scene", _i32),
        ("y2", _vp), ("s2", _vp), ("t2", _vp), ("W1", _vp), ("sbias", _vp), ("Y1", _vp),
        ("s1", _vp), ("t1", _vp), ("keep1", _vp), ("keep_scale", _f), ("W2", _vp), ("Y2", _vp),
        ("stats", _vp),
    ]


class Conv3dGeom(ct.Structure):
    _fields_ = [
        ("B", _i64), ("Di", _i32), ("Hi", _i32), ("Wi", _i32), ("Do", _i32), ("Ho", _i32), ("Wo", _i32),
        ("Cin", _i32), ("Cout", _i32), ("k", _i32), ("s", _i32), ("p", _i32), ("transposed", _i32),
    ]


class PoolBwdArgs(ct.Structure):
    _fields_ = [
        ("num_scenes", _i64), ("scene_rows", _i64),
        ("Cs", _i32), ("Cg", _i32), ("col_off", _i32),
        ("s1_alpha", _vp), ("s1_beta", _vp), ("s1_gamma", _vp),
        ("s1_scene_s1", _vp), ("s1_scene_sum", _vp),
        ("W_s1", _vp), ("ldw", _i64),
        ("g", _vp), ("ysel", _vp), ("g_mean", _vp), ("g_rstd", _vp), ("g_gamma", _vp),
        ("g_scene_sum", _vp),
        ("dW_s1_global", _vp), ("csum", _vp),
        ("alpha", _vp), ("beta_c", _vp), ("gamma_c", _vp),
        ("dgamma", _vp), ("dbeta", _vp), ("dbias", _vp), ("sp", _vp),
    ]


class HeadArgs(ct.Structure):
    _fields_ = [
        ("num_scenes", _i64), ("scene_rows", _i64),
        ("Cin", _i32), ("num_classes", _i32), ("dtype", _i32), ("mode", _i32),
        ("chunks_per_scene", _i32),
        ("Y", _vp), ("s", _vp), ("t", _vp), ("W", _vp), ("bias", _vp), ("logits", _vp),
        ("labels", _vp), ("class_weight", _vp), ("wsum", _vp),
        ("dlogits", _vp), ("dl_stride_row", _i64), ("dl_stride_col", _i64),
        ("dZ", _vp), ("mean", _vp), ("rstd", _vp), ("stats", _vp), ("wpartial", _vp),
        ("loss_partial", _vp),
    ]


# (name, restype, argtypes) of every exported symbol declared in include/pcs.h
SIGNATURES = [
    ("pcs_gemm_geometry", _i64, [ct.POINTER(GemmArgs)]),
    ("pcs_gemm", ct.c_int, [ct.POINTER(GemmArgs), _vp]),
    ("pcs_conv1_fwd", ct.c_int, [ct.POINTER(GemmArgs), _vp]),
    ("pcs_wgrad_workspace", _i64, [ct.POINTER(WgradArgs)]),
    ("pcs_wgrad", ct.c_int, [ct.POINTER(WgradArgs), _vp]),
    ("pcs_conv1_wgrad", ct.c_int, [ct.POINTER(WgradArgs), _vp]),
    ("pcs_bn_fwd_finalize", ct.c_int, [_vp, _i64, _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp,
                                       _vp, _f, _f, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("pcs_bn_eval_coefs", ct.c_int, [_vp, _vp, _vp, _vp, _vp, _f, _i32, _vp, _vp, _vp]),
    ("pcs_bn_bwd_finalize", ct.c_int, [_vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("pcs_pool_finalize", ct.c_int, [_vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("pcs_scene_gemv", ct.c_int, [_vp, _i64, _i32, _vp, _i64, _i32, _vp, _i32, _vp, _vp, _vp]),
    ("pcs_pool_bwd", ct.c_int, [ct.POINTER(PoolBwdArgs), _vp]),
    ("pcs_head_geometry", _i64, [ct.POINTER(HeadArgs)]),
    ("pcs_head", ct.c_int, [ct.POINTER(HeadArgs), _vp]),
    ("pcs_ce_weight_sum", ct.c_int, [_vp, _i64, _vp, _i32, _vp, _vp, _vp]),
    ("pcs_dropout_bits", ct.c_int, [ct.c_uint64, ct.c_uint64, _i64, _i32, _f, _vp, _vp]),
    ("pcs_dropout_bits_bounded", ct.c_int, [ct.c_uint64, ct.c_uint64, _i64, _i32, _f, _vp, _i32, _vp]),
    ("pcs_dropout_bits_independent", ct.c_int, [ct.c_uint64, ct.c_uint64, _i64, _i32, _f, _vp, _vp]),
    ("pcs_reduce_partials", ct.c_int, [_vp, _i64, _i64, _f, _vp, _i64, _i64, _vp]),
    ("pcs_reduce_partials_grouped", ct.c_int, [_vp, _i64, _i64, _i64, _f, _vp, _vp]),
    ("pcs_cast_weight", ct.c_int, [_vp, _i64, _i64, _i64, _i32, _vp, _vp, _vp]),
    ("pcs_adam", ct.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _f, _f, _f, _f, _f, _i64, _vp]),
    ("pcs_colstats_geometry", _i64, [_i64, _i64, _i32, ct.POINTER(_i32)]),
    ("pcs_colstats", ct.c_int, [_vp, _i64, _i64, _i32, _i32, _i32, _i64, _vp, _vp, _vp]),
    ("pcs_bnrelu_bwd", ct.c_int, [_vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32,
                                  _i32, _i64, _vp, _vp]),
    ("pcs_abi_version", ct.c_int, []),
    ("pcs_conv3d", ct.c_int, [ct.POINTER(Conv3dGeom), _vp, _vp, _vp, _vp, _i32, _vp]),
    ("pcs_conv3d_wgrad_workspace", _i64, [ct.POINTER(Conv3dGeom)]),
    ("pcs_conv3d_wgrad", ct.c_int, [ct.POINTER(Conv3dGeom), _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    ("pcs_conv3d_weight_t", ct.c_int, [_vp, _i32, _i32, _i32, _vp, _vp]),
    ("pcs_sparse_conv", ct.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _i32, _vp, _vp, _i32, _i32, _vp]),
    ("pcs_sparse_conv_wgrad_workspace", _i64, [_i64, _i32, _i32, _i32]),
    ("pcs_sparse_conv_wgrad", ct.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _i32, _vp, _i64, _vp, _vp, _vp]),
    ("pcs_sparse_pairs_workspace", _i64, [_i64, _i32]),
    ("pcs_sparse_pairs_count", ct.c_int, [_vp, _i64, _i32, _vp, _vp, _vp]),
    ("pcs_sparse_pairs_build", ct.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("pcs_sparse_conv_pairs", ct.c_int, [_vp, _vp, _vp, _i32, _i64, _vp, _i32, _vp, _i32, _vp, _vp, _vp, _i32, _i32,
                                         _vp]),
    ("pcs_sparse_conv_wgrad_pairs_workspace", _i64, [_vp, _i32, _i64, _i32, _i32]),
    ("pcs_sparse_conv_wgrad_pairs", ct.c_int, [_vp, _vp, _vp, _i32, _i64, _vp, _i32, _vp, _i32, _vp, _i64, _vp, _vp,
                                               _vp]),
    ("pcs_voxel_keys", ct.c_int, [_vp, _vp, _i64, _i64, _i32, _f, _f, _f, _f, _f, _f, _vp, _vp, _vp]),
    ("pcs_voxel_hash_capacity", _i64, [_i64]),
    ("pcs_voxel_hash_build", ct.c_int, [_vp, _i64, _vp, _vp, _i64, _vp]),
    ("pcs_voxel_hash_find", ct.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp]),
    ("pcs_sparse_neighbors", ct.c_int, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _vp]),
    ("pcs_gram_workspace", _i64, [_i64, _i64, _i32, _i32, ct.POINTER(_i32)]),
    ("pcs_gram", ct.c_int, [_vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    ("pcs_pool_rows_add", ct.c_int, [_vp, _i32, _vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _i64, _i32, _vp, _i32,
                                     _vp]),
    ("pcs_quant_fp8_rows", ct.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    ("pcs_gram_raw_workspace", _i64, [_i64, _i32]),
    ("pcs_gram_raw", ct.c_int, [_vp, _i64, _i32, _i32, _vp, _i64, _vp, _vp]),
    ("pcs_gram_wgrad", ct.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32,
                                  _i32, _vp, _vp, _vp, _i64, _vp]),
    ("pcs_bn_fold", ct.c_int, [_vp, _i32, _i32, _i64, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    ("pcs_bn_s2_from_r", ct.c_int, [_vp, _i64, _i32, _vp, _vp, _i32, _i64, _i32, _vp, _vp, _vp]),
    ("pcs_bn_stats_from_gram", ct.c_int, [_vp, _vp, _i64, _vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp]),
    ("pcs_bn_stats_from_gram_scenes_workspace", _i64, [_i32, _i32]),
    ("pcs_sign_rows", ct.c_int, [_vp, _i32, _i64, _i64, _vp, _vp, _vp]),
    ("pcs_dgrad_wgrad_folded_workspace", _i64, [ct.POINTER(WgradArgs)]),
    ("pcs_dgrad_wgrad_folded", ct.c_int, [ct.POINTER(WgradArgs), _vp, _vp, _vp, _vp, _vp, _vp]),
    ("pcs_bn_stats_from_gram_scenes", ct.c_int, [_vp, _vp, _i64, _vp, _i32, _i64, _i32, _i32, _i64, _vp, _i64, _vp,
                                                 _vp]),
    ("pcs_confusion", ct.c_int, [_vp, _i64, _vp, _i64, _i32, _vp, _vp]),
    ("pcs_argmax", ct.c_int, [_vp, _i64, _i64, _i32, _vp, _vp]),
    ("pcs_dgrad_wgrad_workspace", _i64, [ct.POINTER(WgradArgs)]),
    ("pcs_dgrad_wgrad", ct.c_int, [ct.POINTER(WgradArgs), _vp, _vp, _vp]),
    ("pcs_dgrad_wgrad_bn_workspace", _i64, [ct.POINTER(GemmArgs)]),
    ("pcs_dgrad_wgrad_bn", ct.c_int, [ct.POINTER(GemmArgs), _vp, _vp, _i64, _vp]),
    ("pcs_round_weight", ct.c_int, [_vp, _i64, _i32, _vp, _vp]),
    ("pcs_bnrelu_bf16", ct.c_int, [_vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    ("pcs_fwd_seg12_geometry", _i64, [ct.POINTER(Seg12Args)]),
    ("pcs_fwd_seg12", ct.c_int, [ct.POINTER(Seg12Args), _vp]),
    ("pcs_bn_stats_gram_sbias", ct.c_int, [_vp, _vp, _i64, _i64, _vp, _i64, _i32, _i32, _vp, _vp, _vp]),
    ("pcs_voxel_ids", ct.c_int, [_vp, _i64, _i32, _f, _f, _f, _f, _f, _f, _vp, _vp]),
    ("pcs_voxelize_workspace", _i64, [_i64]),
    ("pcs_voxelize", ct.c_int, [_vp, _vp, _vp, _i64, _i64, _i32, _f, _f, _f, _f, _f, _f, _i32, _vp, _i64,
                                _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("pcs_gather_rows", ct.c_int, [_vp, _i64, _vp, _i64, _i32, _vp, _vp]),
    ("pcs_voxel_padded_index", ct.c_int, [_vp, _i64, _vp, _i64, _i64, _vp, _vp]),
    ("pcs_pad_scatter", ct.c_int, [_vp, _vp, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    ("pcs_last_error", ct.c_char_p, []),
]

_lib = None


# include/pcs.h PCS_ABI_VERSION: the layout of the structs mirrored in this file
ABI_VERSION = 2


class PcsError(RuntimeError):
    pass


def load():
    """Load libpcs.so (raises ImportError with build instructions when absent)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("PCS_LIB", LIB_PATH)   # an alternative build, for A/B timing
    if not os.path.exists(path):
        raise ImportError(
            f"pcs_amd HIP library not built: {path} is missing. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or "
            "`make -C point-cloud-cnn-segmentation_amd/csrc`.")
    lib = ct.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    got = lib.pcs_abi_version()
    if got != ABI_VERSION:   # the ctypes structs below mirror one layout of include/pcs.h
        raise ImportError(f"{path} has C ABI version {got}, this binding expects {ABI_VERSION}: rebuild it "
                          "(`make -C point-cloud-cnn-segmentation_amd/csrc`)")
    _lib = lib
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc < 0:
        raise PcsError(f"{name} failed ({rc}): {lib.pcs_last_error().decode()}")
    return rc


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream
