"""ctypes binding of libdqrm's C ABI (include/dqrm.h).

This is the same binding a maintainer would add to the reference:
plain pointers, sizes and an int status per call. There is no CPU fallback: if the
shared library is missing, importing the compute path raises.
"""
from __future__ import annotations

import ctypes as C
import os

from ._build import LIB_PATH

DQRM_OK = 0
DQRM_E_INVALID = -1
DQRM_E_HIP = -2
DQRM_E_CAPACITY = -3
DQRM_E_WORKSPACE = -4

DQRM_BATCH_POOLING_ONE = 1
DQRM_ERRF_INDEX = 1
DQRM_ERRF_OFFSET = 2
DQRM_ERRF_OVERFLOW = 4
DQRM_ERRF_STALL = 8

DQRM_BLOCK_ROWS = 256
DQRM_SBLOCK_ROWS = 65536
DQRM_TABLE_SPLIT = 8
DQRM_SYNC_STRIDE = 64
DQRM_SLOT_KEYS = 8192

DQRM_FWD_REFRESH_SCALE = 1
DQRM_FWD_USE_PACKED = 2
DQRM_FWD_FULL_PRECISION = 4
DQRM_FWD_NT_STORE = 16

DQRM_UPD_DP = 0
DQRM_UPD_SIMULATED = 1
DQRM_UPD_FP32 = 2
DQRM_APPLY_AUTO = 0
DQRM_APPLY_FLAT = 1
DQRM_APPLY_SLOT = 2
DQRM_APPLY_RANGES = 3
DQRM_APPLY_MERGE = 4
DQRM_APPLY_FWD_SEPARATE = 0
DQRM_APPLY_FWD_ONE_LAUNCH = 1
DQRM_APPLY_FWD_FIN_FWD = 2
DQRM_COALESCE_AUTO = 0
DQRM_COALESCE_GENERAL = 1

DQRM_CRITEO_RECORD_INTS = 40
DQRM_CRITEO_DENSE = 13
DQRM_CRITEO_SPARSE = 26

DQRM_WIRE_F16 = 1
DQRM_WIRE_I32 = 2
DQRM_WIRE_F32 = 3

DQRM_ABI_VERSION = 11  # include/dqrm.h
DQRM_PRESUM_MAX_LOOKUPS = 2048

# every symbol include/dqrm.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "dqrm_refresh_absmax",
    "dqrm_refresh_scale_and_pack",
    "dqrm_emb_fwd",
    "dqrm_bwd_workspace_bytes",
    "dqrm_emb_bwd_sgd",
    "dqrm_coalesce_slot_caps",
    "dqrm_emb_bwd_coalesce",
    "dqrm_emb_bwd_coalesce_scaled",
    "dqrm_emb_bwd_lookup_grad",
    "dqrm_rows_changed",
    "dqrm_emb_fwd_after_update",
    "dqrm_payload_bytes",
    "dqrm_grad_quant_pack",
    "dqrm_grad_quant_pack_strided",
    "dqrm_grad_quant_pack_ranked",
    "dqrm_emb_local_update",
    "dqrm_apply_sparse_update",
    "dqrm_apply_sparse_update_strided",
    "dqrm_apply_sparse_update_fwd",
    "dqrm_apply_fwd_is_one_launch",
    "dqrm_apply_fwd_form",
    "dqrm_apply_workspace_bytes",
    "dqrm_apply_local",
    "dqrm_emb_bwd_apply_local",
    "dqrm_bwd_apply_local_is_one_launch",
    "dqrm_emb_bwd_apply_fwd_local",
    "dqrm_bwd_apply_fwd_local_is_one_launch",
    "dqrm_emb_bwd_sgd_fwd",
    "dqrm_bwd_sgd_fwd_is_one_launch",
    "dqrm_dense_wire_type",
    "dqrm_dense_grad_scale",
    "dqrm_dense_grad_quant",
    "dqrm_dense_grad_decode",
    "dqrm_dense_update",
    "dqrm_criteo_unpack",
    "dqrm_rowwise_row_bytes",
    "dqrm_rowwise_prepack",
    "dqrm_rowwise_bag",
    "dqrm_init_uniform",
    "dqrm_checksum64",
    "dqrm_replica_mean",
    "dqrm_comm_unique_id",
    "dqrm_comm_init",
    "dqrm_comm_init_external",
    "dqrm_comm_destroy",
    "dqrm_comm_size",
    "dqrm_comm_allgather",
    "dqrm_exchange_grad",
    "dqrm_exchange_apply",
    "dqrm_exchange_apply_fwd",
    "dqrm_emb_bwd_lookup_grad_presum",
    "dqrm_read_errors",
    "dqrm_last_error",
    "dqrm_set_apply_kernel",
    "dqrm_set_coalesce_kernel",
    "dqrm_abi_version",
)

c_i64p = C.c_void_p  # device pointers are passed as integers

# dqrm_allgather_fn: int (*)(const void* send, void* recv, size_t bytes, void* stream, void* user)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p)


class TableSet(C.Structure):
    """Mirror of ``dqrm_table_set`` (include/dqrm.h)."""

    _fields_ = [
        ("num_tables", C.c_int32),
        ("dim", C.c_int32),
        ("total_rows", C.c_int64),
        ("total_blocks", C.c_int64),
        ("total_sblocks", C.c_int64),
        ("W", C.c_void_p),
        ("packed", C.c_void_p),
        ("rowmax", C.c_void_p),
        ("blkmax", C.c_void_p),
        ("sblkmax", C.c_void_p),
        ("tmax", C.c_void_p),
        ("scale", C.c_void_p),
        ("pscale", C.c_void_p),
        ("meta", C.c_void_p),
        ("err", C.c_void_p),
        ("tflags", C.c_void_p),
        ("sdirty", C.c_void_p),
        ("bdirty", C.c_void_p),
        ("sync", C.c_void_p),
        ("num_rows_host", C.c_void_p),  # host int64 [T] (launch planning), nullable
    ]


class Batch(C.Structure):
    """Mirror of ``dqrm_batch`` (include/dqrm.h)."""

    _fields_ = [
        ("idx", C.c_void_p),
        ("off", C.c_void_p),
        ("idx_base", C.c_void_p),
        ("num_bags", C.c_int64),
        ("max_lookups", C.c_int64),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class DenseSet(C.Structure):
    """Mirror of ``dqrm_dense_set`` (include/dqrm.h)."""

    _fields_ = [
        ("num_channels", C.c_int32),
        ("max_len", C.c_int32),
        ("total_elems", C.c_int64),
        ("grad", C.c_void_p),
        ("param", C.c_void_p),
        ("len", C.c_void_p),
        ("wire_off", C.c_void_p),
    ]


class Exchange(C.Structure):
    """Mirror of ``dqrm_exchange`` (include/dqrm.h): one rank's exchange buffers."""

    _fields_ = [
        ("set", C.POINTER(TableSet)),
        ("comm", C.c_void_p),
        ("num_ranks", C.c_int32),
        ("grad_bits", C.c_int32),
        ("ws_cap_base", C.c_void_p),
        ("ws_cap_total", C.c_int64),
        ("ws_rows", C.c_void_p),
        ("ws_vals", C.c_void_p),
        ("ws_ucount", C.c_void_p),
        ("ws_absmax", C.c_void_p),
        ("absmax_all", C.c_void_p),
        ("cap_base", C.c_void_p),
        ("cap_total", C.c_int64),
        ("s_avg", C.c_void_p),
        ("payload", C.c_void_p),
        ("gathered", C.c_void_p),
        ("payload_bytes", C.c_size_t),
        ("workspace", C.c_void_p),
        ("workspace_bytes", C.c_size_t),
        ("apply_ws", C.c_void_p),
        ("apply_ws_bytes", C.c_size_t),
    ]


class DQRMError(RuntimeError):
    pass


_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load libdqrm.so (in-tree). Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("DQRM_LIB_PATH") or LIB_PATH
    if not os.path.exists(path):
        raise DQRMError(
            f"libdqrm.so not found at {path}: build it with "
            "`python -m deep_quantized_recommendation_model_dqrm_amd._build` "
            "(no CPU fallback exists for the hot path)"
        )
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    P = C.c_void_p
    TS = C.POINTER(TableSet)
    BA = C.POINTER(Batch)
    DS = C.POINTER(DenseSet)
    sig = {
        "dqrm_refresh_absmax": (C.c_int, [TS, P]),
        "dqrm_refresh_scale_and_pack": (C.c_int, [TS, C.c_int, P]),
        "dqrm_emb_fwd": (C.c_int, [TS, BA, C.c_int, C.c_uint32, P, C.c_int64, C.c_int64, P]),
        "dqrm_bwd_workspace_bytes": (C.c_size_t, [C.c_int, C.c_int64]),
        "dqrm_emb_bwd_sgd": (
            C.c_int, [TS, BA, P, C.c_int64, C.c_int64, C.c_int, C.c_float, C.c_int, P, C.c_size_t, P]
        ),
        "dqrm_coalesce_slot_caps": (C.c_int64, [P, C.c_int, C.c_int64, P]),
        "dqrm_emb_bwd_coalesce": (
            C.c_int,
            [TS, BA, P, C.c_int64, C.c_int64, C.c_int, P, P, P, P, P, P, C.c_size_t, P],
        ),
        "dqrm_emb_bwd_coalesce_scaled": (
            C.c_int,
            [TS, BA, P, C.c_int64, C.c_int64, C.c_int, C.c_int, P, P, P, P, P, P, C.c_size_t, P],
        ),
        "dqrm_emb_bwd_lookup_grad": (C.c_int, [TS, BA, P, C.c_int64, C.c_int64, C.c_int, P, P, P]),
        "dqrm_rows_changed": (C.c_int, [TS, P, C.c_int64, C.c_int, P]),
        "dqrm_emb_fwd_after_update": (
            C.c_int,
            [TS, BA, C.c_int, C.c_uint32, P, C.c_int64, C.c_int64, P, C.c_int64, C.c_int, P],
        ),
        "dqrm_payload_bytes": (C.c_size_t, [C.c_int, C.c_int64, C.c_int, C.c_int]),
        "dqrm_grad_quant_pack": (
            C.c_int,
            [C.c_int, C.c_int, P, C.c_int64, P, P, P, P, C.c_int, C.c_int, P, C.c_int64, P, P, P],
        ),
        "dqrm_grad_quant_pack_strided": (
            C.c_int,
            [C.c_int, C.c_int, P, C.c_int64, P, P, P, P, C.c_int64, C.c_int, C.c_int, P, C.c_int64, P, P, P],
        ),
        "dqrm_grad_quant_pack_ranked": (
            C.c_int,
            [C.c_int, C.c_int, P, C.c_int64, P, P, P, P, P, P, C.c_int64, P, P],
        ),
        "dqrm_emb_local_update": (
            C.c_int,
            [TS, BA, P, C.c_int64, C.c_int64, C.c_int, C.c_float, P, C.c_int, P, C.c_size_t, P],
        ),
        "dqrm_apply_sparse_update": (
            C.c_int,
            [TS, P, C.c_int64, P, C.c_size_t, C.c_int, C.c_int, P, C.c_float, C.c_int, C.c_int, P],
        ),
        "dqrm_apply_sparse_update_strided": (
            C.c_int,
            [TS, P, C.c_int64, P, C.c_size_t, C.c_size_t, C.c_int, C.c_int, P, C.c_float, C.c_int, C.c_int, P],
        ),
        "dqrm_apply_sparse_update_fwd": (
            C.c_int,
            [TS, P, C.c_int64, P, C.c_size_t, C.c_size_t, C.c_int, C.c_int, P, C.c_float, C.c_int, C.c_int, P,
             C.c_size_t, BA, C.c_int, C.c_uint32, P, C.c_int64, C.c_int64, P],
        ),
        "dqrm_apply_workspace_bytes": (C.c_size_t, [C.c_int, C.c_int64]),
        "dqrm_apply_fwd_is_one_launch": (C.c_int, [TS, C.c_int, C.c_int64, C.c_size_t, BA, C.c_uint32]),
        "dqrm_apply_fwd_form": (C.c_int, [TS, C.c_int, C.c_int64, C.c_size_t, BA, C.c_uint32]),
        "dqrm_apply_local": (
            C.c_int,
            [TS, P, C.c_int64, P, P, P, P, C.c_int, P, C.c_float, C.c_int, P],
        ),
        "dqrm_emb_bwd_apply_local": (
            C.c_int,
            [TS, BA, P, C.c_int64, C.c_int64, C.c_int, P, C.c_int64, P, P, P, P, C.c_int, P, C.c_float, C.c_int, P,
             C.c_size_t, P],
        ),
        "dqrm_bwd_apply_local_is_one_launch": (C.c_int, [TS, BA, P]),
        "dqrm_emb_bwd_apply_fwd_local": (
            C.c_int,
            [TS, BA, P, C.c_int64, C.c_int64, C.c_int, P, C.c_int64, P, P, P, P, C.c_int, P, C.c_float, C.c_int, P,
             C.c_size_t, BA, C.c_int, C.c_uint32, P, C.c_int64, C.c_int64, P],
        ),
        "dqrm_bwd_apply_fwd_local_is_one_launch": (C.c_int, [TS, BA, BA, C.c_uint32, P]),
        "dqrm_emb_bwd_sgd_fwd": (
            C.c_int,
            [TS, BA, P, C.c_int64, C.c_int64, C.c_int, C.c_float, C.c_int, P, C.c_size_t, BA, C.c_int, C.c_uint32,
             P, C.c_int64, C.c_int64, P],
        ),
        "dqrm_bwd_sgd_fwd_is_one_launch": (C.c_int, [TS, BA, BA, C.c_uint32]),
        "dqrm_dense_wire_type": (C.c_int, [C.c_int, C.c_int]),
        "dqrm_dense_grad_scale": (C.c_int, [DS, C.c_int, P, P]),
        "dqrm_dense_grad_quant": (C.c_int, [DS, C.c_int, P, C.c_int, P, C.c_int, P, P]),
        "dqrm_dense_grad_decode": (C.c_int, [DS, P, C.c_int, C.c_int, P]),
        "dqrm_dense_update": (C.c_int, [DS, P, C.c_float, P]),
        "dqrm_criteo_unpack": (C.c_int, [P, C.c_int64, C.c_int32, P, P, P, P, P]),
        "dqrm_rowwise_row_bytes": (C.c_size_t, [C.c_int, C.c_int]),
        "dqrm_rowwise_prepack": (C.c_int, [C.c_int, P, C.c_int64, C.c_int, P, P]),
        "dqrm_rowwise_bag": (
            C.c_int,
            [C.c_int, P, C.c_int64, C.c_int, P, C.c_int64, P, C.c_int64, C.c_int, P, P, P, P],
        ),
        "dqrm_init_uniform": (C.c_int, [TS, C.c_uint64, P]),
        "dqrm_checksum64": (C.c_int, [P, C.c_int64, P, P]),
        "dqrm_replica_mean": (C.c_int, [P, C.c_int64, C.c_int, C.c_float, P]),
        "dqrm_comm_unique_id": (C.c_int, [P]),
        "dqrm_comm_init": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, P]),
        "dqrm_comm_init_external": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, ALLGATHER_FN, P]),
        "dqrm_comm_destroy": (C.c_int, [P]),
        "dqrm_comm_size": (C.c_int, [P]),
        "dqrm_comm_allgather": (C.c_int, [P, P, P, C.c_size_t, P]),
        "dqrm_exchange_grad": (C.c_int, [C.POINTER(Exchange), BA, P, C.c_int64, C.c_int64, C.c_int, P]),
        "dqrm_exchange_apply": (C.c_int, [C.POINTER(Exchange), C.c_float, C.c_int, C.c_int, P]),
        "dqrm_exchange_apply_fwd": (
            C.c_int,
            [C.POINTER(Exchange), C.c_float, C.c_int, C.c_int, BA, C.c_int, C.c_uint32, P, C.c_int64, C.c_int64, P],
        ),
        "dqrm_emb_bwd_lookup_grad_presum": (C.c_int, [TS, BA, P, C.c_int64, C.c_int64, C.c_int, P, P, P]),
        "dqrm_read_errors": (C.c_int, [TS, C.POINTER(C.c_uint32), C.c_int, P]),
        "dqrm_last_error": (C.c_char_p, []),
        "dqrm_set_apply_kernel": (C.c_int, [C.c_int]),
        "dqrm_set_coalesce_kernel": (C.c_int, [C.c_int]),
        "dqrm_abi_version": (C.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    got = lib.dqrm_abi_version()
    if got != DQRM_ABI_VERSION:  # a stale build would be called with the wrong argument lists
        raise DQRMError(
            f"{path} has ABI version {got}, this package needs {DQRM_ABI_VERSION}: rebuild it with "
            "`python -m deep_quantized_recommendation_model_dqrm_amd._build`"
        )
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != DQRM_OK:
        msg = load().dqrm_last_error().decode(errors="replace")
        raise DQRMError(f"{what} failed ({rc}): {msg}")


def apply_update_form(num_ranks: int = 1) -> str:
    """What dqrm_apply_sparse_update launches under AUTO (for bench lines): the payload decode +
    update kernel and where the |W| hierarchy is finalized."""
    return "the payload decode + update kernel (k_apply_flat) + a short k_table_finalize launch"
