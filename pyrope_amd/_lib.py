"""ctypes binding of libpyrope_hip.so (the C ABI in include/pyrope_ann.h).

The product path has no fallback: if the in-tree library is missing, or no
gfx950 device is present, calls raise instead of computing anything on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# PYR_LIB: another build of the library (measurement only: A/B runs of two builds on one box)
LIB_PATH = os.environ.get("PYR_LIB") or os.path.join(HERE, "libpyrope_hip.so")

(PYR_OK, PYR_E_DIM, PYR_E_ARG, PYR_E_STATE, PYR_E_OOM, PYR_E_DEVICE, PYR_E_DUPLICATE, PYR_E_NOT_FOUND,
 PYR_E_FORMAT, PYR_E_IO) = range(10)
PYR_FLAT, PYR_IVF_FLAT, PYR_IVF_PQ = 0, 1, 2


class PyrError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


# C# exception types the reference raises on this path (mirrored for the tests/shim)
class ArgumentException(ValueError):
    pass


class ArgumentNullException(ArgumentException):
    pass


class ArgumentOutOfRangeException(ArgumentException):
    pass


class FormatException(ValueError):
    """System.FormatException (e.g. JsonElement.GetInt32 on a non-Int32 number)."""


class InvalidOperationException(RuntimeError):
    pass


class DeviceError(RuntimeError):
    pass


class FileNotFoundException(FileNotFoundError):
    """System.IO.FileNotFoundException (Load of a missing snapshot)."""


class JsonException(ValueError):
    """System.Text.Json.JsonException (Load of a file that is not a snapshot of this index)."""


class IOException(OSError):
    """System.IO.IOException (a snapshot could not be written)."""


class IndexDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dim", C.c_int32), ("metric", C.c_int32), ("nlist", C.c_int32),
                ("pq_m", C.c_int32), ("pq_k", C.c_int32), ("device", C.c_int32), ("default_nprobe", C.c_int32),
                ("device_mask", C.c_uint64), ("shards", C.c_int32), ("reserved", C.c_int32)]


class SearchParams(C.Structure):
    _fields_ = [("nprobe", C.c_int32), ("reserved", C.c_int32), ("max_scans", C.c_int64)]


_lib = None
_lock = threading.Lock()

_f = C.POINTER(C.c_float)
_i64 = C.POINTER(C.c_int64)
_i32 = C.POINTER(C.c_int32)
_u8 = C.POINTER(C.c_uint8)
_vp = C.c_void_p

SIGNATURES = {
    "pyr_index_create": (C.c_int, [C.POINTER(IndexDesc), C.POINTER(_vp)]),
    "pyr_index_destroy": (None, [_vp]),
    "pyr_index_add": (C.c_int, [_vp, _f, C.c_int64, _i64]),
    "pyr_index_upsert": (C.c_int, [_vp, _f, C.c_int64, _i64]),
    "pyr_index_remove": (C.c_int, [_vp, _i64, C.c_int64, _u8]),
    "pyr_index_build": (C.c_int, [_vp]),
    "pyr_index_search": (C.c_int, [_vp, _f, C.c_int64, C.c_int32, C.POINTER(SearchParams), _f, _i64, _i32]),
    "pyr_index_search_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(SearchParams), _vp, _vp, _vp,
                                          _vp]),
    "pyr_index_stats": (C.c_int, [_vp, _i64, _i32, _i32]),
    "pyr_index_snapshot": (C.c_int, [_vp, C.c_char_p]),
    "pyr_index_set_coalescing": (C.c_int, [_vp, C.c_int32, C.c_int32]),
    "pyr_index_load": (C.c_int, [_vp, C.c_char_p]),
    "pyr_image_nonce": (C.c_int, [C.c_char_p, _u8]),
    "pyr_index_get_centroids": (C.c_int, [_vp, _f, _i32]),
    "pyr_index_ivf_layout": (C.c_int, [_vp, _i64, _i64, _u8, _i64]),
    "pyr_index_pq_state": (C.c_int, [_vp, _f, _i32, _u8]),
    "pyr_index_scan": (C.c_int, [_vp, _i64, _f, _i64]),
    "pyr_index_labels": (C.c_int, [_vp, _i64, _i64]),
    "pyr_index_set_quantization": (C.c_int, [_vp, C.c_int32]),
    "pyr_index_probe_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, _vp, C.POINTER(C.c_int32), _vp]),
    "pyr_index_search_probed_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(SearchParams), _vp,
                                                 C.c_int32, _vp, _vp, _vp, _vp]),
    "pyr_scalar_quantize": (C.c_int, [C.c_int32, _f, C.c_int64, C.c_int32, _u8]),
    "pyr_scalar_quantize_minmax": (C.c_int, [C.c_int32, _f, C.c_int64, C.c_int32, _u8, _f, _f]),
    "pyr_scalar_dequantize": (C.c_int, [C.c_int32, _u8, C.c_int64, C.c_int32, _f, _f, _f]),
    "pyr_merge_topk_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, C.c_int32, _vp, _vp, _vp]),
    "pyr_merge_topk_parts_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp]),
    "pyr_ivf_memory_plan": (C.c_int, [C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int32,
                                      _i64, _i64]),
    "pyr_generate_synthetic": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, _f]),
    "pyr_generate_synthetic_blocked": (C.c_int, [C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int64, _f]),
    "pyr_index_set_centroids": (C.c_int, [_vp, _f, C.c_int32]),
    "pyr_index_set_codebooks": (C.c_int, [_vp, _f, C.c_int32, C.c_int32]),
    "pyr_index_reserve": (C.c_int, [_vp, C.c_int64]),
    "pyr_kmeans_train": (C.c_int, [C.c_int32, _f, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                   _f, _i32]),
    # list-sharded multi-GPU search (dist.py ListShardedIvf)
    "pyr_assign": (C.c_int, [C.c_int32, _f, C.c_int32, _f, C.c_int64, C.c_int32, C.c_int32, _i32]),
    "pyr_shard_record_bytes": (C.c_int64, [C.c_int32]),
    "pyr_index_set_list_samples": (C.c_int, [_vp, _f, _i64, _i64, C.c_int32]),
    "pyr_index_shard_prepare_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(SearchParams), _vp,
                                                 C.POINTER(C.c_int32), _vp]),
    "pyr_shard_plan_stride": (C.c_int32, [C.c_int32, C.c_int64]),
    "pyr_index_shard_info": (C.c_int, [_vp, _i32, _i32, _i64, _i64, _i64, _i64]),
    "pyr_index_shard_search_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, _vp, C.c_int32, C.c_int32, _vp,
                                                _vp]),
    "pyr_index_shard_rerun_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, _vp, C.c_int32, C.c_int32, _vp,
                                               C.c_int32, C.c_int32, C.c_int64, _vp, _vp]),
    "pyr_shard_merge_device": (C.c_int, [_vp, C.c_int32, C.c_int64, C.c_int32, _vp, C.c_int32, _vp, _vp, _vp, _vp,
                                         C.c_int32, _vp]),
    "pyr_profile_enable": (None, [C.c_int32]),
    "pyr_profile_reset": (None, []),
    "pyr_index_debug_candidates": (C.c_int, [_vp, C.c_int64, C.c_int32, _vp, _vp, _vp]),
    "pyr_profile_get": (C.c_int, [C.c_int32, C.POINTER(C.c_double), _i64, _i64]),
    "pyr_last_error": (C.c_char_p, []),
    "pyr_version": (C.c_char_p, []),
}


def load():
    """Load the in-tree library (building it first when this tree has hipcc and it is stale)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DeviceError(f"{LIB_PATH} is missing: run `python -m pyrope_amd.build` (no CPU fallback exists)")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    return load().pyr_last_error().decode(errors="replace")


def check(status: int, what: str = "") -> None:
    if status == PYR_OK:
        return
    msg = last_error() or what
    if status == PYR_E_DIM:
        raise ArgumentException(msg)
    if status == PYR_E_ARG:
        raise ArgumentOutOfRangeException(msg) if "topK" in msg else ArgumentException(msg)
    if status in (PYR_E_STATE, PYR_E_DUPLICATE):
        raise InvalidOperationException(msg)
    if status == PYR_E_DEVICE:
        raise DeviceError(msg)
    if status == PYR_E_NOT_FOUND:
        raise FileNotFoundException(msg)
    if status == PYR_E_FORMAT:
        raise JsonException(msg)
    if status == PYR_E_IO:
        raise IOException(msg)
    raise PyrError(status, msg)


def ptr(a, ct):
    if a is None:
        return C.cast(None, C.POINTER(ct))
    return a.ctypes.data_as(C.POINTER(ct))
