"""ctypes binding of libhbec.so (include/hbec.h).

There is deliberately no fallback: if the native library is missing or fails
to load, every entry point raises.  The GF arithmetic runs only in the HIP
kernels of libhbec.so.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("HBEC_LIB", _PKG / "libhbec.so"))

HBEC_OK = 0
ERR_INV_SHARD_NUM = -1
ERR_MAX_SHARD_NUM = -2
ERR_TOO_FEW_SHARDS = -3
ERR_SHARD_NO_DATA = -4
ERR_SHARD_SIZE = -5
ERR_SINGULAR = -6
ERR_INVALID_ARG = -7
ERR_DEVICE = -8
ERR_NOMEM = -9
ERR_UNEXPECTED_EOF = -10
ERR_IO = -11
ERR_SCHEME = -12


class View(C.Structure):
    _fields_ = [("base", C.c_void_p), ("obj_stride", C.c_uint64)]


class Stripe(C.Structure):
    _fields_ = [("base", C.c_void_p), ("shard_len", C.c_uint64)]


class Object(C.Structure):
    _fields_ = [("data", C.c_void_p), ("parity", C.c_void_p), ("shard_len", C.c_uint64)]


READ_FN = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t)
WRITE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t)

# every symbol include/hbec.h declares: (name, restype, argtypes)
_P = C.c_void_p
_U8P = C.POINTER(C.c_uint8)
_SIG = [
    ("hbec_strerror", C.c_char_p, [C.c_int]),
    ("hbec_last_error", C.c_char_p, []),
    ("hbec_version", C.c_int, []),
    ("hbec_new", C.c_int, [C.c_int, C.c_int, C.POINTER(_P)]),
    ("hbec_free", None, [_P]),
    ("hbec_data_shards", C.c_int, [_P]),
    ("hbec_parity_shards", C.c_int, [_P]),
    ("hbec_matrix", C.c_int, [_P, _U8P]),
    ("hbec_encode", C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_size_t), C.c_int]),
    ("hbec_reconstruct", C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_size_t), C.c_int, C.c_int]),
    ("hbec_verify", C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_size_t), C.c_int, C.POINTER(C.c_int)]),
    ("hbec_encode_databuf", C.c_int, [_P, _P, C.c_size_t]),
    ("hbec_reconstruct_databuf", C.c_int, [_P, _P, C.c_size_t, _U8P, C.c_int]),
    ("hbec_verify_databuf", C.c_int, [_P, _P, C.c_size_t, C.POINTER(C.c_int)]),
    ("hbec_coalesce_stats", C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_host_md5_stats", C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_verify_batch", C.c_int, [_P, C.POINTER(View), C.c_uint64, C.c_uint64, _P, _P]),
    ("hbec_encode_batch", C.c_int, [_P, C.POINTER(View), C.c_uint64, C.c_uint64, _P]),
    ("hbec_reconstruct_batch", C.c_int,
     [_P, C.POINTER(View), _U8P, C.c_uint64, C.c_uint64, C.c_int, _P]),
    ("hbec_md5_batch", C.c_int, [C.POINTER(View), C.c_int, C.c_uint64, C.c_uint64, _P, _P]),
    ("hbec_md5_list", C.c_int, [C.POINTER(_P), C.POINTER(C.c_uint64), C.c_uint64, _P, _P]),
    ("hbec_md5_host", C.c_int, [C.POINTER(_P), C.POINTER(C.c_uint64), C.c_uint64, _U8P]),
    ("hbec_md5_new", C.c_int, [C.c_int, C.c_uint64, C.POINTER(_P)]),
    ("hbec_md5_free", None, [_P]),
    ("hbec_md5_update", C.c_int, [_P, C.POINTER(View), C.c_uint64, _P]),
    ("hbec_md5_final", C.c_int, [_P, _P, _P]),
    ("hbec_encode_md5_batch", C.c_int, [_P, C.POINTER(View), C.c_uint64, C.c_uint64, _P, _P]),
    ("hbec_decode_rows", C.c_int,
     [_P, _U8P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), _U8P]),
    ("hbec_apply_batch", C.c_int,
     [C.c_int, C.c_int, _U8P, C.POINTER(View), C.POINTER(View), C.c_uint64, C.c_uint64, _P]),
    ("hbec_fill_splitmix", C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P]),
    ("hbec_plan_stripes", C.c_int, [_P, C.POINTER(Stripe), C.c_uint64, C.POINTER(_P)]),
    ("hbec_plan_objects", C.c_int, [_P, C.POINTER(Object), C.c_uint64, C.POINTER(_P)]),
    ("hbec_plan_free", None, [_P]),
    ("hbec_plan_info", C.c_int,
     [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_int), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_encode_plan", C.c_int, [_P, _P, _P]),
    ("hbec_reconstruct_plan", C.c_int, [_P, _P, _U8P, C.c_int, _P]),
    ("hbec_encode_host", C.c_int, [_P, C.POINTER(Stripe), C.c_uint64]),
    ("hbec_host_alloc", C.c_int, [C.c_size_t, C.POINTER(_P)]),
    ("hbec_host_free", None, [_P]),
    ("hbec_host_device_addr", C.c_int, [_P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("hbec_reconstruct_host", C.c_int, [_P, C.POINTER(Stripe), C.c_uint64, _U8P, C.c_int]),
    ("hbec_encode_host_md5", C.c_int, [_P, C.POINTER(Stripe), C.c_uint64, _U8P]),
    ("hbec_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("hbec_set_device", C.c_int, [C.c_int]),
    ("hbec_encode_host_devices", C.c_int, [_P, C.POINTER(Stripe), C.c_uint64, C.POINTER(C.c_int), C.c_int]),
    ("hbec_reconstruct_host_devices", C.c_int,
     [_P, C.POINTER(Stripe), C.c_uint64, _U8P, C.c_int, C.POINTER(C.c_int), C.c_int]),
    ("hbec_batcher_new", C.c_int, [_P, C.c_uint64, C.c_uint32, C.POINTER(_P)]),
    ("hbec_batcher_free", None, [_P]),
    ("hbec_batcher_encode", C.c_int, [_P, C.POINTER(Stripe)]),
    ("hbec_batcher_encode_md5", C.c_int, [_P, C.POINTER(Stripe), _U8P]),
    ("hbec_batcher_reconstruct", C.c_int, [_P, C.POINTER(Stripe), _U8P, C.c_int]),
    ("hbec_batcher_stats", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_set_force_stream", C.c_int, [C.c_int]),
    ("hbec_set_odd_chunk_tiles", C.c_int, [C.c_uint64]),
    ("hbec_kernel_info", C.c_int,
     [C.c_int, C.c_int, C.c_uint64, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("hbec_odd_path_stats", C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_odd_edge_stats", C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_odd_record_cache", C.c_int, [C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("hbec_ec_shard_length", C.c_int64, [C.c_int64, C.c_int64]),
    ("hbec_ec_split", C.c_int, [C.c_int, C.c_int, READ_FN, _P, C.c_int, C.c_int64, WRITE_FN, C.POINTER(_P)]),
    ("hbec_ec_reconstruct", C.c_int,
     [C.c_int, C.c_int, READ_FN, C.POINTER(_P), C.c_int, C.c_int64, WRITE_FN, C.POINTER(_P),
      C.POINTER(C.c_int), C.c_int]),
    ("hbec_ec_glue", C.c_int,
     [C.c_int, C.c_int, READ_FN, C.POINTER(_P), C.c_int, C.c_int64, WRITE_FN, C.POINTER(_P), C.c_int]),
    ("hbec_ec_glue_range", C.c_int,
     [C.c_int, C.c_int, READ_FN, C.POINTER(_P), C.c_int, C.c_int64, C.c_int64, C.c_int64, WRITE_FN, C.POINTER(_P),
      C.c_int]),
    ("hbec_ec_copy_range", C.c_int,
     [C.c_int, C.c_int, READ_FN, C.POINTER(_P), C.c_int, C.c_int64, C.c_int64, C.c_int64, WRITE_FN, C.POINTER(_P),
      C.c_int]),
    ("hbec_parse_ec_scheme", C.c_int,
     [C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("hbec_range_chunk_align", None,
     [C.c_int64, C.c_int64, C.c_int64, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
]
SYMBOLS = [s[0] for s in _SIG]

_lib = None


class NativeLibraryError(RuntimeError):
    pass


def lib():
    """Load libhbec.so once; raise NativeLibraryError if it is absent."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build it with `python -m hummingbird_amd.build` "
                "(there is no CPU fallback)")
        try:
            h = C.CDLL(str(LIB_PATH))
        except OSError as e:  # pragma: no cover - depends on the host
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, res, args in _SIG:
            # an explicitly chosen library (HBEC_LIB: an older build in an
            # interleaved A/B) may lack newer entry points; they raise on use
            if "HBEC_LIB" in os.environ and not hasattr(h, name):
                continue
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def last_error() -> str:
    return lib().hbec_last_error().decode(errors="replace")


def strerror(code: int) -> str:
    return lib().hbec_strerror(code).decode()
