"""ctypes wrapper of oracle/build/libhbec_oracle.so (gf_oracle.c).

TEST INFRASTRUCTURE ONLY — the C restatement of the klauspost codec used as
the fast full-size checker and as bench.py's CPU baseline ("port").  Build it
with ``make -C oracle``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

SCALAR = 0
AVX2 = 1

_LIB_PATH = Path(__file__).resolve().parent / "build" / "libhbec_oracle.so"
_lib = None
_U8P = C.POINTER(C.c_uint8)


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise RuntimeError(f"{_LIB_PATH} missing: run `make -C oracle`")
        h = C.CDLL(str(_LIB_PATH))
        h.orc_gal_mul.restype = C.c_uint8
        h.orc_gal_mul.argtypes = [C.c_uint8, C.c_uint8]
        h.orc_gal_exp.restype = C.c_uint8
        h.orc_gal_exp.argtypes = [C.c_uint8, C.c_int]
        h.orc_invert.restype = C.c_int
        h.orc_invert.argtypes = [C.c_int, _U8P, _U8P]
        h.orc_build_matrix.restype = C.c_int
        h.orc_build_matrix.argtypes = [C.c_int, C.c_int, _U8P]
        h.orc_apply.restype = None
        h.orc_apply.argtypes = [C.c_int, C.c_int, _U8P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_size_t,
                                C.c_int]
        h.orc_encode.restype = C.c_int
        h.orc_encode.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_size_t, C.c_int]
        h.orc_splitmix_fill.restype = None
        h.orc_splitmix_fill.argtypes = [C.c_uint64, C.c_void_p, C.c_size_t]
        h.orc_fill_objects.restype = None
        h.orc_fill_objects.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p]
        h.orc_encode_batch.restype = C.c_double
        h.orc_encode_batch.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int,
                                       C.c_int]
        h.orc_ecsplit_once.restype = C.c_double
        h.orc_ecsplit_once.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int]
        h.orc_have_avx2.restype = C.c_int
        h.orc_apply_batch.restype = C.c_double
        h.orc_apply_batch.argtypes = [C.c_int, C.c_int, _U8P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t, C.c_size_t,
                                      C.c_int, C.c_int]
        _lib = h
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(_U8P)


def build_matrix(k: int, m: int) -> np.ndarray:
    out = np.zeros((k + m) * k, dtype=np.uint8)
    rc = lib().orc_build_matrix(k, m, _u8(out))
    if rc:
        raise ValueError(f"orc_build_matrix rc={rc}")
    return out.reshape(k + m, k)


def invert(m) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(m, dtype=np.uint8))
    n = a.shape[0]
    out = np.zeros((n, n), dtype=np.uint8)
    if lib().orc_invert(n, _u8(a), _u8(out)):
        raise ValueError("singular")
    return out


def apply(coeffs, inputs, impl=AVX2):
    """out[r] = XOR_j coeffs[r][j] * inputs[j] (arrays of equal length)."""
    c = np.ascontiguousarray(np.asarray(coeffs, dtype=np.uint8))
    rows, k = c.shape
    ins = [np.ascontiguousarray(x, dtype=np.uint8) for x in inputs]
    n = ins[0].size
    outs = [np.zeros(n, dtype=np.uint8) for _ in range(rows)]
    ip = (C.c_void_p * k)(*[x.ctypes.data for x in ins])
    op = (C.c_void_p * rows)(*[x.ctypes.data for x in outs])
    lib().orc_apply(rows, k, _u8(c), ip, op, n, impl)
    return outs


def fill_objects(first: int, count: int, obj_len: int, base_seed: int = 0x48424543) -> np.ndarray:
    out = np.empty((count, obj_len), dtype=np.uint8)
    lib().orc_fill_objects(base_seed, first, count, obj_len, obj_len, out.ctypes.data)
    return out


def encode_batch(k: int, m: int, objs: np.ndarray, threads: int = 1, impl=AVX2):
    """objs [n, len] -> (parity [n, m*S], seconds)."""
    n, ln = objs.shape
    s = ln // k
    par = np.empty((n, m * s), dtype=np.uint8)
    t = lib().orc_encode_batch(k, m, objs.ctypes.data, n, ln, par.ctypes.data, threads, impl)
    if t < 0:
        raise ValueError(f"orc_encode_batch rc={t}")
    return par, t


def apply_batch(coeffs, in_views, out_views, n: int, length: int, threads: int = 1, impl=AVX2) -> float:
    """Threaded out[r] = XOR_j coeffs[r][j]*in[j] over n strided objects;
    views are (address, stride) pairs.  Returns wall seconds."""
    c = np.ascontiguousarray(np.asarray(coeffs, dtype=np.uint8))
    rows, k = c.shape
    ib = (C.c_void_p * k)(*[v[0] for v in in_views])
    ist = (C.c_size_t * k)(*[v[1] for v in in_views])
    ob = (C.c_void_p * rows)(*[v[0] for v in out_views])
    ost = (C.c_size_t * rows)(*[v[1] for v in out_views])
    return lib().orc_apply_batch(rows, k, _u8(c), ib, ist, ob, ost, n, length, threads, impl)


def ecsplit_once(k: int, m: int, obj: np.ndarray, chunk: int, impl=AVX2, with_setup=True) -> float:
    return lib().orc_ecsplit_once(k, m, obj.ctypes.data, obj.size, chunk, impl, 1 if with_setup else 0)


def have_avx2() -> bool:
    return bool(lib().orc_have_avx2())


def cpu_threads() -> int:
    """Host threads to use: the process's CPU affinity, capped by
    OMP_NUM_THREADS when set (the GPU box's per-GPU CPU share is 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)
