"""The klauspost/reedsolomon ``Encoder`` surface that objectserver/ecutils.go
uses, backed by libhbec's gfx950 kernels.

Reference call sites: ``reedsolomon.New`` (ecutils.go:27,77,135),
``enc.Encode`` (:59), ``enc.Reconstruct`` (:111), ``enc.ReconstructData``
(:168).  Names, argument meaning and errors follow that API:

    enc = New(4, 2)
    enc.Encode(shards)            # shards: k+m equal-length buffers, parity in place
    enc.Reconstruct(shards)       # missing = None / len 0, filled in place
    enc.ReconstructData(shards)   # data shards only

Shards are writable byte buffers (``bytearray``, ``numpy.uint8`` arrays,
``memoryview``).  Missing shards are refilled with new ``numpy`` arrays, the
way Go allocates when the slice has no capacity.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


class ReedSolomonError(Exception):
    code = None


class ErrInvShardNum(ReedSolomonError):
    code = N.ERR_INV_SHARD_NUM


class ErrMaxShardNum(ReedSolomonError):
    code = N.ERR_MAX_SHARD_NUM


class ErrTooFewShards(ReedSolomonError):
    code = N.ERR_TOO_FEW_SHARDS


class ErrShardNoData(ReedSolomonError):
    code = N.ERR_SHARD_NO_DATA


class ErrShardSize(ReedSolomonError):
    code = N.ERR_SHARD_SIZE


class ErrSingular(ReedSolomonError):
    code = N.ERR_SINGULAR


class ErrDevice(ReedSolomonError):
    code = N.ERR_DEVICE


class ErrInvalidArg(ReedSolomonError):
    code = N.ERR_INVALID_ARG


class ErrUnexpectedEOF(ReedSolomonError):
    code = N.ERR_UNEXPECTED_EOF


class ErrIO(ReedSolomonError):
    code = N.ERR_IO


class ErrScheme(ReedSolomonError):
    code = N.ERR_SCHEME


class ErrNoMem(ReedSolomonError):
    """Host or device allocation failed (HBEC_ERR_NOMEM): like ErrDevice, the
    caller may fall back to its own CPU codec."""
    code = N.ERR_NOMEM


_BY_CODE = {c.code: c for c in (ErrInvShardNum, ErrMaxShardNum, ErrTooFewShards, ErrShardNoData, ErrShardSize,
                                ErrSingular, ErrDevice, ErrInvalidArg, ErrUnexpectedEOF, ErrIO, ErrScheme,
                                ErrNoMem)}


def check(rc: int) -> None:
    if rc != N.HBEC_OK:
        cls = _BY_CODE.get(rc, ReedSolomonError)
        raise cls(f"{N.strerror(rc)}: {N.last_error()}")


def _as_array(buf) -> np.ndarray:
    if buf is None:
        return np.zeros(0, dtype=np.uint8)
    if isinstance(buf, np.ndarray):
        if buf.dtype != np.uint8 or buf.ndim != 1 or not buf.flags.c_contiguous:
            raise TypeError("shards must be 1-D contiguous uint8 arrays")
        return buf
    return np.frombuffer(buf, dtype=np.uint8)


class Encoder:
    """reedsolomon.Encoder over the GPU codec (one matrix per (k, m))."""

    def __init__(self, data_shards: int, parity_shards: int):
        self._h = C.c_void_p()
        check(N.lib().hbec_new(int(data_shards), int(parity_shards), C.byref(self._h)))
        self.DataShards = int(data_shards)
        self.ParityShards = int(parity_shards)
        self.Shards = self.DataShards + self.ParityShards

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and N._lib is not None:
            N._lib.hbec_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def matrix(self) -> np.ndarray:
        out = np.zeros((self.Shards, self.DataShards), dtype=np.uint8)
        check(N.lib().hbec_matrix(self._h, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out

    def _ptrs(self, arrs):
        n = len(arrs)
        ptrs = (C.c_void_p * n)(*[a.ctypes.data if a.size else 0 for a in arrs])
        lens = (C.c_size_t * n)(*[a.size for a in arrs])
        return ptrs, lens

    def Encode(self, shards) -> None:
        arrs = [_as_array(s) for s in shards]
        for a in arrs:
            if a.size and not a.flags.writeable:
                raise ValueError("shards must be writable")
        ptrs, lens = self._ptrs(arrs)
        check(N.lib().hbec_encode(self._h, ptrs, lens, len(arrs)))

    def Verify(self, shards) -> bool:
        """Encoder.Verify: True when the parity shards match the data."""
        arrs = [_as_array(s) for s in shards]
        ptrs, lens = self._ptrs(arrs)
        ok = C.c_int()
        check(N.lib().hbec_verify(self._h, ptrs, lens, len(arrs), C.byref(ok)))
        return bool(ok.value)

    def _reconstruct(self, shards, data_only: int) -> None:
        arrs = [_as_array(s) for s in shards]
        size = next((a.size for a in arrs if a.size), 0)
        if len(arrs) == self.Shards and size:
            # give every missing shard a buffer of the shard size (Go: reuse or allocate)
            for i, a in enumerate(arrs):
                if a.size == 0 and (i < self.DataShards or not data_only):
                    arrs[i] = np.zeros(size, dtype=np.uint8)
        n = len(arrs)
        ptrs = (C.c_void_p * n)(*[a.ctypes.data if a.size else 0 for a in arrs])
        lens = (C.c_size_t * n)(*[(a.size if (shards[i] is not None and len(shards[i])) else 0)
                                  for i, a in enumerate(arrs)])
        check(N.lib().hbec_reconstruct(self._h, ptrs, lens, n, data_only))
        for i in range(n):
            if lens[i] and (shards[i] is None or len(shards[i]) == 0):
                shards[i] = arrs[i]

    def Reconstruct(self, shards) -> None:
        self._reconstruct(shards, 0)

    def ReconstructData(self, shards) -> None:
        self._reconstruct(shards, 1)

    # ---- single-pointer databuf forms (hbec_*_databuf): the k+m shards of one
    # contiguous buffer, shard i at i*S, as every ecutils.go call site builds
    # them (ecutils.go:31-35,55-58,94-101,151-159) ----
    def _databuf(self, databuf, shard_len):
        a = _as_array(databuf)
        if shard_len < 0 or a.size < self.Shards * shard_len:
            raise ValueError("databuf shorter than (k+m) * shard_len")
        return C.c_void_p(a.ctypes.data if a.size else None)

    def EncodeDatabuf(self, databuf, shard_len: int) -> None:
        """Encode(data) where data[i] = databuf[i*S:(i+1)*S] (ecSplit, ecutils.go:55-59)."""
        check(N.lib().hbec_encode_databuf(self._h, self._databuf(databuf, shard_len), int(shard_len)))

    def ReconstructDatabuf(self, databuf, shard_len: int, present, data_only: bool = False) -> None:
        """Reconstruct(data) / ReconstructData(data) with missing shards rebuilt in
        their databuf slots (ecReconstruct ecutils.go:94-111, ecGlue :151-168)."""
        p = (C.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        check(N.lib().hbec_reconstruct_databuf(self._h, self._databuf(databuf, shard_len), int(shard_len), p,
                                               int(data_only)))

    def VerifyDatabuf(self, databuf, shard_len: int) -> bool:
        ok = C.c_int()
        check(N.lib().hbec_verify_databuf(self._h, self._databuf(databuf, shard_len), int(shard_len), C.byref(ok)))
        return bool(ok.value)

    # ---- streaming host path: many host stripes (ecSplit databuf layout) ----
    def _stripes(self, stripes):
        """stripes: list of 1-D uint8 arrays, each (k+m)*S bytes (data then parity)."""
        arr = (N.Stripe * max(1, len(stripes)))()
        for i, st in enumerate(stripes):
            a = _as_array(st)
            if a.size % self.Shards:
                raise ValueError("stripe length must be a multiple of k+m")
            arr[i].base = a.ctypes.data if a.size else None
            arr[i].shard_len = a.size // self.Shards
        return arr

    def EncodeStripes(self, stripes) -> None:
        check(N.lib().hbec_encode_host(self._h, self._stripes(stripes), len(stripes)))

    def EncodeStripesMD5(self, stripes):
        """EncodeStripes + the ShardHash of every shard of every stripe, hashed on
        the GPU (indexdb.go:746-753).  Returns [[hex] * (k+m)] per stripe."""
        n = len(stripes)
        out = (C.c_uint8 * (16 * self.Shards * max(n, 1)))()
        check(N.lib().hbec_encode_host_md5(self._h, self._stripes(stripes), n, out))
        raw = bytes(out)
        return [[raw[16 * (s * self.Shards + i):16 * (s * self.Shards + i + 1)].hex() for i in range(self.Shards)]
                for s in range(n)]

    def EncodeStripesDevices(self, stripes, devices=None) -> None:
        """EncodeStripes spread over several GPUs (one host thread each);
        devices=None: every visible device."""
        d, nd = _devices(devices)
        check(N.lib().hbec_encode_host_devices(self._h, self._stripes(stripes), len(stripes), d, nd))

    def ReconstructStripesDevices(self, stripes, present, data_only: bool = False, devices=None) -> None:
        p = (C.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        d, nd = _devices(devices)
        check(N.lib().hbec_reconstruct_host_devices(self._h, self._stripes(stripes), len(stripes), p, int(data_only),
                                                    d, nd))

    def ReconstructStripes(self, stripes, present, data_only: bool = False) -> None:
        p = (C.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        check(N.lib().hbec_reconstruct_host(self._h, self._stripes(stripes), len(stripes), p, int(data_only)))

    def DecodeRows(self, present, data_only: bool = False):
        """(survivors, outputs, rows) the reconstruct kernels apply."""
        n = self.Shards
        p = (C.c_uint8 * n)(*[1 if x else 0 for x in present])
        surv = (C.c_int * self.DataShards)()
        outs = (C.c_int * n)()
        nout = C.c_int()
        rows = (C.c_uint8 * (n * self.DataShards))()
        check(N.lib().hbec_decode_rows(self._h, p, int(data_only), surv, outs, C.byref(nout), rows))
        r = np.frombuffer(bytes(rows), dtype=np.uint8)[: nout.value * self.DataShards]
        return list(surv), list(outs)[: nout.value], r.reshape(nout.value, self.DataShards)


class Batcher:
    """hbec_batcher: concurrent callers each submit one host stripe (ecSplit
    databuf layout, (k+m)*S bytes) and block; the library codes whatever has
    queued in one streaming host-path call.  ctypes releases the GIL during
    the call, so Python threads really run concurrently."""

    def __init__(self, enc: Encoder, max_batch_bytes: int = 256 << 20, max_wait_us: int = 200):
        self.enc = enc
        self._h = C.c_void_p()
        check(N.lib().hbec_batcher_new(enc.handle, int(max_batch_bytes), int(max_wait_us), C.byref(self._h)))

    def close(self):
        if self._h:
            N.lib().hbec_batcher_free(self._h)
            self._h = None

    __del__ = close

    def _stripe(self, st):
        a = _as_array(st)
        s = N.Stripe()
        s.base = a.ctypes.data
        s.shard_len = a.size // self.enc.Shards
        return s

    def Encode(self, stripe) -> None:
        s = self._stripe(stripe)
        check(N.lib().hbec_batcher_encode(self._h, C.byref(s)))

    def EncodeMD5(self, stripe):
        """Encode + ShardHash of the stripe's k+m shards (hex strings)."""
        s = self._stripe(stripe)
        out = (C.c_uint8 * (16 * self.enc.Shards))()
        check(N.lib().hbec_batcher_encode_md5(self._h, C.byref(s), out))
        raw = bytes(out)
        return [raw[16 * i:16 * (i + 1)].hex() for i in range(self.enc.Shards)]

    def Reconstruct(self, stripe, present, data_only: bool = False) -> None:
        s = self._stripe(stripe)
        p = (C.c_uint8 * self.enc.Shards)(*[1 if x else 0 for x in present])
        check(N.lib().hbec_batcher_reconstruct(self._h, C.byref(s), p, int(data_only)))

    def stats(self):
        b, s = C.c_uint64(), C.c_uint64()
        check(N.lib().hbec_batcher_stats(self._h, C.byref(b), C.byref(s)))
        return {"batches": b.value, "stripes": s.value}


def New(data_shards: int, parity_shards: int) -> Encoder:
    """reedsolomon.New (ecutils.go:27,77,135)."""
    return Encoder(data_shards, parity_shards)


class HostBuffer:
    """Pinned, device-mapped host memory from ``hbec_host_alloc`` — what the
    cgo shim would hand ecSplit as its databuf (ecutils.go:31-35) so that
    ``EncodeStripes`` / ``ReconstructStripes`` code the stripes in place over
    PCIe (zero-copy) instead of staging them through the pinned ring.

    ``.array`` is a numpy uint8 view; keep the HostBuffer alive while it is used."""

    def __init__(self, nbytes: int):
        self._p = C.c_void_p()
        check(N.lib().hbec_host_alloc(int(nbytes), C.byref(self._p)))
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array(C.cast(self._p, C.POINTER(C.c_uint8)), shape=(self.nbytes,))

    @property
    def ptr(self) -> int:
        return self._p.value

    def free(self) -> None:
        if self._p and self._p.value and N._lib is not None:
            self.array = None
            N._lib.hbec_host_free(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        self.free()


def host_device_addr(buf) -> int:
    """Device address of a host buffer when all of it is pinned and device
    mapped (the zero-copy condition), else 0."""
    a = _as_array(buf)
    out = C.c_uint64()
    check(N.lib().hbec_host_device_addr(C.c_void_p(a.ctypes.data), a.size, C.byref(out)))
    return out.value


def _devices(devices):
    if devices is None:
        return None, 0
    arr = (C.c_int * len(devices))(*[int(x) for x in devices])
    return arr, len(devices)


def device_count() -> int:
    n = C.c_int()
    check(N.lib().hbec_device_count(C.byref(n)))
    return n.value
