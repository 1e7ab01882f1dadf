"""Device-resident batches of objects (the GPU hot path) on torch tensors.

torch supplies device memory and streams only; the arithmetic is libhbec's
HIP kernels, called through the C ABI (``hbec_encode_batch`` /
``hbec_reconstruct_batch``).  Layout of a batch of n one-stripe objects with
shard length S (the ecSplit layout, objectserver/ecutils.go:55-58):

    objs   : uint8 [n, k*S]  — object o's data shard j = objs[o, j*S:(j+1)*S]
    parity : uint8 [n, m*S]  — object o's parity shard r = parity[o, r*S:(r+1)*S]

Shards are never copied: the kernels read the data shards in place.
"""
from __future__ import annotations

import ctypes as C

from . import _native as N
from .reedsolomon import Encoder, check

HBEC_SEED = 0x48424543


def _stream_ptr(stream):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


def shard_views(t, n_shards: int, shard_len: int):
    """Views of the n_shards consecutive shards stored in each row of a 2-D tensor."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a 2-D row-contiguous tensor")
    if t.shape[1] < n_shards * shard_len:
        raise ValueError("tensor rows shorter than n_shards * shard_len")
    base = t.data_ptr()
    row = t.stride(0) * t.element_size()
    return [(base + i * shard_len, row) for i in range(n_shards)]


def _views(pairs):
    arr = (N.View * len(pairs))()
    for i, (b, s) in enumerate(pairs):
        arr[i].base = b
        arr[i].obj_stride = s
    return arr


def encode_views(enc: Encoder, views, n_objects: int, shard_len: int, stream=None) -> None:
    v = _views(views)
    check(N.lib().hbec_encode_batch(enc.handle, v, int(n_objects), int(shard_len), _stream_ptr(stream)))


def reconstruct_views(enc: Encoder, views, present, n_objects: int, shard_len: int, data_only: bool = False,
                      stream=None) -> None:
    v = _views(views)
    p = (C.c_uint8 * len(present))(*[1 if x else 0 for x in present])
    check(N.lib().hbec_reconstruct_batch(enc.handle, v, p, int(n_objects), int(shard_len), int(data_only),
                                         _stream_ptr(stream)))


def verify_views(enc: Encoder, views, n_objects: int, shard_len: int, flags, stream=None) -> None:
    """Set flags[o] = 1 (uint32 CUDA tensor, caller-zeroed) for objects whose parity is wrong."""
    v = _views(views)
    check(N.lib().hbec_verify_batch(enc.handle, v, int(n_objects), int(shard_len), C.c_void_p(flags.data_ptr()),
                                    _stream_ptr(stream)))


def encode_objects(enc: Encoder, objs, parity, shard_len: int, stream=None) -> None:
    """Encode every row of ``objs`` [n, k*S] into ``parity`` [n, m*S]."""
    n = objs.shape[0]
    if parity.shape[0] != n:
        raise ValueError("objs and parity disagree on the batch size")
    views = shard_views(objs, enc.DataShards, shard_len) + shard_views(parity, enc.ParityShards, shard_len)
    encode_views(enc, views, n, shard_len, stream)


def fill_splitmix(t, obj_len: int, base_seed: int = HBEC_SEED, first: int = 0, stream=None) -> None:
    """Fill row o of a 2-D uint8 tensor with synthetic object (first + o)."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a 2-D row-contiguous tensor")
    check(N.lib().hbec_fill_splitmix(C.c_void_p(t.data_ptr()), t.shape[0], int(obj_len),
                                     t.stride(0) * t.element_size(), int(base_seed), int(first),
                                     _stream_ptr(stream)))


def apply_views(rows: int, cols: int, coeffs, in_views, out_views, n_objects: int, shard_len: int,
                stream=None) -> None:
    """Generic GF(2^8) matrix apply: out[r] = XOR_c coeffs[r][c] * in[c]."""
    flat = bytes(int(x) for row in coeffs for x in row)
    cbuf = (C.c_uint8 * len(flat)).from_buffer_copy(flat)
    check(N.lib().hbec_apply_batch(int(rows), int(cols), cbuf, _views(in_views), _views(out_views),
                                   int(n_objects), int(shard_len), _stream_ptr(stream)))


class StripePlan:
    """A device-side plan over stripes of mixed shard lengths (hbec_plan_*).
    `stripes` = [(device address, shard_len)], each stripe being k+m shards
    back to back (ecSplit's databuf layout).  Buffers must outlive the plan's
    queued work."""

    def __init__(self, enc: Encoder, stripes=None, objects=None):
        """stripes = [(base, shard_len)] (ecSplit databuf layout), or
        objects = [(data, parity, shard_len)] (data and parity in separate
        regions, hbec_plan_objects)."""
        self.enc = enc
        self._h = C.c_void_p()
        if objects is not None:
            arr = (N.Object * max(1, len(objects)))()
            for i, (d, p, s) in enumerate(objects):
                arr[i].data, arr[i].parity, arr[i].shard_len = d, p, s
            check(N.lib().hbec_plan_objects(enc.handle, arr, len(objects), C.byref(self._h)))
            return
        arr = (N.Stripe * max(1, len(stripes)))()
        for i, (b, s) in enumerate(stripes):
            arr[i].base = b
            arr[i].shard_len = s
        check(N.lib().hbec_plan_stripes(enc.handle, arr, len(stripes), C.byref(self._h)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and N._lib is not None:
            N._lib.hbec_plan_free(h)
            self._h = None

    def info(self):
        nt, fb, sb = C.c_uint64(), C.c_uint64(), C.c_uint64()
        tb = C.c_int()
        check(N.lib().hbec_plan_info(self._h, C.byref(nt), C.byref(tb), C.byref(fb), C.byref(sb)))
        return {"n_tiles": nt.value, "tile_bytes": tb.value, "n_fallback": fb.value, "shard_bytes": sb.value}

    def encode(self, stream=None):
        check(N.lib().hbec_encode_plan(self.enc.handle, self._h, _stream_ptr(stream)))

    def reconstruct(self, present, data_only=False, stream=None):
        p = (C.c_uint8 * len(present))(*[1 if x else 0 for x in present])
        check(N.lib().hbec_reconstruct_plan(self.enc.handle, self._h, p, int(data_only), _stream_ptr(stream)))


KERNEL_KINDS = {0: "unrolled", 1: "pipelined", 2: "streaming", 3: "packed", 4: "records"}


def kernel_info(k: int, r: int, shard_len: int):
    tb, kind, bpc = C.c_int(), C.c_int(), C.c_int()
    check(N.lib().hbec_kernel_info(k, r, int(shard_len), C.byref(tb), C.byref(kind), C.byref(bpc)))
    return {"tile_bytes": tb.value, "kind": KERNEL_KINDS[kind.value], "blocks_per_cu": bpc.value}


def odd_path_stats():
    """Launches since load of the odd-shard main kernels, by family:
    bit-plane (compiled encode XOR networks), table-multiply records, strided;
    and the guard bands: separate edge-kernel launches (`edges`) and main
    launches that coded their own (`fused`)."""
    b, r, s = C.c_uint64(), C.c_uint64(), C.c_uint64()
    check(N.lib().hbec_odd_path_stats(C.byref(b), C.byref(r), C.byref(s)))
    e, f = C.c_uint64(), C.c_uint64()
    check(N.lib().hbec_odd_edge_stats(C.byref(e), C.byref(f)))
    return {"bitplane": b.value, "records": r.value, "strided": s.value, "edges": e.value, "fused": f.value}


def odd_record_cache(clear: bool = False):
    """(cached view sets, calls that reused one) of the strided record
    passes' record cache; clear=True drops it (test hook, device synchronised)."""
    e, h = C.c_uint64(), C.c_uint64()
    check(N.lib().hbec_odd_record_cache(1 if clear else 0, C.byref(e), C.byref(h)))
    return e.value, h.value


def set_odd_chunk_tiles(tiles: int) -> None:
    """Test hook: odd-shard strided launches of at most `tiles` tiles (0 = default)."""
    N.lib().hbec_set_odd_chunk_tiles(int(tiles))


def set_force_stream(on: bool) -> None:
    N.lib().hbec_set_force_stream(1 if on else 0)
