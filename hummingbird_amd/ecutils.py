"""objectserver/ecutils.go (and the ecobj.go helpers it pairs with) over libhbec.

    ec_shard_length(length, k)                                 ecutils.go:14-24
    ec_split(k, m, fp, chunk_size, content_length, writers)    ecutils.go:26-72
    ec_reconstruct(k, m, bodies, chunk_size, content_length,
                   dsts, dst_chunk_num)                        ecutils.go:74-132
    ec_glue(k, m, bodies, chunk_size, content_length, *dsts)   ecutils.go:134-186
    ec_copy_range(k, m, bodies, chunk_size, content_length,
                  start, end, *dsts)                           ecobj.go:207-267 (CopyRange, byte-exact)
    ec_glue_range(k, m, bodies, chunk_size, content_length,
                  start, end, *dsts)                           CopyRange decode, corrected units (opt-in)
    parse_ec_scheme(scheme)                                    ecobj.go:82-98
    range_chunk_align(start, end, chunk_size, k)               ecobj.go:814-824

Readers are objects with ``read(n) -> bytes`` (b"" at EOF; raising = error);
writers have ``write(b)`` (raising = error).  ``None`` is Go's nil.  The stripe
loops run in C++ (hummingbird_amd/csrc/ecutils.cpp) and every GF step runs on
the GPU.
"""
from __future__ import annotations

import ctypes as C

from . import _native as N
from .reedsolomon import check

_objs: dict[int, object] = {}


def _register(objs):
    ids = []
    for o in objs:
        if o is None:
            ids.append(None)
        else:
            key = id(o)
            _objs[key] = o
            ids.append(key)
    return ids


@N.READ_FN
def _read_cb(ctx, buf, n):
    try:
        data = _objs[ctx].read(n)
    except Exception:
        return -1
    if not data:
        return 0
    ln = len(data)
    C.memmove(buf, data, ln)
    return ln


@N.WRITE_FN
def _write_cb(ctx, buf, n):
    try:
        _objs[ctx].write(C.string_at(buf, n))
    except Exception:
        return 1
    return 0


def _ctx_array(ids):
    return (C.c_void_p * len(ids))(*[i if i is not None else None for i in ids])


def ec_shard_length(length: int, data_shards: int) -> int:
    return int(N.lib().hbec_ec_shard_length(int(length), int(data_shards)))


def ec_split(data_chunks, parity_chunks, fp, chunk_size, content_length, writers):
    ids = _register([fp, *writers])
    try:
        check(N.lib().hbec_ec_split(int(data_chunks), int(parity_chunks), _read_cb, ids[0], int(chunk_size),
                                    int(content_length), _write_cb, _ctx_array(ids[1:])))
    finally:
        for i in ids:
            _objs.pop(i, None)


def ec_reconstruct(data_chunks, parity_chunks, bodies, chunk_size, content_length, dsts, dst_chunk_num):
    b_ids = _register(bodies)
    d_ids = _register(dsts)
    try:
        nums = (C.c_int * len(dst_chunk_num))(*dst_chunk_num)
        check(N.lib().hbec_ec_reconstruct(int(data_chunks), int(parity_chunks), _read_cb, _ctx_array(b_ids),
                                          int(chunk_size), int(content_length), _write_cb, _ctx_array(d_ids),
                                          nums, len(d_ids)))
    finally:
        for i in b_ids + d_ids:
            _objs.pop(i, None)


def ec_glue(data_chunks, parity_chunks, bodies, chunk_size, content_length, *dsts):
    b_ids = _register(bodies)
    d_ids = _register(dsts)
    try:
        check(N.lib().hbec_ec_glue(int(data_chunks), int(parity_chunks), _read_cb, _ctx_array(b_ids),
                                   int(chunk_size), int(content_length), _write_cb, _ctx_array(d_ids),
                                   len(d_ids)))
    finally:
        for i in b_ids + d_ids:
            _objs.pop(i, None)


def ec_glue_range(data_chunks, parity_chunks, bodies, chunk_size, content_length, start, end, *dsts):
    """Object bytes [start, end) (CopyRange, ecobj.go:207-267): bodies are the
    shard streams from rangeChunkAlign's shardStart on."""
    b_ids = _register(bodies)
    d_ids = _register(dsts)
    try:
        check(N.lib().hbec_ec_glue_range(int(data_chunks), int(parity_chunks), _read_cb, _ctx_array(b_ids),
                                         int(chunk_size), int(content_length), int(start), int(end), _write_cb,
                                         _ctx_array(d_ids), len(d_ids)))
    finally:
        for i in b_ids + d_ids:
            _objs.pop(i, None)


def ec_copy_range(data_chunks, parity_chunks, bodies, chunk_size, content_length, start, end, *dsts):
    """ecObject.CopyRange's decode byte for byte as the reference does it
    (ecobj.go:238-265, shard/object unit mix included): bodies are the ranged
    shard streams "bytes=shardStart-shardEnd".  Returns the glue's status
    code (the reference ignores it) instead of raising."""
    b_ids = _register(bodies)
    d_ids = _register(dsts)
    try:
        return int(N.lib().hbec_ec_copy_range(int(data_chunks), int(parity_chunks), _read_cb, _ctx_array(b_ids),
                                              int(chunk_size), int(content_length), int(start), int(end), _write_cb,
                                              _ctx_array(d_ids), len(d_ids)))
    finally:
        for i in b_ids + d_ids:
            _objs.pop(i, None)


def parse_ec_scheme(scheme: str):
    """Returns (algo, data_shards, parity_shards, chunk_size); raises ErrScheme."""
    algo = C.create_string_buffer(len(scheme.encode()) + 1)
    k, m, c = C.c_int64(), C.c_int64(), C.c_int64()  # Go int
    check(N.lib().hbec_parse_ec_scheme(scheme.encode(), algo, len(algo), C.byref(k), C.byref(m), C.byref(c)))
    return algo.value.decode(), k.value, m.value, c.value


def range_chunk_align(start: int, end: int, chunk_size: int, data_shards: int):
    s, e = C.c_int64(), C.c_int64()
    N.lib().hbec_range_chunk_align(int(start), int(end), int(chunk_size), int(data_shards), C.byref(s), C.byref(e))
    return s.value, e.value
