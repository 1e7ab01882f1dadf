"""ShardHash on the GPU: MD5 of shard bodies (objectserver/indexdb.go:746-753,
``hex.EncodeToString(md5(body))``; re-checked by the auditor,
objectserver/auditor.go:100-156), computed by libhbec's md5 kernel — one GPU
lane per (object, shard) chain.

Digest layout everywhere: uint8 [n_objects, n_views, 16] (raw MD5), device
memory.  ``hexdigests`` turns it into the strings the index DB stores.
"""
from __future__ import annotations

import ctypes as C

from . import _native as N
from .batch import _stream_ptr, _views, shard_views
from .reedsolomon import Encoder, check


def _digest_tensor(n_objects: int, n_views: int, device):
    import torch

    return torch.empty((n_objects, n_views, 16), dtype=torch.uint8, device=device)


def md5_views(views, n_objects: int, length: int, digests=None, device="cuda", stream=None):
    """MD5 of `length` bytes at every (base + o*stride) of every view."""
    n = len(views)
    if digests is None:
        digests = _digest_tensor(n_objects, n, device)
    check(N.lib().hbec_md5_batch(_views(views), n, int(n_objects), int(length), C.c_void_p(digests.data_ptr()),
                                 _stream_ptr(stream)))
    return digests


def md5_rows(t, n_shards: int, shard_len: int, stream=None):
    """MD5 of each of the n_shards consecutive shards in every row of a 2-D tensor."""
    return md5_views(shard_views(t, n_shards, shard_len), t.shape[0], shard_len, device=t.device, stream=stream)


def encode_md5_views(enc: Encoder, views, n_objects: int, shard_len: int, digests=None, device="cuda",
                     stream=None):
    """hbec_encode_md5_batch: parity of every object plus the MD5 of all k+m shards."""
    n = enc.DataShards + enc.ParityShards
    if len(views) != n:
        raise ValueError("need k+m views")
    if digests is None:
        digests = _digest_tensor(n_objects, n, device)
    check(N.lib().hbec_encode_md5_batch(enc.handle, _views(views), int(n_objects), int(shard_len),
                                        C.c_void_p(digests.data_ptr()), _stream_ptr(stream)))
    return digests


def encode_objects_md5(enc: Encoder, objs, parity, shard_len: int, stream=None):
    """encode_objects (batch.py) + ShardHash of every data and parity shard."""
    views = shard_views(objs, enc.DataShards, shard_len) + shard_views(parity, enc.ParityShards, shard_len)
    return encode_md5_views(enc, views, objs.shape[0], shard_len, device=objs.device, stream=stream)


def md5_list(buffers, digests=None, device="cuda", stream=None):
    """MD5 of device buffers of any lengths: `buffers` = [(device address, length)]
    or 1-D uint8 CUDA tensors.  Returns uint8 [n, 16] digests (device)."""
    import torch

    pairs = [(b.data_ptr(), b.numel()) if hasattr(b, "data_ptr") else (int(b[0]), int(b[1])) for b in buffers]
    n = len(pairs)
    if digests is None:
        digests = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=device)
    addrs = (C.c_void_p * max(n, 1))(*[a for a, _ in pairs])
    lens = (C.c_uint64 * max(n, 1))(*[ln for _, ln in pairs])
    check(N.lib().hbec_md5_list(addrs, lens, n, C.c_void_p(digests.data_ptr()), _stream_ptr(stream)))
    return digests[:n]


def md5_host(buffers):
    """ShardHash of host buffers (bytes / numpy uint8 arrays) of any lengths,
    hashed on the GPU (an auditor pass).  Returns hex strings."""
    import numpy as np

    arrs = [np.ascontiguousarray(np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else b,
                                 dtype=np.uint8) for b in buffers]
    n = len(arrs)
    ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrs])
    lens = (C.c_uint64 * max(n, 1))(*[a.size for a in arrs])
    out = (C.c_uint8 * (16 * max(n, 1)))()
    check(N.lib().hbec_md5_host(ptrs, lens, n, out))
    raw = bytes(out)
    return [raw[16 * i:16 * (i + 1)].hex() for i in range(n)]


class MD5Chains:
    """Streaming MD5 chains (hbec_md5_*): n_views x n_objects chains fed one
    stripe's sub-chunks per update — a multi-stripe shard file's hash."""

    def __init__(self, n_views: int, n_objects: int):
        h = C.c_void_p()
        check(N.lib().hbec_md5_new(int(n_views), int(n_objects), C.byref(h)))
        self._h = h
        self.n_views = n_views
        self.n_objects = n_objects

    def close(self):
        if getattr(self, "_h", None):
            N.lib().hbec_md5_free(self._h)
            self._h = None

    __del__ = close

    def update(self, views, length: int, stream=None):
        if len(views) != self.n_views:
            raise ValueError("need n_views views")
        check(N.lib().hbec_md5_update(self._h, _views(views), int(length), _stream_ptr(stream)))

    def final(self, digests=None, device="cuda", stream=None):
        if digests is None:
            digests = _digest_tensor(self.n_objects, self.n_views, device)
        check(N.lib().hbec_md5_final(self._h, C.c_void_p(digests.data_ptr()), _stream_ptr(stream)))
        return digests


def hexdigests(digests):
    """uint8 [..., 16] digests -> nested lists of hex strings (ShardHash form)."""
    import numpy as np

    a = np.ascontiguousarray(digests.cpu().numpy() if hasattr(digests, "cpu") else digests)
    flat = a.reshape(-1, 16)
    out = [bytes(r).hex() for r in flat]
    shape = a.shape[:-1]
    if len(shape) == 1:
        return out
    res, i = [], 0
    for _ in range(shape[0]):
        res.append(out[i:i + shape[1]])
        i += shape[1]
    return res


def audit_ec_shard(body, content_length: str, ec_scheme: str, index_hash: str):
    """ecAuditor.AuditItem for a stable EC shard (objectserver/auditor.go:100-158,
    the md5BytesPerSec > 0 branch) over the library: the shard file must be
    ecShardLength(Content-Length, k) bytes (hbec_parse_ec_scheme +
    hbec_ec_shard_length), then its MD5, hashed on the GPU (hbec_md5_host),
    must equal the index's ShardHash.  Returns (bytes, error or None), as
    AuditItem returns (int64, error): (0, err) on a size mismatch, (n, err)
    on a hash mismatch."""
    import re

    from . import ecutils as E
    from .reedsolomon import ErrScheme

    if not re.fullmatch(r"[+-]?[0-9]+", content_length or ""):  # strconv.ParseInt(s, 10, 64)
        return 0, f"Error parsing content-length from metadata: {content_length!r}"
    try:
        _, ds, _, _ = E.parse_ec_scheme(ec_scheme)
    except ErrScheme as e:
        return 0, f"Error decoding ec-scheme: {e}"
    f_bytes = E.ec_shard_length(int(content_length), ds)
    if f_bytes != len(body):
        return 0, f"File size ({len(body)}) doesn't match metadata ({f_bytes})"
    (calc,) = md5_host([body])
    if calc != index_hash:
        return len(body), "File contents don't match object hash"
    return len(body), None
