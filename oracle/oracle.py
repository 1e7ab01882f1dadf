"""CPU oracle for the Hummingbird EC hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``hummingbird_amd`` over ``libhbec.so``) never calls it.

What it restates
----------------
The reference's EC arithmetic is not in the reference tree:
``objectserver/ecutils.go:9`` imports ``github.com/klauspost/reedsolomon``,
which is NOT vendored and NOT pinned (no go.mod / Gopkg; ``Makefile:13`` does
``go get -u``; Go 1.10.2 era per ``.travis.yml:7-8`` => klauspost/reedsolomon
~v1.6-v1.9, 2018).  This file restates that library's *default* codec (the
only one ``reedsolomon.New(k, m)`` builds) from its published algorithm:

* GF(2^8), reducing polynomial 0x11D, generator 2   (klauspost galois.go)
* systematic matrix = Vandermonde(k+m, k) x inv(top k x k)  (matrix.go buildMatrix)
* Encode: parity_r = XOR_j M[k+r][j] * data_j       (reedsolomon.go Encode)
* Reconstruct / ReconstructData: first k present shards, invert their rows
  (reedsolomon.go reconstruct)

plus the byte-level striping of the reference's own code:

* ``ec_shard_length``  <- objectserver/ecutils.go:14-24
* ``ec_split``         <- objectserver/ecutils.go:26-72
* ``ec_reconstruct``   <- objectserver/ecutils.go:74-132
* ``ec_glue``          <- objectserver/ecutils.go:134-186
* ``parse_ec_scheme``  <- objectserver/ecobj.go:82-98
* ``range_chunk_align``<- objectserver/ecobj.go:814-824
* ``ec_copy_range``     <- objectserver/ecobj.go:207-267 (CopyRange, byte-exact)
* ``shard_hash``       <- objectserver/indexdb.go:746-753 (hex MD5 of a shard body)

Parity pinning
--------------
The reference's own tests pin only shard LENGTHS, scheme parsing and range
alignment (ecutils_test.go:9-21, ecobj_test.go:196-205,317-330,360-379).  The
codec bytes are pinned by the upstream klauspost / Backblaze known-answer tests
(galois_test.go, matrix_test.go, reedsolomon_test.go TestOneEncode), restated
in ``tests/golden/kats.json`` and checked by ``tests/test_oracle.py``.
"""
from __future__ import annotations

import numpy as np

# --------------------------------------------------------------------------
# GF(2^8) field (klauspost galois.go: logTable / expTable, poly 29 = 0x11D)
# --------------------------------------------------------------------------
GF_POLY = 0x11D


def _build_tables():
    exp = np.zeros(510, dtype=np.int32)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        exp[i + 255] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= GF_POLY
    return exp, log


EXP, LOG = _build_tables()

# full 256x256 multiplication table (mulTable in klauspost galois.go)
_a = np.arange(256)
MUL = np.zeros((256, 256), dtype=np.uint8)
_nz = _a[1:]
MUL[1:, 1:] = EXP[(LOG[_nz][:, None] + LOG[_nz][None, :])].astype(np.uint8)


def gal_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gal_divide(a: int, b: int) -> int:
    if a == 0:
        return 0
    if b == 0:
        raise ZeroDivisionError("divide by zero")
    d = LOG[a] - LOG[b]
    if d < 0:
        d += 255
    return int(EXP[d])


def gal_exp(a: int, n: int) -> int:
    """klauspost galois.go galExp."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(int(LOG[a]) * n) % 255])


# --------------------------------------------------------------------------
# Matrices (klauspost matrix.go)
# --------------------------------------------------------------------------
class SingularMatrix(Exception):
    pass


def vandermonde(rows: int, cols: int) -> list[list[int]]:
    return [[gal_exp(r, c) for c in range(cols)] for r in range(rows)]


def mat_mul(a, b):
    rows, inner, cols = len(a), len(b), len(b[0])
    out = [[0] * cols for _ in range(rows)]
    for r in range(rows):
        for c in range(cols):
            v = 0
            for i in range(inner):
                v ^= gal_mul(a[r][i], b[i][c])
            out[r][c] = v
    return out


def mat_invert(m):
    """Gauss-Jordan over GF(2^8) on [m | I] (matrix.go Invert /
    gaussianElimination).  The inverse is unique, so only the result matters."""
    n = len(m)
    if any(len(row) != n for row in m):
        raise ValueError("only square matrices can be inverted")
    w = [list(m[r]) + [1 if c == r else 0 for c in range(n)] for r in range(n)]
    for r in range(n):
        if w[r][r] == 0:
            for below in range(r + 1, n):
                if w[below][r] != 0:
                    w[r], w[below] = w[below], w[r]
                    break
        if w[r][r] == 0:
            raise SingularMatrix("matrix is singular")
        if w[r][r] != 1:
            scale = gal_divide(1, w[r][r])
            w[r] = [gal_mul(scale, v) for v in w[r]]
        for below in range(r + 1, n):
            if w[below][r] != 0:
                scale = w[below][r]
                w[below] = [x ^ gal_mul(scale, y) for x, y in zip(w[below], w[r])]
    for d in range(n):
        for above in range(d):
            if w[above][d] != 0:
                scale = w[above][d]
                w[above] = [x ^ gal_mul(scale, y) for x, y in zip(w[above], w[d])]
    return [row[n:] for row in w]


def build_matrix(data_shards: int, total_shards: int):
    """matrix.go buildMatrix: Vandermonde(total, data) x inv(top data x data)."""
    vm = vandermonde(total_shards, data_shards)
    top = [row[:] for row in vm[:data_shards]]
    return mat_mul(vm, mat_invert(top))


# --------------------------------------------------------------------------
# Codec (klauspost reedsolomon.go)
# --------------------------------------------------------------------------
class ErrInvShardNum(ValueError):
    pass


class ErrMaxShardNum(ValueError):
    pass


class ErrTooFewShards(ValueError):
    pass


class ErrShardNoData(ValueError):
    pass


class ErrShardSize(ValueError):
    pass


def gf_apply(coeffs, inputs):
    """out[r] = XOR_j coeffs[r][j] * inputs[j] over byte arrays (codeSomeShards)."""
    n = len(inputs[0])
    outs = []
    for row in coeffs:
        acc = np.zeros(n, dtype=np.uint8)
        for c, x in zip(row, inputs):
            if c:
                acc ^= MUL[c][x]
        outs.append(acc)
    return outs


class Encoder:
    """Restatement of klauspost ``reedSolomon`` (default options)."""

    def __init__(self, data_shards: int, parity_shards: int):
        if data_shards <= 0 or parity_shards < 0:
            raise ErrInvShardNum("cannot create Encoder with zero or less data/parity shards")
        if data_shards + parity_shards > 256:
            raise ErrMaxShardNum("cannot create Encoder with more than 256 data+parity shards")
        self.data_shards = data_shards
        self.parity_shards = parity_shards
        self.shards = data_shards + parity_shards
        self.m = build_matrix(data_shards, self.shards)
        self.parity = [self.m[data_shards + i] for i in range(parity_shards)]
        self._inv_cache = {}

    # reedsolomon.go checkShards / shardSize
    @staticmethod
    def _check_shards(shards, nilok):
        size = 0
        for s in shards:
            if len(s) != 0:
                size = len(s)
                break
        if size == 0:
            raise ErrShardNoData("no shard data")
        for s in shards:
            if len(s) != size and (len(s) != 0 or not nilok):
                raise ErrShardSize("shard sizes do not match")
        return size

    def encode(self, shards):
        """Encode in place: shards[k:] are overwritten with parity."""
        if len(shards) != self.shards:
            raise ErrTooFewShards("too few shards given")
        self._check_shards(shards, False)
        data = [np.asarray(s, dtype=np.uint8) for s in shards[: self.data_shards]]
        for i, out in enumerate(gf_apply(self.parity, data)):
            shards[self.data_shards + i][:] = out
        return shards

    def decode_matrix(self, present):
        """Rows of inv(sub) for the first k present shards; returns
        (survivor indices, inverse).  Cached by erasure set like klauspost's
        inversion tree (the cache does not change results)."""
        valid = [i for i in range(self.shards) if present[i]][: self.data_shards]
        key = tuple(valid)
        if key not in self._inv_cache:
            sub = [self.m[i][:] for i in valid]
            self._inv_cache[key] = mat_invert(sub)
        return valid, self._inv_cache[key]

    def _reconstruct(self, shards, data_only):
        if len(shards) != self.shards:
            raise ErrTooFewShards("too few shards given")
        size = self._check_shards(shards, True)
        present = [len(s) != 0 for s in shards]
        n_present = sum(present)
        data_present = sum(present[: self.data_shards])
        if n_present == self.shards or (data_only and data_present == self.data_shards):
            return shards
        if n_present < self.data_shards:
            raise ErrTooFewShards("too few shards given")
        valid, inv = self.decode_matrix(present)
        survivors = [np.asarray(shards[i], dtype=np.uint8) for i in valid]
        miss_data = [i for i in range(self.data_shards) if not present[i]]
        if miss_data:
            outs = gf_apply([inv[i] for i in miss_data], survivors)
            for i, o in zip(miss_data, outs):
                shards[i] = o
        if data_only:
            return shards
        miss_par = [i for i in range(self.data_shards, self.shards) if not present[i]]
        if miss_par:
            data = [np.asarray(shards[i], dtype=np.uint8) for i in range(self.data_shards)]
            outs = gf_apply([self.m[i] for i in miss_par], data)
            for i, o in zip(miss_par, outs):
                shards[i] = o
        assert all(len(s) == size for s in shards if len(s))
        return shards

    def reconstruct(self, shards):
        return self._reconstruct(shards, False)

    def reconstruct_data(self, shards):
        return self._reconstruct(shards, True)


# --------------------------------------------------------------------------
# ecutils.go / ecobj.go byte semantics
# --------------------------------------------------------------------------
def shard_hash(body) -> str:
    """StablePut's ShardHash (objectserver/indexdb.go:746-753): md5.New() fed
    the whole shard body by common.Copy, hex.EncodeToString of the sum.  The
    MD5 itself is Python's hashlib (RFC 1321), pinned by the RFC 1321 test
    suite in tests/golden/kats.json."""
    import hashlib

    return hashlib.md5(bytes(body)).hexdigest()


def ec_split_hashes(k: int, m: int, data: bytes, chunk_size: int) -> list[str]:
    """ShardHash of every shard file ec_split produces (what the k+m receiving
    StablePut calls compute, ecobj.go:756-774 -> indexdb.go:746-753)."""
    return [shard_hash(f) for f in ec_split(k, m, data, chunk_size)]


def ec_shard_length(length: int, data_shards: int) -> int:
    """objectserver/ecutils.go:14-24."""
    if length < 0:
        return 0
    s = length // data_shards
    if length % data_shards > 0:
        s += 1
    return s


def ec_split(k: int, m: int, data: bytes, chunk_size: int):
    """objectserver/ecutils.go:26-72 on an in-memory object.  Returns the k+m
    shard files (the concatenation of each shard's per-stripe sub-chunks)."""
    enc = Encoder(k, m)
    files = [bytearray() for _ in range(k + m)]
    total = 0
    content_length = len(data)
    while total < content_length:
        expected = min(k * chunk_size, content_length - total)
        stripe = bytearray(data[total : total + expected])
        total += expected
        while len(stripe) % k:  # pad with zeros to a multiple of k (:51-54)
            stripe.append(0)
        s = len(stripe) // k
        arr = np.frombuffer(bytes(stripe), dtype=np.uint8)
        shards = [arr[i * s : (i + 1) * s].copy() for i in range(k)]
        shards += [np.zeros(s, dtype=np.uint8) for _ in range(m)]
        enc.encode(shards)
        for i in range(k + m):
            files[i] += shards[i].tobytes()
    return [bytes(f) for f in files]


def _stripe_sizes(k, chunk_size, content_length):
    """Per-stripe shard sub-chunk sizes used by ecReconstruct / ecGlue
    (ecutils.go:86-92 / :144-150)."""
    sizes = []
    done = 0
    while done < content_length:
        s = chunk_size
        if content_length - done < chunk_size * k:
            rem = content_length - done
            s = rem // k + (1 if rem % k else 0)
        sizes.append(s)
        done += min(s * k, content_length - done)
    return sizes


def ec_reconstruct(k, m, shard_files, chunk_size, content_length, dst_chunk_nums):
    """objectserver/ecutils.go:74-132: shard_files[i] is bytes or None (missing).
    Returns the reconstructed shard files for dst_chunk_nums."""
    enc = Encoder(k, m)
    outs = [bytearray() for _ in dst_chunk_nums]
    off = 0
    for s in _stripe_sizes(k, chunk_size, content_length):
        shards = []
        for i in range(k + m):
            f = shard_files[i]
            if f is not None and len(f) >= off + s:
                shards.append(np.frombuffer(f[off : off + s], dtype=np.uint8).copy())
            else:
                shards.append(np.zeros(0, dtype=np.uint8))
        enc.reconstruct(shards)
        for o, c in zip(outs, dst_chunk_nums):
            o += shards[c].tobytes()
        off += s
    return [bytes(o) for o in outs]


def ec_glue(k, m, shard_files, chunk_size, content_length):
    """objectserver/ecutils.go:134-186: returns the object bytes."""
    enc = Encoder(k, m)
    out = bytearray()
    off = 0
    for s in _stripe_sizes(k, chunk_size, content_length):
        shards = []
        for i in range(k + m):
            f = shard_files[i]
            if f is not None and len(f) >= off + s:
                shards.append(np.frombuffer(f[off : off + s], dtype=np.uint8).copy())
            else:
                shards.append(np.zeros(0, dtype=np.uint8))
        enc.reconstruct_data(shards)
        for i in range(k):
            d = shards[i].tobytes()
            rem = content_length - len(out)
            out += d[:rem]
        off += s
    return bytes(out)


class RangeBytesWriter:
    """rangeBytesWriter (objectserver/ecobj.go:826-850): keeps the bytes after
    the first start_offset, at most `length` of them."""

    def __init__(self, start_offset: int, length: int):
        self.start_offset, self.length, self.out = start_offset, length, bytearray()

    def write(self, b: bytes) -> int:
        n = len(b)
        if self.start_offset > n:
            self.start_offset -= n
            return n
        if self.length <= 0:
            return n
        b = b[self.start_offset:]
        self.start_offset = 0
        if len(b) > self.length:
            b = b[:self.length]
        self.length -= len(b)
        self.out += b
        return n


def ec_glue_range(k, m, shard_files, chunk_size, content_length, start, end):
    """Range GET decode (ecObject.CopyRange, objectserver/ecobj.go:207-267) in
    object-byte units: glue the stripes covering [start, end) from the shard
    bytes at rangeChunkAlign's shardStart on, then keep [start, end) through a
    RangeBytesWriter.  (The reference passes a shard-byte length and start %
    chunk_size, ecobj.go:238-265; restated here with the object-byte
    quantities those stand for.)"""
    stripe = k * chunk_size
    obj0 = start // stripe * stripe
    obj1 = min(content_length, -(-end // stripe) * stripe)
    shard_start, _ = range_chunk_align(start, end, chunk_size, k)
    files = [None if f is None else f[shard_start:] for f in shard_files]
    w = RangeBytesWriter(start - obj0, end - start)
    body = ec_glue(k, m, files, chunk_size, obj1 - obj0)
    for i in range(0, len(body), chunk_size):  # the glue writes shard-sized pieces
        w.write(body[i:i + chunk_size])
    return bytes(w.out)


def http_range_body(f, first: int, last: int):
    """The shard server's answer to "Range: bytes=first-last" (inclusive) over
    shard file f, as CopyRange sees it (ecobj.go:241-257): bytes [first,
    last] clipped at EOF, or None (no body: a 416 is skipped at :253-255)
    when first is past the end of the file."""
    if f is None or first >= len(f):
        return None
    return f[first:last + 1]


def ec_copy_range(k, m, shard_files, chunk_size, content_length, start, end):
    """ecObject.CopyRange (objectserver/ecobj.go:207-267) byte for byte, the
    reference's unit mix included: rangeChunkAlign's shard-byte span (capped
    at the object's content length, :239-241) is glued as if it were the
    content length, through a rangeBytesWriter that starts at start %
    chunk_size (:264-265).  ecGlue's error is ignored there (CopyRange
    returns end - start, nil), so a stripe that cannot be rebuilt just ends
    the output."""
    shard_start, shard_end = range_chunk_align(start, end, chunk_size, k)
    if shard_end > content_length:
        shard_end = content_length
    files = [http_range_body(f, shard_start, shard_end) for f in shard_files]
    w = RangeBytesWriter(start % chunk_size, end - start)
    glue_len = shard_end - shard_start
    enc = Encoder(k, m)
    written = 0
    failed = [False] * (k + m)
    off = 0
    for s in _stripe_sizes(k, chunk_size, glue_len):  # ecutils.go:142-186
        shards = []
        for i in range(k + m):
            f = files[i]
            if f is not None and not failed[i] and len(f) >= off + s:
                shards.append(np.frombuffer(f[off:off + s], dtype=np.uint8).copy())
            else:
                if f is not None:
                    failed[i] = True
                shards.append(np.zeros(0, dtype=np.uint8))
        try:
            enc.reconstruct_data(shards)
        except ValueError:
            break  # ecGlue returns the error; CopyRange drops it
        for i in range(k):
            d = shards[i].tobytes()[:glue_len - written]
            w.write(d)
            written += len(d)
        off += s
    return bytes(w.out)


def _shard_positions(k, chunk_size, length):
    """ecSplit's layout (ecutils.go:26-72) as index arithmetic: for every data
    shard, the object position each shard byte holds (-1 = zero padding)."""
    shards = [[] for _ in range(k)]
    done = 0
    while done < length:
        e = chunk_size
        if length - done < chunk_size * k:
            e = (length - done) // k + (1 if (length - done) % k else 0)
        for i in range(k):
            shards[i] += [p if p < length else -1 for p in range(done + i * e, done + (i + 1) * e)]
        done += min(e * k, length - done)
    return shards


def copy_range_positions(k, chunk_size, content_length, start, end):
    """The object positions CopyRange (ec_copy_range, all shards healthy)
    writes, in order: the same glue and writer arithmetic on position labels
    instead of bytes (-1 = a padding byte)."""
    pos = _shard_positions(k, chunk_size, content_length)
    shard_start, shard_end = range_chunk_align(start, end, chunk_size, k)
    if shard_end > content_length:
        shard_end = content_length
    glue_len = shard_end - shard_start
    stream, off = [], 0
    for s in _stripe_sizes(k, chunk_size, glue_len):
        if any(shard_start + off + s > len(p) for p in pos):
            break  # a short shard body: the stripe cannot be rebuilt from data alone (parity has the same length)
        for i in range(k):
            stream += pos[i][shard_start + off:shard_start + off + s][:glue_len - len(stream)]
        off += s
    a = start % chunk_size
    return stream[a:a + (end - start)] if a <= len(stream) else []


def copy_range_is_object_slice(k: int, chunk_size: int, content_length: int, start: int, end: int) -> bool:
    """True where CopyRange's bytes equal object[start:end]."""
    return copy_range_positions(k, chunk_size, content_length, start, end) == list(range(start, end))


def parse_ec_scheme(scheme: str):
    """objectserver/ecobj.go:82-98."""
    sections = scheme.split("/")
    if len(sections) != 4:
        raise ValueError(f"{len(sections)} scheme sections")
    algo = sections[0]
    names = ["Invalid data shard count", "Invalid parity shard count", "Invalid chunk size"]
    vals = []
    for sec, name in zip(sections[1:], names):
        try:
            vals.append(_go_atoi(sec))
        except ValueError:
            raise ValueError(name) from None
    return (algo, *vals)


def _go_atoi(s: str) -> int:
    # strconv.Atoi: optional sign, decimal digits only, no spaces/underscores;
    # Go's int is 64-bit on the reference's amd64 build (ErrRange beyond it)
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        raise ValueError(s)
    v = int(s)
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError(s)
    return v


def range_chunk_align(start: int, end: int, chunk_size: int, data_shards: int):
    """objectserver/ecobj.go:814-824."""
    stripe = chunk_size * data_shards
    start_chunk = start // stripe
    end_chunk = end // stripe
    start = start_chunk * chunk_size
    if end % stripe == 0:
        end = end_chunk * chunk_size
    else:
        end = (end_chunk + 1) * chunk_size
    return start, end


# --------------------------------------------------------------------------
# Synthetic inputs: splitmix64 stream, little-endian bytes
# --------------------------------------------------------------------------
HBEC_SEED = 0x48424543
_GOLDEN = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


def splitmix_bytes(seed: int, n: int) -> np.ndarray:
    """Bytes of the splitmix64 stream seeded with ``seed`` (vectorised)."""
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(1, words + 1, dtype=np.uint64)
        z = np.uint64(seed & _M64) + idx * np.uint64(_GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def object_seed(base_seed: int, i: int) -> int:
    return (base_seed ^ ((i * _GOLDEN) & _M64)) & _M64


def object_bytes(i: int, n: int, base_seed: int = HBEC_SEED) -> np.ndarray:
    return splitmix_bytes(object_seed(base_seed, i), n)


def audit_ec_shard(body: bytes, content_length: str, ec_scheme: str, index_hash: str):
    """ecAuditor.AuditItem for a stable EC shard (objectserver/auditor.go:100-158,
    md5BytesPerSec > 0): the file must be ecShardLength(Content-Length, k)
    bytes, then its MD5 must equal the index's ShardHash.  Returns
    (bytes, error message or None) as AuditItem returns (int64, error)."""
    import re

    if not re.fullmatch(r"[+-]?[0-9]+", content_length or ""):  # strconv.ParseInt(s, 10, 64)
        return 0, f"Error parsing content-length from metadata: {content_length!r}"
    cl = int(content_length)
    try:
        _, ds, _, _ = parse_ec_scheme(ec_scheme)
    except ValueError as e:
        return 0, f"Error decoding ec-scheme: {e}"
    f_bytes = ec_shard_length(cl, ds)
    if f_bytes != len(body):
        return 0, f"File size ({len(body)}) doesn't match metadata ({f_bytes})"
    if shard_hash(body) != index_hash:
        return len(body), "File contents don't match object hash"
    return len(body), None
