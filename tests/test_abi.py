"""C-ABI boundary checks that need no GPU: the library loads, exports exactly
what include/hbec.h declares, and its host-side logic (matrix build, decode
rows, argument validation, ecutils helpers) matches the oracle / reference
tests.  No GF compute call here (that needs the GPU: test_gpu_parity.py)."""
import ctypes as C
import itertools
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from hummingbird_amd import _native as N
from hummingbird_amd import ecutils as E
from hummingbird_amd import reedsolomon as RS
from oracle import oracle as O

ROOT = Path(__file__).resolve().parents[1]


def header_symbols():
    text = (ROOT / "include" / "hbec.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hbec_[a-z0-9_]+)\s*\(", text)) - {"hbec_read_fn", "hbec_write_fn"})


def test_library_exports_every_header_symbol():
    N.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (hbec_[a-z0-9_]+)$", out, flags=re.M))
    declared = set(header_symbols())
    assert declared, "no symbols parsed from include/hbec.h"
    assert declared <= exported, sorted(declared - exported)
    assert declared == set(N.SYMBOLS)


def test_version_and_strerror():
    assert N.lib().hbec_version() == 2  # 2: int64 data_shards in hbec_ec_shard_length
    assert N.strerror(N.ERR_TOO_FEW_SHARDS) == "too few shards given"
    assert N.strerror(N.ERR_SHARD_SIZE) == "shard sizes do not match"


@pytest.mark.parametrize("k,m,exc", [(0, 2, RS.ErrInvShardNum), (-1, 2, RS.ErrInvShardNum),
                                     (4, -1, RS.ErrInvShardNum), (200, 57, RS.ErrMaxShardNum)])
def test_new_errors(k, m, exc):
    with pytest.raises(exc):
        RS.New(k, m)


@pytest.mark.parametrize("k,m", [(1, 0), (2, 1), (3, 2), (4, 2), (8, 3), (10, 4), (17, 3), (200, 56)])
def test_matrix_matches_oracle(k, m):
    enc = RS.New(k, m)
    want = O.build_matrix(k, k + m) if k + m <= 20 else None
    got = enc.matrix()
    assert np.array_equal(got[:k], np.eye(k, dtype=np.uint8))
    if want is not None:
        assert got.tolist() == want


@pytest.mark.parametrize("k,m", [(4, 2), (8, 3)])
def test_decode_rows_match_oracle(k, m):
    enc = RS.New(k, m)
    oenc = O.Encoder(k, m)
    for e in range(1, m + 1):
        for missing in itertools.combinations(range(k + m), e):
            present = [0 if i in missing else 1 for i in range(k + m)]
            surv, outs, rows = enc.DecodeRows(present)
            osurv, inv = oenc.decode_matrix(present)
            assert surv == osurv
            assert outs == list(missing)
            for o, row in zip(outs, rows):
                if o < k:
                    want = inv[o]
                else:  # parity rows fused with the inverse
                    want = O.mat_mul([oenc.m[o]], inv)[0]
                assert row.tolist() == want
            surv_d, outs_d, _ = enc.DecodeRows(present, data_only=True)
            assert outs_d == [i for i in missing if i < k]


def test_encode_validation_before_device():
    enc = RS.New(4, 2)
    good = [np.ones(8, np.uint8) for _ in range(6)]
    with pytest.raises(RS.ErrTooFewShards):
        enc.Encode(good[:5])
    with pytest.raises(RS.ErrShardSize):
        enc.Encode(good[:5] + [np.ones(7, np.uint8)])
    with pytest.raises(RS.ErrShardSize):
        enc.Encode(good[:5] + [np.zeros(0, np.uint8)])
    with pytest.raises(RS.ErrShardNoData):
        enc.Encode([np.zeros(0, np.uint8)] * 6)


def test_reconstruct_validation_before_device():
    enc = RS.New(4, 2)
    z = np.zeros(0, np.uint8)
    with pytest.raises(RS.ErrShardNoData):
        enc.Reconstruct([z] * 6)
    with pytest.raises(RS.ErrShardSize):
        enc.Reconstruct([np.ones(4, np.uint8)] * 5 + [np.ones(3, np.uint8)])
    with pytest.raises(RS.ErrTooFewShards):
        enc.Reconstruct([z, z, z] + [np.ones(4, np.uint8)] * 3)
    with pytest.raises(RS.ErrTooFewShards):
        enc.Reconstruct([np.ones(4, np.uint8)] * 5)
    # nothing missing / all data present with ReconstructData: no work, no error, no GPU
    full = [np.ones(4, np.uint8)] * 6
    enc.Reconstruct(full)
    enc.ReconstructData([np.ones(4, np.uint8)] * 4 + [z, z])


def test_product_path_has_no_cpu_fallback():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_gpu_parity")
    enc = RS.New(4, 2)
    with pytest.raises(RS.ErrDevice):
        enc.Encode([np.ones(8, np.uint8) for _ in range(6)])


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(N, "LIB_PATH", tmp_path / "nope.so")
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(N.NativeLibraryError):
        N.lib()


def test_ecutils_host_kats(kats):
    for length, k, want in kats["shard_length"]:
        assert E.ec_shard_length(length, k) == want
    for s, e, cs, k, ws, we in kats["range_chunk_align"]:
        assert E.range_chunk_align(s, e, cs, k) == (ws, we)
    for scheme, algo, k, m, c in kats["parse_ec_scheme"]["ok"]:
        assert E.parse_ec_scheme(scheme) == (algo, k, m, c)
    for scheme in kats["parse_ec_scheme"]["err"] + ["", "a/b", "reedsolomon/1/2/3/4", "reedsolomon/ 1/2/3",
                                                    "reedsolomon/1/2/", "reedsolomon/1/+/3"]:
        with pytest.raises(RS.ErrScheme):
            E.parse_ec_scheme(scheme)
    assert E.parse_ec_scheme("reedsolomon/+4/-2/0") == ("reedsolomon", 4, -2, 0)
    assert E.parse_ec_scheme("xor/4/2/1048576") == ("xor", 4, 2, 1048576)


def test_ec_split_zero_length_needs_no_device():
    out = []

    class W:
        def write(self, b):
            out.append(b)

    E.ec_split(4, 2, None, 1 << 20, 0, [W() for _ in range(6)])
    assert out == []


def test_copy_range_refuses_negative_or_inverted_ranges():
    """A negative start (Go would panic on b[negative:], ecobj.go:826-850) or
    end < start is an argument error before any body is read (advisor r03)."""
    read = []

    class Body:
        def read(self, n):
            read.append(n)
            return b""

    class W:
        def write(self, b):
            raise AssertionError("nothing may be written")

    for start, end in [(-1, 10), (-4096, 0), (10, 5)]:
        rc = E.ec_copy_range(4, 2, [Body() for _ in range(6)], 1 << 20, 100, start, end, W())
        assert rc == N.ERR_INVALID_ARG, (start, end)
    assert read == []


def test_ec_split_short_read_is_unexpected_eof():
    import io
    with pytest.raises(RS.ErrUnexpectedEOF):
        E.ec_split(4, 2, io.BytesIO(b""), 1 << 20, 10, [None] * 6)


def test_header_has_c_linkage():
    text = (ROOT / "include" / "hbec.h").read_text()
    assert 'extern "C"' in text
    assert "torch" not in text.lower()


def test_plan_build_needs_no_kernel_launch_for_empty():
    # an empty plan allocates nothing on the device
    enc = RS.New(4, 2)
    import ctypes as C
    h = C.c_void_p()
    arr = (N.Stripe * 1)()
    assert N.lib().hbec_plan_stripes(enc.handle, arr, 0, C.byref(h)) == 0
    nt, fb, sb, tb = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_int()
    assert N.lib().hbec_plan_info(h, C.byref(nt), C.byref(tb), C.byref(fb), C.byref(sb)) == 0
    assert (nt.value, fb.value, sb.value) == (0, 0, 0) and tb.value in (1024, 2048, 3072, 4096)
    N.lib().hbec_plan_free(h)


def test_pure_c_client(tmp_path):
    """The header compiles as C11 with gcc and the library links and answers
    from a plain C program (what cgo does)."""
    exe = tmp_path / "abi_smoke"
    lib_dir = N.LIB_PATH.parent
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "native" / "abi_smoke.c"), "-L", str(lib_dir), "-lhbec",
                    f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, (out.returncode, out.stderr)
    assert "abi ok v2" in out.stdout


def test_shardhash_validation_before_device():
    """hbec_md5_* argument checks answer without a GPU; the
    hashing itself has no CPU fallback."""
    L = N.lib()
    v = (N.View * 1)()
    v[0].base = 4096
    dig = (C.c_uint8 * 64)()
    assert L.hbec_md5_batch(None, 1, 1, 16, C.cast(dig, C.c_void_p), None) == N.ERR_INVALID_ARG
    assert L.hbec_md5_batch(v, 0, 1, 16, C.cast(dig, C.c_void_p), None) == N.ERR_INVALID_ARG
    assert L.hbec_md5_batch(v, 1, 1, 16, None, None) == N.ERR_INVALID_ARG
    odd = C.c_void_p(C.addressof(dig) + 1)
    assert L.hbec_md5_batch(v, 1, 1, 16, odd, None) == N.ERR_INVALID_ARG
    assert "aligned" in N.last_error()
    v[0].base = None
    assert L.hbec_md5_batch(v, 1, 1, 16, C.cast(dig, C.c_void_p), None) == N.ERR_INVALID_ARG
    h = C.c_void_p()
    assert L.hbec_md5_new(0, 1, C.byref(h)) == N.ERR_INVALID_ARG
    assert L.hbec_md5_update(None, v, 16, None) == N.ERR_INVALID_ARG
    assert L.hbec_md5_final(None, C.cast(dig, C.c_void_p), None) == N.ERR_INVALID_ARG
    enc = RS.New(4, 2)
    assert L.hbec_encode_md5_batch(enc.handle, None, 1, 16, C.cast(dig, C.c_void_p), None) == N.ERR_INVALID_ARG
    assert L.hbec_md5_list(None, None, 2, C.cast(dig, C.c_void_p), None) == N.ERR_INVALID_ARG
    assert L.hbec_md5_list(None, None, 0, C.cast(dig, C.c_void_p), None) == N.HBEC_OK
    assert L.hbec_md5_host(None, None, 3, dig) == N.ERR_INVALID_ARG
    st = (N.Stripe * 1)()
    st[0].base = 4096
    st[0].shard_len = 0
    assert L.hbec_encode_host_md5(enc.handle, st, 1, None) == N.ERR_INVALID_ARG
    assert L.hbec_encode_host_md5(enc.handle, st, 1, dig) == N.ERR_SHARD_NO_DATA


def test_object_plan_validation_needs_no_device():
    """hbec_plan_objects: argument checks and an empty plan answer without a GPU."""
    import ctypes as C
    enc = RS.New(4, 2)
    h = C.c_void_p()
    arr = (N.Object * 1)()
    assert N.lib().hbec_plan_objects(None, arr, 1, C.byref(h)) == N.ERR_INVALID_ARG
    assert N.lib().hbec_plan_objects(enc.handle, None, 1, C.byref(h)) == N.ERR_INVALID_ARG
    arr[0].data, arr[0].parity, arr[0].shard_len = 4096, None, 16
    assert N.lib().hbec_plan_objects(enc.handle, arr, 1, C.byref(h)) == N.ERR_INVALID_ARG  # m > 0, no parity
    assert N.lib().hbec_plan_objects(enc.handle, arr, 0, C.byref(h)) == 0
    nt, fb, sb, tb = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_int()
    assert N.lib().hbec_plan_info(h, C.byref(nt), C.byref(tb), C.byref(fb), C.byref(sb)) == 0
    assert (nt.value, fb.value, sb.value) == (0, 0, 0)
    N.lib().hbec_plan_free(h)


def test_host_devices_validation_needs_no_device():
    import ctypes as C
    enc = RS.New(4, 2)
    devs = (C.c_int * 1)(0)
    assert N.lib().hbec_encode_host_devices(enc.handle, None, 1, devs, 1) == N.ERR_INVALID_ARG
    assert N.lib().hbec_encode_host_devices(enc.handle, None, 0, devs, 0) == N.ERR_INVALID_ARG  # n_devices <= 0
    assert N.lib().hbec_reconstruct_host_devices(enc.handle, None, 0, None, 0, devs, 1) == N.ERR_INVALID_ARG
    assert N.lib().hbec_host_alloc(0, C.byref(C.c_void_p())) == N.ERR_INVALID_ARG
    out = C.c_uint64(7)
    buf = (C.c_uint8 * 64)()
    assert N.lib().hbec_host_device_addr(buf, 64, C.byref(out)) == 0 and out.value == 0  # pageable


def test_all_missing_stripe_is_shard_no_data_without_device():
    """klauspost's checkShards precedes the shard count, so a stripe with no
    shard at all is ErrShardNoData in ecReconstruct / ecGlue
    (ecutils.go:111,168) and in the databuf entry points; it is decided
    before any device work."""
    with pytest.raises(RS.ErrShardNoData):
        E.ec_reconstruct(4, 2, [None] * 6, 1024, 10_000, [], [])
    with pytest.raises(RS.ErrShardNoData):
        E.ec_glue(4, 2, [None] * 6, 1024, 10_000)
    with pytest.raises(O.ErrShardNoData):
        O.ec_reconstruct(4, 2, [None] * 6, 1024, 10_000, [0])
    with pytest.raises(O.ErrShardNoData):
        O.ec_glue(4, 2, [None] * 6, 1024, 10_000)
    enc = RS.New(4, 2)
    buf = np.zeros(6 * 16, np.uint8)
    with pytest.raises(RS.ErrShardNoData):
        enc.EncodeDatabuf(buf, 0)
    with pytest.raises(RS.ErrShardNoData):
        enc.ReconstructDatabuf(buf, 16, [0] * 6)
    with pytest.raises(RS.ErrTooFewShards):
        enc.ReconstructDatabuf(buf, 16, [1, 1, 1, 0, 0, 0])
    enc.ReconstructDatabuf(buf, 16, [1] * 6)          # nothing missing: no device work
    enc.ReconstructDatabuf(buf, 16, [1] * 4 + [0, 0], data_only=True)
    with pytest.raises(ValueError):
        enc.EncodeDatabuf(buf, 17)                    # buffer shorter than (k+m)*S
    ok = C.c_int(9)
    assert N.lib().hbec_verify_databuf(enc.handle, None, 16, C.byref(ok)) == N.ERR_INVALID_ARG


def test_verify_validation_before_device():
    """Encoder.Verify's argument checks (klauspost: shard count, then
    checkShards without nil) answer without a GPU."""
    enc = RS.New(4, 2)
    with pytest.raises(RS.ErrTooFewShards):
        enc.Verify([np.ones(8, np.uint8)] * 5)
    with pytest.raises(RS.ErrShardSize):
        enc.Verify([np.ones(8, np.uint8)] * 5 + [np.ones(9, np.uint8)])
    with pytest.raises(RS.ErrShardSize):
        enc.Verify([np.ones(8, np.uint8)] * 5 + [np.zeros(0, np.uint8)])  # a missing shard is not allowed
    with pytest.raises(RS.ErrShardNoData):
        enc.Verify([np.zeros(0, np.uint8)] * 6)


def test_environment_knobs_are_the_documented_table():
    """The library reads the environment in one place (env_knob, hbec.cpp);
    the variables it reads in the product build are exactly the table in
    include/hbec.h (tuning knobs are tune_knob, compiled
    to their defaults unless HBEC_TUNE=1)."""
    csrc = ROOT / "hummingbird_amd" / "csrc"
    src = "\n".join(p.read_text() for p in sorted(csrc.glob("*")) if p.suffix in (".cpp", ".hip", ".h"))
    assert src.count("getenv(") == 1
    read = set(re.findall(r'env_(?:knob|size)\("(HBEC_[A-Z0-9_]+)"', src))
    header = (ROOT / "include" / "hbec.h").read_text()
    table = header[header.index("/* Environment."):header.index("*/", header.index("/* Environment."))]
    documented = set(re.findall(r"\*\s+(HBEC_[A-Z0-9_]+)\s+\d", table))
    assert read == documented, (sorted(read - documented), sorted(documented - read))
    assert len(documented) <= 10
