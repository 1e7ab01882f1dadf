"""Property tests (hypothesis) of the C-ABI's host-side logic against the
oracle restatements — no GPU:

* ecShardLength (ecutils.go:14-24) and rangeChunkAlign (ecobj.go:814-824)
  through libhbec equal the oracle for arbitrary integers;
* parseECScheme (ecobj.go:82-98) accepts exactly what the oracle accepts and
  returns the same fields, including Go strconv.Atoi's sign handling;
* the product's decode rows (hbec_decode_rows) equal the Lagrange closed form
  for random shapes and random present masks (survivors = first k present),
  and the too-few-shards boundary matches klauspost's;
* the product's coding matrix equals the Lagrange matrix for random shapes.
"""
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from hummingbird_amd import ecutils as E
from hummingbird_amd import reedsolomon as RS
from oracle import lagrange as L
from oracle import oracle as O

SETTINGS = settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
i64 = st.integers(min_value=-(1 << 62), max_value=(1 << 62))


@SETTINGS
@given(length=i64, k=st.integers(min_value=1, max_value=256))
def test_shard_length_matches_oracle(length, k):
    assert E.ec_shard_length(length, k) == O.ec_shard_length(length, k)


@SETTINGS
@given(start=st.integers(0, 1 << 40), span=st.integers(1, 1 << 30), chunk=st.integers(1, 1 << 24),
       k=st.integers(1, 64))
def test_range_chunk_align_matches_oracle(start, span, chunk, k):
    end = start + span
    assert E.range_chunk_align(start, end, chunk, k) == O.range_chunk_align(start, end, chunk, k)


field = st.one_of(st.integers(-(1 << 31), (1 << 31) - 1).map(str),
                  st.sampled_from(["+4", "-2", "007", "", " 3", "3 ", "1e3", "0x10", "++1", "4294967296"]))


@SETTINGS
@given(algo=st.sampled_from(["reedsolomon", "xor", "", "reed/solomon"]), a=field, b=field, c=field,
       extra=st.sampled_from(["", "/", "/1"]))
def test_parse_ec_scheme_matches_oracle(algo, a, b, c, extra):
    scheme = f"{algo}/{a}/{b}/{c}{extra}"
    try:
        want = O.parse_ec_scheme(scheme)
    except Exception:  # noqa: BLE001 - the oracle rejects: so must the library
        with pytest.raises(RS.ErrScheme):
            E.parse_ec_scheme(scheme)
        return
    assert E.parse_ec_scheme(scheme) == want


@st.composite
def shape_and_mask(draw):
    k = draw(st.integers(1, 24))
    m = draw(st.integers(1, 12))
    present = draw(st.lists(st.booleans(), min_size=k + m, max_size=k + m))
    return k, m, present, draw(st.booleans())


@SETTINGS
@given(case=shape_and_mask())
def test_decode_rows_match_lagrange(case):
    k, m, present, data_only = case
    enc = RS.New(k, m)
    mask = [1 if p else 0 for p in present]
    if sum(mask) == 0:
        return  # ErrShardNoData is decided before the rows (test_abi)
    if sum(mask) < k:
        with pytest.raises(RS.ErrTooFewShards):
            enc.DecodeRows(mask, data_only=data_only)
        return
    surv, outs, rows = enc.DecodeRows(mask, data_only=data_only)
    lsurv, louts, lrows = L.decode_rows(k, m, mask, data_only)
    assert surv == lsurv and outs == louts
    assert [list(map(int, r)) for r in rows] == lrows


@SETTINGS
@given(k=st.integers(1, 40), m=st.integers(0, 20))
def test_coding_matrix_matches_lagrange(k, m):
    got = RS.New(k, m).matrix()
    assert [list(map(int, r)) for r in got] == L.coding_matrix(k, m)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(k=st.integers(1, 10), m=st.integers(1, 4), chunk=st.integers(1, 300), length=st.integers(0, 3000),
       data=st.data())
def test_oracle_stripe_loops_round_trip(k, m, chunk, length, data):
    """The oracle's ecSplit / ecGlue / ecReconstruct restatements are
    consistent with each other: any <= m lost shard files still glue to the
    object, and rebuilt shard files equal the split's (ecutils.go:26-186)."""
    body = bytes(O.object_bytes(k * 131 + m * 7 + chunk, length))
    files = O.ec_split(k, m, body, chunk)
    assert all(len(f) == O.ec_shard_length(length, k) for f in files) or length == 0
    lost = data.draw(st.lists(st.integers(0, k + m - 1), max_size=m, unique=True))
    kept = [None if i in lost else f for i, f in enumerate(files)]
    if length:
        assert O.ec_glue(k, m, kept, chunk, length) == body
        if lost:
            rebuilt = O.ec_reconstruct(k, m, kept, chunk, length, lost)
            assert [bytes(x) for x in rebuilt] == [bytes(files[i]) for i in lost]
