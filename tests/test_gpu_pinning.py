"""Oracle pinning inside the GPU run (`pytest -m gpu`): the reference-held and
upstream fixtures re-checked against the product on the GPU box, and the GPU
Verify kernel fed parity that the GPU did NOT produce.

* Verify: parity from the CPU oracle (oracle/gf_oracle.c)
  and from the committed golden seeded vectors -> every object verifies;
  one flipped byte in any data or parity shard -> exactly that object flagged.
* Host-integer KATs of the reference's own tests: ecShardLength
  (ecutils_test.go:9-21), parseECScheme (ecobj_test.go:317-330),
  rangeChunkAlign (ecobj_test.go:360-379), the auditor's EC shard rule with
  the GPU MD5 (auditor_test.go:583-661).
* The coding matrix and every decode row the kernels apply, against the
  closed-form Lagrange derivation (oracle/lagrange.py: no matrix inversion,
  structurally different from the product's Gauss-Jordan)."""
import hashlib
import itertools

import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import ecutils as E
from hummingbird_amd import reedsolomon as RS
from hummingbird_amd import shardhash as H
from oracle import coracle as CO
from oracle import lagrange as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    yield


def sha(b):
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


@pytest.mark.parametrize("k,m,size,n", [(4, 2, MiB, 48), (8, 3, MiB, 24), (8, 3, 4096, 2000), (10, 4, 40960, 64),
                                        (3, 2, 3 * 4096, 33)])
def test_verify_batch_on_oracle_parity(k, m, size, n):
    s = size // k
    enc = RS.New(k, m)
    objs = CO.fill_objects(1234 + k, n, size)
    par, _ = CO.encode_batch(k, m, objs, threads=CO.cpu_threads())
    d_objs = torch.from_numpy(objs).cuda()
    d_par = torch.from_numpy(par).cuda()
    views = B.shard_views(d_objs, k, s) + B.shard_views(d_par, m, s)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0
    rng = np.random.default_rng(k * 100 + m)
    bad = sorted(set(rng.integers(0, n, 6).tolist()) | {0, n - 1})
    for o in bad:
        if rng.integers(0, 2):
            d_objs[o, int(rng.integers(0, k * s))] ^= 0x80
        else:
            d_par[o, int(rng.integers(0, m * s))] ^= 0x01
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert torch.nonzero(flags).flatten().tolist() == bad


def test_verify_host_on_golden_seeded_vectors(vectors):
    """The committed seeded objects: oracle parity must hash to the golden
    shard digests, then Encoder.Verify on the GPU accepts it and rejects one
    flipped byte in each shard."""
    for case in vectors["seeded"]:
        k, m, size = case["k"], case["m"], case["size"]
        s = size // k
        obj = CO.fill_objects(case["index"], 1, size)
        par, _ = CO.encode_batch(k, m, obj)
        shards = [obj[0][j * s:(j + 1) * s].copy() for j in range(k)] + [par[0][r * s:(r + 1) * s].copy()
                                                                       for r in range(m)]
        assert [sha(x) for x in shards] == case["shard_sha256"]
        enc = RS.New(k, m)
        assert enc.Verify(shards)
        for i in (0, k - 1, k, k + m - 1):
            bad = [x.copy() for x in shards]
            bad[i][s // 3] ^= 0x10
            assert not enc.Verify(bad), (case["k"], case["m"], i)


def test_verify_databuf_on_testing_3_2(vectors):
    """The TESTING 3+2 stripe (ecobj_test.go:144-206) with the golden shard files."""
    files = [bytes.fromhex(f) if isinstance(f, str) else bytes(f) for f in vectors["testing_3_2"]["files"]]
    buf = np.frombuffer(b"".join(files), dtype=np.uint8).copy()
    enc = RS.New(3, 2)
    assert enc.VerifyDatabuf(buf, 3)
    buf[13] ^= 1
    assert not enc.VerifyDatabuf(buf, 3)


def test_reference_host_kats_in_gpu_run(kats):
    """ecutils_test.go:9-21, ecobj_test.go:317-330, :360-379 through the library."""
    for length, k, want in kats["shard_length"]:
        assert E.ec_shard_length(length, k) == want
    for s, e, cs, k, ws, we in kats["range_chunk_align"]:
        assert E.range_chunk_align(s, e, cs, k) == (ws, we)
    for scheme, algo, k, m, c in kats["parse_ec_scheme"]["ok"]:
        assert E.parse_ec_scheme(scheme) == (algo, k, m, c)
    for scheme in kats["parse_ec_scheme"]["err"]:
        with pytest.raises(RS.ErrScheme):
            E.parse_ec_scheme(scheme)


def test_auditor_fixtures_with_gpu_md5(kats):
    """auditor_test.go:583-661: size rule + ShardHash, the MD5 computed by the
    GPU kernel (hbec_md5_host), same (bytes, pass/fail) as the reference test."""
    for c in kats["auditor_ec"]["cases"]:
        got, err = H.audit_ec_shard(c["body"].encode(), c["content_length"], c["ec_scheme"], c["shard_hash"])
        assert got == c["bytes"], c["test"]
        assert (err is None) == c["ok"], (c["test"], err)


@pytest.mark.parametrize("k,m,max_e", [(4, 2, 2), (8, 3, 3), (10, 4, 2), (17, 3, 1)])
def test_rows_the_kernels_apply_equal_closed_form(k, m, max_e):
    """hbec_matrix and hbec_decode_rows (what the kernels are launched with)
    against the Lagrange closed form; then one reconstruct per pattern on
    the GPU with the closed-form rows applied by the oracle."""
    enc = RS.New(k, m)
    assert enc.matrix().tolist() == L.coding_matrix(k, m)
    s = 1024
    obj = CO.fill_objects(77 + k, 1, k * s)[0]
    full = [obj[j * s:(j + 1) * s].copy() for j in range(k)]
    full += CO.apply(L.parity_rows(k, m), full)
    for e in range(1, max_e + 1):
        for missing in itertools.combinations(range(k + m), e):
            present = [0 if i in missing else 1 for i in range(k + m)]
            surv, outs, rows = enc.DecodeRows(present)
            lsurv, louts, lrows = L.decode_rows(k, m, present)
            assert (surv, outs, rows.tolist()) == (lsurv, louts, lrows)
    for missing in [tuple(range(max_e)), tuple(range(k, k + min(m, max_e))), (k - 1,)]:
        sh = [x.copy() if i not in missing else None for i, x in enumerate(full)]
        enc.Reconstruct(sh)
        for i in range(k + m):
            assert np.array_equal(sh[i], full[i]), (missing, i)
