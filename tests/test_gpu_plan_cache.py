"""Plans keep the gf_odd_rec records of the passes they ran (plan.cpp
OddRecCache): the records depend on the stripes and on which shards a pass
reads and writes, never on the data or the coefficients.  Repeated Encode
(objectserver/ecutils.go:59) over changed data, Reconstruct
(ecutils.go:111) with alternating erasure patterns, and calls from a second
stream must all still equal the oracle byte for byte."""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,m", [(4, 2), (8, 3), (10, 4), (14, 3)])
def test_plan_records_reused_across_calls_patterns_and_streams(k, m):
    rng = np.random.default_rng(1000 * k + m)
    sizes = [int(x) | 1 for x in rng.integers(200, 9000, 40)]
    data = torch.empty(sum(k * s for s in sizes) + 64, dtype=torch.uint8, device="cuda")
    parity = torch.empty(sum(m * s for s in sizes) + 64, dtype=torch.uint8, device="cuda")
    objs, do, po = [], 3, 5
    for s in sizes:
        objs.append((data.data_ptr() + do, parity.data_ptr() + po, s))
        do += k * s
        po += m * s
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, objects=objs)
    rows = CO.build_matrix(k, m)[k:]

    def check_parity():
        torch.cuda.synchronize()
        d, p = data.cpu().numpy(), parity.cpu().numpy()
        do, po = 3, 5
        for s in sizes:
            want = CO.apply(rows, [d[do + j * s:do + (j + 1) * s] for j in range(k)])
            for r in range(m):
                assert np.array_equal(p[po + r * s:po + (r + 1) * s], want[r])
            do += k * s
            po += m * s

    side = torch.cuda.Stream()
    for rep in range(3):
        B.fill_splitmix(data.view(1, -1), data.numel(), first=77 + rep)
        if rep == 1:  # the same plan from another stream
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                plan.encode(stream=side)
            side.synchronize()
        else:
            plan.encode()
        check_parity()
    keep_d, keep_p = data.clone(), parity.clone()
    for lost in ([0, k], [1], [0, k], [k + m - 1, 2][:m]):
        present = [0 if i in lost else 1 for i in range(k + m)]
        do, po = 3, 5
        for s in sizes:
            for i in lost:
                if i < k:
                    data[do + i * s:do + (i + 1) * s] = 0x6B
                else:
                    parity[po + (i - k) * s:po + (i - k + 1) * s] = 0x6B
            do += k * s
            po += m * s
        plan.reconstruct(present)
        torch.cuda.synchronize()
        assert torch.equal(data, keep_d) and torch.equal(parity, keep_p), lost


# Strided record passes keep the per-object records of views they code again
# (hbec.cpp objrec_cached: cached on a key's second sighting), chunked
# launches included (hbec_set_odd_chunk_tiles).
@pytest.mark.parametrize("k,m,s,chunk", [(8, 3, 8191, 0), (10, 4, 8193, 0), (8, 3, 8191, 60)])
def test_strided_records_reused_across_calls_and_streams(k, m, s, chunk):
    n = 40
    pitch = (k + m) * s + 9
    buf = torch.empty(3 + n * pitch + 64, dtype=torch.uint8, device="cuda")
    views = [(buf.data_ptr() + 3 + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    rows = CO.build_matrix(k, m)[k:]
    side = torch.cuda.Stream()
    B.set_odd_chunk_tiles(chunk)
    B.odd_record_cache(clear=True)
    try:
        for rep in range(4):
            B.fill_splitmix(buf.view(1, -1), buf.numel(), first=500 + rep)
            p0 = B.odd_path_stats()
            if rep == 2:
                torch.cuda.synchronize()
                with torch.cuda.stream(side):
                    B.encode_views(enc, views, n, s, stream=side)
                side.synchronize()
            else:
                B.encode_views(enc, views, n, s)
            torch.cuda.synchronize()
            p1 = B.odd_path_stats()
            launches = sum(p1[x] - p0[x] for x in ("bitplane", "records", "strided"))
            got = buf.cpu().numpy()
            for o in range(n):
                b = 3 + o * pitch
                want = CO.apply(rows, [got[b + j * s:b + (j + 1) * s] for j in range(k)])
                for r in range(m):
                    assert np.array_equal(got[b + (k + r) * s:b + (k + r + 1) * s], want[r]), (rep, o, r)
        entries, hits = B.odd_record_cache()
        assert launches >= (2 if chunk else 1)
        assert entries == launches and hits == 2 * launches, (entries, hits)  # built on call 2, reused on 3 and 4
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        for rep in range(3):  # Verify's own records, cached from the second call
            flags.zero_()
            hit = {5 + rep: (k, 1), 30 - rep: (1, s - 2)}
            for o, (i, p) in hit.items():
                buf[3 + o * pitch + i * s + p] ^= 0x11
            B.verify_views(enc, views, n, s, flags)
            torch.cuda.synchronize()
            assert flags.nonzero().flatten().tolist() == sorted(hit), rep
            for o, (i, p) in hit.items():
                buf[3 + o * pitch + i * s + p] ^= 0x11
    finally:
        B.set_odd_chunk_tiles(0)
