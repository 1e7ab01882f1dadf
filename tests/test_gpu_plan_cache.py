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
