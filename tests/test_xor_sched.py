"""The compiled XOR schedules of the bit-plane encode kernels (CPU only).

hummingbird_amd/gen_xor.py writes csrc/xor_sched.h: for each compiled (k, m)
the parity rows of reedsolomon.New(k, m) (objectserver/ecutils.go:27,59) as a
fixed XOR network over bit-planes.  Checked here against the oracle:
- the generator's matrix restatement equals oracle.build_matrix;
- every network, evaluated on random bit-planes, equals the oracle's GF(2^8)
  multiply of the same bytes (the generator also self-checks before writing);
- the committed header is exactly what the generator writes (no hand edits,
  no stale schedule), and its coefficient table is the one the networks code.
"""
from __future__ import annotations

import re

import numpy as np
import pytest

from hummingbird_amd import gen_xor as G
from oracle import oracle as O


@pytest.mark.parametrize("k,m", G.SHAPES)
def test_generator_matrix_is_the_oracle_matrix(k, m):
    assert G.encode_matrix(k, m) == [list(r) for r in O.build_matrix(k, k + m)]


def _planes(data):
    """data: k x 32 bytes -> 8 k planes (plane 8 j + b: bit q = bit b of byte q)"""
    return [sum(((int(data[j][q]) >> b) & 1) << q for q in range(32)) for j in range(len(data)) for b in range(8)]


@pytest.mark.parametrize("k,m", G.SHAPES)
def test_schedule_equals_field_multiply(k, m):
    mat = O.build_matrix(k, k + m)
    rng = np.random.default_rng(k * 16 + m)
    for r0 in range(0, m, 4):
        coef = [list(mat[k + r]) for r in range(r0, min(m, r0 + 4))]
        temps, rows = G.schedule(G.bit_rows(coef), 8 * k, 10_000)
        # the network never reads an operand before it is defined
        for t, ops in enumerate(temps):
            assert all(o < 8 * k + t for o in ops)
        for _ in range(4):
            data = rng.integers(0, 256, (k, 32), dtype=np.uint8)
            got = G.simulate(temps, rows, 8 * k, _planes(data))
            want = O.gf_apply(coef, [d for d in data])
            for r in range(len(coef)):
                wb = want[r]
                for i in range(8):
                    assert got[8 * r + i] == sum(((int(wb[q]) >> i) & 1) << q for q in range(32)), (r, i)


def test_committed_header_is_generated():
    assert G.OUT.read_text() == G.generate(), "csrc/xor_sched.h differs: run python -m hummingbird_amd.gen_xor"


def test_header_table_matches_networks():
    text = G.OUT.read_text()
    nets = re.findall(r"struct XorNet<(\d+)> \{\n    static constexpr int K = (\d+), R = (\d+);", text)
    table = re.findall(r"\{(\d+), (\d+), (\d+), (\d+), (?:true|false), (?:true|false), (?:true|false), \{(.*?)\}\},  // XorNet<(\d+)>",
                       text)
    assert len(nets) == len(table) == sum((m + 3) // 4 for _, m in G.SHAPES)
    shapes = {int(i): (int(k), int(r)) for i, k, r in nets}
    for k, m, r0, R, coefs, i in table:
        k, m, r0, R, i = map(int, (k, m, r0, R, i))
        assert shapes[i] == (k, R)
        rows = [list(map(int, c.strip("{} ").split(","))) for c in re.findall(r"\{[^{}]*\}", "{" + coefs + "}")]
        mat = O.build_matrix(k, k + m)
        for r in range(R):
            assert rows[r][:k] == list(mat[k + r0 + r])
