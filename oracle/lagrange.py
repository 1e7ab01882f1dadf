"""Second, structurally different derivation of klauspost's default code —
TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

oracle.py and the product's gf256.h both build the systematic matrix the way
klauspost's matrix.go does: Vandermonde(k+m, k) times the Gauss-Jordan
inverse of its top k x k block.  A misreading shared by those two
restatements would not be caught by comparing them.  This module never
inverts a matrix.  It uses what that construction MEANS:

  V[r][c] = galExp(r, c) = r^c, with the row index r read as a GF(2^8)
  element.  The top block is V_top[a][c] = a^c for a < k, so
  M = V x inv(V_top) is the matrix whose row r evaluates at the point r
  the unique polynomial p of degree < k with p(a) = data_a (a < k).
  Row r of M is therefore the Lagrange basis over the points 0..k-1
  evaluated at r:

      M[r][a] = prod_{b != a, b < k} (r - b) / (a - b)      (in GF(2^8), - = XOR)

Reconstruct (klauspost reconstruct: the first k present shards s_0..s_{k-1}
are the survivors) recovers p from its values at the survivor points, so
the decode row of any shard e (data or parity) over the survivors is the
Lagrange basis over the survivor points evaluated at e:

      D[e][t] = prod_{u != t} (e - s_u) / (s_t - s_u)

This equals the product's fused rows (inv(sub) row e for a data shard,
M[e] x inv(sub) for a parity shard), since both are the unique linear map
from the survivors to shard e.  Only field multiply / divide are shared with
oracle.py (GF(2^8), poly 0x11D, the KAT-pinned galMul).
"""
from __future__ import annotations

from .oracle import gal_divide, gal_mul


def lagrange_row(points, x):
    """[L_t(x) for t] over distinct GF(2^8) points."""
    row = []
    for t, pt in enumerate(points):
        num, den = 1, 1
        for u, pu in enumerate(points):
            if u != t:
                num = gal_mul(num, x ^ pu)
                den = gal_mul(den, pt ^ pu)
        row.append(gal_divide(num, den))
    return row


def parity_rows(k: int, m: int):
    """Rows k..k+m-1 of klauspost's default systematic matrix, no inversion."""
    pts = list(range(k))
    return [lagrange_row(pts, r) for r in range(k, k + m)]


def coding_matrix(k: int, m: int):
    return [lagrange_row(list(range(k)), r) for r in range(k + m)]


def decode_rows(k: int, m: int, present, data_only: bool = False):
    """(survivors, outputs, rows) for a present mask, as Encoder.Reconstruct /
    ReconstructData apply them: survivors = first k present shards, outputs
    = missing shards (data only when data_only)."""
    surv = [i for i in range(k + m) if present[i]][:k]
    if len(surv) < k:
        raise ValueError("too few shards")
    outs = [i for i in range(k + m) if not present[i] and (i < k or not data_only)]
    return surv, outs, [lagrange_row(surv, e) for e in outs]
