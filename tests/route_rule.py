"""Which 16-B-aligned shards the library codes on the record kernels instead
of the aligned ones: a mirror of csrc/hbec.cpp rec_route (thresholds read
from csrc/tuning.h), for tests that count a plan's tiled / record stripes."""
import re
from pathlib import Path

_T = (Path(__file__).resolve().parents[1] / "hummingbird_amd" / "csrc" / "tuning.h").read_text()
MIN_S = int(re.search(r"#define HBEC_REC_ROUTE_MIN_S (\d+)", _T).group(1))
MIN_S_BIG = int(re.search(r"#define HBEC_REC_ROUTE_MIN_S_BIG (\d+)", _T).group(1))
POS32_MAX = (1 << 31) - (1 << 16)


def rec_route(k, s, *addrs, rows=3, bitplane=False):
    """rows: the pass's output rows; bitplane: they have a compiled schedule"""
    line = s % 128 == 0 and all(a % 128 == 0 for a in addrs)
    if not 5 <= k <= 12 or s > POS32_MAX:
        return False
    if k > 8:
        return s >= MIN_S_BIG
    r = min(rows, 4)
    return s >= MIN_S and (not line or r >= 4) and (k * r <= 24 or bitplane)


def _plan_bp(k, m):
    from hummingbird_amd import gen_xor
    return gen_xor.USE.get((k, min(m, 4)), (False, False, False))[1] and m <= 4


def stripe_on_records(k, m, base, s):
    """hbec_plan_stripes: not tiled (plan.cpp aligned_stripe, plan_rec_route)"""
    return bool(base % 16 or s % 16) or rec_route(k, s, base, rows=m, bitplane=_plan_bp(k, m))


def object_on_records(k, m, data, parity, s):
    """hbec_plan_objects' obj_fallback count (k <= 8; k > 8 objects are all
    on records but not counted there)"""
    return bool(data % 16 or parity % 16 or s % 16 or s >= 1 << 32) or (
        k <= 8 and rec_route(k, s, data, parity, rows=m, bitplane=_plan_bp(k, m)))
