#!/usr/bin/env python3
"""Build the MD5 depth variants md5_sweep.sh times (CPU side)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from hummingbird_amd import build as Bd  # noqa: E402

VARIANTS = {"d1": ["HBEC_MD5_DEPTH=1"], "d2": ["HBEC_MD5_DEPTH=2"], "d4": ["HBEC_MD5_DEPTH=4"],
            "d2rot": ["HBEC_MD5_DEPTH=2", "HBEC_MD5_PINGPONG=0"], "d4rot": ["HBEC_MD5_DEPTH=4", "HBEC_MD5_PINGPONG=0"]}
for name, defs in VARIANTS.items():
    out = ROOT / "tune_build" / f"md5_{name}"
    Bd.build(defs=defs, lib=out / "libhbec.so", objdir=out / "obj", verbose=False)
    print("built", out)
