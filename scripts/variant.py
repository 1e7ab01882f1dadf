#!/usr/bin/env python3
"""Build a tuning variant of libhbec.so into tune_build/NAME/ with extra -D
definitions, recompiling only the units that read them (the others' objects
are copied from the product build).

    python scripts/variant.py NAME DEF[=VAL] ... [--units odd_bp.hip,odd.hip]
"""
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from hummingbird_amd import build as hb  # noqa: E402

args = sys.argv[1:]
units = ["all"]  # every unit: a -D that one unit reads and another does not would build an ODR-inconsistent hybrid
if "--units" in args:
    i = args.index("--units")
    units = args[i + 1].split(",")
    del args[i:i + 2]
name, defs = args[0], args[1:]
hb.build(verbose=False)
od = ROOT / "tune_build" / name / "obj"
od.mkdir(parents=True, exist_ok=True)
for o in hb.OBJ.glob("*.o"):
    shutil.copy2(o, od / o.name)
for u in (hb.SOURCES if units == ["all"] else units):
    (od / (u.rsplit(".", 1)[0] + ".o")).unlink(missing_ok=True)
lib = ROOT / "tune_build" / name / "libhbec.so"
lib.unlink(missing_ok=True)
hb.build(verbose=False, defs=defs, lib=lib, objdir=od)
# what this variant is: its -D definitions and the units rebuilt with them
rebuilt = list(hb.SOURCES) if units == ["all"] else units
(lib.parent / "variant.json").write_text(json.dumps({"defs": defs, "units_rebuilt": [str(u) for u in rebuilt]}, indent=1) + "\n")
print(lib)
