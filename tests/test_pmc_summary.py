"""scripts/pmc_summary.py splits the PMC dispatches at bench.py's leg marker
launches (a fill_splitmix of PMC_MARK_BLOCKS + i blocks starts leg i), so two
legs launching the same kernel get their own bytes (CPU only, synthetic
rocprofv3 CSVs)."""
import csv
import importlib.util
from pathlib import Path

import bench

ROOT = Path(__file__).resolve().parents[1]
spec = importlib.util.spec_from_file_location("pmc_summary", ROOT / "scripts" / "pmc_summary.py")
PS = importlib.util.module_from_spec(spec)
spec.loader.exec_module(PS)

COLS = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
        "End_Timestamp"]


def _write(d: Path, counter, rows):
    d.mkdir(parents=True, exist_ok=True)
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLS)
        w.writeheader()
        for i, (kernel, grid, value) in enumerate(rows):
            w.writerow({"Dispatch_Id": i + 1, "Grid_Size": grid, "Kernel_Name": f"void hbec::{kernel}(args)",
                        "Counter_Name": counter, "Counter_Value": value, "Start_Timestamp": 10 * i,
                        "End_Timestamp": 10 * i + 5})


def _mark(leg):
    return ("fill_splitmix", (bench.PMC_MARK_BLOCKS + bench.PMC_LEGS.index(leg)) * 256, 1.0)


def test_legs_get_their_own_launches(tmp_path):
    plan = "gf_odd_rec<8, 3, 0, 2, true>"
    grid = 256 * 256
    rows = [("gf_apply_vec_pipe2<4, 2>", 4096 * 256, 100.0),
            _mark("random_objects"), (plan, grid, 3000.0), (plan, grid, 3000.0), (plan, 64, 1.0),
            _mark("mid_objects"), (plan, grid, 1000.0), (plan, grid, 1000.0), (plan, grid, 1000.0),
            ("fill_splitmix", 16384 * 256, 7.0)]
    _write(tmp_path / "f", "FETCH_SIZE", rows)
    _write(tmp_path / "w", "WRITE_SIZE", [(k, g, v / 2) for k, g, v in rows])
    fr = PS.dispatches(tmp_path / "f", "FETCH_SIZE")
    wr = PS.dispatches(tmp_path / "w", "WRITE_SIZE")
    legs_f = PS.by_leg(fr, bench.PMC_LEGS, bench.PMC_MARK_BLOCKS)
    legs_w = PS.by_leg(wr, bench.PMC_LEGS, bench.PMC_MARK_BLOCKS)
    assert set(legs_f) == {"random_objects", "mid_objects"}
    rnd = PS.summarize(PS.per_kernel(legs_f["random_objects"]), PS.per_kernel(legs_w["random_objects"]))
    mid = PS.summarize(PS.per_kernel(legs_f["mid_objects"]), PS.per_kernel(legs_w["mid_objects"]))
    # read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB; the one-object launch (grid 64) is not a bench launch
    assert rnd[plan]["hbm_bytes_per_launch"] == (2 * 3000 + 1500) * 1024
    assert rnd[plan]["launches_fetch_pass"] == 2
    assert mid[plan]["hbm_bytes_per_launch"] == (2 * 1000 + 500) * 1024
    # the whole-run view mixes both legs (what bench.py no longer uses for them)
    whole = PS.summarize(PS.per_kernel(fr), PS.per_kernel(wr))
    assert whole[plan]["launches_fetch_pass"] == 5
    # the headline (before any marker) is in no leg; a fill after a leg stays in it, the markers in none
    assert "gf_apply_vec_pipe2<4, 2>" not in rnd and "gf_apply_vec_pipe2<4, 2>" in whole
    assert "fill_splitmix" not in rnd and mid["fill_splitmix"]["launches_fetch_pass"] == 1
