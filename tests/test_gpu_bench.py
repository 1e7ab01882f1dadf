"""bench.py end to end on one GPU at a reduced size: the JSON line the driver
parses carries the metric, a roofline with the dominant kernel and fresh (or
explicitly stale) traffic, and every BASELINE-config leg with its parity flag."""
import json

import pytest
import torch

import bench

pytestmark = pytest.mark.gpu


def test_bench_line_small(capsys):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    rc = bench.main(["--steps", "3", "--warmup", "1", "--objects", "128", "--config5-objects", "512",
                     "--no-cpu-baseline", "--no-host-path", "--settle-ms", "5"])
    out = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert rc == 0 and len(out) == 1
    d = json.loads(out[0])
    assert d["metric"] == bench.METRIC and d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["parity_ok"] and d["value"] > 0 and d["settle_steps"] >= 1
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == bench.HBM_PEAK_GBS and 0 < r["frac"] < 1
    assert r["kernel"] == bench.KERNEL_NAME
    assert (r["traffic"] is None) == (r["traffic_note"] is not None)
    assert d["config5"]["parity_ok"] and d["config5"]["objects"] == 512
    assert d["config4"]["parity_ok"] and 0 < d["config4"]["frac"] < 1
    assert all(sh["parity_ok"] for sh in d["small_objects"]["shapes"])
    assert d["odd_objects"]["parity_ok"] and d["odd_objects"]["shard_bytes"] % 16 != 0
    assert all(0 < d["odd_objects"][op]["frac"] < 1 for op in ("encode", "reconstruct", "verify"))
