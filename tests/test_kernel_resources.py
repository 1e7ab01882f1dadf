"""Register / LDS contract of the shipped gfx950 kernels (CPU only).

Reads the AMDGPU metadata of every gfx950 code object embedded in
hummingbird_amd/libhbec.so (the clang offload bundles of its HIP TUs) with
llvm-readelf and pins the resource facts the round-3 tuning depends on
("Plan record ids as scalars", "Pinned outputs"):

- gf_odd_plan keeps its record ids in SGPRs: no kernel of that family uses
  LDS (the compiler once promoted the URec copies to LDS, 59 -> 66 % when
  fixed);
- the pinned instances fit two waves per SIMD: 10+4 / 9+4 apply and the plan
  kernel at <= 256 VGPRs (a few dwords of spill allowed), 8+3 / 6+3 Verify
  likewise without spill;
- the headline kernel gf_apply_vec_pipe2<4,2> has no scratch.
"""
from __future__ import annotations

import shutil
import struct
import subprocess
import tempfile
from pathlib import Path

import pytest
import yaml

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "hummingbird_amd" / "libhbec.so"
READELF = Path("/opt/rocm/lib/llvm/bin/llvm-readelf")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(blob: bytes):
    i = 0
    while True:
        i = blob.find(MAGIC, i)
        if i < 0:
            return
        n = struct.unpack_from("<Q", blob, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                yield blob[i + off:i + off + size]
        i += len(MAGIC)


@pytest.fixture(scope="module")
def kernels():
    if not LIB.exists():
        pytest.skip("libhbec.so not built")
    readelf = str(READELF) if READELF.exists() else shutil.which("llvm-readelf")
    if not readelf:
        pytest.skip("llvm-readelf not found")
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(_code_objects(LIB.read_bytes())):
            f = Path(td) / f"co{n}.o"
            f.write_bytes(co)
            text = subprocess.run([readelf, "--notes", str(f)], capture_output=True, text=True,
                                  check=True).stdout
            body = text.split("---", 1)[1].split("\n...", 1)[0]
            meta = yaml.safe_load(body)
            for k in meta["amdhsa.kernels"]:
                out[k[".name"]] = k
    assert out, "no gfx950 code objects found in libhbec.so"
    return out


def _one(kernels, mangled):
    assert mangled in kernels, f"{mangled} not in libhbec.so"
    return kernels[mangled]


def test_odd_plan_kernels_use_no_lds(kernels):
    plans = {n: k for n, k in kernels.items() if "gf_odd_planILi" in n}
    assert len(plans) >= 12 * 4
    bad = {n: k[".group_segment_fixed_size"] for n, k in plans.items() if k[".group_segment_fixed_size"] != 0}
    assert not bad, bad


@pytest.mark.parametrize("name", [
    "_ZN4hbec6gf_oddILi10ELi4ELi0EEEvNS_8PassArgsEPj",
    "_ZN4hbec6gf_oddILi9ELi4ELi0EEEvNS_8PassArgsEPj",
    "_ZN4hbec11gf_odd_planILi10ELi4ELi0ELb0ELb0EEEvNS_9UPlanArgsEPKNS_4URecE",
])
def test_pinned_apply_fits_two_waves_per_simd(kernels, name):
    k = _one(kernels, name)
    assert k[".vgpr_count"] <= 256, k[".vgpr_count"]
    assert k[".private_segment_fixed_size"] <= 64, k[".private_segment_fixed_size"]


@pytest.mark.parametrize("name", [
    "_ZN4hbec6gf_oddILi8ELi3ELi2EEEvNS_8PassArgsEPj",
    "_ZN4hbec6gf_oddILi6ELi3ELi2EEEvNS_8PassArgsEPj",
])
def test_pinned_verify_fits_two_waves_per_simd(kernels, name):
    k = _one(kernels, name)
    assert k[".vgpr_count"] <= 256, k[".vgpr_count"]
    assert k[".private_segment_fixed_size"] == 0


def test_headline_kernel_has_no_scratch(kernels):
    k = _one(kernels, "_ZN4hbec18gf_apply_vec_pipe2ILi4ELi2EEEvNS_8PassArgsE")
    assert k[".private_segment_fixed_size"] == 0
    assert k[".group_segment_fixed_size"] == 0


def test_record_loads_unread_before_wait():
    """gf_odd_rec issues its record loads by hand and waits for them after the
    next tile's arithmetic; the control-flow-aware check of
    hummingbird_amd/isa_check.py (run by build() on every library it links)
    finds no instruction touching a pending load destination in any shipped
    instance (tests/test_isa_check.py pins the analysis itself)."""
    from hummingbird_amd import isa_check

    if not LIB.exists():
        pytest.skip("libhbec.so not built")
    checked, bad = isa_check.check_library(LIB)
    assert not bad, {k: v[:4] for k, v in bad.items()}
    assert checked >= 12 * 4 * 3 // 2, checked
