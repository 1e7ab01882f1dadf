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


OBJDUMP = Path("/opt/rocm/lib/llvm/bin/llvm-objdump")


def _sregs(tok: str) -> set:
    import re
    m = re.match(r"s\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _early_reads(lines):
    """Instructions (in code order) that read an SGPR an s_load is still
    filling: after the load, before an s_waitcnt lgkmcnt(0)."""
    pend, bad = set(), []
    for ins in lines:
        op = ins.split()[0]
        args = [a.strip() for a in ins[len(op):].split(",")]
        if op.startswith("s_waitcnt"):
            if "lgkmcnt(0)" in ins:
                pend = set()
            continue
        if op.startswith("s_load_dword"):
            if any(_sregs(a) & pend for a in args[1:]):
                bad.append(ins)
            pend |= _sregs(args[0])
            continue
        if not pend:
            continue
        srcs = args if op.startswith("s_cmp") else args[1:]
        if any(_sregs(a.split()[0]) & pend for a in srcs if a):
            bad.append(ins)
        pend -= _sregs(args[0]) if args else set()
    return bad


def test_record_loads_unread_before_wait():
    """gf_odd_rec issues its record loads by hand (odd_impl.h odd_sload: the
    compiler's own scalar loads sat right before their use) and waits for them
    after the next tile's arithmetic, on the shapes odd_rec_prefetch allows.
    That is only correct if the compiler never copies or spills a record
    register in between (v_writelane of a destination before its wait read
    unfilled registers: a memory fault at 12+4 in round 4).  Every shipped
    instance's code is checked for such a read."""
    if not LIB.exists():
        pytest.skip("libhbec.so not built")
    if not OBJDUMP.exists():
        pytest.skip("llvm-objdump not found")
    checked = 0
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(_code_objects(LIB.read_bytes())):
            if b"gf_odd_rec" not in co:
                continue
            f = Path(td) / f"co{n}.o"
            f.write_bytes(co)
            syms = subprocess.run([str(OBJDUMP), "-t", str(f)], capture_output=True, text=True, check=True).stdout
            names = sorted({ln.split()[-1] for ln in syms.splitlines()
                            if "gf_odd_rec" in ln and ln.split()[-1].startswith("_Z") and ".kd" not in ln})
            text = subprocess.run([str(OBJDUMP), "-d", "--mcpu=gfx950", "--disassemble-symbols=" + ",".join(names),
                                   str(f)], capture_output=True, text=True, check=True).stdout
            cur, body = None, {}
            for ln in text.splitlines():
                if ln.endswith(">:"):
                    cur = ln.split("<", 1)[1][:-2]
                    body[cur] = []
                elif cur and ln.strip():
                    ins = ln.split("//")[0].strip()
                    if ins:
                        body[cur].append(ins)
            for name, lines in body.items():
                checked += 1
                assert not _early_reads(lines), (name, _early_reads(lines)[:4])
    assert checked >= 12 * 4 * 3 // 2, checked
