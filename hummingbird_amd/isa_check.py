"""Build-time check of the hand-issued scalar loads in the record kernels.

gf_odd_rec (csrc/odd_impl.h) issues the next tile's record loads by inline
asm (`s_load_dwordx8`, odd_sload) and waits for them (`s_waitcnt
lgkmcnt(0)`, odd_swait) only after the current tile's arithmetic.  The asm
declares the destination registers as written when the load ISSUES, so the
code is correct only if the compiler neither reads nor writes those SGPRs
before the wait.  In round 4 it spilled them into VGPR lanes (`v_writelane`)
right after the load, before the data had landed: a memory fault at 12+4.

This module proves the property on the shipped machine code.  It
disassembles every selected kernel of libhbec.so's gfx950 code objects,
builds the control-flow graph from the branch targets, and runs a forward
may-analysis to a fixed point: the set of SGPRs an `s_load*` is still
filling, propagated along every edge (loop back-edges included; a block's
entry set is the union of its predecessors' exit sets).  `s_waitcnt` with
`lgkmcnt(0)` clears the set (scalar loads return out of order, so a non-zero
count proves nothing).  Any other instruction naming a pending SGPR as an
operand, read or write (a write would race with the landing load), is a
violation, and so is an `s_load` whose address registers are pending.

`hummingbird_amd.build.build()` runs it on every library it links and
refuses one with a violation; tests/test_isa_check.py pins the analysis on
synthetic listings (a loop-carried early read, a write before the wait, a
read on one branch only).
"""
from __future__ import annotations

import re
import shutil
import struct
import subprocess
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
OBJDUMP = Path("/opt/rocm/lib/llvm/bin/llvm-objdump")

_SREG = re.compile(r"(?<![\w\]])s\[(\d+):(\d+)\]|(?<![\w\]])s(\d+)\b")
_TARGET = re.compile(r"<([^<>+]+)\+0x([0-9a-fA-F]+)>")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]{8,16}):")


def code_objects(blob: bytes, arch: str = "gfx950"):
    """The `arch` code objects of the clang offload bundles inside a host
    shared library (one per HIP translation unit)."""
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
            if arch in triple and size:
                yield blob[i + off:i + off + size]
        i += len(MAGIC)


def sregs(text: str) -> set[int]:
    out: set[int] = set()
    for a, b, c in _SREG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


@dataclass
class Ins:
    addr: int
    op: str
    args: str  # operand text (no comment)
    target: int | None = None  # branch target address


@dataclass
class Block:
    ins: list = field(default_factory=list)
    succ: list = field(default_factory=list)


def parse_listing(text: str) -> dict[str, list[Ins]]:
    """llvm-objdump -d output -> {symbol: instructions}.  Each line carries its
    address in the trailing comment; branch targets print as <sym+0xOFF>."""
    out: dict[str, list[Ins]] = {}
    cur, base = None, 0
    for ln in text.splitlines():
        m = re.match(r"^([0-9a-fA-F]+) <(.+)>:$", ln.strip())
        if m:
            cur, base = m.group(2), int(m.group(1), 16)
            out[cur] = []
            continue
        if cur is None or not ln.strip():
            continue
        code, _, cmt = ln.partition("//")
        code = code.strip()
        if not code:
            continue
        am = _ADDR.search("//" + cmt)
        addr = int(am.group(1), 16) if am else (out[cur][-1].addr + 4 if out[cur] else base)
        op, _, args = code.partition(" ")
        t = None
        tm = _TARGET.search(cmt)
        if tm and (op.startswith("s_branch") or op.startswith("s_cbranch")):
            t = base + int(tm.group(2), 16) if tm.group(1) == cur else None
        out[cur].append(Ins(addr, op, args.strip(), t))
    return out


_TERM = ("s_endpgm", "s_setpc", "s_trap", "s_rfe")


def cfg(ins: list[Ins]) -> list[Block]:
    if not ins:
        return []
    leaders = {ins[0].addr}
    for i, x in enumerate(ins):
        if x.op.startswith(("s_branch", "s_cbranch")) or x.op.startswith(_TERM):
            if x.target is not None:
                leaders.add(x.target)
            if i + 1 < len(ins):
                leaders.add(ins[i + 1].addr)
    blocks, start = [], {}
    for x in ins:
        if x.addr in leaders:
            start[x.addr] = len(blocks)
            blocks.append(Block())
        blocks[-1].ins.append(x)
    for bi, b in enumerate(blocks):
        last = b.ins[-1]
        fall = bi + 1 if bi + 1 < len(blocks) else None
        if last.op.startswith(_TERM):
            continue
        if last.op.startswith("s_branch"):
            if last.target in start:
                b.succ.append(start[last.target])
            continue
        if last.op.startswith("s_cbranch") and last.target in start:
            b.succ.append(start[last.target])
        if fall is not None:
            b.succ.append(fall)
    return blocks


def _step(x: Ins, pend: set[int], bad: list | None) -> set[int]:
    if x.op.startswith("s_waitcnt"):
        return set() if "lgkmcnt(0)" in x.args else pend
    if x.op.startswith(("s_load_", "s_buffer_load_")):
        parts = x.args.split(",", 1)
        dst, src = sregs(parts[0]), sregs(parts[1] if len(parts) > 1 else "")
        if bad is not None and (src & pend or dst & pend):
            bad.append(x)
        return pend | dst
    if pend and bad is not None and sregs(x.args) & pend:
        bad.append(x)
    return pend


def violations(ins: list[Ins]) -> list[Ins]:
    """Instructions that touch an SGPR a scalar load may still be filling on
    some path (fixed point over the CFG, back-edges included)."""
    blocks = cfg(ins)
    if not blocks:
        return []
    preds: list[list[int]] = [[] for _ in blocks]
    for i, b in enumerate(blocks):
        for s in b.succ:
            preds[s].append(i)
    out: list[set[int]] = [set() for _ in blocks]
    work = list(range(len(blocks)))
    while work:
        i = work.pop(0)
        p: set[int] = set()
        for q in preds[i]:
            p |= out[q]
        for x in blocks[i].ins:
            p = _step(x, p, None)
        if p != out[i]:
            out[i] = p
            work += [s for s in blocks[i].succ if s not in work]
    bad: list[Ins] = []
    for i, b in enumerate(blocks):
        p: set[int] = set()
        for q in preds[i]:
            p |= out[q]
        for x in b.ins:
            p = _step(x, p, bad)
    return bad


def _objdump() -> str:
    if OBJDUMP.exists():
        return str(OBJDUMP)
    w = shutil.which("llvm-objdump")
    if not w:
        raise FileNotFoundError("llvm-objdump not found (needed to check the record kernels)")
    return w


def check_library(lib: Path, pattern: str = "gf_odd_rec", arch: str = "gfx950") -> tuple[int, dict]:
    """(kernels checked, {kernel: [violating instructions]}) for every kernel
    whose symbol contains `pattern` in the library's `arch` code objects."""
    objdump = _objdump()
    checked, found = 0, {}
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(code_objects(Path(lib).read_bytes(), arch)):
            if pattern.encode() not in co:
                continue
            f = Path(td) / f"co{n}.o"
            f.write_bytes(co)
            syms = subprocess.run([objdump, "-t", str(f)], capture_output=True, text=True, check=True).stdout
            names = sorted({ln.split()[-1] for ln in syms.splitlines()
                            if pattern in ln and ln.split()[-1].startswith("_Z") and ".kd" not in ln})
            if not names:
                continue
            text = subprocess.run([objdump, "-d", f"--mcpu={arch}", "--disassemble-symbols=" + ",".join(names),
                                   str(f)], capture_output=True, text=True, check=True).stdout
            for name, ins in parse_listing(text).items():
                checked += 1
                v = violations(ins)
                if v:
                    found[name] = [f"{x.addr:#x}: {x.op} {x.args}" for x in v]
    return checked, found


if __name__ == "__main__":
    import sys

    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parent / "libhbec.so"
    n, bad = check_library(lib)
    for k, v in bad.items():
        print(k, v[:4])
    print(f"{n} kernels checked, {len(bad)} with early scalar-load reads")
    sys.exit(1 if bad or n == 0 else 0)
