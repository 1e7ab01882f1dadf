"""The build-time scalar-load check (hummingbird_amd/isa_check.py) on
synthetic listings and on the shipped library (CPU only).

The record kernels issue their next tile's `s_load_dwordx8` by hand and wait
for it after the current tile's arithmetic (csrc/odd_impl.h odd_sload /
odd_swait).  Touching a destination SGPR before `s_waitcnt lgkmcnt(0)`
reads (or races with) a register the load has not filled: round 4's 12+4
memory fault (a `v_writelane` spill of such a register).  The analysis walks
the control-flow graph to a fixed point, so a read reached only through a
loop back-edge or only on one branch is caught.
"""
from __future__ import annotations

import pytest

from hummingbird_amd import build as hb
from hummingbird_amd import isa_check as IC

SYM = "_ZN4hbec10gf_odd_recILi12ELi4ELi0EEEvNS_8PassArgsEPjPKj"


def _listing(lines):
    """objdump-style text: one instruction per 4 bytes, branch targets as
    <SYM+0xOFF>; `lines` are (instruction, target offset or None)."""
    out = [f"0000000000001000 <{SYM}>:"]
    for i, (ins, tgt) in enumerate(lines):
        addr = 0x1000 + 4 * i
        t = f" <{SYM}+0x{tgt * 4:x}>" if tgt is not None else ""
        out.append(f"\t{ins:58s}// {addr:012X}: 00000000{t}")
    return "\n".join(out)


def _bad(lines):
    ins = IC.parse_listing(_listing(lines))[SYM]
    return [f"{x.op} {x.args}" for x in IC.violations(ins)]


def test_wait_before_use_is_clean():
    assert _bad([("s_load_dwordx8 s[8:15], s[2:3], 0x0", None),
                 ("v_mov_b32 v0, v1", None),
                 ("s_waitcnt lgkmcnt(0)", None),
                 ("s_add_u32 s4, s8, s9", None),
                 ("s_endpgm", None)]) == []


def test_read_before_wait_is_flagged():
    assert _bad([("s_load_dwordx8 s[8:15], s[2:3], 0x0", None),
                 ("v_writelane_b32 v7, s9, 3", None),  # the round-4 spill
                 ("s_waitcnt lgkmcnt(0)", None),
                 ("s_endpgm", None)]) == ["v_writelane_b32 v7, s9, 3"]


def test_write_before_wait_is_flagged():
    assert _bad([("s_load_dwordx8 s[8:15], s[2:3], 0x0", None),
                 ("s_mov_b32 s12, 0", None),
                 ("s_waitcnt lgkmcnt(0)", None),
                 ("s_endpgm", None)]) == ["s_mov_b32 s12, 0"]


def test_nonzero_lgkmcnt_proves_nothing():
    # scalar loads return out of order: lgkmcnt(1) does not cover the first load
    assert _bad([("s_load_dwordx8 s[8:15], s[2:3], 0x0", None),
                 ("s_load_dwordx8 s[16:23], s[2:3], 0x20", None),
                 ("s_waitcnt lgkmcnt(1)", None),
                 ("s_add_u32 s4, s8, 1", None),
                 ("s_waitcnt lgkmcnt(0)", None),
                 ("s_endpgm", None)]) == ["s_add_u32 s4, s8, 1"]


def test_loop_carried_early_read_is_flagged():
    """The load is issued at the bottom of the loop and waited for only at the
    bottom; the read at the top of the NEXT iteration comes first.  A scan in
    code order sees the read before the load and misses it."""
    lines = [("s_mov_b32 s0, 0", None),                       # 0
             ("s_add_u32 s5, s10, s11", None),                # 1: loop head, reads s[8:15]
             ("v_add_u32 v0, v0, v1", None),                  # 2
             ("s_load_dwordx8 s[8:15], s[2:3], 0x0", None),   # 3: next tile's record
             ("s_add_u32 s0, s0, 1", None),                   # 4
             ("s_cmp_lt_u32 s0, 8", None),                    # 5
             ("s_cbranch_scc1 65530", 1),                     # 6: back-edge to 1
             ("s_waitcnt lgkmcnt(0)", None),                  # 7
             ("s_endpgm", None)]
    # (re-issuing the load into registers it is still filling is flagged too)
    assert _bad(lines) == ["s_add_u32 s5, s10, s11", "s_load_dwordx8 s[8:15], s[2:3], 0x0"]


def test_read_on_one_branch_only_is_flagged():
    lines = [("s_load_dwordx8 s[8:15], s[2:3], 0x0", None),   # 0
             ("s_cmp_eq_u32 s4, 0", None),                    # 1
             ("s_cbranch_scc1 2", 5),                         # 2: -> 5
             ("s_waitcnt lgkmcnt(0)", None),                  # 3
             ("s_branch 1", 6),                               # 4: -> 6
             ("v_readfirstlane_b32 s13, v2", None),           # 5: write of a pending register
             ("s_waitcnt lgkmcnt(0)", None),                  # 6
             ("s_endpgm", None)]
    assert _bad(lines) == ["v_readfirstlane_b32 s13, v2"]


def test_load_address_pending_is_flagged():
    assert _bad([("s_load_dwordx2 s[8:9], s[2:3], 0x0", None),
                 ("s_load_dwordx8 s[16:23], s[8:9], 0x0", None),
                 ("s_waitcnt lgkmcnt(0)", None),
                 ("s_endpgm", None)]) == ["s_load_dwordx8 s[16:23], s[8:9], 0x0"]


def test_register_names_are_not_mnemonics():
    assert IC.sregs("s[8:11], s4, vcc, exec, s_nop, v[0:1], ttmp2") == {8, 9, 10, 11, 4}


def test_shipped_library_has_no_early_reads():
    """Every record kernel of the product library (the same check build()
    runs before it accepts a library)."""
    if not hb.LIB.exists():
        pytest.skip("libhbec.so not built")
    n, bad = IC.check_library(hb.LIB)
    assert n >= 100, n
    assert not bad, {k: v[:4] for k, v in bad.items()}
