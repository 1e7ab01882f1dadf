#!/usr/bin/env python3
"""Generate hummingbird_amd/csrc/xor_sched.h: compile-time XOR schedules for
the fixed encode matrices (bit-plane field multiply, odd_impl.h).

    python -m hummingbird_amd.gen_xor [--check]

Why.  Multiplying a byte by a constant c in GF(2^8) is a linear map over
GF(2): an 8 x 8 bit matrix B_c with B_c[i][b] = bit i of c * 2^b.  The parity
rows of reedsolomon.New(k, m) (objectserver/ecutils.go:27,59; klauspost's
default Vandermonde-derived matrix) are fixed per (k, m), so the whole encode
of one 32-byte bit-plane group is a fixed (8R x 8K) bit matrix: every output
bit-plane is the XOR of a fixed set of input bit-planes.  The kernel
transposes each input's 32 bytes (two 16-B columns per lane) into 8 planes,
runs the straight-line XOR network generated here, and transposes the 8R
output planes back.  The bytes are identical to the table multiply's.

The network is the matrix's rows after greedy common-subexpression
elimination (Paar's algorithm, extended to 3-input terms because gfx950's
v_bitop3_b32 XORs three operands in one instruction): at each step the pair
or triple of terms whose shared temporary saves the most v_bitop3 / v_xor
instructions over all rows becomes a temporary.  Each row is then folded
with 3-input XORs.

The field and matrix are restated here (the same construction as
csrc/gf256.h build_matrix); tests/test_xor_sched.py checks them and every
schedule against the oracle, and that this file regenerates the committed
header byte for byte.
"""
from __future__ import annotations

import argparse
import itertools
import sys
from pathlib import Path

OUT = Path(__file__).resolve().parent / "csrc" / "xor_sched.h"

# (k, m) encode shapes that get a compiled schedule.  Output groups of <= 4
# rows (kMaxR); k <= kOddMaxK (12).  Chosen where the table multiply fills
# the issue slots (K * R >= 18 and the BASELINE / hec shapes).
SHAPES = [(6, 3), (7, 3), (8, 3), (8, 4), (9, 3), (10, 4), (12, 4), (6, 2), (8, 2), (4, 2),
          (5, 3), (6, 4), (10, 2), (10, 3), (12, 2), (12, 3)]
# Where the bit-plane kernel is the one launched (interleaved A/Bs against the
# v_perm table kernels, profiles/r05_ab_bitplane.jsonl, r05_ab_plans_verify.jsonl):
# strided batches / plans / Verify (the parity rows are the encode matrix).  The others keep the table kernels there (their schedule is still
# compiled, so a tuning build can A/B it).
USE = {  # (k, m): (strided, plan, verify)
    (6, 3): (True, True, True), (7, 3): (False, False, True), (8, 3): (False, True, True),
    (8, 4): (True, True, True), (9, 3): (True, True, True), (10, 4): (True, True, True),
    (12, 4): (True, True, True), (6, 2): (False, True, True), (8, 2): (False, True, True),
    (4, 2): (False, False, False),
    (5, 3): (True, True, True), (6, 4): (True, True, True), (10, 2): (True, True, True),
    (10, 3): (True, True, True), (12, 2): (False, True, True), (12, 3): (True, True, True),
}


# ---- GF(2^8), poly 0x11D, generator 2 (klauspost galois.go) ----
def _tables():
    exp, log = [0] * 510, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = exp[i + 255] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    return exp, log


EXP, LOG = _tables()


def gmul(a: int, b: int) -> int:
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def gpow(a: int, n: int) -> int:
    if n == 0:
        return 1
    if a == 0:
        return 0
    return EXP[(LOG[a] * n) % 255]


def ginv_mat(a):
    n = len(a)
    w = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(a)]
    for r in range(n):
        if w[r][r] == 0:
            for b in range(r + 1, n):
                if w[b][r]:
                    w[r], w[b] = w[b], w[r]
                    break
        if w[r][r] == 0:
            raise ValueError("singular")
        s = EXP[(255 - LOG[w[r][r]]) % 255]
        w[r] = [gmul(s, v) for v in w[r]]
        for b in range(n):
            if b != r and w[b][r]:
                f = w[b][r]
                w[b] = [u ^ gmul(f, v) for u, v in zip(w[b], w[r])]
    return [row[n:] for row in w]


def encode_matrix(k: int, m: int):
    """(k+m) x k systematic matrix: Vandermonde x inv(top k x k)."""
    vm = [[gpow(r, c) for c in range(k)] for r in range(k + m)]
    inv = ginv_mat(vm[:k])
    out = []
    for r in range(k + m):
        row = []
        for c in range(k):
            v = 0
            for i in range(k):
                v ^= gmul(vm[r][i], inv[i][c])
            row.append(v)
        out.append(row)
    return out


def bit_rows(coef):
    """coef: R x K.  Row (r, i) = set of input planes 8 j + b with bit i of
    coef[r][j] * 2^b."""
    rows = []
    for cr in coef:
        for i in range(8):
            rows.append({8 * j + b for j, c in enumerate(cr) for b in range(8) if (gmul(c, 1 << b) >> i) & 1})
    return rows


def _cost(n: int) -> int:
    """instructions to XOR n terms with 2/3-input XORs"""
    return 0 if n <= 1 else (n - 1 + 1) // 2


def schedule(rows, n_in: int, max_temps: int):
    """Greedy CSE.  Returns (temps, rows): temps[t] = tuple of 2 or 3 operand
    ids (inputs 0..n_in-1, temps n_in + t), rows = final operand lists."""
    rows = [set(r) for r in rows]
    temps = []
    while len(temps) < max_temps:
        cnt2, cnt3 = {}, {}
        for r in rows:
            s = sorted(r)
            for c in itertools.combinations(s, 2):
                cnt2[c] = cnt2.get(c, 0) + 1
        best, gain = None, 0
        # gain of a temp T (|T| terms) = sum over rows containing T of
        # cost(n) - cost(n - |T| + 1), minus the temp's own instruction
        for c, n in cnt2.items():
            if n < 2:
                continue
            g = -1
            for r in rows:
                if c[0] in r and c[1] in r:
                    g += _cost(len(r)) - _cost(len(r) - 1)
            if g > gain or (g == gain and best is not None and (len(c), c) < (len(best), best)):
                best, gain = c, g
        # triples built from the frequent pairs only (bounded search)
        top = sorted((c for c, n in cnt2.items() if n >= 2), key=lambda c: (-cnt2[c], c))[:64]
        for a, b in top:
            cands = {}
            for r in rows:
                if a in r and b in r:
                    for x in r:
                        if x != a and x != b:
                            cands[x] = cands.get(x, 0) + 1
            for x, n in cands.items():
                if n < 2:
                    continue
                t = tuple(sorted((a, b, x)))
                if t in cnt3:
                    continue
                g = -1
                for r in rows:
                    if t[0] in r and t[1] in r and t[2] in r:
                        g += _cost(len(r)) - _cost(len(r) - 2)
                cnt3[t] = g
                if g > gain or (g == gain and best is not None and (len(t), t) < (len(best), best)):
                    best, gain = t, g
        if best is None or gain <= 0:
            break
        tid = n_in + len(temps)
        temps.append(best)
        for r in rows:
            if all(x in r for x in best):
                for x in best:
                    r.discard(x)
                r.add(tid)
    return temps, [sorted(r) for r in rows]


def simulate(temps, rows, n_in, planes):
    vals = list(planes) + [0] * len(temps)
    for t, ops in enumerate(temps):
        v = 0
        for o in ops:
            v ^= vals[o]
        vals[n_in + t] = v
    out = []
    for r in rows:
        v = 0
        for o in r:
            v ^= vals[o]
        out.append(v)
    return out


def emit_net(sid, k, m, r0, coef, temps, rows):
    n_in, R = 8 * k, len(coef)
    name = lambda o: f"p[{o}]" if o < n_in else f"t{o - n_in}"  # noqa: E731
    lines = [f"// {k}+{m}, parity rows {r0}..{r0 + R - 1}: {len(temps)} temporaries, "
             f"{len(temps) + sum(_cost(len(r)) for r in rows)} XOR instructions",
             "template <>",
             f"struct XorNet<{sid}> {{",
             f"    static constexpr int K = {k}, R = {R};",
             f"    __device__ static __forceinline__ void run(const uint32_t (&p)[{n_in}], uint32_t (&o)[{8 * R}]) {{"]
    for t, ops in enumerate(temps):
        args = ", ".join(name(x) for x in ops)
        lines.append(f"        const uint32_t t{t} = x{len(ops)}({args});")
    for i, r in enumerate(rows):
        if not r:
            lines.append(f"        o[{i}] = 0u;")
            continue
        # balanced 3-ary tree: the same instruction count as a chain, depth
        # log3(n) instead of n / 2 (a lone wave stalls on dependent VALU)
        terms = [name(x) for x in r]
        while len(terms) > 2:
            nxt = []
            while len(terms) >= 3:
                nxt.append(f"x3({terms[0]}, {terms[1]}, {terms[2]})")
                terms = terms[3:]
            terms = nxt + terms  # 0-2 leftovers join the next level
        if len(terms) == 2:
            terms = [f"x2({terms[0]}, {terms[1]})"]
        lines.append(f"        o[{i}] = {terms[0]};")
    lines += ["    }", "};", ""]
    return lines


def generate(max_temps: int = 10_000) -> str:
    hdr = ['// xor_sched.h — GENERATED by hummingbird_amd/gen_xor.py; do not edit.',
           '// Compile-time XOR networks of the fixed encode matrices (reedsolomon.New(k, m)',
           '// parity rows, objectserver/ecutils.go:27,59) over bit-planes: output plane',
           '// 8 r + i = XOR of input planes 8 j + b with bit i of C[r][j] * 2^b.  Used by',
           '// the bit-plane record kernels (odd_impl.h) when a pass\'s coefficients equal',
           '// one of kXorShapes (checked on the host, odd.hip).',
           '#pragma once',
           '#include <hip/hip_runtime.h>',
           '#include <stdint.h>',
           '',
           'namespace hbec {',
           '',
           '__device__ __forceinline__ uint32_t x2(uint32_t a, uint32_t b) { return a ^ b; }',
           '// v_bitop3_b32 0x96: a ^ b ^ c in one instruction (the compiler emits two v_xor_b32)',
           '__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {',
           '    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);',
           '}',
           '',
           'template <int ID>',
           'struct XorNet;',
           '',
           'struct XorShape {',
           '    int k, m, r0, R;  // shape, first parity row, rows',
           '    bool strided, plan, verify;  // launched for strided batches / plans / Verify (else the table kernels)',
           '    uint8_t coef[4][12];  // C[r][j]',
           '};',
           '']
    body, table = [], []
    sid = 0
    for k, m in SHAPES:
        mat = encode_matrix(k, m)
        for r0 in range(0, m, 4):
            coef = [mat[k + r] for r in range(r0, min(m, r0 + 4))]
            rows = bit_rows(coef)
            temps, frows = schedule(rows, 8 * k, max_temps)
            # self-check on random planes against the field multiply
            import random
            rnd = random.Random(sid + 1)
            for _ in range(8):
                data = [[rnd.randrange(256) for _ in range(32)] for _ in range(k)]
                planes = [sum(((data[j][q] >> b) & 1) << q for q in range(32)) for j in range(k) for b in range(8)]
                got = simulate(temps, frows, 8 * k, planes)
                for r, cr in enumerate(coef):
                    outb = [0] * 32
                    for q in range(32):
                        v = 0
                        for j in range(k):
                            v ^= gmul(cr[j], data[j][q])
                        outb[q] = v
                    for i in range(8):
                        want = sum(((outb[q] >> i) & 1) << q for q in range(32))
                        assert got[8 * r + i] == want, (k, m, r0, r, i)
            body += emit_net(sid, k, m, r0, coef, temps, frows)
            cs = ", ".join("{" + ", ".join(str(c) for c in (cr + [0] * (12 - k))) + "}" for cr in coef)
            st, pl, ve = (str(x).lower() for x in USE[(k, m)])
            table.append(f"    {{{k}, {m}, {r0}, {len(coef)}, {st}, {pl}, {ve}, {{{cs}}}}},  // XorNet<{sid}>")
            sid += 1
    foot = ['// XorNet<i> codes kXorShapes[i]',
            f'constexpr int kXorShapeCount = {sid};',
            'constexpr XorShape kXorShapes[kXorShapeCount] = {', *table, '};', '',
            '}  // namespace hbec', '']
    return "\n".join(hdr + body + foot)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="exit 1 if the committed header differs")
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    text = generate()
    if a.stats:
        for line in text.splitlines():
            if line.startswith("// ") and "XOR instructions" in line:
                print(line)
        return
    if a.check:
        sys.exit(0 if OUT.exists() and OUT.read_text() == text else 1)
    OUT.write_text(text)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
