#!/usr/bin/env python3
"""Generate the plane-sliced BCH remainder kernels' constant code (csrc/gen/ezbch_ps_tables.inc).

The BCH remainder of a row (Djelic encode_bch / decode_bch, wrapped by c++/ezpwd/bch:196-205,
316-331): data bits MSB first, ECC = d(x) x^E mod g(x) left-justified big-endian (E = ecc_bits).
Bit b (LSB = 0) of the byte q places from a row's end is the coefficient of x^(8q + b), so with
r_b(y) = sum_q bit_b(byte_q) y^q ("plane" b of the row, a binary polynomial in y = x^8)

    r(x) mod g = sum_b x^b U_b,    U_b = sum_q bit_b(byte_q) w(q),    w(q) = x^(8q) mod g.

Every plane has the same weights w(q): a 32-bit word holding one byte position of four rows
(byte k = row k, bit 8k + b = plane b of row k) is added into the E state words U[i] (bit i of
the E-bit weights) whole -- XOR only, like the RS plane-sliced syndromes (gen_ps.py) but with a
state of E words instead of 128.  Per 8 byte positions the 15 XOR combinations of positions
0..3 and of 4..7 are formed once and every state word takes one 3-input XOR.

Fold: sum_b x^b U_b in three levels inside each byte (planes 2m + x plane 2m+1, then x^2, then
x^4: shift the word by 1, 2, 4 and multiply by x^s mod g, a sparse E x E map), leaving remainder
bit i of row k at bit 8k of U[i].

Frame: F byte positions, right-aligned: position F - 1 holds the byte Q0 places from the row's end
(q = F - 1 - f + Q0).  Encode reads the data alone (Q0 = ECC bytes: the ECC positions that follow
are zero), decode the data and the received ECC (Q0 = 0): the remainder of the whole row is then
the data's remainder XOR the received ECC, the difference decode_bch works from.  Codecs: E a
multiple of 8 (ECC bytes exactly E / 8), E <= 64.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

# init_bch's default primitive polynomials, m = 5..15 (as csrc/ezbch.hip)
DEFAULT_POLY = {5: 0x25, 6: 0x43, 7: 0x83, 8: 0x11d, 9: 0x211, 10: 0x409, 11: 0x805, 12: 0x1053,
                13: 0x201b, 14: 0x402b, 15: 0x8003}

# (name, m, t): BCH(1023, 983, 4) is SURVEY 8(d) config C5; BCH(255, 239, 2) the Itron SCM codec of
# the reference's fixtures (bch_itron.C)
CODECS = [("BCH_10_4", 10, 4), ("BCH_8_2", 8, 2)]


def generator(m, t, poly):
    """g(x) of init_bch(m, t, poly): the product of the minimal polynomials of alpha^j over the
    cyclotomic cosets of 1, 3, .., 2t - 1 (as HostBch::build).  Bit k of the result = x^k."""
    n = (1 << m) - 1
    ex, lg = [0] * (2 * n), [0] * (n + 1)
    x = 1
    for i in range(n):
        ex[i] = ex[i + n] = x
        lg[x] = i
        x <<= 1
        if x >> m:
            x ^= poly
    root = [False] * n
    for i in range(t):
        j = 2 * i + 1
        for _ in range(m):
            root[j] = True
            j = (2 * j) % n
    gc = [1]

    def mul(a, b):
        return ex[lg[a] + lg[b]] if a and b else 0
    for j in range(n):
        if not root[j]:
            continue
        r = ex[j]
        gc.append(0)
        for k in range(len(gc) - 1, 0, -1):
            gc[k] = gc[k - 1] ^ mul(gc[k], r)
        gc[0] = mul(gc[0], r)
    assert all(c in (0, 1) for c in gc)
    return sum(c << k for k, c in enumerate(gc)), len(gc) - 1


def polymod(a, g, E):
    """a(x) mod g(x) over GF(2), g of degree E."""
    while a.bit_length() > E:
        a ^= g << (a.bit_length() - 1 - E)
    return a


class BpsCodec:
    def __init__(self, name, m, t):
        self.name, self.m, self.t = name, m, t
        self.poly = DEFAULT_POLY[m]
        self.g, self.E = generator(m, t, self.poly)
        assert self.E % 8 == 0 and self.E <= 64, "plane-sliced BCH: ECC bits a multiple of 8, <= 64"
        self.EB = self.E // 8
        n = (1 << m) - 1
        self.max_len = (n - self.E) // 8                 # data bytes (bch_test.C:89-92)
        self.F = 8 * (-(-(self.max_len + self.EB) // 8))  # frame bytes
        self.NB = self.F // 8

    def w(self, q):
        return polymod(1 << (8 * q), self.g, self.E)

    def xs(self, s):
        """x^(E + i) mod g for i < s: the reduction of x^s * y."""
        return [polymod(1 << (self.E + i), self.g, self.E) for i in range(s)]


def emit_combos(out, name, srcs, ind):
    a = srcs
    out.append(f"{ind}const uint32_t {name}1 = {a[0]}, {name}2 = {a[1]}, {name}4 = {a[2]}, {name}8 = {a[3]};")
    out.append(f"{ind}const uint32_t {name}3 = {name}1 ^ {name}2, {name}5 = {name}1 ^ {name}4, "
               f"{name}6 = {name}2 ^ {name}4, {name}9 = {name}1 ^ {name}8, {name}10 = {name}2 ^ {name}8, "
               f"{name}12 = {name}4 ^ {name}8;")
    out.append(f"{ind}const uint32_t {name}7 = {name}3 ^ {name}4, {name}11 = {name}3 ^ {name}8, "
               f"{name}13 = {name}5 ^ {name}8, {name}14 = {name}6 ^ {name}8;")
    out.append(f"{ind}const uint32_t {name}15 = {name}7 ^ {name}8;")
    out.append(f"{ind}(void){name}1; (void){name}2; (void){name}3; (void){name}4; (void){name}5; "
               f"(void){name}6; (void){name}7; (void){name}8; (void){name}9; (void){name}10; "
               f"(void){name}11; (void){name}12; (void){name}13; (void){name}14; (void){name}15;")


def xor_expr(terms):
    if not terms:
        return "0u"
    acc, rest = terms[0], terms[1:]
    while rest:
        if len(rest) >= 2:
            acc, rest = f"xor3({acc}, {rest[0]}, {rest[1]})", rest[2:]
        else:
            acc, rest = f"({acc} ^ {rest[0]})", rest[1:]
    return acc


def gen_codec(c: BpsCodec):
    st = f"BPS_{c.name}"
    E, F, NB = c.E, c.F, c.NB
    out = [f"struct {st} {{",
           f"    static constexpr int M = {c.m}, T = {c.t}, E = {E}, EB = {c.EB}, F = {F}, NB = {NB};",
           f"    static constexpr unsigned G_LO = {c.g & 0xffffffff:#x}u, POLY = {c.poly:#x};",
           "    // frame block B (byte positions 8B .. 8B+7, words X) into the state (FIRST: set it);",
           "    // position F - 1 is the byte Q0 places from the row's end (encode Q0 = EB, decode 0)",
           "    template <int B, bool FIRST, int Q0>",
           "    static __device__ void block(uint32_t (&U)[E], const uint32_t (&X)[8]);",
           "    // sum_b x^b U_b: remainder bit i of row k left at bit 8k of U[i]",
           "    static __device__ void fold(uint32_t (&U)[E]);",
           "};"]
    I = "    "
    for q0, B, first in ((q0, B, first) for q0 in (c.EB, 0) for B in range(NB) for first in (True, False)):
            out.append(f"template <> __device__ __forceinline__ void {st}::block<{B}, {str(first).lower()}, {q0}>("
                       "uint32_t (&U)[E], const uint32_t (&X)[8]) {")
            emit_combos(out, "l", [f"X[{t}]" for t in range(4)], I)
            emit_combos(out, "h", [f"X[{t}]" for t in range(4, 8)], I)
            ws = [c.w(F - 1 - (8 * B + t) + q0) for t in range(8)]
            for k in range(E):
                m1 = sum(((ws[t] >> k) & 1) << t for t in range(4))
                m2 = sum(((ws[4 + t] >> k) & 1) << t for t in range(4))
                terms = ([f"l{m1}"] if m1 else []) + ([f"h{m2}"] if m2 else [])
                if first:
                    out.append(f"{I}U[{k}] = " + (" ^ ".join(terms) if terms else "0u") + ";")
                elif len(terms) == 2:
                    out.append(f"{I}U[{k}] = acc_xor3(U[{k}], {terms[0]}, {terms[1]});")
                elif terms:
                    out.append(f"{I}U[{k}] = acc_xor2(U[{k}], {terms[0]});")
            out.append("}")
    # fold: levels s = 1, 2, 4 -- U[k] ^= (x^s * (U >> s))[k] mod g
    out.append(f"__device__ __forceinline__ void {st}::fold(uint32_t (&U)[E]) {{")
    for s in (1, 2, 4):
        red = c.xs(s)
        out.append(f"{I}{{ // x^{s}")
        out.append(f"{I}    uint32_t y[E];")
        out.append(f"{I}    #pragma unroll")
        out.append(f"{I}    for (int k = 0; k < E; ++k) y[k] = U[k] >> {s};")
        for k in range(E):
            terms = [f"U[{k}]"] + ([f"y[{k - s}]"] if k >= s else [])
            terms += [f"y[{E - s + i}]" for i in range(s) if (red[i] >> k) & 1]
            out.append(f"{I}    U[{k}] = {xor_expr(terms)};")
        out.append(f"{I}}}")
    out.append("}")
    return "\n".join(out)


def main(dst=None):
    dst = dst or os.path.join(HERE, "..", "csrc", "gen", "ezbch_ps_tables.inc")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    body = ["// GENERATED by codegen/gen_bch_ps.py -- do not edit.",
            "// Plane-sliced BCH remainder networks (see ezbch_ps.hip).",
            "#pragma once", "#include <cstdint>", "namespace ezrs { namespace bps {",
            "__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {",
            "    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);", "}",
            "// state accumulation: opaque to the compiler's XOR reassociation (gen_ps.py)",
            "__device__ __forceinline__ uint32_t acc_xor3(uint32_t a, uint32_t b, uint32_t c) {",
            "    uint32_t r;",
            "    asm(\"v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96\" : \"=v\"(r) : \"v\"(a), \"v\"(b), \"v\"(c));",
            "    return r;",
            "}",
            "__device__ __forceinline__ uint32_t acc_xor2(uint32_t a, uint32_t b) {",
            "    uint32_t r;",
            "    asm(\"v_xor_b32 %0, %1, %2\" : \"=v\"(r) : \"v\"(a), \"v\"(b));",
            "    return r;",
            "}"]
    for cd in CODECS:
        body.append(gen_codec(BpsCodec(*cd)))
    body.append("// codecs with the plane-sliced remainder kernels: X(name, m, t)")
    body.append("#define EZBCH_PS_CODEC_LIST(X) " + " ".join(f"X({n}, {m}, {t})" for n, m, t in CODECS))
    body.append("} } // namespace ezrs::bps")
    txt = "\n".join(body) + "\n"
    old = open(dst).read() if os.path.exists(dst) else None
    if old != txt:
        with open(dst, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
