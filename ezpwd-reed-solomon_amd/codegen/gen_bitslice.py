#!/usr/bin/env python3
"""Generate the constant tables of the bit-sliced GF(2^8) RS kernels (csrc/gen/ezrs_bs_tables.inc).

The kernels evaluate syndromes S_i = r(g_i), g_i = alpha^((fcr+i)*prim) (c++/ezpwd/rs_base:1390-1414),
on 32 slots per 32-bit register: 4 codewords x 8 interleaved segments (positions p = 8y + sigma).
Slot bit 8s + k holds codeword k & 3, segment sigma = 4 (k >> 2) + s.  Per segment, Horner in
d_i = g_i^8 runs in blocks of 16 y-steps (128 positions, one LDS chunk):

    G_i <- G_i * d_i^16 + sum_{t<16} c_{8(16k+t)+sigma} * d_i^(15-t)

and the segments are folded in three levels (x g^4, << 4; x g, << 8; x g^2, << 16), leaving
S_i = sum_sigma g_i^(7-sigma) G_sigma at bits 28..31.  Every constant multiplication is a
GF(2)-linear 8x8 bit map; the tables below give, for every output bit, the 4-bit masks of input
bits 0-3 and 4-7 it XORs (the kernels precompute all 15 XOR-combinations of each input nibble once
and spend one v_bitop3 per output bit and input byte).

Encode evaluates the data word only and maps the syndromes to parity with the GF(2) matrix Q of
parity = into_dual?( V^-1 (g^NR * H(data)) ) (see gf8.Codec8.q_rows), in passes of 8 parity
symbols over full 32-codeword registers (q_pass).

Dual-basis codecs fold from_dual into every input map and into_dual into Q, so the kernels never
touch the dual-basis tables (rs_base:109-146, 1312, 1324-1326).
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gf8 import Codec8  # noqa: E402

# (name, poly, fcr, prim, nroots, dual) -- the codecs with a bit-sliced fast path
CODECS = [
    ("RS_255_223", 0x11d, 1, 1, 32, False),
    ("RS_255_239", 0x11d, 1, 1, 16, False),
    ("RS_255_251", 0x11d, 1, 1, 4, False),
    ("CCSDS_255_223", 0x187, 112, 11, 32, True),
    ("CCSDS_CONV_255_223", 0x187, 112, 11, 32, False),
]

NROLES = 4
BLOCK = 16     # y-steps per Horner block (= one LDS chunk of 128 positions)
SEG = 8        # positions per y-step (segments per codeword slot group)


def plane_off(b):
    """LDS dword offset of bit-plane b from a lane's base (see ezrs_bitslice.hip: the 4 row pieces
    of a lane sit 64 dwords apart, plane b in row piece b & 3, dword b >> 2 of the y-step)."""
    return 64 * (b & 3) + (b >> 2)


def split(nr):
    """Syndromes per role: NROLES contiguous ranges (first, count)."""
    h = (nr + NROLES - 1) // NROLES
    out = []
    for r in range(NROLES):
        a = min(nr, r * h)
        out.append((a, min(nr, a + h) - a))
    return out


def nib(row):
    return (row & 15) | ((row >> 4) & 15) << 4


def fmt(arr, depth=0):
    if isinstance(arr, list):
        return "{" + ",".join(fmt(a, depth + 1) for a in arr) + "}"
    return str(arr)


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


def upd(dst, acc, m, lo="l", hi="h"):
    ml, mh = m & 15, m >> 4
    terms = ([f"{lo}{ml}"] if ml else []) + ([f"{hi}{mh}"] if mh else [])
    if acc is None:
        if not terms:
            return f"{dst} = 0u;"
        if len(terms) == 1:
            return f"{dst} = {terms[0]};"
        return f"{dst} = {terms[0]} ^ {terms[1]};"
    if not terms:
        return None
    if len(terms) == 1:
        return f"{dst} ^= {terms[0]};"
    return f"{dst} = xor3({acc}, {terms[0]}, {terms[1]});"


def gen_codec(name, poly, fcr, prim, nr, dual):
    C = Codec8(poly, fcr, prim, nr, dual)
    gf = C.gf
    roles = split(nr)
    Q = C.q_rows()
    npass = (nr + 7) // 8
    st = f"BS_{name}"
    out = [f"struct {st} {{",
           f"    static constexpr unsigned POLY = {poly:#x}, FCR = {fcr}, PRIM = {prim}, NR = {nr};",
           f"    static constexpr bool DUAL = {'true' if dual else 'false'};",
           f"    static constexpr int NROLES = {NROLES};",
           f"    static constexpr int S0[{NROLES}] = {{{', '.join(str(a) for a, _ in roles)}}};",
           f"    static constexpr int NS[{NROLES}] = {{{', '.join(str(n) for _, n in roles)}}};",
           f"    static constexpr int NPASS = {npass};   // parity passes of 8 symbols",
           "    // s *= d_i^16 (one Horner block) for syndrome S0[R] + I",
           "    template <int R, int I> static __device__ void mul(uint32_t (&s)[8]);",
           "    // one Horner block of 16 y-steps",
           "    template <int R> static __device__ void horner_block(uint32_t (&S)[16][8], "
           "const uint32_t *p);",
           "    // fold the 8 segment partials of syndrome S0[R] + I into bits 28..31",
           "    template <int R, int I> static __device__ void fold(uint32_t (&s)[8]);",
           "    template <int P> static __device__ void q_pass(uint32_t (&O)[8][8], "
           "const uint32_t *in, int ld);",
           "};"]
    for r, (r0, n) in enumerate(roles):
        I = "    "
        # ---- s *= d^16, one function per syndrome
        for i in range(n):
            rows = C.mul_rows(gf.pow(gf.pow(C.roots[r0 + i], SEG), BLOCK))
            out.append(f"template <> __device__ __forceinline__ void {st}::mul<{r}, {i}>(uint32_t (&s)[8]) {{")
            emit_combos(out, "l", [f"s[{q}]" for q in range(4)], I)
            emit_combos(out, "h", [f"s[{q}]" for q in range(4, 8)], I)
            for q in range(8):
                out.append(f"{I}" + upd(f"s[{q}]", None, nib(rows[q])))
            out.append("}")
        # ---- one block of BLOCK y-steps, constants d^(BLOCK-1-t), straight-line (pad positions
        # are zero data: from a zero state they leave it zero).  Plane loads are not prefetched
        # across y-steps: with 4 waves per SIMD the other waves cover the LDS latency, and 8 VGPRs
        # fewer keep the kernel spill-free at 128.
        out.append(f"template <> __device__ __forceinline__ void {st}::horner_block<{r}>("
                   "uint32_t (&S)[16][8], const uint32_t *p) {")
        for t in range(BLOCK):
            out.append(f"{I}{{")
            out.append(f"{I}    uint32_t P[8];")
            for bb in range(8):
                out.append(f"{I}    P[{bb}] = p[{plane_off(bb) + 2 * t}];")
            emit_combos(out, "l", ["P[0]", "P[1]", "P[2]", "P[3]"], I + "    ")
            emit_combos(out, "h", ["P[4]", "P[5]", "P[6]", "P[7]"], I + "    ")
            for i in range(n):
                d = gf.pow(C.roots[r0 + i], SEG)
                rows = C.input_rows(gf.pow(d, BLOCK - 1 - t))
                for q in range(8):
                    ln = upd(f"S[{i}][{q}]", f"S[{i}][{q}]", nib(rows[q]))
                    if ln:
                        out.append(f"{I}    " + ln)
            out.append(f"{I}    __builtin_amdgcn_sched_barrier(0);")
            out.append(f"{I}}}")
        out.append("}")
        # ---- segment fold, one function per syndrome
        for i in range(n):
            g = C.roots[r0 + i]
            out.append(f"template <> __device__ __forceinline__ void {st}::fold<{r}, {i}>(uint32_t (&s)[8]) {{")
            for c, sh in ((gf.pow(g, 4), 4), (g, 8), (gf.mul(g, g), 16)):
                rows = C.mul_rows(c)
                out.append(f"{I}{{")
                emit_combos(out, "l", [f"(s[{q}] << {sh})" for q in range(4)], I + "    ")
                emit_combos(out, "h", [f"(s[{q}] << {sh})" for q in range(4, 8)], I + "    ")
                for q in range(8):
                    ln = upd(f"s[{q}]", f"s[{q}]", nib(rows[q]))
                    if ln:
                        out.append(f"{I}    " + ln)
                out.append(f"{I}    __builtin_amdgcn_sched_barrier(0);")
                out.append(f"{I}}}")
            out.append("}")
    # ---- encode parity map, one pass of up to 8 parity symbols over full 32-slot registers:
    # O[jl][b] = bit b of parity symbol 8P+jl; in[(8 i + q) * ld] = bit q of syndrome i.
    for P in range(npass):
        I = "    "
        j0, nj = 8 * P, min(8, nr - 8 * P)
        out.append(f"template <> __device__ __forceinline__ void {st}::q_pass<{P}>("
                   "uint32_t (&O)[8][8], const uint32_t *in, int ld) {")
        first = [[True] * 8 for _ in range(nj)]
        out.append(f"{I}uint32_t N[8];")
        out.append(f"{I}#pragma unroll")
        out.append(f"{I}for (int q = 0; q < 8; ++q) N[q] = in[q * ld];")
        for i in range(nr):
            out.append(f"{I}{{ // syndrome {i}")
            out.append(f"{I}    uint32_t P[8];")
            out.append(f"{I}    #pragma unroll")
            out.append(f"{I}    for (int q = 0; q < 8; ++q) P[q] = N[q];")
            if i + 1 < nr:
                out.append(f"{I}    #pragma unroll")
                out.append(f"{I}    for (int q = 0; q < 8; ++q) N[q] = in[({8 * (i + 1)} + q) * ld];")
            out.append(f"{I}    __builtin_amdgcn_sched_barrier(0);")
            emit_combos(out, "l", ["P[0]", "P[1]", "P[2]", "P[3]"], I + "    ")
            emit_combos(out, "h", ["P[4]", "P[5]", "P[6]", "P[7]"], I + "    ")
            for jl in range(nj):
                for b in range(8):
                    row = Q[8 * (j0 + jl) + b]
                    m = nib((row >> (8 * i)) & 0xFF)
                    if first[jl][b]:
                        out.append(f"{I}    " + upd(f"O[{jl}][{b}]", None, m))
                        first[jl][b] = False
                    else:
                        ln = upd(f"O[{jl}][{b}]", f"O[{jl}][{b}]", m)
                        if ln:
                            out.append(f"{I}    " + ln)
            out.append(f"{I}    __builtin_amdgcn_sched_barrier(0);")
            out.append(f"{I}}}")
        out.append("}")
    return "\n".join(out)


def main(dst=None):
    dst = dst or os.path.join(HERE, "..", "csrc", "gen", "ezrs_bs_tables.inc")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    body = ["// GENERATED by codegen/gen_bitslice.py -- do not edit.",
            "// Straight-line XOR networks of the bit-sliced GF(2^8) RS kernels (see ezrs_bitslice.hip).",
            "#pragma once", "#include <cstdint>", "namespace ezrs { namespace bs {",
            "__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {",
            "    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);", "}",
            "// In-place 8x8 bit transpose of (register index) x (bit position mod 8): afterwards",
            "// D[b] bit 8s+c holds what D[c] bit 8s+b held (3 delta-swap stages, 4 ops per pair).",
            "__device__ __forceinline__ void transpose8(uint32_t (&D)[8]) {",
            "#pragma unroll",
            "    for (int k = 0; k < 3; ++k) {",
            "        const int sh = 1 << k;",
            "        const uint32_t M = k == 0 ? 0x55555555u : k == 1 ? 0x33333333u : 0x0F0F0F0Fu;",
            "#pragma unroll",
            "        for (int c = 0; c < 8; ++c) {",
            "            if (c & sh) continue;",
            "            const uint32_t x = D[c], y = D[c | sh];",
            "            D[c] = (x & M) | ((y << sh) & ~M);",
            "            D[c | sh] = ((x >> sh) & M) | (y & ~M);",
            "        }",
            "    }",
            "}"]
    for c in CODECS:
        body.append(gen_codec(*c))
    body.append("#define EZRS_BS_CODEC_LIST(X) \\")
    for i, (name, poly, fcr, prim, nr, dual) in enumerate(CODECS):
        sep = " \\" if i + 1 < len(CODECS) else ""
        body.append(f"    X(BS_{name}){sep}")
    body.append("} } // namespace ezrs::bs")
    txt = "\n".join(body) + "\n"
    old = open(dst).read() if os.path.exists(dst) else None
    if old != txt:
        with open(dst, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
