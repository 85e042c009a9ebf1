#!/usr/bin/env python3
"""Generate gen/ezrs_wide_tables.inc: the GF(2)-linear remainder networks of the GF(2^16) syndrome
kernels (ezrs_wide.hip).

Derivation.  The syndromes of decode_symbols (c++/ezpwd/rs_base:1390-1414) are
S_i = r(beta_i), beta_i = alpha^(e_i), e_i = (fcr + i) * prim mod NN, with r(x) the received word
(data[0] the highest-degree coefficient).  Let M_e(x) be the minimal polynomial of alpha^e over
GF(2) (binary coefficients, degree 16 for every e that occurs here) and R_e = r mod M_e.  Then
r(beta) = R_e(beta) for every conjugate beta = alpha^(e 2^k), so one remainder per cyclotomic coset
("leader") serves all the syndromes of that coset.  Because M_e is binary, R_e is computed with
XORs of whole 16-bit symbols only: a GF(2)-linear shift register whose taps are the 1-bits of M_e.

Blocks of CB symbols c_0..c_(CB-1) (c_0 first) update the 16 remainder words s[0..15]
(R = sum_k s[k] x^k) as
    R' = R x^CB + sum_t c_t x^(CB-1-t)  (mod M_e)
so s'[k] is the XOR of the s[i] with bit k of x^(CB+i) mod M_e set and of the c_t with bit k of
x^(CB-1-t) mod M_e set.  A cost-driven greedy elimination forms shared pairs and triples once
(one v_xor / v_bitop3 each), and every row is a chain of three-input XORs.  check_network()
evaluates each generated network against the bit-serial remainder.  Per 16 symbols and 16 leaders:
CB = 16 costs 719 ops (828 with the earlier pair-only elimination), CB = 32 615, CB = 64 533 --
more inputs per row to share; the kernel holds CB inputs plus its leaders' states in VGPRs.

A 32-bit word packs the same position of two codewords (low half: even codeword of the lane's
pair, high half: odd), so every XOR advances two codewords.

Run from the repo root: python3 ezpwd-reed-solomon_amd/codegen/gen_wide.py
"""
import itertools
import os
import sys

# (m, poly, fcr, prim, nroots): the GF(2^16) codecs with a fast path.  RS<65535,65503> is BASELINE
# config C4 (rs:47-104 maps RS<N,K> to poly 0x1100b, fcr 1, prim 1).
CODECS = [
    (16, 0x1100B, 1, 1, 32),
    (16, 0x1100B, 1, 1, 16),
]
CB = 64                                       # symbols per network block


class GF:
    def __init__(self, m, poly):
        self.m, self.nn = m, (1 << m) - 1
        self.exp = [0] * (2 * self.nn)
        self.log = [0] * (self.nn + 1)
        x = 1
        for i in range(self.nn):
            self.exp[i] = self.exp[i + self.nn] = x
            self.log[x] = i
            x <<= 1
            if x >> m:
                x ^= poly
        assert x == 1

    def mul(self, a, b):
        if not a or not b:
            return 0
        return self.exp[self.log[a] + self.log[b]]


def min_poly(gf, e):
    """Binary minimal polynomial of alpha^e as an int (bit k = coefficient of x^k)."""
    conj, x = [], e % gf.nn
    while x not in conj:
        conj.append(x)
        x = 2 * x % gf.nn
    p = [1]                                   # coefficients, low to high, in GF(2^m)
    for c in conj:
        r = gf.exp[c]
        q = [0] * (len(p) + 1)
        for k, a in enumerate(p):             # p * (x + r)
            q[k + 1] ^= a
            q[k] ^= gf.mul(a, r)
        p = q
    assert all(a in (0, 1) for a in p), "minimal polynomial not binary"
    return sum(a << k for k, a in enumerate(p)), len(conj)


def leaders(m, poly, fcr, prim, nr):
    gf = GF(m, poly)
    seen, lead, syn_leader = {}, [], []
    for i in range(nr):
        e = (fcr + i) * prim % gf.nn
        c, x = [], e
        while x not in c:
            c.append(x)
            x = 2 * x % gf.nn
        ld = min(c)
        if ld not in seen:
            seen[ld] = len(lead)
            lead.append(ld)
        syn_leader.append(seen[ld])
    return gf, lead, syn_leader


def block_rows(mp, d, B):
    """rows[k] = the terms of s'[k] for a block of B symbols c_0..c_(B-1) (c_0 first):
    R' = R x^B + sum_t c_t x^(B-1-t) (mod M), so s'[k] is the XOR of the s_i whose x^(B+i) mod M
    has bit k set and of the c_t whose x^(B-1-t) mod M has bit k set."""
    def reduce(v):
        for b in range(v.bit_length() - 1, d - 1, -1):
            if v >> b & 1:
                v ^= mp << (b - d)
        return v
    rows = [[] for _ in range(d)]
    for i in range(d):
        v = reduce(1 << (B + i))
        for k in range(d):
            if v >> k & 1:
                rows[k].append(f"s{i}")
    for t in range(B):
        v = reduce(1 << (B - 1 - t))
        for k in range(d):
            if v >> k & 1:
                rows[k].append(f"c[{t}]")
    return rows


def xor_ops(n):
    """v_bitop3 / v_xor count of an XOR of n terms."""
    return n // 2


def cse(rows):
    """Greedy common-subexpression elimination on XOR rows, cost-driven: at each step form the
    pair or triple (one v_xor / v_bitop3) that lowers the total op count the most, counting each
    row as xor_ops(terms).  Returns (temps, rows) with temps = [(name, *terms)]."""
    rows = [list(r) for r in rows]
    temps = []
    while True:
        cands = {}
        for ri, r in enumerate(rows):
            rs = sorted(r)
            for k in (2, 3):
                for comb in itertools.combinations(rs, k):
                    cands.setdefault(comb, []).append(ri)
        best = None
        for comb, users in cands.items():
            if len(users) < 2:
                continue
            k = len(comb)
            gain = -xor_ops(k) + sum(xor_ops(len(rows[ri])) - xor_ops(len(rows[ri]) - k + 1) for ri in users)
            key = (gain, len(users), -k, comb)
            if gain > 0 and (best is None or key > best[0]):
                best = (key, comb, users)
        if best is None:
            break
        _, comb, users = best
        t = f"t{len(temps)}"
        temps.append((t,) + comb)
        for ri in users:
            for x in comb:
                rows[ri].remove(x)
            rows[ri].append(t)
    return temps, rows


def xor_chain(terms):
    terms = list(terms)
    acc, rest = terms[0], terms[1:]
    while rest:
        if len(rest) >= 2:
            acc, rest = f"xor3({acc}, {rest[0]}, {rest[1]})", rest[2:]
        else:
            acc, rest = f"({acc} ^ {rest[0]})", rest[1:]
    return acc


def check_network(mp, d, B, temps, rows, trials=64):
    """Evaluate the network on random words and compare with the remainder computed bit by bit."""
    import random
    rnd = random.Random(mp * 131 + B)
    for _ in range(trials):
        sv = [rnd.getrandbits(32) for _ in range(d)]
        cv = [rnd.getrandbits(32) for _ in range(B)]
        env = {f"s{i}": sv[i] for i in range(d)}
        env.update({f"c[{t}]": cv[t] for t in range(B)})
        for t in temps:
            v = 0
            for x in t[1:]:
                v ^= env[x]
            env[t[0]] = v
        got = []
        for r in rows:
            v = 0
            for x in r:
                v ^= env[x]
            got.append(v)
        for bit in range(32):                    # each bit plane is a GF(2) polynomial
            R = sum(((sv[i] >> bit) & 1) << i for i in range(d))
            for t in range(B):
                R = (R << 1) | ((cv[t] >> bit) & 1)
                if R >> d & 1:
                    R ^= mp
            assert all(((got[k] >> bit) & 1) == (R >> k & 1) for k in range(d)), "network mismatch"


def gen_block(name, mp, d, B):
    temps, rows = cse(block_rows(mp, d, B))
    check_network(mp, d, B, temps, rows)
    ops = 0
    out = [f"__device__ __forceinline__ void {name}(uint32_t (&s)[{d}], const uint32_t (&c)[{B}]) {{"]
    out += [f"    const uint32_t s{i} = s[{i}];" for i in range(d)]
    for t in temps:
        out.append(f"    const uint32_t {t[0]} = {xor_chain(t[1:])};")
        ops += xor_ops(len(t) - 1)
    for k in range(d):
        out.append(f"    s[{k}] = {xor_chain(rows[k])};")
        ops += xor_ops(len(rows[k]))
    out.append("}")
    return out, ops


def gen_codec(m, poly, fcr, prim, nr):
    gf, lead, syn_leader = leaders(m, poly, fcr, prim, nr)
    tag = f"RS_{gf.nn}_{gf.nn - nr}" if (poly, fcr, prim) == (0x1100B, 1, 1) else \
        f"C{m}_{poly:x}_{fcr}_{prim}_{nr}"
    out = [f"// ---- {tag}: m={m} poly={poly:#x} fcr={fcr} prim={prim} nroots={nr}: "
           f"{len(lead)} coset leaders ----"]
    # slot order: waves take consecutive slots (kLPW per wave); alternate the costliest networks with the cheapest so
    # that the waves of a workgroup reach each window's barrier together
    cost = {}
    for e in lead:
        mp, d = min_poly(gf, e)
        assert d == m, f"leader {e}: degree {d}"
        cost[e] = gen_block("x", mp, d, CB)[1]
    by = sorted(lead, key=lambda e: (-cost[e], e))
    order = []
    while by:
        order.append(by.pop(0))
        if by:
            order.append(by.pop())
    costs = []
    for li, e in enumerate(order):
        mp, d = min_poly(gf, e)
        body, ops = gen_block(f"wb_{tag}_{li}", mp, d, CB)
        costs.append(ops)
        out.append(f"// slot {li}: leader {e}: M(x) = {mp:#x}, {ops} ops per {CB}-symbol block")
        out += body
    nl = len(order)
    out.append(f"struct WC_{tag} {{")
    out.append(f"    static constexpr unsigned M = {m}, POLY = {poly:#x}, FCR = {fcr}, PRIM = {prim}, NR = {nr};")
    out.append(f"    static constexpr int NL = {nl};")
    out.append(f"    static constexpr int CB = {CB};  // symbols per block")
    out.append(f"    static constexpr uint16_t LEADER[{nl}] = {{{', '.join(str(e) for e in order)}}};  // slot -> coset leader")
    out.append("    template <int L>")
    out.append(f"    static __device__ __forceinline__ void block(uint32_t (&s)[16], const uint32_t (&c)[{CB}]) {{")
    for li in range(nl):
        kw = "if" if li == 0 else "else if"
        out.append(f"        {kw} constexpr (L == {li}) wb_{tag}_{li}(s, c);")
    out.append("    }")
    out.append("};")
    out.append(f"// total {sum(costs)} ops per {CB} symbols x 2 codewords "
               f"({sum(costs) / (2 * CB):.2f} per codeword-symbol)")
    return tag, out


def main(dst=None):
    here = os.path.dirname(os.path.abspath(__file__))
    dst = dst or os.path.join(here, "..", "csrc", "gen", "ezrs_wide_tables.inc")
    body = ["// Generated by codegen/gen_wide.py -- do not edit.",
            "#pragma once",
            "namespace ezrs {",
            "namespace wide {",
            "__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {",
            "    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);",
            "}"]
    tags = []
    for cd in CODECS:
        tag, out = gen_codec(*cd)
        tags.append(tag)
        body += out
    body.append("#define EZRS_WIDE_CODEC_LIST(X) \\")
    cont = " \\"
    body += [f"    X({t})" + (cont if i + 1 < len(tags) else "") for i, t in enumerate(tags)]
    body += ["} // namespace wide", "} // namespace ezrs", ""]
    with open(dst, "w") as f:
        f.write("\n".join(body))
    if "-v" in sys.argv:
        print("\n".join(l for l in body if l.startswith("//")))


if __name__ == "__main__":
    main(next((a for a in sys.argv[1:] if a != "-v"), None))
