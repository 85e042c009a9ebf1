#!/usr/bin/env python3
"""Generate the plane-sliced GF(2^8) RS kernels' constant code (csrc/gen/ezrs_ps_tables.inc).

Word layout.  A 32-bit word holds ONE position of FOUR codewords: byte k = the symbol of codeword
k, so bit 8k + b is bit-plane b of codeword k.  Every bit of the word is an independent GF(2)
stream (codeword k, plane b); the kernels never separate the planes of a symbol.

Plane slicing.  With r_p = sum_b bit_b(r_p) alpha^b (polynomial basis), a syndrome is

    S_e = r(alpha^e) = sum_b alpha^b V_{b,e},     V_{b,e} = sum_p bit_b(r_p) w_e(p),
    w_e(p) = alpha^(e (N-1-p))                          (c++/ezpwd/rs_base:1390-1414)

and, because the V's coefficients are bits, V_{b,2e} = V_{b,e}^2.  So only one root per
cyclotomic coset ("leader") is evaluated in the main loop -- 16 of the 32 roots of RS(255,223) --
and the others follow by squaring in the epilogue.

Main loop (tile kernel k_pt, PT_<codec>).  Per 8 positions and leader bit q the state word takes
one 3-input XOR of two Four-Russians combinations (all 15 XORs of four position words are formed
once per 4 positions).  A workgroup of 8 waves covers a tile of 256 codewords (4 per lane): wave
(g, q) evaluates leader group g over the 16-position pieces of quarter q, each piece with its own
networks, and a recursive-halving exchange sums the quarters' partials.

Epilogue: expansion (squarings) and the plane fold S = sum_b alpha^b V_b inside each byte (3
levels: x alpha, x alpha^2, x alpha^4 with shifts 1,2,4), four syndromes packed per word.

Encode: syndromes of the data symbols (positions 0..K-1 of the full frame) go to a workspace; the
parity kernel (PS_<codec>::q_pass4) maps them to parity with the GF(2) matrix of parity = V^-1 S
(V_{e,j} = alpha^(e (NR-1-j))), applied bit-sliced over 32 codewords per lane.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gf8 import GF8, gf_mat_inv, lin_rows  # noqa: E402

N = 255

# (name, poly, fcr, prim, nroots): codecs with a plane-sliced path.  Every RS(255,K) with
# NROOTS <= 32 that the reference validates (rsvalidate.C:46-62), plus the conventional-basis
# CCSDS codec RS_CCSDS_CONV(255,239) (rs:101-104; RS_CCSDS(255,223) has 27 cosets, above the
# 16-leader tile design: it keeps the bit-sliced kernels).
CODECS = [
    ("RS_255_223", 0x11d, 1, 1, 32),
    ("RS_255_239", 0x11d, 1, 1, 16),
    ("RS_255_251", 0x11d, 1, 1, 4),
    ("RS_255_254", 0x11d, 1, 1, 1),
    ("RS_255_253", 0x11d, 1, 1, 2),
    ("RS_255_252", 0x11d, 1, 1, 3),
    ("RS_255_248", 0x11d, 1, 1, 7),
    ("RS_255_247", 0x11d, 1, 1, 8),
    ("RS_255_246", 0x11d, 1, 1, 9),
    ("RS_255_243", 0x11d, 1, 1, 12),
    ("RS_255_238", 0x11d, 1, 1, 17),
    ("RS_255_228", 0x11d, 1, 1, 27),
    ("CCSDS_CONV_255_239", 0x187, 120, 11, 16),
]


def fmt_list(xs):
    return "{" + ", ".join(str(x) for x in xs) + "}"


class PsCodec:
    def __init__(self, name, poly, fcr, prim, nr):
        self.name, self.poly, self.fcr, self.prim, self.nr = name, poly, fcr, prim, nr
        gf = self.gf = GF8(poly)
        self.exps = [((fcr + i) * prim) % N for i in range(nr)]   # syndrome i <-> alpha^exps[i]
        # cyclotomic cosets: leader = first syndrome index of each coset hit by the roots
        leaders, members = [], {}
        for i, e in enumerate(self.exps):
            for l in leaders:
                x, found = self.exps[l], None
                for k in range(8):
                    if x == e:
                        found = k
                        break
                    x = (2 * x) % N
                if found is not None:
                    members[l].append((i, found))
                    break
            else:
                leaders.append(i)
                members[i] = [(i, 0)]
        self.leaders, self.members = leaders, members
        assert len(leaders) <= 16, "plane-sliced path supports at most 16 leaders"
        # parity map: p = Vinv S  (S with the x^NR factor included)
        V = [[gf.pow_alpha(e * (nr - 1 - j)) for j in range(nr)] for e in self.exps]
        self.Vinv = gf_mat_inv(gf, V)

    # weight of full-frame position p for syndrome i
    def w(self, i, p):
        return self.gf.pow_alpha(self.exps[i] * (N - 1 - p))

    def q_rows(self):
        """8 NR rows (parity symbol j, bit b) as masks over input bits 8 i + q (syndrome i, bit q)."""
        gf, nr = self.gf, self.nr
        rows = []
        for j in range(nr):
            for b in range(8):
                m = 0
                for i in range(nr):
                    for q in range(8):
                        if gf.mul(self.Vinv[j][i], 1 << q) >> b & 1:
                            m |= 1 << (8 * i + q)
                rows.append(m)
        return rows


def xor_chain(dst, terms, ind):
    """dst = XOR of terms, folded left with v_bitop3 three-input XORs."""
    if not terms:
        return [f"{ind}{dst} = 0u;"]
    acc, rest = terms[0], terms[1:]
    while rest:
        if len(rest) >= 2:
            acc, rest = f"xor3({acc}, {rest[0]}, {rest[1]})", rest[2:]
        else:
            acc, rest = f"({acc} ^ {rest[0]})", rest[1:]
    return [f"{ind}{dst} = {acc};"]


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


def mat_apply(out, dst, src, rows, ind, extra=None):
    """dst[q] = (extra[q] ^) XOR over b in rows[q] of src[b]; src and dst distinct arrays."""
    for q in range(8):
        terms = ([extra[q]] if extra else []) + [src[b] for b in range(8) if rows[q] >> b & 1]
        out.extend(xor_chain(dst[q], terms, ind))


def gen_parity(c: PsCodec):
    """PS_<codec>: the codec's constants and the parity map passes over 32-codeword bit-sliced
    syndromes, q_pass4<P> = parity symbols 4P .. 4P+3 (k_ps_parity8, wave P).  Before it reads
    syndrome i's planes (i >= 1) a pass calls ready(std::integral_constant<int, i>): the kernel
    makes staged planes visible there, and interleaves other work (k_ps_parity8)."""
    st = f"PS_{c.name}"
    npass = (c.nr + 3) // 4
    out = [f"struct {st} {{",
           f"    static constexpr unsigned POLY = {c.poly:#x}, FCR = {c.fcr}, PRIM = {c.prim}, NR = {c.nr};",
           f"    static constexpr int NPASS4 = {npass};"]
    out += [f"    template <class R> static __device__ void q4_{P}(uint32_t (&O)[4][8], const uint32_t *in, int ld, "
            "R &&ready);" for P in range(npass)]
    out.append("    template <int P, class R> static __device__ __forceinline__ void q_pass4(uint32_t (&O)[4][8], "
               "const uint32_t *in, int ld, R &&ready) {")
    out.append("        " + " else ".join(f"if constexpr (P == {P}) q4_{P}(O, in, ld, ready);" for P in range(npass)))
    out.append("    }")
    out.append("};")
    I = "    "
    Q = c.q_rows()
    nr = c.nr
    PW = 4
    for P in range(npass):
        j0, nj = PW * P, min(PW, nr - PW * P)
        out.append(f"template <class R> __device__ __forceinline__ void {st}::q4_{P}("
                   f"uint32_t (&O)[{PW}][8], const uint32_t *in, int ld, R &&ready) {{")
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
                out.append(f"{I}    ready(std::integral_constant<int, {i + 1}>{{}});")
                out.append(f"{I}    #pragma unroll")
                out.append(f"{I}    for (int q = 0; q < 8; ++q) N[q] = in[({8 * (i + 1)} + q) * ld];")
            out.append(f"{I}    __builtin_amdgcn_sched_barrier(0);")
            emit_combos(out, "l", ["P[0]", "P[1]", "P[2]", "P[3]"], I + "    ")
            emit_combos(out, "h", ["P[4]", "P[5]", "P[6]", "P[7]"], I + "    ")
            for jl in range(nj):
                for b in range(8):
                    row = Q[8 * (j0 + jl) + b]
                    m = (row >> (8 * i)) & 0xFF
                    ml, mh = m & 15, m >> 4
                    terms = ([f"l{ml}"] if ml else []) + ([f"h{mh}"] if mh else [])
                    dst = f"O[{jl}][{b}]"
                    if first[jl][b]:
                        out.append(f"{I}    {dst} = " + (" ^ ".join(terms) if terms else "0u") + ";")
                        first[jl][b] = False
                    elif len(terms) == 2:
                        out.append(f"{I}    {dst} = acc_xor3({dst}, {terms[0]}, {terms[1]});")
                    elif terms:
                        out.append(f"{I}    {dst} = acc_xor2({dst}, {terms[0]});")
            out.append(f"{I}    __builtin_amdgcn_sched_barrier(0);")
            out.append(f"{I}}}")
        out.append("}")
    return "\n".join(out)


def emit_fold_epilogue(out, gf, fname, T, nlw_expr, seq):
    """A device function fname(T, emit) folding the syndromes listed in seq = [(local leader,
    syndrome index, squarings)] four per quad."""
    I = "    "
    sq_cache = {}

    def sqk(k):
        if k not in sq_cache:
            sq_cache[k] = lin_rows(lambda x, k=k: gf.pow(x, 1 << k) if x else 0)
        return sq_cache[k]

    def cost(rows):
        return sum(max(0, bin(r).count("1") - 1) for r in rows)

    a1 = lin_rows(lambda x: gf.mul(2, x))
    a2 = lin_rows(lambda x: gf.mul(4, x))
    a4 = lin_rows(lambda x: gf.mul(16, x))

    def fold_level(dst, src, rows, sh, ind, up=False):
        """dst = src + alpha^k (src one step up), at the lower bit positions of each pair of
        positions sh apart -- or, up, at the upper ones (src shifted up instead), so that the
        next pack needs no shift."""
        out.append(f"{ind}{{")
        out.append(f"{ind}    uint32_t y[8];")
        if up:
            out.append(f"{ind}    for (int b = 0; b < 8; ++b) y[b] = {src}[b] << {sh};")
            mat_apply(out, [f"{dst}[{q}]" for q in range(8)], [f"{src}[{b}]" for b in range(8)], rows,
                      ind + "    ", extra=[f"y[{q}]" for q in range(8)])
        else:
            out.append(f"{ind}    for (int b = 0; b < 8; ++b) y[b] = {src}[b] >> {sh};")
            mat_apply(out, [f"{dst}[{q}]" for q in range(8)], [f"y[{b}]" for b in range(8)], rows,
                      ind + "    ", extra=[f"{src}[{q}]" for q in range(8)])
        out.append(f"{ind}}}")

    out.append(f"template <class F, class HK> __device__ __forceinline__ void {fname}("
               f"const uint32_t (&{T})[{nlw_expr}][8], F &&emit, HK &&hook) {{")
    prev = {}

    def expand(li, m, k, ind):
        if k == 0:
            prev[li] = (f"{T}[{li}]", 0)
            return f"{T}[{li}]"
        src, kp = prev.get(li, (f"{T}[{li}]", 0))
        direct = cost(sqk(k))
        chained = cost(sqk(k - kp)) if kp else direct
        out.append(f"{ind}uint32_t W{m}[8];")
        if kp and chained < direct:
            mat_apply(out, [f"W{m}[{b}]" for b in range(8)], [f"{src}[{b}]" for b in range(8)], sqk(k - kp), ind)
        else:
            mat_apply(out, [f"W{m}[{b}]" for b in range(8)], [f"{T}[{li}][{b}]" for b in range(8)], sqk(k), ind)
        prev[li] = (f"W{m}", k)
        return f"W{m}"

    for qd in range((len(seq) + 3) // 4):
        part = seq[4 * qd:4 * qd + 4]
        srcs = [expand(li, m, k, I) for li, m, k in part]
        out.append(f"{I}{{ // quad {qd}: syndromes {[m for _, m, _ in part]}")
        for j in range(4):
            out.append(f"{I}    uint32_t F{j}[8];")
            if j < len(part):
                fold_level(f"F{j}", srcs[j], a1, 1, I + "    ", up=j % 2 == 1)
            else:
                out.append(f"{I}    for (int b = 0; b < 8; ++b) F{j}[b] = 0u;")
            out.append(f"{I}    hook(std::integral_constant<int, {4 * qd + j}>{{}});   // other work may go here")
        for pj in range(2):
            out.append(f"{I}    uint32_t P{pj}[8], G{pj}[8];")
            out.append(f"{I}    for (int b = 0; b < 8; ++b) P{pj}[b] = bfi(0x55555555u, "
                       f"F{2 * pj}[b], F{2 * pj + 1}[b]);")
            fold_level(f"G{pj}", f"P{pj}", a2, 2, I + "    ", up=pj == 1)
        out.append(f"{I}    uint32_t H[8], Q[8];")
        out.append(f"{I}    for (int b = 0; b < 8; ++b) H[b] = bfi(0x33333333u, G0[b], G1[b]);")
        fold_level("Q", "H", a4, 4, I + "    ")
        out.append(f"{I}    emit(std::integral_constant<int, {qd}>{{}}, Q);")
        out.append(f"{I}}}")
    out.append("}")


def emit_weight_block(out, fname_sig, weights, B, I="    ", first=False, opaque=False):
    """One main-loop block: positions 8B..8B+7 (X[0..7]) into state V[s][q] for the GF(2^8)
    weight functions weights[s](p) (V[s] accumulates sum_p bit_b(x_p) weights[s](p)).
    first: set the state instead of accumulating (a wave's first block).  opaque: accumulate
    through inline-asm XORs (acc_xor3 / acc_xor2), so the compiler cannot reassociate the state
    chains across blocks (which keeps every block's combinations live to the end and spills)."""
    xf3, xf2 = ("acc_xor3", "acc_xor2") if opaque else ("xor3", None)
    out.append(fname_sig + " {")
    emit_combos(out, "l", [f"X[{t}]" for t in range(4)], I)
    emit_combos(out, "h", [f"X[{t}]" for t in range(4, 8)], I)
    acc, first_rows = [], []
    for s_, wf in enumerate(weights):
        for q in range(8):
            m1 = sum(((wf(8 * B + t) >> q) & 1) << t for t in range(4))
            m2 = sum(((wf(8 * B + 4 + t) >> q) & 1) << t for t in range(4))
            terms = ([f"l{m1}"] if m1 else []) + ([f"h{m2}"] if m2 else [])
            if len(terms) == 2:
                acc.append(f"V[{s_}][{q}] = {xf3}(V[{s_}][{q}], {terms[0]}, {terms[1]});")
                first_rows.append(f"V[{s_}][{q}] = {terms[0]} ^ {terms[1]};")
            elif terms:
                acc.append(f"V[{s_}][{q}] = {xf2}(V[{s_}][{q}], {terms[0]});" if opaque else f"V[{s_}][{q}] ^= {terms[0]};")
                first_rows.append(f"V[{s_}][{q}] = {terms[0]};")
            else:
                first_rows.append(f"V[{s_}][{q}] = 0u;")
    out.extend(f"{I}{x}" for x in (first_rows if first else acc))
    out.append("}")


# ---- tile kernel (k_pt): 8 waves share one 256-codeword tile ------------------------------------
PT_WAVES = 8
PT_XCAP = 5               # items (8 words each) a wave sends per exchange sub-round (80 KiB area)


def pt_exchange(groups_need, qn):
    """Recursive-halving reduce-scatter over the qn position-split waves of one item group.
    groups_need[q] = set of item slots wave q needs at the end.  Round r pairs q with q ^ (1 << r);
    after round r wave q holds the sums over its 2^(r+1)-wave block of the items needed by the
    waves that agree with q on bits 0..r.  Returns per wave, per round (send list, recv list)."""
    rounds = qn.bit_length() - 1
    allitems = set().union(*groups_need) if groups_need else set()

    def resp(q, r):                     # items wave q must hold after round r (r = -1: all)
        if r < 0:
            return set(allitems)
        mask = (1 << (r + 1)) - 1
        return set().union(*[groups_need[x] for x in range(qn) if (x & mask) == (q & mask)])
    plan = []
    for q in range(qn):
        per = []
        for r in range(rounds):
            p = q ^ (1 << r)
            send = sorted(resp(p, r) & resp(q, r - 1))
            recv = sorted(resp(q, r) & resp(p, r - 1))
            per.append((send, recv))
        plan.append(per)
    return plan


def pt_xcost(plan, qn, xcap=PT_XCAP):
    rounds = qn.bit_length() - 1
    return sum(max(-(-len(plan[q][r][0]) // xcap) for q in range(qn)) for r in range(rounds))


class PtRole:
    """One direction of the tile kernel for one codec: items (decode: coset leaders; encode: parity
    symbols) of 8 state words each, split into GN groups of NI items; each group's QN = 8 / GN
    waves split the positions; a recursive-halving exchange leaves every wave the totals of the
    items its epilogue folds (seq = [(item slot, output index, squarings)])."""

    def __init__(self, c: PsCodec, enc: bool, waves=PT_WAVES, gn=None, xcap=PT_XCAP):
        from itertools import combinations, permutations
        self.c, self.enc = c, enc
        self.nwaves, self.xcap = waves, xcap
        gf = c.gf
        K = N - c.nr
        self.hi = K if enc else N
        if enc:
            nitems = c.nr
            def G(p, j):
                if p >= K:
                    return 0
                acc = 0
                for i in range(c.nr):
                    acc ^= gf.mul(c.Vinv[j][i], gf.pow_alpha(c.exps[i] * (N - 1 - p)))
                return acc
            self.wfun = [(lambda p, j=j: G(p, j)) for j in range(nitems)]
            outs = [[(j, 0)] for j in range(nitems)]            # item j -> output j, no squaring
        else:
            nitems = len(c.leaders)
            self.wfun = [(lambda p, l=l: c.w(l, p) if p < N else 0) for l in c.leaders]
            outs = [sorted(c.members[l], key=lambda x: x[1]) for l in c.leaders]
        self.gn = gn if gn else max(1, -(-nitems // 8))
        while waves % self.gn:
            self.gn += 1
        self.qn = waves // self.gn
        size = [len(o) for o in outs]
        # 1. items -> GN groups of (nearly) equal item and output counts; 2. per group, outputs ->
        #    QN waves by recursive halving of the group's output multiset, which is the exchange's
        #    own structure: at each level choose how many outputs of every item go to each half
        #    (equal output counts), minimising the distinct items per half (what the exchange
        #    round of that level sends).  The group split is chosen by the resulting exchange cost.
        from functools import lru_cache
        from itertools import product
        items = list(range(nitems))

        def split(counts, n):
            """counts: tuple of (item, outputs); n waves -> (cost, [per-wave (item, outputs) lists]).
            Halves take whole items, at most one item split between them."""
            if n == 1:
                return (len(counts),), [list(counts)]
            tot = sum(k for _, k in counts)
            half = -(-tot // 2)
            m = len(counts)
            best = None
            for mask in range(1 << m):
                inA = [k for j, (_, k) in enumerate(counts) if mask >> j & 1]
                sa = sum(inA)
                opts = []
                if sa == half:
                    opts.append(None)
                elif sa < half:
                    for j, (_, k) in enumerate(counts):      # split item j: half - sa of it to A
                        if not (mask >> j & 1) and k > half - sa:
                            opts.append((j, half - sa))
                for o in opts:
                    A, B = [], []
                    for j, (i, k) in enumerate(counts):
                        if o is not None and o[0] == j:
                            A.append((i, o[1]))
                            B.append((i, k - o[1]))
                        elif mask >> j & 1:
                            A.append((i, k))
                        else:
                            B.append((i, k))
                    here = max(len(A), len(B))
                    if best is not None and here > best[0][0]:
                        continue
                    ca, ga = split(tuple(A), n // 2)
                    cb, gb = split(tuple(B), n // 2)
                    key = (here,) + tuple(max(x, y) for x, y in zip(ca, cb))
                    if best is None or key < best[0]:
                        best = (key, ga + gb)
            return best

        def plan_group(gitems):
            counts = tuple((s, size[i]) for s, i in enumerate(gitems))
            _, parts = split(counts, self.qn)
            # part j of the recursion: bit r from the top selects the half at level r; wave q meets
            # q ^ 1 in round 0 (the top split), so q = bit-reverse(j)
            nbits = self.qn.bit_length() - 1
            bins, used = [None] * self.qn, {}
            for j, part in enumerate(parts):
                q = int(format(j, f"0{nbits}b")[::-1], 2) if nbits else 0
                b = []
                for s, k in part:
                    u = used.get(s, 0)
                    b += [(s, m, kk) for m, kk in outs[gitems[s]][u:u + k]]
                    used[s] = u + k
                bins[q] = b
            plan = pt_exchange([set(s for s, _, _ in b) for b in bins], self.qn)
            return (pt_xcost(plan, self.qn, xcap), max(-(-len(b) // 4) for b in bins),
                    sum(len(x[0]) for pq in plan for x in pq)), bins, plan

        if self.gn == 1:
            cands = [[items]]
        elif enc:
            per = -(-nitems // self.gn)
            cands = [[items[i:i + per] for i in range(0, nitems, per)]]
        else:
            per = -(-nitems // self.gn)
            target = sum(size) / self.gn
            cands = []
            assert self.gn == 2, "decode tile plan: at most two leader groups"
            for comb in combinations(items[1:], per - 1):
                grp = [0] + list(comb)
                if sum(size[i] for i in grp) == round(target):
                    cands.append([grp, [i for i in items if i not in grp]])
                if len(cands) >= 60:
                    break
            if not cands:
                cands = [[items[0::2], items[1::2]]]
        best = None
        for groups in cands:
            res = [plan_group(gi) for gi in groups]
            key = tuple(max(r[0][x] for r in res) for x in range(3))
            if best is None or key < best[0]:
                best = (key, groups, res)
        _, groups, res = best
        self.groups = groups
        self.ni = max(len(g) for g in groups)
        self.waves = {}                                       # wave -> dict
        for g, (gitems, (_, bins, plan)) in enumerate(zip(groups, res)):
            for q in range(self.qn):
                w = g + self.gn * q
                seq = bins[q]
                own = sorted(set(s for s, _, _ in seq))
                self.waves[w] = {"g": g, "q": q, "plan": plan[q], "own": own,
                                 "seq": [(own.index(s), m, k) for s, m, k in seq]}
        self.rounds = self.qn.bit_length() - 1
        # sub-rounds: <= xcap items per wave at a time (the exchange area)
        self.subs = []                                        # (round, chunk index)
        for r in range(self.rounds):
            nch = max(-(-len(self.waves[w]["plan"][r][0]) // xcap) for w in range(waves))
            self.subs += [(r, ch) for ch in range(nch)]
        self.nown = max(1, max(len(v["own"]) for v in self.waves.values()))
        self.nq = max(1, max(-(-len(v["seq"]) // 4) for v in self.waves.values()))
        # 4. pieces (16 positions) per wave: half 0 = pieces 0..7, half 1 = 8..; round-robin
        npieces = -(-self.hi // 16)
        self.pieces = {}
        for w in range(waves):
            q = self.waves[w]["q"]
            h0 = [p for p in range(0, min(8, npieces)) if p % self.qn == q % self.qn]
            h1 = [p for p in range(8, npieces) if (p - 8) % self.qn == q % self.qn]
            self.pieces[w] = (h0, h1)


def gen_pt(c: PsCodec):
    """Tile-kernel tables and straight-line code, PT_<codec>: syndromes by coset leaders, the
    leaders split into GN groups, the positions into QN quarters.  Wave (g, q) reads pieces
    q, q + QN, q + 2 QN, ... and runs each piece's own networks on them (block index = the piece's
    absolute 8-position block).  Encode evaluates the same syndromes over the data positions (the
    kernel masks positions >= K) for k_ps_parity8."""
    out = []
    R = PtRole(c, False)
    st = f"PT_{c.name}"
    W = PT_WAVES
    mp = max(max(len(R.pieces[w][0]) + len(R.pieces[w][1]) for w in range(W)), 1)
    nsub = max(len(R.subs), 1)

    def pad(xs, n, v=-1):
        return list(xs) + [v] * (n - len(xs))
    X = PT_XCAP
    xs = [[pad(R.waves[w]["plan"][r][0][X * ch:X * ch + X], X) for (r, ch) in R.subs] or [[-1] * X]
          for w in range(W)]
    xv = [[pad(R.waves[w]["plan"][r][1][X * ch:X * ch + X], X) for (r, ch) in R.subs] or [[-1] * X]
          for w in range(W)]
    syn = [[[R.waves[w]["seq"][4 * qd + j][1] if 4 * qd + j < len(R.waves[w]["seq"]) else -1
             for j in range(4)] for qd in range(R.nq)] for w in range(W)]
    for w in range(W):                                  # pieces of wave (g, q) = quarter 0's + q
        q = R.waves[w]["q"]
        p0 = R.pieces[R.waves[w]["g"]][0] + R.pieces[R.waves[w]["g"]][1]
        mine = R.pieces[w][0] + R.pieces[w][1]
        assert mine == [p + q for p in p0][:len(mine)], (w, mine, p0)
    hdr = [f"struct {st} {{",
           f"    static constexpr unsigned POLY = {c.poly:#x}, FCR = {c.fcr}, PRIM = {c.prim}, NR = {c.nr};",
           f"    static constexpr int GN = {R.gn}, QN = {R.qn}, NI = {R.ni}, NOWN = {R.nown}, NQ = {R.nq};",
           f"    static constexpr int NSUB = {len(R.subs)}, MP = {mp}, XCAP = {X};",
           "    // pieces (16 positions) of wave W: NP0 in half 0, then NP1 in half 1 (decode: 255",
           "    // positions; encode stops at the data positions)",
           f"    static constexpr int NP0[{W}] = {fmt_list([len(R.pieces[w][0]) for w in range(W)])};",
           f"    static constexpr int NP1[{W}] = {fmt_list([len(R.pieces[w][1]) for w in range(W)])};",
           f"    static constexpr int PIECE[{W}][{mp}] = " + "{" + ", ".join(
               fmt_list(pad(R.pieces[w][0] + R.pieces[w][1], mp)) for w in range(W)) + "};",
           "    // exchange sub-round s (round XR[s]): wave W sends item slots XS[W][s], adds the",
           "    // partner's words into slots XV[W][s] (partner = W ^ (GN << XR[s]))",
           f"    static constexpr int XR[{nsub}] = {fmt_list([r for r, _ in R.subs] or [0])};",
           f"    static constexpr int XS[{W}][{nsub}][{X}] = " + "{" + ", ".join(
               "{" + ", ".join(fmt_list(x) for x in xs[w]) + "}" for w in range(W)) + "};",
           f"    static constexpr int XV[{W}][{nsub}][{X}] = " + "{" + ", ".join(
               "{" + ", ".join(fmt_list(x) for x in xv[w]) + "}" for w in range(W)) + "};",
           "    // item slots whose totals wave W folds (T[i] <-> slot OWN[W][i])",
           f"    static constexpr int OWN[{W}][{R.nown}] = " + "{" + ", ".join(
               fmt_list(pad(R.waves[w]["own"], R.nown)) for w in range(W)) + "};",
           "    // syndrome index of quad slot (W, quad, j), -1 = none",
           f"    static constexpr int SYN[{W}][{R.nq}][4] = " + "{" + ", ".join(
               "{" + ", ".join(fmt_list(q) for q in syn[w]) + "}" for w in range(W)) + "};",
           "    // positions 8B..8B+7 (words X) into group G's state (B: the absolute 8-position block;",
           "    // F: the wave's first block, which sets the state instead of accumulating into it)",
           "    template <int G, int B, bool F> static __device__ void block(uint32_t (&V)[NI][8], const uint32_t (&X)[8]);",
           "    template <int W, class F, class H> static __device__ void epilogue(const uint32_t (&T)[NOWN][8], F &&emit, "
           "H &&hook);",
           "};"]
    out += hdr
    gf = c.gf
    for g, gitems in enumerate(R.groups):
        ws = [R.wfun[i] for i in gitems]
        # every wave of group g runs its own pieces' networks (block index = absolute 8-position
        # block), so no quarter needs a fix-up
        pall = sorted(set(p for w in range(W) if R.waves[w]["g"] == g for p in R.pieces[w][0] + R.pieces[w][1]))
        for pc in pall:
            for B in (2 * pc, 2 * pc + 1):
                for F in ((True, False) if B == 2 * pc else (False,)):
                    emit_weight_block(out, f"template <> __device__ __forceinline__ void {st}::block<{g}, {B}, {str(F).lower()}>("
                                      "uint32_t (&V)[NI][8], const uint32_t (&X)[8])", ws, B, first=F, opaque=True)
    for w in range(W):
        emit_fold_epilogue(out, c.gf, f"{st}_epi{w}", "T", f"{st}::NOWN", R.waves[w]["seq"])
    out.append(f"template <int W, class F, class H> __device__ __forceinline__ void {st}::epilogue("
               "const uint32_t (&T)[NOWN][8], F &&emit, H &&hook) {")
    out.append("    " + " else ".join(f"if constexpr (W == {w}) {st}_epi{w}(T, emit, hook);" for w in range(W)))
    out.append("}")
    return "\n".join(out)


# ---- 4-wave tile kernel (k_pq): each wave evaluates ALL leaders over its own run of positions ------
PQ_WAVES = 4
PQ_XCAP = 8               # items a wave sends per exchange sub-round (4 x 8 x 2 KiB = the 64 KiB image)
PQ_CODECS = {"RS_255_223", "RS_255_251", "RS_255_239", "RS_255_247", "RS_255_243", "RS_255_238", "RS_255_228", "CCSDS_CONV_255_239"}


def gen_pq(c: PsCodec):
    """PQ_<codec>: the 4-wave tile kernel's tables and straight-line code.  Wave W evaluates every
    coset leader (NI x 8 state words) over its own contiguous run of 8-position blocks, with each
    block's own network (no quarter fix-ups, no leader groups: reads and Four-Russians combinations
    are done once per position); a two-round recursive-halving exchange then leaves every wave the
    totals of the leaders whose syndromes (two quads) it folds.  Encode runs the same networks over
    the data positions (the kernel masks positions >= K) for k_ps_parity8."""
    out = []
    R = PtRole(c, False, waves=PQ_WAVES, gn=1, xcap=PQ_XCAP)
    st = f"PQ_{c.name}"
    W = PQ_WAVES
    X = PQ_XCAP
    nsub = max(len(R.subs), 1)

    def pad(xs, n, v=-1):
        return list(xs) + [v] * (n - len(xs))
    xs = [[pad(R.waves[w]["plan"][r][0][X * ch:X * ch + X], X) for (r, ch) in R.subs] or [[-1] * X]
          for w in range(W)]
    xv = [[pad(R.waves[w]["plan"][r][1][X * ch:X * ch + X], X) for (r, ch) in R.subs] or [[-1] * X]
          for w in range(W)]
    syn = [[[R.waves[w]["seq"][4 * qd + j][1] if 4 * qd + j < len(R.waves[w]["seq"]) else -1
             for j in range(4)] for qd in range(R.nq)] for w in range(W)]
    # 8-position blocks per direction, split into W contiguous runs (decode: all N positions;
    # encode: the data positions)
    runs = []
    for hi in (N, N - c.nr):
        nb = -(-hi // 8)
        cut = [round(nb * w / W) for w in range(W + 1)]
        runs.append((nb, cut))
    hdr = [f"struct {st} {{",
           f"    static constexpr unsigned POLY = {c.poly:#x}, FCR = {c.fcr}, PRIM = {c.prim}, NR = {c.nr};",
           f"    static constexpr int NI = {R.ni}, NOWN = {R.nown}, NQ = {R.nq};",
           f"    static constexpr int NSUB = {len(R.subs)}, XCAP = {X};",
           "    // 8-position blocks of wave W: [B0[E][W], B0[E][W + 1]) (E = 0 decode, 1 encode)",
           f"    static constexpr int NB[2] = {{{runs[0][0]}, {runs[1][0]}}};",
           f"    static constexpr int B0[2][{W + 1}] = {{{fmt_list(runs[0][1])}, {fmt_list(runs[1][1])}}};",
           "    // exchange sub-round s (round XR[s]): wave W sends item slots XS[W][s], adds the",
           "    // partner's words into slots XV[W][s] (partner = W ^ (1 << XR[s]))",
           f"    static constexpr int XR[{nsub}] = {fmt_list([r for r, _ in R.subs] or [0])};",
           f"    static constexpr int XS[{W}][{nsub}][{X}] = " + "{" + ", ".join(
               "{" + ", ".join(fmt_list(x) for x in xs[w]) + "}" for w in range(W)) + "};",
           f"    static constexpr int XV[{W}][{nsub}][{X}] = " + "{" + ", ".join(
               "{" + ", ".join(fmt_list(x) for x in xv[w]) + "}" for w in range(W)) + "};",
           "    // item slots whose totals wave W folds (T[i] <-> slot OWN[W][i])",
           f"    static constexpr int OWN[{W}][{R.nown}] = " + "{" + ", ".join(
               fmt_list(pad(R.waves[w]["own"], R.nown)) for w in range(W)) + "};",
           "    // syndrome index of quad slot (W, quad, j), -1 = none",
           f"    static constexpr int SYN[{W}][{R.nq}][4] = " + "{" + ", ".join(
               "{" + ", ".join(fmt_list(q) for q in syn[w]) + "}" for w in range(W)) + "};",
           "    // positions 8B..8B+7 (words X) into every leader's state",
           "    // F: the wave's first block (sets the state instead of accumulating into it)",
           "    template <int B, bool F> static __device__ void block(uint32_t (&V)[NI][8], const uint32_t (&X)[8]);",
           "    template <int W, class F, class H> static __device__ void epilogue(const uint32_t (&T)[NOWN][8], F &&emit, "
           "H &&hook);",
           "};"]
    out += hdr
    ws = [R.wfun[i] for i in R.groups[0]]
    for B in range(runs[0][0]):
        for F in (True, False):
            emit_weight_block(out, f"template <> __device__ __forceinline__ void {st}::block<{B}, {str(F).lower()}>("
                              "uint32_t (&V)[NI][8], const uint32_t (&X)[8])", ws, B, first=F, opaque=True)
    for w in range(W):
        emit_fold_epilogue(out, c.gf, f"{st}_epi{w}", "T", f"{st}::NOWN", R.waves[w]["seq"])
    out.append(f"template <int W, class F, class H> __device__ __forceinline__ void {st}::epilogue("
               "const uint32_t (&T)[NOWN][8], F &&emit, H &&hook) {")
    out.append("    " + " else ".join(f"if constexpr (W == {w}) {st}_epi{w}(T, emit, hook);" for w in range(W)))
    out.append("}")
    return "\n".join(out)


def main(dst=None):
    dst = dst or os.path.join(HERE, "..", "csrc", "gen", "ezrs_ps_tables.inc")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    body = ["// GENERATED by codegen/gen_ps.py -- do not edit.",
            "// Plane-sliced GF(2^8) RS syndrome kernels' straight-line code (see ezrs_ps.hip).",
            "#pragma once", "#include <cstdint>", "namespace ezrs { namespace ps {",
            "__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {",
            "    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);", "}",
            "// state accumulation of the 4-wave kernel: opaque to the compiler's XOR reassociation",
            "__device__ __forceinline__ uint32_t acc_xor3(uint32_t a, uint32_t b, uint32_t c) {",
            "    uint32_t r;",
            "    asm(\"v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96\" : \"=v\"(r) : \"v\"(a), \"v\"(b), \"v\"(c));",
            "    return r;",
            "}",
            "__device__ __forceinline__ uint32_t acc_xor2(uint32_t a, uint32_t b) {",
            "    uint32_t r;",
            "    asm(\"v_xor_b32 %0, %1, %2\" : \"=v\"(r) : \"v\"(a), \"v\"(b));",
            "    return r;",
            "}",
            "// (m & a) | (~m & b): v_bfi_b32",
            "__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {",
            "    return (m & a) | (~m & b);", "}"]
    for cd in CODECS:
        c = PsCodec(*cd)
        body.append(gen_parity(c))
        body.append(gen_pt(c))
        if c.name in PQ_CODECS:
            body.append(gen_pq(c))

    body.append("// codecs with the 4-wave tile kernel (PQ_<codec>)")
    body.append("#define EZRS_PQ_CODEC_LIST(X) " + " ".join(f"X({cd[0]})" for cd in CODECS if cd[0] in PQ_CODECS))
    body.append("#define EZRS_PS_CODEC_LIST(X) \\")
    for i, cd in enumerate(CODECS):
        sep = " \\" if i + 1 < len(CODECS) else ""
        body.append(f"    X({cd[0]}){sep}")
    body.append("} } // namespace ezrs::ps")
    txt = "\n".join(body) + "\n"
    old = open(dst).read() if os.path.exists(dst) else None
    if old != txt:
        with open(dst, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
