"""GF(2^8) helpers for the bit-sliced kernel generator (host-side, build time only).

Field, generator roots and dual-basis conventions follow c++/ezpwd/rs_base:537-635 (tables),
1263-1285 (roots alpha^((fcr+i)*prim)) and 109-146 (CCSDS dual basis)."""
from __future__ import annotations


class GF8:
    def __init__(self, poly):
        self.poly = poly
        self.exp = [0] * 512
        self.log = [0] * 256
        x = 1
        for i in range(255):
            self.exp[i] = x
            self.log[x] = i
            x <<= 1
            if x & 0x100:
                x ^= poly
        assert x == 1, "polynomial not primitive"
        for i in range(255, 512):
            self.exp[i] = self.exp[i - 255]

    def mul(self, a, b):
        if a == 0 or b == 0:
            return 0
        return self.exp[self.log[a] + self.log[b]]

    def pow_alpha(self, e):
        return self.exp[e % 255]

    def pow(self, a, e):
        if a == 0:
            return 0 if e else 1
        return self.exp[(self.log[a] * e) % 255]

    def inv(self, a):
        assert a
        return self.exp[(255 - self.log[a]) % 255]


DUAL_COLS = (0x7b, 0xaf, 0x99, 0xfa, 0x86, 0xec, 0xef, 0x8d)


def into_dual_map():
    into = []
    for x in range(256):
        y = 0
        for b in range(8):
            if x >> b & 1:
                y ^= DUAL_COLS[b]
        into.append(y)
    frm = [0] * 256
    for x, y in enumerate(into):
        frm[y] = x
    return into, frm


def lin_rows(f):
    """Rows (8-bit input masks) of the GF(2)-linear byte map f: out bit q = XOR of input bits p
    with row[q] bit p."""
    cols = [f(1 << p) for p in range(8)]
    return [sum(((cols[p] >> q) & 1) << p for p in range(8)) for q in range(8)]


def apply_rows(rows, x):
    y = 0
    for q, r in enumerate(rows):
        y |= (bin(r & x).count("1") & 1) << q
    return y


def gf2_inv(mat, n):
    """Invert an n x n GF(2) matrix given as a list of n row bitmasks."""
    a = [(mat[i], 1 << i) for i in range(n)]
    for col in range(n):
        piv = next(r for r in range(col, n) if a[r][0] >> col & 1)
        a[col], a[piv] = a[piv], a[col]
        for r in range(n):
            if r != col and a[r][0] >> col & 1:
                a[r] = (a[r][0] ^ a[col][0], a[r][1] ^ a[col][1])
    return [a[i][1] for i in range(n)]


def gf_mat_inv(gf, A):
    """Invert a square matrix over GF(2^8) (list of rows)."""
    n = len(A)
    M = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(A)]
    for col in range(n):
        piv = next(r for r in range(col, n) if M[r][col])
        M[col], M[piv] = M[piv], M[col]
        iv = gf.inv(M[col][col])
        M[col] = [gf.mul(iv, v) for v in M[col]]
        for r in range(n):
            if r != col and M[r][col]:
                f = M[r][col]
                M[r] = [a ^ gf.mul(f, b) for a, b in zip(M[r], M[col])]
    return [row[n:] for row in M]


class Codec8:
    """An RS code over GF(2^8) as the bit-sliced kernels see it."""

    def __init__(self, poly, fcr, prim, nroots, dual):
        self.gf = GF8(poly)
        self.poly, self.fcr, self.prim, self.nroots, self.dual = poly, fcr, prim, nroots, dual
        self.into, self.frm = into_dual_map()
        self.roots = [self.gf.pow_alpha((fcr + i) * prim) for i in range(nroots)]
        # parity p solves  sum_q p_q g_i^(NR-1-q) = g_i^NR * H_i(data)   for every root g_i
        V = [[self.gf.pow(g, nroots - 1 - q) for q in range(nroots)] for g in self.roots]
        self.Vinv = gf_mat_inv(self.gf, V)

    def input_rows(self, c):
        """Rows of 'multiply the (raw, possibly dual-basis) input symbol by c'."""
        pre = self.frm if self.dual else None
        return lin_rows(lambda x: self.gf.mul(c, pre[x] if pre else x))

    def mul_rows(self, c):
        return lin_rows(lambda x: self.gf.mul(c, x))

    def q_rows(self):
        """Encode map: 8*NR output bits (parity symbol j, bit b) as masks over 8*NR input bits
        (syndrome i, bit q), input bit index 8*i + q."""
        nr = self.nroots
        cols = []
        for i in range(nr):
            for q in range(8):
                w = [0] * nr
                w[i] = self.gf.mul(self.gf.pow(self.roots[i], nr), 1 << q)
                p = [0] * nr
                for j in range(nr):
                    v = 0
                    for ii in range(nr):
                        v ^= self.gf.mul(self.Vinv[j][ii], w[ii])
                    p[j] = self.into[v] if self.dual else v
                cols.append(p)
        rows = []
        for j in range(nr):
            for b in range(8):
                m = 0
                for k, p in enumerate(cols):
                    if p[j] >> b & 1:
                        m |= 1 << k
                rows.append(m)
        return rows
