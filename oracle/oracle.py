"""ctypes front-end to the parity checkers (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg import this module.
It loads

* ``oracle/_build/libezrs_oracle.so`` -- the clean-room C restatement of c++/ezpwd/rs_base, and
* ``oracle/_ref/libezrs_ref.so`` -- the reference codec compiled from /root/reference (optional;
  present only where oracle/Makefile could build it, or where a prebuilt copy travelled along).

Parity status: pinned (see oracle/ezrs_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "libezrs_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libezrs_ref.so")
KARN_SO = os.path.join(HERE, "_ref", "libkarn.so")

_vp, _sz, _u, _i = C.c_void_p, C.c_size_t, C.c_uint, C.c_int


def build(quiet: bool = True) -> None:
    """Compile the restatement (and the reference shim when /root/reference exists)."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.check_call(["make", "-s", "-C", HERE, "all"], stdout=out)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_vp)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = C.CDLL(ORACLE_SO)
        L.ezo_create.restype = _vp
        L.ezo_create.argtypes = [_u, _u, _u, _u, _u, _i]
        L.ezo_destroy.argtypes = [_vp]
        for f in ("ezo_size", "ezo_nroots", "ezo_load", "ezo_datum_bytes", "ezo_iprim"):
            getattr(L, f).restype = _u
            getattr(L, f).argtypes = [_vp]
        L.ezo_tables.argtypes = [_vp, _vp, _vp, _vp]
        L.ezo_encode.argtypes = [_vp, _vp, _u, _vp]
        L.ezo_decode.argtypes = [_vp, _vp, _u, _vp, _vp, _u, _vp]
        L.ezo_encode_batch.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _i]
        L.ezo_decode_batch.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _sz, _vp, _vp, _vp,
                                       _sz, _vp, _sz, _sz, _i]
        L.ezo_set_karn.argtypes = [_vp, _i]
        L.ezo_into_dual.restype = C.POINTER(C.c_uint8)
        L.ezo_from_dual.restype = C.POINTER(C.c_uint8)
        _lib = L
    return _lib


class Codec:
    """RS codec in the restatement: Codec(mm, poly, fcr, prim, nroots, dual)."""

    def __init__(self, mm, poly, fcr, prim, nroots, dual=False, karn=False):
        self.mm, self.poly, self.fcr, self.prim, self.nroots, self.dual = (
            mm, poly, fcr, prim, nroots, bool(dual))
        self._h = lib().ezo_create(mm, poly, fcr, prim, nroots, int(bool(dual)))
        if not self._h:
            raise ValueError("invalid RS codec parameters")
        if karn:      # decode with libfec's semantics (ezrs_oracle.c decode_symbols)
            lib().ezo_set_karn(self._h, 1)
        self.nn = (1 << mm) - 1
        self.load = self.nn - nroots
        self.dtype = np.uint8 if mm <= 8 else np.uint16

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().ezo_destroy(h)
            self._h = None

    @property
    def iprim(self):
        return lib().ezo_iprim(self._h)

    def tables(self):
        a = np.zeros(self.nn + 1, np.uint16)
        i = np.zeros(self.nn + 1, np.uint16)
        g = np.zeros(self.nroots + 1, np.uint16)
        lib().ezo_tables(self._h, _ptr(a), _ptr(i), _ptr(g))
        return a, i, g

    # -- single codeword --------------------------------------------------------------------
    def encode(self, data):
        data = np.ascontiguousarray(data, self.dtype)
        par = np.zeros(self.nroots, self.dtype)
        r = lib().ezo_encode(self._h, _ptr(data), len(data), _ptr(par))
        return r, par

    def decode(self, data, parity, erasures=(), corr=None):
        """In-place decode of numpy arrays; returns (count, positions)."""
        eras = np.zeros(max(self.nroots, len(erasures)), np.uint32)
        eras[:len(erasures)] = erasures
        r = lib().ezo_decode(self._h, _ptr(data), len(data), _ptr(parity), _ptr(eras),
                             len(erasures), _ptr(corr))
        return r, eras[:max(r, 0)].copy()

    # -- batch ---------------------------------------------------------------------------------
    def encode_batch(self, data, length=None, parity=None, nthreads=1):
        """data: [ncw, stride] array.  Writes parity into ``parity`` ([ncw, nroots]) or, when
        None, into columns length..length+nroots of ``data``."""
        ncw, stride = data.shape
        length = stride - self.nroots if length is None else length
        pstride = parity.shape[1] if parity is not None else 0
        return lib().ezo_encode_batch(self._h, _ptr(data), stride, length, _ptr(parity), pstride,
                                      ncw, nthreads)

    def decode_batch(self, data, length=None, parity=None, eras=None, neras=None,
                     positions=None, nthreads=1):
        ncw, stride = data.shape
        length = stride - self.nroots if length is None else length
        result = np.zeros(ncw, np.int32)
        lib().ezo_decode_batch(
            self._h, _ptr(data), stride, length, _ptr(parity),
            parity.shape[1] if parity is not None else 0,
            _ptr(eras), eras.shape[1] if eras is not None else 0, _ptr(neras), _ptr(result),
            _ptr(positions), positions.shape[1] if positions is not None else 0, None, 0, ncw,
            nthreads)
        return result


def dual_tables():
    L = lib()
    return (np.ctypeslib.as_array(L.ezo_into_dual(), (256,)).copy(),
            np.ctypeslib.as_array(L.ezo_from_dual(), (256,)).copy())


# ---------------------------------------------------------------------------------------------
# Standard codec families (c++/ezpwd/rs:74-104)
STD_POLY = {2: 0x7, 3: 0xb, 4: 0x13, 5: 0x25, 6: 0x43, 7: 0x89, 8: 0x11d, 9: 0x211, 10: 0x409,
            11: 0x805, 12: 0x1053, 13: 0x201b, 14: 0x4443, 15: 0x8003, 16: 0x1100b}


def rs_params(n, k):
    """(mm, poly, fcr, prim, nroots, dual) of ezpwd::RS<N,K> (rs:75-89)."""
    mm = (n + 1).bit_length() - 1
    assert (1 << mm) - 1 == n, "N must be 2^m - 1"
    return mm, STD_POLY[mm], 1, 1, n - k, False


def ccsds_params(k, dual=True):
    """(mm, poly, fcr, prim, nroots, dual) of RS_CCSDS[_CONV]<255,K> (rs:101-104)."""
    return 8, 0x187, 128 - (255 - k) // 2, 11, 255 - k, dual


# ---------------------------------------------------------------------------------------------
class Ref:
    """The reference codec compiled from /root/reference by oracle/Makefile (oracle/_ref)."""

    _L = None

    @classmethod
    def available(cls):
        return os.path.exists(REF_SO)

    @classmethod
    def lib(cls):
        if cls._L is None:
            L = C.CDLL(REF_SO)
            L.ezref_count.restype = _u
            L.ezref_describe.restype = C.c_char_p
            L.ezref_describe.argtypes = [_u, _vp]
            L.ezref_encode.argtypes = [_u, _vp, _u, _vp]
            L.ezref_decode.argtypes = [_u, _vp, _u, _vp, _vp, _u, _vp]
            L.ezref_encode_batch.argtypes = [_u, _vp, _sz, _u, _vp, _sz, _sz, _u]
            L.ezref_decode_batch.argtypes = [_u, _vp, _sz, _u, _vp, _sz, _vp, _sz, _vp, _vp,
                                             _vp, _sz, _sz, _u]
            L.ezref_dual_tables.argtypes = [_vp, _vp]
            cls._L = L
        return cls._L

    @classmethod
    def codecs(cls):
        L = cls.lib()
        out = []
        for i in range(L.ezref_count()):
            p = np.zeros(6, np.uint32)
            name = L.ezref_describe(i, _ptr(p)).decode()
            out.append((i, name, tuple(int(x) for x in p[:5]) + (bool(p[5]),)))
        return out

    @classmethod
    def index(cls, name):
        for i, n, _ in cls.codecs():
            if n == name:
                return i
        raise KeyError(name)

    @classmethod
    def encode(cls, idx, data, nroots, dtype):
        data = np.ascontiguousarray(data, dtype)
        par = np.zeros(nroots, dtype)
        r = cls.lib().ezref_encode(idx, _ptr(data), len(data), _ptr(par))
        return r, par

    @classmethod
    def decode(cls, idx, data, parity, nroots, erasures=(), corr=None):
        eras = np.zeros(max(nroots, len(erasures)), np.uint32)
        eras[:len(erasures)] = erasures
        r = cls.lib().ezref_decode(idx, _ptr(data), len(data), _ptr(parity), _ptr(eras),
                                   len(erasures), _ptr(corr))
        return r, eras[:max(r, 0)].copy()

    @classmethod
    def encode_batch(cls, idx, data, length, parity):
        ncw, stride = data.shape
        w = data.dtype.itemsize
        return cls.lib().ezref_encode_batch(idx, _ptr(data), stride, length, _ptr(parity),
                                            parity.shape[1], ncw, w)

    @classmethod
    def decode_batch(cls, idx, data, length, parity, eras=None, neras=None, positions=None):
        ncw, stride = data.shape
        result = np.zeros(ncw, np.int32)
        cls.lib().ezref_decode_batch(
            idx, _ptr(data), stride, length, _ptr(parity), parity.shape[1], _ptr(eras),
            eras.shape[1] if eras is not None else 0, _ptr(neras), _ptr(result), _ptr(positions),
            positions.shape[1] if positions is not None else 0, ncw, data.dtype.itemsize)
        return result

    @classmethod
    def dual_tables(cls):
        a = np.zeros(256, np.uint8)
        b = np.zeros(256, np.uint8)
        cls.lib().ezref_dual_tables(_ptr(a), _ptr(b))
        return a, b


# ---------------------------------------------------------------------------------------------
class Karn:
    """Phil Karn's libfec RS codecs (fec-3.0.1: init/encode/decode_rs_char, encode/decode_rs_8,
    encode/decode_rs_ccsds) compiled from the reference's tarball by oracle/Makefile (karn); only
    tests/golden/make_karn_fixtures.py calls it -- the committed fixtures carry its outputs."""

    _L = None

    @classmethod
    def available(cls):
        return os.path.exists(KARN_SO)

    @classmethod
    def lib(cls):
        if cls._L is None:
            L = C.CDLL(KARN_SO)
            L.karn_init_char.restype = _vp
            L.karn_init_char.argtypes = [_i, _i, _i, _i, _i, _i]
            L.karn_free_char.argtypes = [_vp]
            L.karn_encode_char_batch.argtypes = [_vp, _vp, C.c_long, _vp, C.c_long, C.c_long, _i]
            L.karn_decode_char_batch.argtypes = [_vp, _vp, C.c_long, C.c_long, _i, _vp, _vp, _vp]
            L.karn_init_int.restype = _vp
            L.karn_init_int.argtypes = [_i, _i, _i, _i, _i, _i]
            L.karn_free_int.argtypes = [_vp]
            L.karn_encode_int_batch.argtypes = [_vp, _vp, C.c_long, _vp, C.c_long, C.c_long, _i, _i]
            L.karn_decode_int_batch.argtypes = [_vp, _vp, C.c_long, C.c_long, _i, _i, _vp, _vp, _vp]
            for f in ("karn_encode_8_batch", "karn_encode_ccsds_batch"):
                getattr(L, f).argtypes = [_vp, C.c_long, _vp, C.c_long, C.c_long, _i]
            for f in ("karn_decode_8_batch", "karn_decode_ccsds_batch"):
                getattr(L, f).argtypes = [_vp, C.c_long, C.c_long, _vp, _vp, _vp, _i]
            cls._L = L
        return cls._L

    @classmethod
    def encode_char(cls, params, data, length):
        """params = (symsize, gfpoly, fcr, prim, nroots, pad); data uint8 [ncw, >= length]."""
        L = cls.lib()
        rs = L.karn_init_char(*params)
        assert rs, "init_rs_char rejected the parameters"
        ncw = data.shape[0]
        par = np.zeros((ncw, params[4]), np.uint8)
        L.karn_encode_char_batch(rs, _ptr(data), data.shape[1], _ptr(par), par.shape[1], ncw, length)
        L.karn_free_char(rs)
        return par

    @classmethod
    def decode_char(cls, params, rows, eras, neras):
        """rows uint8 [ncw, len + nroots] corrected in place; eras int32 [ncw, nroots] in/out."""
        L = cls.lib()
        rs = L.karn_init_char(*params)
        ncw = rows.shape[0]
        result = np.zeros(ncw, np.int32)
        L.karn_decode_char_batch(rs, _ptr(rows), rows.shape[1], ncw, params[4], _ptr(eras), _ptr(neras),
                                 _ptr(result))
        L.karn_free_char(rs)
        return result

    @classmethod
    def encode_int(cls, params, data, length):
        """init_rs_int codec; data uint16 [ncw, >= length]; returns uint16 parity [ncw, nroots]."""
        L = cls.lib()
        rs = L.karn_init_int(*params)
        assert rs, "init_rs_int rejected the parameters"
        ncw = data.shape[0]
        par = np.zeros((ncw, params[4]), np.uint16)
        L.karn_encode_int_batch(rs, _ptr(data), data.shape[1], _ptr(par), par.shape[1], ncw, length, params[4])
        L.karn_free_int(rs)
        return par

    @classmethod
    def decode_int(cls, params, rows, eras, neras):
        """rows uint16 [ncw, len + nroots] corrected in place; eras int32 [ncw, nroots] in/out."""
        L = cls.lib()
        rs = L.karn_init_int(*params)
        ncw = rows.shape[0]
        result = np.zeros(ncw, np.int32)
        L.karn_decode_int_batch(rs, _ptr(rows), rows.shape[1], ncw, params[4], rows.shape[1], _ptr(eras),
                                _ptr(neras), _ptr(result))
        L.karn_free_int(rs)
        return result

    @classmethod
    def encode_fixed(cls, kind, data, pad=0):
        """kind "8" (conventional basis, 0x187 / fcr 112 / prim 11) or "ccsds" (dual basis)."""
        ncw = data.shape[0]
        par = np.zeros((ncw, 32), np.uint8)
        getattr(cls.lib(), f"karn_encode_{kind}_batch")(_ptr(data), data.shape[1], _ptr(par), 32, ncw, pad)
        return par

    @classmethod
    def decode_fixed(cls, kind, rows, eras, neras, pad=0):
        ncw = rows.shape[0]
        result = np.zeros(ncw, np.int32)
        getattr(cls.lib(), f"karn_decode_{kind}_batch")(_ptr(rows), rows.shape[1], ncw, _ptr(eras), _ptr(neras),
                                                        _ptr(result), pad)
        return result


# ---------------------------------------------------------------------------------------------
# Binary BCH (oracle/ezbch_oracle.c): the restatement of the Djelic codec behind ezpwd::bch_base
_bch_ready = False


def _bch_lib():
    global _bch_ready
    L = lib()
    if not _bch_ready:
        L.ezb_create.restype = _vp
        L.ezb_create.argtypes = [_i, _i, _u]
        L.ezb_destroy.argtypes = [_vp]
        L.ezb_info.argtypes = [_vp, _vp]
        L.ezb_genpoly.argtypes = [_vp, _vp]
        L.ezb_encode.argtypes = [_vp, _vp, _u, _vp]
        L.ezb_decode.argtypes = [_vp, _vp, _u, _vp, _vp]
        L.ezb_correct.argtypes = [_vp, _vp, _u, _vp, _vp]
        L.ezb_encode_batch.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _i]
        L.ezb_decode_batch.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _vp, _sz, _sz, _i]
        L.ezb_syndromes.argtypes = [_vp, _vp, _u, _vp, _vp]
        L.ezb_decode_syn.argtypes = [_vp, _u, _vp, _vp]
        _bch_ready = True
    return L


class BCH:
    """BCH codec in the restatement: BCH(m, t, prim_poly=0), i.e. ezpwd::bch_base(m, t, prim_poly)
    (c++/ezpwd/bch:54-61).  Parity status: pinned by the reference's BCH fixtures only."""

    def __init__(self, m, t, poly=0):
        L = _bch_lib()
        self._h = L.ezb_create(m, t, poly)
        if not self._h:
            raise ValueError("invalid BCH parameters")
        info = np.zeros(6, np.uint32)
        L.ezb_info(self._h, _ptr(info))
        self.m, self.n, self.t, self.ecc_bits, self.ecc_bytes, self.poly = (int(x) for x in info)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _bch_lib().ezb_destroy(h)
            self._h = None

    @property
    def max_len(self):
        """Longest data (whole bytes) decode accepts: 8*len <= n - ecc_bits."""
        return (self.n - self.ecc_bits) // 8

    def genpoly(self):
        g = np.zeros(self.ecc_bits + 1, np.uint8)
        _bch_lib().ezb_genpoly(self._h, _ptr(g))
        return g

    def encode(self, data):
        data = np.ascontiguousarray(data, np.uint8)
        ecc = np.zeros(self.ecc_bytes, np.uint8)
        _bch_lib().ezb_encode(self._h, _ptr(data), len(data), _ptr(ecc))
        return ecc

    def correct(self, data, ecc):
        """correct_bch in place on contiguous uint8 arrays; returns (result, error locations)."""
        loc = np.zeros(2 * self.t + 1, np.uint32)
        r = _bch_lib().ezb_correct(self._h, _ptr(data), len(data), _ptr(ecc), _ptr(loc))
        return r, loc[:max(r, 0)].copy()

    def syndromes(self, data, ecc):
        """S_1..S_2t of (data, received ecc) as uint32[2t]."""
        data = np.ascontiguousarray(data, np.uint8)
        ecc = np.ascontiguousarray(ecc, np.uint8)
        syn = np.zeros(2 * self.t, np.uint32)
        _bch_lib().ezb_syndromes(self._h, _ptr(data), len(data), _ptr(ecc), _ptr(syn))
        return syn

    def decode_syn(self, length, syn):
        """decode_bch's hardware-syndrome form: (result, ascending error locations)."""
        syn = np.ascontiguousarray(syn, np.uint32)
        loc = np.zeros(2 * self.t + 1, np.uint32)
        r = _bch_lib().ezb_decode_syn(self._h, length, _ptr(syn), _ptr(loc))
        return r, loc[:max(r, 0)].copy()

    def encode_batch(self, data, length, ecc=None, nthreads=1):
        ncw, stride = data.shape
        _bch_lib().ezb_encode_batch(self._h, _ptr(data), stride, length, _ptr(ecc),
                                    ecc.shape[1] if ecc is not None else 0, ncw, nthreads)

    def decode_batch(self, data, length, ecc=None, errloc=None, nthreads=1):
        ncw, stride = data.shape
        result = np.zeros(ncw, np.int32)
        _bch_lib().ezb_decode_batch(self._h, _ptr(data), stride, length, _ptr(ecc),
                                    ecc.shape[1] if ecc is not None else 0, _ptr(result),
                                    _ptr(errloc), errloc.shape[1] if errloc is not None else 0,
                                    ncw, nthreads)
        return result
