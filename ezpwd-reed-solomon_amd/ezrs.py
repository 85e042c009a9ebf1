"""Python host mirror of the MI355X RS engine (ctypes over lib/libezrs_hip.so, include/ezrs.h).

Mirrors the reference's RS codec surface for the batch hot path:

* ``Codec.rs(n, k)``          -- ezpwd::RS<N,K>                  (c++/ezpwd/rs:74-89)
* ``Codec.ccsds(k, dual)``    -- ezpwd::RS_CCSDS[_CONV]<255,K>   (c++/ezpwd/rs:101-104)
* ``Codec.encode(...)``       -- encode<TYP>(data, len, parity)  (c++/ezpwd/rs_base:868-904) per row
* ``Codec.decode(...)``       -- decode<TYP>(data, len, parity, eras_pos, no_eras, corr)
                                                                 (c++/ezpwd/rs_base:1170-1242) per row

Device forms take torch tensors on the codec's device (PyTorch is only the allocator/stream
provider here); host forms take numpy arrays and go through the library's pinned, double-buffered
copy pipeline.  There is no CPU fallback: if the HIP library is missing or no GPU is visible,
constructing a codec raises.
"""
from __future__ import annotations

import ctypes as C
import errno
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libezrs_hip.so")
# timing experiments only: a variant build of the same library (tools/build_variant.sh)
LIB_PATH = os.environ.get("EZRS_LIB_VARIANT") or LIB_PATH
HEADER = os.path.join(os.path.dirname(HERE), "include", "ezrs.h")
BCH_HEADER = os.path.join(os.path.dirname(HERE), "include", "ezbch.h")

_vp, _sz, _u, _i = C.c_void_p, C.c_size_t, C.c_uint, C.c_int


class EzrsError(RuntimeError):
    pass


class Info(C.Structure):
    _fields_ = [("symbol_bits", _u), ("size", _u), ("nroots", _u), ("load", _u), ("poly", _u),
                ("fcr", _u), ("prim", _u), ("datum_bytes", _u), ("dual", _i), ("device", _i)]


class BCHInfo(C.Structure):
    _fields_ = [("m", _u), ("n", _u), ("t", _u), ("ecc_bits", _u), ("ecc_bytes", _u),
                ("prim_poly", _u), ("device", _i)]


_lib = None


def lib():
    """Load libezrs_hip.so; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EzrsError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                            "(make -C ezpwd-reed-solomon_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        L.ezrs_abi_version.restype = _i
        L.ezrs_device_count.restype = _i
        L.ezrs_last_error.restype = C.c_char_p
        L.ezrs_create.argtypes = [C.POINTER(_vp), _u, _u, _u, _u, _u, _i, _i]
        L.ezrs_create_rs.argtypes = [C.POINTER(_vp), _u, _u, _i]
        L.ezrs_create_ccsds.argtypes = [C.POINTER(_vp), _u, _i, _i]
        L.ezrs_destroy.argtypes = [_vp]
        L.ezrs_get_info.argtypes = [_vp, C.POINTER(Info)]
        L.ezrs_reserve.argtypes = [_vp, _sz]
        L.ezrs_reserve_stream.argtypes = [_vp, _sz, _vp]
        L.ezrs_workspace_bytes.argtypes = [_vp, _sz]
        L.ezrs_workspace_bytes.restype = _sz
        L.ezrs_encode.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _vp]
        L.ezrs_encode_rows.argtypes = [_vp, _vp, _sz, _u, _sz, _vp]
        L.ezrs_encode_ws.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _vp, _sz, _vp]
        L.ezrs_encode_rows_ws.argtypes = [_vp, _vp, _sz, _u, _sz, _vp, _sz, _vp]
        L.ezrs_decode.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _sz,
                                  _vp, _sz, _sz, _vp]
        L.ezrs_decode_ws.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _sz,
                                     _vp, _sz, _sz, _vp, _sz, _vp]
        L.ezrs_encode_host.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _sz]
        L.ezrs_encode_rows_host.argtypes = [_vp, _vp, _sz, _u, _sz, _sz]
        L.ezrs_decode_host.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _sz, _vp, _vp, _vp,
                                       _sz, _vp, _sz, _sz, _sz]
        L.ezrs_stream_encoded_bound.argtypes = [_vp, _sz, _u]
        L.ezrs_stream_encoded_bound.restype = _sz
        L.ezrs_stream_encode.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, C.POINTER(_sz)]
        L.ezrs_stream_decode.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, C.POINTER(_sz),
                                         C.POINTER(_sz)]
        L.ezrs_shard_codewords.restype = _sz
        L.ezrs_shard_codewords.argtypes = [_vp, _sz, _u]
        L.ezrs_shard_encoded_len.restype = _sz
        L.ezrs_shard_encoded_len.argtypes = [_vp, _sz, _u]
        L.ezrs_encode_shards.argtypes = [_vp, _vp, _sz, _sz, _u, _sz, _vp]
        L.ezrs_decode_shards.argtypes = [_vp, _vp, _sz, _sz, _u, _sz, _vp, _sz, _vp, _vp, _vp, _sz,
                                         _vp, _sz, _vp]
        L.ezrs_kernel_path.argtypes = [_vp]
        L.ezrs_set_launch_rows.argtypes = [_vp, _sz]
        L.ezrs_set_semantics.argtypes = [_vp, _i]
        L.ezrs_get_semantics.argtypes = [_vp]
        L.ezrs_host_alloc.argtypes = [C.POINTER(_vp), _sz]
        L.ezrs_host_free.argtypes = [_vp]
        L.ezbch_last_error.restype = C.c_char_p
        L.ezbch_create.argtypes = [C.POINTER(_vp), _u, _u, _u, _i]
        L.ezbch_create_nkt.argtypes = [C.POINTER(_vp), _u, _u, _u, _i]
        L.ezbch_destroy.argtypes = [_vp]
        L.ezbch_get_info.argtypes = [_vp, C.POINTER(BCHInfo)]
        L.ezbch_encode.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _vp]
        L.ezbch_encode_rows.argtypes = [_vp, _vp, _sz, _u, _sz, _vp]
        L.ezbch_encode_rows_host.argtypes = [_vp, _vp, _sz, _u, _sz, _sz]
        L.ezbch_decode.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _vp, _sz, _sz, _vp]
        L.ezbch_decode_ecc.argtypes = [_vp, _vp, _sz, _u, _vp, _vp, _sz, _sz, _vp]
        L.ezbch_decode_syn.argtypes = [_vp, _vp, _sz, _u, _vp, _vp, _sz, _sz, _vp]
        L.ezbch_encode_host.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _sz, _sz]
        L.ezbch_decode_host.argtypes = [_vp, _vp, _sz, _u, _vp, _sz, _vp, _vp, _sz, _sz, _sz]
        _lib = L
    return _lib


def _check(rc, what, bch=False):
    if rc < 0:
        msg = (lib().ezbch_last_error() if bch else lib().ezrs_last_error()).decode(errors="replace")
        raise EzrsError(f"{what} failed: {errno.errorcode.get(-rc, rc)} {msg}")
    return rc


def _tp(t):
    """Device pointer of a torch tensor (or None)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def _np(a):
    return None if a is None else a.ctypes.data_as(_vp)


_ITEM = {"uint8": 1, "int8": 1, "uint16": 2, "int16": 2, "uint32": 4, "int32": 4}


def _dev_rows(t, what, device, itemsize, ndim=2):
    """Validate a device tensor argument: on the codec's device, rows of contiguous elements of the
    expected width; returns its row stride in elements (0 for None)."""
    if t is None:
        return 0
    if not getattr(t, "is_cuda", False):
        raise EzrsError(f"{what}: expected a GPU tensor")
    if t.device.index != device:
        raise EzrsError(f"{what}: tensor on cuda:{t.device.index}, codec on cuda:{device}")
    if t.element_size() != itemsize:
        raise EzrsError(f"{what}: expected {itemsize}-byte elements, got {t.dtype}")
    if t.dim() != ndim or (ndim == 2 and t.shape[1] > 1 and t.stride(1) != 1):
        raise EzrsError(f"{what}: expected a {ndim}-D tensor with contiguous rows")
    return t.stride(0) if ndim == 2 else 1


def _host_rows(a, what, itemsize, ndim=2):
    """Validate a numpy argument of the host forms; returns its row stride in elements."""
    if a is None:
        return 0
    if not isinstance(a, np.ndarray):
        raise EzrsError(f"{what}: expected a numpy array")
    if a.itemsize != itemsize:
        raise EzrsError(f"{what}: expected {itemsize}-byte elements, got {a.dtype}")
    if a.ndim != ndim or (ndim == 2 and a.shape[1] > 1 and a.strides[1] != itemsize) or \
            (ndim == 2 and a.strides[0] % itemsize):
        raise EzrsError(f"{what}: expected a {ndim}-D array with contiguous rows")
    if ndim == 1 and a.strides[0] != itemsize:
        raise EzrsError(f"{what}: expected a contiguous array")
    if ndim == 2 and a.strides[0] < 0:
        raise EzrsError(f"{what}: rows in reverse order (negative row stride) are not supported")
    return a.strides[0] // itemsize if ndim == 2 else 1


def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream) if hasattr(stream, "cuda_stream") else C.c_void_p(stream)


class Codec:
    """An RS(N,K) codec resident on one HIP device."""

    def __init__(self, symbol_bits, poly, fcr, prim, nroots, dual=False, device=0, _h=None):
        h = _vp()
        if _h is None:
            _check(lib().ezrs_create(C.byref(h), symbol_bits, poly, fcr, prim, nroots,
                                     int(bool(dual)), device), "ezrs_create")
        else:
            h = _h
        self._h = h
        info = Info()
        _check(lib().ezrs_get_info(self._h, C.byref(info)), "ezrs_get_info")
        self.info = info
        self.symbol_bits, self.nn, self.nroots, self.load = (info.symbol_bits, info.size,
                                                             info.nroots, info.load)
        self.dual, self.device = bool(info.dual), info.device
        self.dtype = np.uint8 if info.datum_bytes == 1 else np.uint16

    @classmethod
    def rs(cls, n, k, device=0):
        h = _vp()
        _check(lib().ezrs_create_rs(C.byref(h), n, k, device), f"ezrs_create_rs({n},{k})")
        return cls(0, 0, 0, 0, 0, _h=h)

    @classmethod
    def ccsds(cls, k, dual=True, device=0):
        h = _vp()
        _check(lib().ezrs_create_ccsds(C.byref(h), k, int(bool(dual)), device), "ezrs_create_ccsds")
        return cls(0, 0, 0, 0, 0, _h=h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().ezrs_destroy(h)
            except Exception:
                pass
            self._h = None

    def __repr__(self):
        i = self.info
        kind = ("RS_CCSDS" if i.dual else "RS_CCSDS_CONV") if i.poly == 0x187 else "RS"
        return f"{kind}({i.size},{i.load})"

    @property
    def torch_dtype(self):
        import torch
        return torch.uint8 if self.dtype == np.uint8 else torch.uint16

    @property
    def kernel_path(self):
        """'generic' | 'bitslice' | 'planeslice' | 'wide' (ezrs_kernel_path)."""
        return ("generic", "bitslice", "planeslice", "wide")[_check(lib().ezrs_kernel_path(self._h),
                                                                      "ezrs_kernel_path")]

    @property
    def semantics(self):
        """'ezpwd' (decode_symbols, the default) or 'karn' (libfec decode_rs_*: full-NN-frame
        erasures and positions, none of ezpwd's extra failure checks) -- ezrs_set_semantics."""
        return ("ezpwd", "karn")[_check(lib().ezrs_get_semantics(self._h), "ezrs_get_semantics")]

    @semantics.setter
    def semantics(self, mode):
        _check(lib().ezrs_set_semantics(self._h, {"ezpwd": 0, "karn": 1}[mode]), "ezrs_set_semantics")

    def set_launch_rows(self, rows):
        """Test hook (ezrs_set_launch_rows): cap the codewords one plane-sliced launch of this codec
        takes; 0 = the default.  Results never depend on it."""
        _check(lib().ezrs_set_launch_rows(self._h, int(rows)), "ezrs_set_launch_rows")

    def reserve(self, ncw, stream=None):
        """Pre-size the workspace of `stream` (default: the current torch stream)."""
        _check(lib().ezrs_reserve_stream(self._h, ncw, _stream_ptr(stream)), "ezrs_reserve_stream")

    def workspace_bytes(self, ncw):
        return int(lib().ezrs_workspace_bytes(self._h, ncw))

    # -- device batch forms ------------------------------------------------------------------
    def encode(self, data, length=None, parity=None, stream=None):
        """data: [ncw, stride] device tensor; parity: [ncw, >=nroots] tensor, or None: each row
        carries its parity in columns length..length+nroots (ezrs_encode_rows)."""
        w = self.info.datum_bytes
        ncw = data.shape[0]
        ds = _dev_rows(data, "data", self.device, w)
        ps = _dev_rows(parity, "parity", self.device, w)
        length = data.shape[1] - self.nroots if length is None else length
        if parity is None:
            _check(lib().ezrs_encode_rows(self._h, _tp(data), ds, length, ncw, _stream_ptr(stream)),
                   "ezrs_encode_rows")
        else:
            _check(lib().ezrs_encode(self._h, _tp(data), ds, length, _tp(parity), ps, ncw,
                                     _stream_ptr(stream)), "ezrs_encode")

    def decode(self, data, length=None, parity=None, eras=None, neras=None, result=None,
               positions=None, corr=None, stream=None):
        """In-place batch decode; returns the int32 result tensor."""
        import torch
        w = self.info.datum_bytes
        ncw = data.shape[0]
        ds = _dev_rows(data, "data", self.device, w)
        ps = _dev_rows(parity, "parity", self.device, w)
        es = _dev_rows(eras, "eras", self.device, 4)
        _dev_rows(neras, "neras", self.device, 4, ndim=1)
        qs = _dev_rows(positions, "positions", self.device, 4)
        cs = _dev_rows(corr, "corr", self.device, w)
        length = data.shape[1] - self.nroots if length is None else length
        if result is None:
            result = torch.empty(ncw, dtype=torch.int32, device=data.device)
        _dev_rows(result, "result", self.device, 4, ndim=1)
        _check(lib().ezrs_decode(
            self._h, _tp(data), ds, length, _tp(parity), ps, _tp(eras), es, _tp(neras),
            _tp(result), _tp(positions), qs, _tp(corr), cs, ncw, _stream_ptr(stream)),
            "ezrs_decode")
        return result

    # -- shard batches (rsencode layout per shard) --------------------------------------------
    def shard_codewords(self, shard_len, chunk=None):
        """Codewords per shard of shard_len data symbols cut into chunks (default: the load)."""
        return int(lib().ezrs_shard_codewords(self._h, shard_len, chunk or self.load))

    def shard_encoded_len(self, shard_len, chunk=None):
        return int(lib().ezrs_shard_encoded_len(self._h, shard_len, chunk or self.load))

    def encode_shards(self, shards, shard_len, chunk=None, stream=None):
        """shards: [nshards, pitch] device tensor, each row one shard in the rsencode layout
        (chunks of `chunk` data symbols, each followed by its parity; the last chunk shorter);
        writes every codeword's parity (ezrs_encode_shards)."""
        w = self.info.datum_bytes
        sp = _dev_rows(shards, "shards", self.device, w)
        _check(lib().ezrs_encode_shards(self._h, _tp(shards), sp, shard_len, chunk or self.load,
                                        shards.shape[0], _stream_ptr(stream)), "ezrs_encode_shards")

    def decode_shards(self, shards, shard_len, chunk=None, eras=None, neras=None, result=None,
                      positions=None, corr=None, stream=None):
        """In-place decode of every codeword of every shard; returns the int32 result tensor
        [nshards * codewords per shard] (shard-major)."""
        import torch
        w = self.info.datum_bytes
        chunk = chunk or self.load
        sp = _dev_rows(shards, "shards", self.device, w)
        es = _dev_rows(eras, "eras", self.device, 4)
        _dev_rows(neras, "neras", self.device, 4, ndim=1)
        qs = _dev_rows(positions, "positions", self.device, 4)
        cs = _dev_rows(corr, "corr", self.device, w)
        ncw = shards.shape[0] * self.shard_codewords(shard_len, chunk)
        if result is None:
            result = torch.empty(ncw, dtype=torch.int32, device=shards.device)
        _dev_rows(result, "result", self.device, 4, ndim=1)
        _check(lib().ezrs_decode_shards(
            self._h, _tp(shards), sp, shard_len, chunk, shards.shape[0], _tp(eras), es, _tp(neras),
            _tp(result), _tp(positions), qs, _tp(corr), cs, _stream_ptr(stream)), "ezrs_decode_shards")
        return result

    # -- host batch forms ----------------------------------------------------------------------
    def encode_host(self, data, length=None, parity=None, chunk=0):
        """data: [ncw, stride] numpy rows (only read); parity: [ncw, >=nroots] array, or None:
        each row carries its parity after its data (ezrs_encode_rows_host)."""
        w = self.info.datum_bytes
        ncw = data.shape[0]
        ds = _host_rows(data, "data", w)
        ps = _host_rows(parity, "parity", w)
        length = data.shape[1] - self.nroots if length is None else length
        if parity is None:
            _check(lib().ezrs_encode_rows_host(self._h, _np(data), ds, length, ncw, chunk),
                   "ezrs_encode_rows_host")
        else:
            _check(lib().ezrs_encode_host(self._h, _np(data), ds, length, _np(parity), ps, ncw,
                                          chunk), "ezrs_encode_host")

    def decode_host(self, data, length=None, parity=None, eras=None, neras=None,
                    positions=None, corr=None, chunk=0):
        w = self.info.datum_bytes
        ncw = data.shape[0]
        ds = _host_rows(data, "data", w)
        ps = _host_rows(parity, "parity", w)
        es = _host_rows(eras, "eras", 4)
        _host_rows(neras, "neras", 4, ndim=1)
        qs = _host_rows(positions, "positions", 4)
        cs = _host_rows(corr, "corr", w)
        length = data.shape[1] - self.nroots if length is None else length
        result = np.zeros(ncw, np.int32)
        _check(lib().ezrs_decode_host(
            self._h, _np(data), ds, length, _np(parity), ps, _np(eras), es, _np(neras),
            _np(result), _np(positions), qs, _np(corr), cs, ncw, chunk), "ezrs_decode_host")
        return result


    # -- rsencode wire format -------------------------------------------------------------------
    def stream_encode(self, data, chunk=128):
        """bytes -> rsencode-format bytes (each chunk followed by its parity; include/ezrs.h
        ezrs_stream_encode).  Returns (encoded, ok); ok is False when a trailing partial symbol
        stopped the stream (the whole chunks before it are encoded, as rsencode does)."""
        src = np.frombuffer(bytes(data), np.uint8)
        cap = int(lib().ezrs_stream_encoded_bound(self._h, src.size, chunk)) or 1
        out = np.zeros(cap, np.uint8)
        n = _sz(0)
        rc = lib().ezrs_stream_encode(self._h, _np(src) if src.size else None, src.size, chunk,
                                      _np(out), cap, C.byref(n))
        if rc not in (0, -errno.EMSGSIZE):
            _check(rc, "ezrs_stream_encode")
        return out[:n.value].tobytes(), rc == 0

    def stream_decode(self, data, chunk=128):
        """rsencode-format bytes -> (decoded bytes, chunks that failed to decode, ok)."""
        src = np.frombuffer(bytes(data), np.uint8)
        out = np.zeros(max(src.size, 1), np.uint8)
        n, nf = _sz(0), _sz(0)
        rc = lib().ezrs_stream_decode(self._h, _np(src) if src.size else None, src.size, chunk,
                                      _np(out), out.size, C.byref(n), C.byref(nf))
        if rc not in (0, -errno.EMSGSIZE):
            _check(rc, "ezrs_stream_decode")
        return out[:n.value].tobytes(), nf.value, rc == 0


class BCH:
    """A binary BCH codec resident on one HIP device: ezpwd::bch_base(m, t, prim_poly) /
    ezpwd::BCH<N,K,T> (c++/ezpwd/bch:48-463) over include/ezbch.h.

    * ``encode(data, length, ecc)`` -- bch_base::encode(data, len, parity) per row (bch:196-205)
    * ``decode(data, length, ecc)`` -- bch_base::decode(data, len, parity, &position), i.e.
      correct_bch (bch:316-331, bch_base:168-199): int32 result per row, bits fixed in place."""

    def __init__(self, m, t, prim_poly=0, device=0, _h=None):
        h = _vp()
        if _h is None:
            _check(lib().ezbch_create(C.byref(h), m, t, prim_poly, device), "ezbch_create", True)
        else:
            h = _h
        self._h = h
        info = BCHInfo()
        _check(lib().ezbch_get_info(self._h, C.byref(info)), "ezbch_get_info", True)
        self.info = info
        self.m, self.n, self.t, self.ecc_bits, self.ecc_bytes = (info.m, info.n, info.t,
                                                                 info.ecc_bits, info.ecc_bytes)
        self.device = info.device

    @classmethod
    def nkt(cls, n, k, t, device=0):
        h = _vp()
        _check(lib().ezbch_create_nkt(C.byref(h), n, k, t, device), f"ezbch_create_nkt({n},{k},{t})",
               True)
        return cls(0, 0, _h=h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().ezbch_destroy(h)
            except Exception:
                pass
            self._h = None

    def __repr__(self):   # bch_base:204-215
        return f"BCH({self.n},{self.n - self.ecc_bits},{self.t})"

    @property
    def max_len(self):
        return (self.n - self.ecc_bits) // 8

    def encode(self, data, length=None, ecc=None, stream=None):
        """data: [ncw, stride] uint8 device tensor; ecc: [ncw, >=ecc_bytes] tensor, or None: the ECC
        goes to columns length..length+ecc_bytes of each row (ezbch_encode_rows)."""
        ncw = data.shape[0]
        ds = _dev_rows(data, "data", self.device, 1)
        es = _dev_rows(ecc, "ecc", self.device, 1)
        length = data.shape[1] - self.ecc_bytes if length is None else length
        if ecc is None:
            _check(lib().ezbch_encode_rows(self._h, _tp(data), ds, length, ncw, _stream_ptr(stream)),
                   "ezbch_encode_rows", True)
        else:
            _check(lib().ezbch_encode(self._h, _tp(data), ds, length, _tp(ecc), es, ncw,
                                      _stream_ptr(stream)), "ezbch_encode", True)

    def decode(self, data, length=None, ecc=None, result=None, errloc=None, stream=None):
        import torch
        ncw = data.shape[0]
        ds = _dev_rows(data, "data", self.device, 1)
        es = _dev_rows(ecc, "ecc", self.device, 1)
        ls = _dev_rows(errloc, "errloc", self.device, 4)
        length = data.shape[1] - self.ecc_bytes if length is None else length
        if result is None:
            result = torch.empty(ncw, dtype=torch.int32, device=data.device)
        _dev_rows(result, "result", self.device, 4, ndim=1)
        _check(lib().ezbch_decode(self._h, _tp(data), ds, length, _tp(ecc), es, _tp(result),
                                  _tp(errloc), ls, ncw, _stream_ptr(stream)), "ezbch_decode", True)
        return result

    def decode_ecc(self, ecc, length, result=None, errloc=None, stream=None):
        """decode_bch's recv XOR calc form: ecc rows hold the ECC differences; returns the int32
        results (errors found, or a negative errno); nothing is corrected (ezbch_decode_ecc)."""
        import torch
        ncw = ecc.shape[0]
        es = _dev_rows(ecc, "ecc", self.device, 1)
        ls = _dev_rows(errloc, "errloc", self.device, 4)
        if result is None:
            result = torch.empty(ncw, dtype=torch.int32, device=ecc.device)
        _dev_rows(result, "result", self.device, 4, ndim=1)
        _check(lib().ezbch_decode_ecc(self._h, _tp(ecc), es, length, _tp(result), _tp(errloc), ls,
                                      ncw, _stream_ptr(stream)), "ezbch_decode_ecc", True)
        return result

    def decode_syn(self, syn, length, result=None, errloc=None, stream=None):
        """decode_bch's syndrome form: syn rows hold S_1..S_2t (int32/uint32, 2t per row); returns
        the int32 results; nothing is corrected (ezbch_decode_syn)."""
        import torch
        ncw = syn.shape[0]
        ss = _dev_rows(syn, "syn", self.device, 4)
        ls = _dev_rows(errloc, "errloc", self.device, 4)
        if result is None:
            result = torch.empty(ncw, dtype=torch.int32, device=syn.device)
        _dev_rows(result, "result", self.device, 4, ndim=1)
        _check(lib().ezbch_decode_syn(self._h, _tp(syn), ss, length, _tp(result), _tp(errloc), ls,
                                      ncw, _stream_ptr(stream)), "ezbch_decode_syn", True)
        return result

    def encode_host(self, data, length=None, ecc=None, chunk=0):
        ncw = data.shape[0]
        ds = _host_rows(data, "data", 1)
        es = _host_rows(ecc, "ecc", 1)
        length = data.shape[1] - self.ecc_bytes if length is None else length
        if ecc is None:
            _check(lib().ezbch_encode_rows_host(self._h, _np(data), ds, length, ncw, chunk),
                   "ezbch_encode_rows_host", True)
        else:
            _check(lib().ezbch_encode_host(self._h, _np(data), ds, length, _np(ecc), es, ncw, chunk),
                   "ezbch_encode_host", True)

    def decode_host(self, data, length=None, ecc=None, errloc=None, chunk=0):
        ncw = data.shape[0]
        ds = _host_rows(data, "data", 1)
        es = _host_rows(ecc, "ecc", 1)
        ls = _host_rows(errloc, "errloc", 4)
        length = data.shape[1] - self.ecc_bytes if length is None else length
        result = np.zeros(ncw, np.int32)
        _check(lib().ezbch_decode_host(self._h, _np(data), ds, length, _np(ecc), es, _np(result),
                                       _np(errloc), ls, ncw, chunk), "ezbch_decode_host", True)
        return result


def exported_symbols():
    """Function names declared in include/ezrs.h and include/ezbch.h."""
    import re
    names = set()
    for fn in (HEADER, BCH_HEADER):
        txt = open(fn).read()
        names |= set(re.findall(
            r"^\s*(?:int|void|const char \*|size_t)\s*\*?\s*(ez(?:rs|bch)_\w+)\s*\(", txt, re.M))
    return sorted(names)
