"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every function that
include/ezrs.h declares, and rejects invalid codecs without touching a GPU."""
import ctypes as C
import errno
import os
import subprocess

import pytest

import ezrs


def test_library_exports_every_declared_symbol():
    L = ezrs.lib()
    declared = ezrs.exported_symbols()
    assert len(declared) >= 24
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", ezrs.LIB_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(declared) <= exported


def test_abi_version():
    assert ezrs.lib().ezrs_abi_version() == 5


def test_invalid_codecs_rejected_before_device():
    L = ezrs.lib()
    h = C.c_void_p()
    assert L.ezrs_create(C.byref(h), 8, 0x11d, 1, 1, 0, 0, 0) == -errno.EINVAL
    assert L.ezrs_create(C.byref(h), 8, 0x101, 1, 1, 32, 0, 0) == -errno.EINVAL
    assert L.ezrs_create(C.byref(h), 10, 0x409, 1, 1, 32, 1, 0) == -errno.EINVAL
    assert L.ezrs_create_rs(C.byref(h), 256, 223, 0) == -errno.EINVAL
    assert L.ezrs_create_ccsds(C.byref(h), 224, 1, 0) == -errno.EINVAL
    # wide symbols: at most 256 parity symbols (engine limit), rejected before any device work
    assert L.ezrs_create(C.byref(h), 10, 0x409, 1, 1, 257, 0, 0) == -errno.ENOTSUP
    assert L.ezrs_create_rs(C.byref(h), 65535, 65000, 0) == -errno.ENOTSUP
    assert not h.value


def test_null_codec_calls_are_einval():
    L = ezrs.lib()
    assert L.ezrs_encode(None, None, 0, 1, None, 0, 1, None) == -errno.EINVAL
    assert L.ezrs_encode_rows(None, None, 0, 1, 1, None) == -errno.EINVAL
    assert L.ezrs_encode_ws(None, None, 0, 1, None, 0, 1, None, 0, None) == -errno.EINVAL
    assert L.ezrs_decode_ws(None, None, 0, 1, None, 0, None, 0, None, None, None, 0, None, 0, 1,
                            None, 0, None) == -errno.EINVAL
    assert L.ezrs_encode_host(None, None, 0, 1, None, 0, 1, 0) == -errno.EINVAL
    assert L.ezrs_encode_rows_host(None, None, 0, 1, 1, 0) == -errno.EINVAL
    assert L.ezrs_reserve_stream(None, 1, None) == -errno.EINVAL
    assert L.ezrs_workspace_bytes(None, 1) == 0
    assert L.ezrs_decode(None, None, 0, 1, None, 0, None, 0, None, None, None, 0, None, 0, 1,
                         None) == -errno.EINVAL
    assert L.ezrs_destroy(None) == 0


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and
                    os.path.exists("/dev/kfd"), reason="a GPU is visible here")
def test_no_device_reports_enodev():
    L = ezrs.lib()
    h = C.c_void_p()
    rc = L.ezrs_create_rs(C.byref(h), 255, 223, 0)
    assert rc == -errno.ENODEV
    with pytest.raises(ezrs.EzrsError):
        ezrs.Codec.rs(255, 223)


def test_bch_invalid_codecs_rejected_before_device():
    L = ezrs.lib()
    h = C.c_void_p()
    assert L.ezbch_create(C.byref(h), 4, 1, 0, 0) == -errno.EINVAL          # m < 5
    assert L.ezbch_create(C.byref(h), 5, 7, 0, 0) == -errno.EINVAL          # m*t >= n
    assert L.ezbch_create(C.byref(h), 8, 2, 0x101, 0) == -errno.EINVAL      # not primitive
    assert L.ezbch_create_nkt(C.byref(h), 255, 240, 2, 0) == -errno.EINVAL  # BCH<255,240,2> mismatch
    assert L.ezbch_create_nkt(C.byref(h), 254, 239, 2, 0) == -errno.EINVAL
    assert not h.value
    assert L.ezbch_destroy(None) == 0
    assert L.ezbch_encode(None, None, 0, 1, None, 0, 1, None) == -errno.EINVAL


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and
                    os.path.exists("/dev/kfd"), reason="a GPU is visible here")
def test_bch_no_device_reports_enodev():
    L = ezrs.lib()
    h = C.c_void_p()
    assert L.ezbch_create_nkt(C.byref(h), 1023, 983, 4, 0) == -errno.ENODEV
    assert L.ezbch_create(C.byref(h), 10, 65, 0, 0) == -errno.ENODEV        # valid, t > 64: wave path
    assert L.ezbch_create(C.byref(h), 15, 200, 0, 0) == -errno.ENODEV
    with pytest.raises(ezrs.EzrsError):
        ezrs.BCH(8, 2)


def test_fec_library_exports_every_declared_symbol():
    """libezrs_fec.so (Phil Karn's libfec RS ABI over the engine) exports every function that
    include/ezrs_fec.h declares (fec-3.0.1/fec.h:229-257, phil-karn/rs.h:22-23, batch forms)."""
    import re
    hdr = os.path.join(os.path.dirname(ezrs.HEADER), "ezrs_fec.h")
    txt = open(hdr).read()
    declared = set(re.findall(r"^\s*(?:int|void|void \*|ezrs_codec \*)\s*\*?\s*(\w+)\s*\(", txt, re.M))
    assert {"init_rs_char", "decode_rs_int", "encode_rs_8", "decode_rs_ccsds", "pad_rs_char",
            "decode_rs_char_batch", "ezrs_fec_codec"} <= declared
    so = os.path.join(os.path.dirname(ezrs.LIB_PATH), "libezrs_fec.so")
    out = subprocess.check_output(["nm", "-D", "--defined-only", so], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared <= exported, declared - exported


def test_fec_init_fails_without_device():
    """No GPU: init_rs_char returns NULL (Karn's failure value); invalid parameters too."""
    so = os.path.join(os.path.dirname(ezrs.LIB_PATH), "libezrs_fec.so")
    L = C.CDLL(so)
    L.init_rs_char.restype = C.c_void_p
    assert not L.init_rs_char(8, 0x11d, 1, 1, 300, 0)        # nroots >= 2^symsize
    assert not L.init_rs_char(8, 0x11d, 1, 1, 32, 223)       # pad leaves no data symbol
    assert not L.init_rs_char(9, 0x211, 1, 1, 32, 0)         # char containers hold m <= 8
