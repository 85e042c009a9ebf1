"""The C++ drop-in header (include/ezpwd_amd/rs, the ezpwd::RS<N,K> call surface of c++/ezpwd/rs and
rs_base) -- compiled with g++ against libezrs_hip.so.  CPU: it builds, links, and fails loudly
(constructor throws, exit 3) when no GPU is usable.  GPU: every record tests/cpp/rs_dropin.cpp prints
(string / vector / array / pair / pointer overloads, erasure + position vectors) matches the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "ezpwd-reed-solomon_amd", "lib")
SRC = os.path.join(ROOT, "tests", "cpp", "rs_dropin.cpp")

CODECS = {"RS255_223": O.rs_params(255, 223), "RS31_27": O.rs_params(31, 27),
          "RS1023_1007": O.rs_params(1023, 1007), "CCSDS255_223": O.ccsds_params(223, True)}


def _build(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libezrs_hip.so")):
        pytest.skip("libezrs_hip.so not built")
    exe = str(tmp_path / "rs_dropin")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
           "-L", LIBDIR, "-lezrs_hip", f"-Wl,-rpath,{LIBDIR}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_header_builds_and_fails_loudly_without_gpu(tmp_path):
    exe = _build(tmp_path)
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present; covered by the gpu test")
    p = subprocess.run([exe, "1"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, p.stdout + p.stderr
    lines = p.stdout.splitlines()
    # codec objects construct without a GPU (the GPU codec is created lazily, so a static codec
    # costs nothing at start-up); the first call fails loudly
    assert lines[0].startswith("# RS(255,223)"), p.stdout
    assert lines[1].startswith("NODEV"), p.stdout


REF_RSENCODE = "/root/reference/rsencode.C"


def build_reference_rsencode(out, extra=()):
    """Compile the reference's own rsencode.C, UNCHANGED, against this repository's drop-in: the
    include path puts include/ (whose ezpwd/rs forwards to ezpwd_amd/rs) before the reference's
    c++/ directory, which still supplies <ezpwd/output>.  Returns the executable path."""
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", *extra, "-I", os.path.join(ROOT, "include"),
           "-I", "/root/reference/c++", REF_RSENCODE, "-L", LIBDIR, "-lezrs_hip",
           f"-Wl,-rpath,{LIBDIR}", "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


@pytest.mark.skipif(not os.path.exists(REF_RSENCODE), reason="reference tree absent")
def test_reference_rsencode_builds_unchanged(tmp_path):
    """rsencode.C:93-163 uses RS_t::symbol_t, rs.NROOTS, rs.SYMBOL and the string / vector
    encode/decode overloads: it must compile against the drop-in with only the include path
    switched, for 8- and 16-bit symbols (GNUmakefile's rsencode / rsencode_16)."""
    if not os.path.exists(os.path.join(LIBDIR, "libezrs_hip.so")):
        pytest.skip("libezrs_hip.so not built")
    exe = build_reference_rsencode(str(tmp_path / "rsencode"))
    build_reference_rsencode(str(tmp_path / "rsencode_16"),
                             ("-DRSCODEWORD=65535", "-DRSPARITY=64"))
    if not os.path.exists("/dev/kfd"):
        p = subprocess.run([exe], input=b"abcd\n", capture_output=True, timeout=60)
        assert p.returncode == 1 and b"cannot create codec on the GPU" in p.stderr


def _parse(line):
    f = line.split()
    rec = {"name": f[1]}
    for kv in f[2:]:
        k, v = kv.split("=", 1)
        rec[k] = int(v) if k in ("len", "r") else [int(x, 16) for x in v.split(",") if x]
    return rec


@pytest.mark.gpu
def test_dropin_matches_oracle(tmp_path):
    exe = _build(tmp_path)
    p = subprocess.run([exe, "12"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    recs = [_parse(l) for l in p.stdout.splitlines() if l.startswith("REC ")]
    assert len(recs) == 48
    for rec in recs:
        oc = O.Codec(*CODECS[rec["name"]])
        L = rec["len"]
        data = np.array(rec["data"], oc.dtype)
        _, par = oc.encode(data)
        assert list(par) == rec["parity"], rec["name"]
        bad = np.array(rec["bad"], oc.dtype)
        d, q = bad[:L].copy(), bad[L:].copy()
        r, pos = oc.decode(d, q, rec["eras"])
        assert r == rec["r"], rec
        assert list(np.concatenate([d, q])) == rec["fixed"], rec["name"]
        assert list(pos) == rec["pos"], rec
