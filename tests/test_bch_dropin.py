"""The C++ BCH drop-in (include/ezpwd_amd/bch, forwarded by include/ezpwd/bch): the reference's own
BCH programs build UNCHANGED against it -- bchsimple.C (ezpwd::BCH<255,239,2> container API),
bchclassic.C (the classic init_bch / encode_bch / correct_bch API) and bch_test.C (init_bch
enumeration) -- and, on a GPU, run to "All tests passed."."""
import os
import re
import subprocess

import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "ezpwd-reed-solomon_amd", "lib")
REF = "/root/reference"


def _build(tmp_path, name):
    out = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(REF, "c++"), os.path.join(REF, name + ".C"), "-L", LIBDIR,
           "-lezrs_hip", f"-Wl,-rpath,{LIBDIR}", "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


needs_ref = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "bchsimple.C")),
                               reason="reference tree absent")
needs_lib = pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libezrs_hip.so")),
                               reason="libezrs_hip.so not built")


@needs_ref
@needs_lib
def test_reference_bch_programs_build_unchanged(tmp_path):
    for name in ("bchsimple", "bchclassic", "bch_test"):
        _build(tmp_path, name)


@needs_ref
@needs_lib
def test_bch_test_enumeration_matches(tmp_path):
    """bch_test.C's init_bch enumeration (host side of the drop-in): every BCH(N, K, T) line and
    its ECC bits/bytes equal the restatement's codec, and the BCH(255,k,t) rows equal the table the
    reference records in swig/python/BCH/BCH.i:83-90."""
    exe = _build(tmp_path, "bch_test")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    rows = re.findall(r"BCH\(\s*(\d+),\s*(\d+),\s*(\d+) \); ECC =\s*(\d+) /\s*(\d+)", p.stdout)
    assert len(rows) > 40
    for n, k, t, bits, nbytes in rows:
        n, k, t, bits, nbytes = map(int, (n, k, t, bits, nbytes))
        m = (n + 1).bit_length() - 1
        c = O.BCH(m, t)
        assert (c.n, c.ecc_bits, c.ecc_bytes) == (n, bits, nbytes) and n - bits == k
    with open(os.path.join(REF, "swig/python/BCH/BCH.i")) as f:
        recorded = re.findall(r"// (BCH\( 255,.*)", f.read())
    got = [l for l in p.stdout.splitlines() if l.startswith("BCH( 255,")]
    assert recorded and got[:len(recorded)] == recorded
    if not os.path.exists("/dev/kfd"):
        assert p.returncode != 0                     # BCH<255,239,2> needs the GPU: fails loudly


@pytest.mark.gpu
@needs_lib
@pytest.mark.parametrize("name", ["bchsimple", "bchclassic"])
def test_reference_bch_programs_pass_on_gpu(tmp_path, name):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    prebuilt = os.path.join(ROOT, "tests", "cpp", "_bin", name)
    exe = prebuilt if os.path.exists(prebuilt) else _build(tmp_path, name)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "All tests passed." in p.stdout, p.stdout[-3000:]
