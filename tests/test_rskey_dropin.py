"""The reference's rskey / rspwd password correctors (c++/ezpwd/corrector over ezpwd::RS<31,..> and
RS<63,..>; rskey.C, rspwd.C) built UNCHANGED against this repository's include/ -- the forwarding
header include/ezpwd/corrector defuses corrector's sibling `#include "rs"` (its guard _EZPWD_RS,
c++/ezpwd/rs:16-17) so every codec call runs on the GPU.  The programs are the reference's own
self-checking tests: rskey_test.C asserts the known encodings ("000G4-0YYYU-XYQWE", ...) and the
strength<> confidences 100 / 50 / 60 (rskey_test.C:77-130), rspwd_test.C round trips with 1..5
parity symbols; both print "...all tests passed." only when every assertion holds."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "_bin")
LIBDIR = os.path.join(ROOT, "ezpwd-reed-solomon_amd", "lib")
REF = "/root/reference"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "rskey.C")), reason="reference tree absent")
@pytest.mark.parametrize("name", ["rskey", "rspwd"])
def test_corrector_sources_build_unchanged(tmp_path, name):
    """rskey.C / rspwd.C (the C APIs over ezpwd::corrector) compile with only the include path
    switched to this repository's include/ (first) and the reference's c++/ (second)."""
    if not os.path.exists(os.path.join(LIBDIR, "libezrs_hip.so")):
        pytest.skip("libezrs_hip.so not built")
    cmd = ["g++", "-std=c++17", "-O1", "-w", "-c", "-I", os.path.join(ROOT, "include"), "-I",
           os.path.join(REF, "c++"), "-I", REF, os.path.join(REF, name + ".C"), "-o",
           str(tmp_path / (name + ".o"))]
    subprocess.run(cmd, check=True, capture_output=True, text=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rskey_test", "rspwd_test"])
def test_reference_corrector_tests_pass_on_gpu(name):
    exe = os.path.join(BIN, name)
    if not os.path.exists(exe):
        pytest.skip(f"{name} not built (needs /root/reference at build time)")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert "...all tests passed." in p.stdout, p.stdout[-3000:]
    assert "FAILURE" not in p.stdout, p.stdout[-3000:]
