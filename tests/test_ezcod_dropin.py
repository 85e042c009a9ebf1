"""The reference's ezcod C API (ezcod.C, ezpwd::ezcod over RS<31,31-P> with 5-bit symbols in
8-bit datums: the masked path of SURVEY 8f3) built UNCHANGED against this repository's include/,
so its Reed-Solomon work runs on the GPU: encodings and decodes (0-3 corrupted characters) equal
the reference build's (tests/golden/ezcod_ref.txt, from oracle/_ref/ezcod_ref)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_bin", "ezcod_gpu")
GOLD = os.path.join(ROOT, "tests", "golden", "ezcod_ref.txt")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(EXE), reason="ezcod_gpu not built (needs /root/reference)")
def test_ezcod_on_gpu_matches_reference():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    got, exp = p.stdout.splitlines(), open(GOLD).read().splitlines()
    assert len(got) == len(exp) == 1800
    bad = [(g, e) for g, e in zip(got, exp) if g != e]
    assert not bad, bad[:5]


def test_ezcod_fixture_shape():
    lines = open(GOLD).read().splitlines()
    enc = [l for l in lines if l.startswith("E ")]
    dec = [l for l in lines if l.startswith("D ")]
    assert len(enc) == 360 and len(dec) == 4 * 360
    assert all(int(l.split()[3]) == 100 for l in dec if l.split()[2] == "0")   # clean: 100 %
