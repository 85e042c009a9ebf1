"""The reference's own RS harnesses, compiled unchanged against the drop-in (tests/cpp/harness.mk,
built by __graft_entry__.build()), run on the GPU:

  rsexercise  rsexercise.C + exercise.H: 12 codecs (RS(255,K), RS_CCSDS, RS_CCSDS_CONV, RS<511>,
              RS<1023>, RS<65535,65503>, RS<65535,65279>) through the 7-parameter reed_solomon type;
              no decoder errors (exercise.H:212-245 prints one line per error)
  rsvalidate  rsvalidate.C: 10 000 trials over 17 codecs held as ezpwd::reed_solomon_base, parity and
              decode cross-checked against Phil Karn's CPU libfec; zero failures (rsvalidate.C:382-385)
  rsspeed     rsspeed.C: the same pairing on 11 codecs, asserting identical corrections
  rstest      phil-karn/rstest.c + exercise.c linked against libezrs_fec.so: Karn's ABI over the
              engine; every Tab row prints OK and the run ends "All codec tests passed!".
              exercise.c is built with the reference's own -DDEBUG=1 knob (exercise.c:136-138),
              which runs 10 trials per (pad, load) class instead of rstest.c's Tab counts (up to
              100 000): each trial is a single-codeword call, a PCIe round trip through the GPU.
              This run is therefore a thin check of the ABI; the bulk of the Karn-mode coverage is
              the batch-form fixture test tests/test_karn_abi_gpu.py (libfec's own outputs over
              shortened codewords, pad erasures, loads to 1.6x the parity, every Tab symbol size).
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "_bin")


def _run(name, timeout):
    exe = os.path.join(BIN, name)
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built (needs /root/reference at build time)")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def test_rsexercise():
    rc, out = _run("rsexercise", 240)
    assert rc == 0, out[-3000:]
    bad = [ln for ln in out.splitlines()
           if "decoder says" in ln or "without error" in ln or "uncorrected errors" in ln]
    assert not bad, "\n".join(bad[:20])
    for codec in ("RS(255,253)", "RS(255,223)", "RS_CCSDS(255,223)", "RS_CCSDS_CONV(255,223)",
                  "RS(511,479)", "RS(1023,991)", "RS(65535,65503)", "RS(65535,65279)"):
        assert f"{codec} Enc/Decoding" in out, codec


def test_rsvalidate():
    rc, out = _run("rsvalidate", 600)
    assert rc == 0, out[-4000:]
    assert "parity-(era+2*err)" in out


def test_rsspeed():
    rc, out = _run("rsspeed", 300)
    assert rc == 0, out[-3000:]
    assert out.count("(EZPWD's)") == 11 and "different results" not in out


def test_rstest_karn_abi():
    rc, out = _run("rstest", 600)
    assert rc == 0, out[-3000:]
    lines = out.splitlines()
    # exercise.c's DEBUG=1 trial lines follow each "Testing ..." header; every codec then prints a
    # line "OK" (rstest.c:77-79, 84-86, 111-113)
    assert any(ln.startswith("Testing fixed (255,223) RS codec...") for ln in lines)
    assert any(ln.startswith("Testing CCSDS standard (255,223) RS codec...") for ln in lines)
    tested = [ln for ln in lines if ln.startswith("Testing (")]
    assert len(tested) == 24, tested
    assert sum(ln == "OK" for ln in lines) == 26, [ln for ln in lines if "OK" in ln][:30]
    bad = [ln for ln in lines if "decoder says" in ln or "without error" in ln or "uncorrected" in ln
           or "failed" in ln]
    assert not bad, "\n".join(bad[:20])
    assert "All codec tests passed!" in lines
