"""The committed straight-line kernel tables (csrc/gen/*.inc) are exactly what codegen/ produces:
each generator is re-run into a scratch file and the bytes compared, so a generator change that is
not regenerated (or a hand edit of a generated file) fails here, on the CPU."""
import filecmp
import importlib.util
import os

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CODEGEN = os.path.join(ROOT, "ezpwd-reed-solomon_amd", "codegen")
GEN = os.path.join(ROOT, "ezpwd-reed-solomon_amd", "csrc", "gen")


def _load(name):
    spec = importlib.util.spec_from_file_location(f"_codegen_{name}", os.path.join(CODEGEN, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    import sys
    sys.path.insert(0, CODEGEN)
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(CODEGEN)
    return mod


@pytest.mark.parametrize("gen,inc", [("gen_bitslice", "ezrs_bs_tables.inc"),
                                     ("gen_ps", "ezrs_ps_tables.inc"),
                                     ("gen_wide", "ezrs_wide_tables.inc")])
def test_generated_tables_are_reproduced(tmp_path, gen, inc):
    dst = str(tmp_path / inc)
    _load(gen).main(dst)
    assert filecmp.cmp(dst, os.path.join(GEN, inc), shallow=False), \
        f"csrc/gen/{inc} differs from codegen/{gen}.py's output: regenerate it"
