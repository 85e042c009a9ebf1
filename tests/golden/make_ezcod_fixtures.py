"""Generate tests/golden/ezcod_ref.txt FROM THE REFERENCE'S OWN ezcod.C.

    make -C oracle ezcod && python tests/golden/make_ezcod_fixtures.py

oracle/_ref/ezcod_ref is tests/cpp/ezcod_driver.cpp linked with the reference's ezcod.C compiled
against the reference's unmodified headers; its output (ezcod 3:10/3:11/3:12 encodings of 120
positions each, and decodes of each with 0-3 corrupted characters) is the fixture.  Data only.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
out = subprocess.run([os.path.join(HERE, "..", "..", "oracle", "_ref", "ezcod_ref")],
                     capture_output=True, text=True, check=True, timeout=120).stdout
with open(os.path.join(HERE, "ezcod_ref.txt"), "w") as f:
    f.write(out)
print(len(out.splitlines()), "lines")
