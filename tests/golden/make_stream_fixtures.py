"""Generate tests/golden/stream_rsencode.npz FROM THE REFERENCE'S OWN rsencode.

Run in the build container (where /root/reference exists):

    make -C oracle rsencode && python tests/golden/make_stream_fixtures.py

oracle/_ref/rsencode_ref (RS(255,223)) and oracle/_ref/rsencode16_ref (RS(65535,65503), 16-bit
big-endian symbols) are the reference's rsencode.C compiled from its unmodified source.  Each case
stores: the input bytes, the reference's encoded stream and exit status, a corrupted copy of that
stream (symbol errors per chunk, some chunks beyond the correction capacity), and the reference's
decoded output and exit status.  Data only: inputs and the reference's outputs.
"""
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "..", "oracle", "_ref")

# name, binary, codeword, parity, chunk, input bytes
CASES = [
    ("rs255_c128_empty", "rsencode_ref", 255, 32, 128, 0),
    ("rs255_c128_1", "rsencode_ref", 255, 32, 128, 1),
    ("rs255_c128_exact", "rsencode_ref", 255, 32, 128, 1280),
    ("rs255_c128_tail", "rsencode_ref", 255, 32, 128, 20000 + 77),
    ("rs255_c223", "rsencode_ref", 255, 32, 223, 9999),
    ("rs255_c50", "rsencode_ref", 255, 32, 50, 3001),
    ("rs65535_c128", "rsencode16_ref", 65535, 32, 128, 6000),
    ("rs65535_c1000_tail", "rsencode16_ref", 65535, 32, 1000, 2 * 3333),
    ("rs65535_odd", "rsencode16_ref", 65535, 32, 128, 601),          # encode stops: odd byte
    ("rs255_c128_trunc", "rsencode_ref", 255, 32, 128, 1000),        # 3 extra bytes join the tail
    ("rs255_c128_short_trunc", "rsencode_ref", 255, 32, 128, 1280),  # decode stops: 3-byte chunk
]


def run(exe, args, data):
    p = subprocess.run([os.path.join(REF, exe), *args], input=data, capture_output=True,
                       timeout=120)
    return p.stdout, p.returncode


def corrupt(rng, enc, codeword, parity, chunk, w):
    """Symbol errors per wire chunk: 0..parity/2 + 4 (beyond parity/2 the chunk is uncorrectable)."""
    buf = bytearray(enc)
    row = (chunk + parity) * w
    off = 0
    while off < len(buf):
        n = min(row, len(buf) - off) // w
        e = int(rng.integers(0, parity // 2 + 5))
        e = min(e, n)
        for s in rng.choice(n, e, replace=False):
            for b in range(w):
                buf[off + s * w + b] ^= int(rng.integers(0, 256))
            if all(buf[off + s * w + b] == enc[off + s * w + b] for b in range(w)):
                buf[off + s * w + w - 1] ^= 1
        off += row
    return bytes(buf)


def main():
    rng = np.random.default_rng(0x52534543)
    out, meta = {}, []
    for i, (name, exe, cw, par, chunk, nbytes) in enumerate(CASES):
        data = rng.integers(0, 256, nbytes).astype(np.uint8).tobytes()
        args = ["-c", str(chunk)]
        enc, erc = run(exe, args, data)
        w = 2 if cw > 255 else 1
        bad = corrupt(rng, enc, cw, par, chunk, w) if erc == 0 else enc
        if name.endswith("_trunc"):
            bad += bytes([1, 2, 3])              # fewer than NROOTS + 1 symbols after the chunks
        dec, drc = run(exe, ["-d", *args], bad)
        meta.append({"name": name, "codeword": cw, "parity": par, "chunk": chunk,
                     "enc_rc": erc, "dec_rc": drc})
        for k, v in (("in", data), ("enc", enc), ("bad", bad), ("dec", dec)):
            out[f"c{i}_{k}"] = np.frombuffer(v, np.uint8)
        print(f"{name}: in {len(data)} enc {len(enc)} (rc {erc}) dec {len(dec)} (rc {drc}) "
              f"restored={dec == data}")
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "stream_rsencode.npz"), **out)


if __name__ == "__main__":
    main()
