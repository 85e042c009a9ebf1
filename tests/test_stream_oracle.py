"""The rsencode wire format (rsencode.C:52-163) restated over the oracle, against the streams the
reference's own rsencode produced (tests/golden/stream_rsencode.npz): chunking, big-endian 16-bit
serialization, parity placement, in-place partial corrections of chunks that fail to decode, and
the two 'Insufficient data' stops.  CPU only."""
import numpy as np
import pytest

import oracle as O
from stream_util import case_ids, cases


def _syms(b, w):
    a = np.frombuffer(b, np.uint8)
    if w == 1:
        return a.copy()
    return (a[0::2].astype(np.uint16) << 8) | a[1::2]


def _bytes(s, w):
    if w == 1:
        return np.asarray(s, np.uint8).tobytes()
    s = np.asarray(s, np.uint16)
    return np.stack([(s >> 8).astype(np.uint8), (s & 0xFF).astype(np.uint8)], 1).tobytes()


def restate_encode(oc, data, chunk, w):
    out, cb = b"", chunk * w
    for off in range(0, len(data), cb):
        piece = data[off:off + cb]
        if len(piece) % w:
            return out, 1                                  # rsencode.C:110-111
        d = _syms(piece, w)
        _, par = oc.encode(d)
        out += piece + _bytes(par, w)
    return out, 0


def restate_decode(oc, enc, chunk, w):
    out, row, nr = b"", (chunk + oc.nroots) * w, oc.nroots
    for off in range(0, len(enc), row):
        piece = enc[off:off + row]
        if len(piece) < (nr + 1) * w or len(piece) % w:
            return out, 1                                  # rsencode.C:140-141
        s = _syms(piece, w)
        d, p = s[:-nr].copy(), s[-nr:].copy()
        oc.decode(d, p)
        out += _bytes(d, w)
    return out, 0


@pytest.mark.parametrize("case", cases(), ids=case_ids())
def test_wire_format_restatement(case):
    n, nr = case["codeword"], case["parity"]
    oc = O.Codec(*O.rs_params(n, n - nr))
    w = 2 if n > 255 else 1
    enc, erc = restate_encode(oc, case["in"], case["chunk"], w)
    assert (enc, erc) == (case["enc"], case["enc_rc"])
    dec, drc = restate_decode(oc, case["bad"], case["chunk"], w)
    assert drc == case["dec_rc"]
    assert dec == case["dec"]
