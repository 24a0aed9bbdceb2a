"""Pin the oracle (oracle/b64_oracle.c) against every fixture we hold.

The oracle restates src/base64encoder.c and src/base64decoder.c.  These
tests check it against the golden files in tests/golden/ (stdlib base64 +
the survey's observations of the compiled reference; see make_golden.py)
and against the reference test's own topology
(test/asynctest-base64encoder.c:123-151).  CPU only.
"""
import base64
import hashlib
import random

import pytest

from oracle import pyoracle as orc
from tests import util


def _case_input(c):
    if "gen" in c:
        assert c["gen"] == "splitmix64"
        return util.splitmix64(c["seed"], c["n"]).tobytes()
    return bytes.fromhex(c["in"])


def test_encode_kat():
    cases = util.golden("kat_encode.json")
    assert len(cases) > 400
    for c in cases:
        data = _case_input(c)
        got = orc.encode(data, c["pos62"], c["pos63"], c["pad"], c["padchar"])
        if "out" in c:
            assert got.hex() == c["out"], (c["mode"], len(data))
        else:
            assert len(got) == c["out_len"]
            assert hashlib.sha256(got).hexdigest() == c["out_sha256"]


def test_decode_kat():
    cases = util.golden("kat_decode.json")
    assert len(cases) > 200
    for c in cases:
        got = orc.decode(bytes.fromhex(c["in"]), c["pos62"], c["pos63"])
        assert got.hex() == c["out"], (c["mode"], c["variant"], c["in"][:40])


def test_leniency_table():
    """SURVEY.md Appendix B, observed on the compiled reference."""
    t = util.golden("leniency.json")
    for c in t["decode"]:
        got = orc.decode(bytes.fromhex(c["in"]), c["pos62"], c["pos63"])
        assert got.hex() == c["out"], c
    for c in t["encode"]:
        got = orc.encode(bytes.fromhex(c["in"]), c["pos62"], c["pos63"], c["pad"],
                         c["padchar"])
        assert got.decode() == c["out"], c


def test_digests_g1_g2_g4():
    d = util.golden("digests.json")
    g1 = orc.encode(util.counting(1000001), ".", "_", True, "-")
    assert len(g1) == d["G1"]["out_len"]
    assert hashlib.sha256(g1).hexdigest() == d["G1"]["out_sha256"]
    g2 = orc.encode(util.counting(1 << 20))
    assert hashlib.sha256(g2).hexdigest() == d["G2"]["out_sha256"]
    assert util.splitmix64(0x5EED, 16).tobytes().hex() == d["splitmix64_head"]["first16"]
    for key in ("G4_4096", "G4_1024"):
        e = orc.encode(util.splitmix64(0x5EED, d[key]["n"]))
        assert len(e) == d[key]["out_len"]
        assert hashlib.sha256(e).hexdigest().startswith(d[key]["out_sha256_prefix"])


@pytest.mark.slow
def test_digest_g3_1gib():
    d = util.golden("digests.json")["G3"]
    x = util.splitmix64(0x5EED, d["n"])
    assert hashlib.sha256(x).hexdigest() == d["in_sha256"]
    e = orc.encode(x, as_array=True)
    assert e.size == d["out_len"]
    assert hashlib.sha256(e).hexdigest() == d["out_sha256"]
    assert e[-4:].tobytes().decode() == d["out_tail"]


def test_reference_test_topology():
    """test/asynctest-base64encoder.c:123-151 restated: the 1,000,001-byte
    counting stream through nice(113) -> encode('.', '_', '-') -> nice(91)
    -> decode -> nice(97), drained 200 bytes at a time."""
    d = util.golden("digests.json")["G1"]
    enc, dec = orc.reftest(1000001)
    assert hashlib.sha256(enc).hexdigest() == d["out_sha256"]
    assert enc[:16].decode() == d["out_head"] and enc[-8:].decode() == d["out_tail"]
    assert dec == util.counting(1000001).tobytes()


@pytest.mark.parametrize("read_size", [4, 8, 12, 64, 200, 4096])
@pytest.mark.parametrize("src_chunk,burst", [(0, 0), (1, 0), (3, 0), (113, 0), (997, 50)])
def test_stream_patterns_agree(read_size, src_chunk, burst):
    """Output is independent of the read pattern inside the parity domain
    (reader counts divisible by 4, SURVEY.md §0 finding 3)."""
    rng = random.Random(read_size * 1000 + src_chunk + burst)
    for n in (0, 1, 2, 3, 5, 100, 1001):
        data = bytes(rng.randrange(256) for _ in range(n))
        for pad in (True, False):
            e = orc.encode_stream(data, src_chunk, burst, read_size, pad=pad)
            assert e == orc.encode(data, pad=pad)
            std = base64.b64encode(data)
            assert e == (std if pad else std.rstrip(b"="))
            junked = b"\r\n".join(e[i:i + 7] for i in range(0, len(e), 7))
            assert orc.decode_stream(junked, src_chunk, burst, read_size) == data


def test_assert_domain_is_detected():
    """Odd reader counts make the reference overrun the caller's buffer
    (assert at src/base64encoder.c:140); the oracle reports it."""
    data = bytes(range(256)) * 4
    with pytest.raises(orc.AssertDomain):
        orc.encode_stream(data, read_size=3)
    assert orc.encode_stream(data, read_size=8) == base64.b64encode(data)


def test_decode_table_rules():
    t = orc.decode_table()
    assert [t[c] for c in b"AZaz09+/"] == [0, 25, 26, 51, 52, 61, 62, 63]
    assert t[ord("=")] == -1 and t[ord("\n")] == -1 and t[0x80] == -1
    t = orc.decode_table(".", "_")
    assert t[ord(".")] == 62 and t[ord("_")] == 63 and t[ord("+")] == -1
    t = orc.decode_table(0xE9, 0xE8)       # signed-char comparison: never matches
    assert t[0xE9] == -1 and t[0xE8] == -1
    t = orc.decode_table("A", "*")          # the table shadows pos62
    assert t[ord("A")] == 0 and t[ord("*")] == 63
    t = orc.decode_table("*", "*")          # 62 wins
    assert t[ord("*")] == 62


def test_oracle_rows_match_stdlib():
    """The oracle's row-batch entry points (bench.py's all-core CPU
    baseline) agree with the single-buffer ones and with stdlib base64."""
    import base64

    import numpy as np

    from oracle import pyoracle

    rng = np.random.default_rng(3)
    for L in (1, 2, 3, 4, 1023, 1024, 1025):
        rows = rng.integers(0, 256, (37, L), dtype=np.uint8)
        E = (L + 2) // 3 * 4
        enc = np.zeros((37, E + 5), np.uint8)
        assert pyoracle.encode_rows(rows, enc) == 37 * E
        for i in (0, 17, 36):
            assert enc[i, :E].tobytes() == base64.b64encode(rows[i].tobytes())
        dec = np.zeros((37, (E + 3) // 4 * 3), np.uint8)
        assert pyoracle.decode_rows(np.ascontiguousarray(enc[:, :E]), dec) == 37 * L
        assert np.array_equal(dec[:, :L], rows)


def _rows_parallel(fn, src, dst, threads=8):
    """Run an oracle row function over slices of rows on `threads` threads
    (ctypes drops the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    n = src.shape[0]
    sl = [slice(i * n // threads, (i + 1) * n // threads) for i in range(threads)]
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda q: fn(src[q], dst[q]), sl))


@pytest.mark.slow
@pytest.mark.parametrize("cfg", ["cfg3", "cfg4"])
def test_batch_whole_output_digests(cfg):
    """SURVEY.md §8(d) configs 3 and 4 pinned by their whole outputs: the
    oracle (one reference encoder per buffer, read with one full read)
    reproduces tests/golden/batch_digests.json -- the digest of all
    characters, of the per-buffer digests and of every chunk -- and its
    decoder gives the input back; for config 4 also from the rows in
    CRLF-76 lines (decode digest = the input's)."""
    import numpy as np
    g = util.golden("batch_digests.json")[cfg]
    nbuf, L, E = g["nbuf"], g["len"], g["out_len"]
    x = util.splitmix64(g["seed"], nbuf * L).reshape(nbuf, L)
    assert hashlib.sha256(x).hexdigest() == g["in_sha256"]
    enc = np.empty((nbuf, E), dtype=np.uint8)
    _rows_parallel(orc.encode_rows, x, enc)
    assert hashlib.sha256(enc).hexdigest() == g["out_sha256"]
    per = hashlib.sha256()
    for i in range(nbuf):
        per.update(hashlib.sha256(enc[i]).digest())
    assert per.hexdigest() == g["per_buffer_sha256_of_sha256"]
    c = g["chunk_buffers"]
    assert [hashlib.sha256(enc[i:i + c]).hexdigest()
            for i in range(0, nbuf, c)] == g["chunk_out_sha256"]
    if "crlf76" in g:
        lines = E // 76
        crlf = np.broadcast_to(np.frombuffer(b"\r\n", np.uint8), (nbuf, lines, 2))
        text = np.concatenate([enc.reshape(nbuf, lines, 76), crlf], axis=2).reshape(nbuf, -1)
        del enc
        assert text.shape[1] == g["crlf76"]["row_bytes"]
        assert hashlib.sha256(text).hexdigest() == g["crlf76"]["text_sha256"]
        enc = text
    dec = np.empty((nbuf, (enc.shape[1] + 3) // 4 * 3), dtype=np.uint8)
    _rows_parallel(orc.decode_rows, enc, dec)
    assert hashlib.sha256(np.ascontiguousarray(dec[:, :L])).hexdigest() == g["in_sha256"]
