"""Config-5 host pieces on CPU: the product's
chunkencoder and queuestream (async_amd/csrc/framing.c) on the product
loop, the oracle's restatement of the whole egress stack, the encoder
read-count model, and the Zipf generator -- all against the committed
fixtures of tests/golden/make_golden.py."""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle as orc
from tests import util

FX = util.golden("chunk.json")


def dechunk(framed: bytes, termination=0):
    """The reference test's framing validator (test/asynctest-chunkencoder.c
    :28-151) as a parser: returns (payload, chunk sizes) or raises."""
    pos, sizes, payload = 0, [], bytearray()
    first = True
    while True:
        if not first:
            assert framed[pos:pos + 2] == b"\r\n", "CRLF expected after chunk"
            pos += 2
        first = False
        end = pos
        while framed[end:end + 1] in tuple(b"0123456789abcdefABCDEF"[i:i + 1] for i in range(22)):
            end += 1
        assert end > pos, "chunk length expected"
        n = int(framed[pos:end], 16)
        pos = end
        if n == 0:
            tail = {0: b"\r\n\r\n", 1: b"\r\n", 2: b""}[termination]
            assert framed[pos:] == tail, "bad termination"
            return bytes(payload), sizes
        assert framed[pos:pos + 2] == b"\r\n", "LF expected after chunk length"
        pos += 2
        payload += framed[pos:pos + n]
        assert len(framed) >= pos + n
        pos += n
        sizes.append(n)


def _rle(pairs):
    return [v for v, k in pairs for _ in range(k)]


def test_zipf_lengths_match_fixture():
    z = FX["zipf"]
    lens = util.zipf_lengths()
    assert lens[:64].tolist() == z["first64"]
    assert int(lens.sum()) == z["total"] and lens.size == z["n_msgs"]
    assert int(lens.max()) == z["max"] and int(lens.min()) == z["min"]
    assert hashlib.sha256(",".join(map(str, lens.tolist())).encode()).hexdigest() == z["sha256"]


@pytest.mark.parametrize("case", FX["enc_counts"], ids=lambda c: f"n{c['n']}_c{c['count']}")
def test_oracle_encoder_read_counts(case):
    data = util.splitmix64(0x5EED, case["n"]).tobytes()
    got = orc.encode_counts(data, case["count"], pad=case["pad"])
    assert got == _rle(case["counts_rle"])


def test_oracle_stack_matches_fixture():
    items = FX["stacks"]["items"]
    lens = [it["len"] for it in items[::2]]
    payload = util.splitmix64(0x5EED, sum(lens)).tobytes()
    off = 0
    for i, L in enumerate(lens):
        msg = payload[off:off + L]
        off += L
        for it in items[2 * i:2 * i + 2]:
            framed = orc.chunked_encode(msg, max_chunk=it["max_chunk"])
            assert len(framed) == it["framed_len"]
            assert hashlib.sha256(framed).hexdigest() == it["framed_sha256"]
            body, sizes = dechunk(framed)
            assert body == orc.encode(msg)
            assert all(s == it["max_chunk"] for s in sizes[:-2])


def test_oracle_stack_pieces_equal_whole():
    """A queue of pieces reads like one blob (queuestream.c:162-183)."""
    data = util.splitmix64(7, 10000).tobytes()
    whole = orc.chunked_encode(data, max_chunk=1000)
    pieces = orc.chunked_encode(data, piece_lens=[1, 0, 2999, 5000, 2000], max_chunk=1000)
    assert whole == pieces


@pytest.mark.parametrize("burst", [0, 7, 113])
@pytest.mark.parametrize("read_size", [1, 7, 100, 4096])
def test_chunkencoder_reference_test(burst, read_size):
    """test/asynctest-chunkencoder.c:160-220 on the product chunkencoder:
    the reference's text, MAX_CHUNK 30, reads of 100 (and others)."""
    rt = FX["ref_test"]
    text = bytes.fromhex(rt["text_hex"])
    got, err = util.chunk_stream(text, rt["max_chunk"], 0, read_size, burst)
    assert err == 0
    assert got.hex() == rt["framed_hex"]
    body, sizes = dechunk(got)
    assert body == text and max(sizes) == 30


@pytest.mark.parametrize("t", FX["terminations"], ids=lambda t: f"t{t['termination']}"
                         f"{'_empty' if t.get('empty') else ''}")
def test_chunkencoder_terminations(t):
    data = b"" if t.get("empty") else b"abc"
    got, err = util.chunk_stream(data, 30, t["termination"], 100)
    assert err == 0 and got.hex() == t["framed_hex"]


def test_chunkencoder_clamps_max_chunk():
    data = bytes(range(256)) * 4
    got, _ = util.chunk_stream(data, 1, 0, 4096)  # clamped to 2 (chunkencoder.c:180)
    _, sizes = dechunk(got)
    assert set(sizes) == {2}
    got, _ = util.chunk_stream(data, 1 << 30, 0, 4096)  # clamped to 16 MiB
    _, sizes = dechunk(got)
    assert sizes == [len(data)]


@pytest.mark.parametrize("push", [False, True])
@pytest.mark.parametrize("burst", [0, 5])
def test_queuestream_concatenates(push, burst):
    rng = np.random.default_rng(3)
    pieces = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes()
              for k in (0, 1, 17, 0, 300, 4096, 2)]
    got, err, eagains = util.queue_stream(pieces, push=push, burst=burst, read_size=64)
    assert err == 0
    assert got == b"".join(pieces)
    # The queue is terminated 2 ms after the start: the reader must have
    # seen EAGAIN at least once (queuestream.c:185-189) and been notified.
    assert eagains >= 1


def test_queuestream_empty_terminated():
    got, err, eagains = util.queue_stream([], read_size=64)
    assert err == 0 and got == b""
