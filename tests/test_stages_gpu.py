"""The drop-in bytestream_1 stages (include/base64encoder.h,
base64decoder.h) on the GPU, driven through the product's event loop by
tests/csrc/stage_harness.c -- including the reference's own test topology
(test/asynctest-base64encoder.c:123-151)."""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle as orc
from tests import util

pytestmark = pytest.mark.gpu


def test_reference_topology_on_gpu_stages():
    """1,000,001 counting bytes -> nice(113) -> GPU encoder('.', '_', '-')
    -> nice(91) -> GPU decoder -> nice(97), read 200 at a time."""
    d = util.golden("digests.json")["G1"]
    res, err, eagains = util.stage_reftest(1000001)
    assert err == 0 and res is not None
    enc, dec = res
    assert len(enc) == d["out_len"]
    assert hashlib.sha256(enc).hexdigest() == d["out_sha256"]
    assert dec == util.counting(1000001).tobytes()
    assert eagains > 0  # the nicestreams did push back


def test_reference_topology_leak_check_on_gpu():
    """The same test with the reference runner's counting allocator wired in
    (test/asynctest.c:111-147, 276-278): after destroy_async() no object is
    outstanding, so the reference's posttest_check would pass.  Stages and
    hub come from fsalloc() and go back through async_wound() -> fsfree()."""
    d = util.golden("digests.json")["G1"]
    (res, err, _), left = util.counted(util.stage_reftest, 1000001)
    assert err == 0 and res is not None
    assert hashlib.sha256(res[0]).hexdigest() == d["out_sha256"]
    assert res[1] == util.counting(1000001).tobytes()
    assert left == 0


@pytest.mark.parametrize("read_size", [1, 3, 4, 5, 200, 4096, 1 << 20])
@pytest.mark.parametrize("burst", [0, 113])
def test_encoder_stage_any_read_size(read_size, burst):
    """Same characters as the oracle for every read size -- including the
    odd sizes the reference cannot serve (its assert, base64encoder.c:140)."""
    rng = np.random.default_rng(read_size + burst)
    for n, abc in ((0, (-1, -1, True, -1)), (1, (-1, -1, True, -1)),
                   (2, (".", "_", True, "-")), (70001, (-1, -1, False, -1)),
                   (300000, ("-", "_", True, "#"))):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        got, err = util.stage_encode(data, burst, read_size, *abc)
        assert err == 0
        assert got == orc.encode(data, *abc), (n, abc)


@pytest.mark.parametrize("read_size", [1, 2, 3, 200, 65536])
@pytest.mark.parametrize("burst", [0, 91])
def test_decoder_stage_vs_oracle(read_size, burst):
    rng = np.random.default_rng(read_size * 3 + burst)
    for n in (0, 1, 2, 3, 1000, 250001):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        chars = orc.encode(data, pad=bool(n % 2))
        dirty = b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76))
        if n == 1000:
            dirty = b"QQ==" + dirty + b"=QU"  # bits carried across '='
        got, err = util.stage_decode(dirty, burst, read_size)
        assert err == 0
        assert got == orc.decode_stream(dirty, 0, 0, 200), n
        if n not in (1000,):
            assert got == data


@pytest.mark.parametrize("abc", [(-1, -1), (".", "_"), ("\n", "\r")])
def test_many_short_decoder_streams_on_one_loop(abc):
    """Short decoder streams (each ends inside its first block) are decoded
    as jobs of shared hub batches: every stream's bytes equal the oracle's,
    including dirty, padded-in-the-middle, ragged and empty messages."""
    rng = np.random.default_rng(17 + len(str(abc)))
    msgs = []
    for i in range(700):
        n = int(rng.integers(0, 3000)) if i % 50 else 0
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        chars = orc.encode(data, abc[0], abc[1], bool(i % 3), -1)
        if i % 4 == 1:
            chars = b"\r\n".join(chars[j:j + 76] for j in range(0, len(chars), 76))
        if i % 7 == 2:
            chars = b"QU=" + chars + b"*Q"
        if i % 11 == 3:
            chars = chars[:max(len(chars) - int(rng.integers(0, 4)), 0)]
        msgs.append(chars)
    for big in (70000, 300000):  # whole message still inside one block
        msgs.append(orc.encode(rng.integers(0, 256, big, dtype=np.uint8).tobytes(),
                               abc[0], abc[1], True, -1))
    got, err = util.ingress_stacks(msgs, 200, *abc)
    assert err == 0
    for i, m in enumerate(msgs):
        assert got[i] == orc.decode_stream(m, 0, 0, 200, *abc), i


def test_many_long_decoder_streams_on_one_loop(monkeypatch):
    """600 decoder streams that each outgrow their first block (1 KiB
    staging, so they continue on chained sessions) on one loop: their
    completions all come back through the loop's one hub eventfd."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", "1024")
    rng = np.random.default_rng(23)
    msgs = [orc.encode(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes())
            for n in rng.integers(1500, 5000, 600)]
    msgs[7] = b"\r\n".join(msgs[7][i:i + 76] for i in range(0, len(msgs[7]), 76))
    got, err = util.ingress_stacks(msgs, 4096)
    assert err == 0
    bad = []
    for i, m in enumerate(msgs):
        want = orc.decode(m)
        if got[i] != want:
            g = got[i] or b""
            first = next((j for j in range(min(len(g), len(want))) if g[j] != want[j]),
                         min(len(g), len(want)))
            last = max((j for j in range(min(len(g), len(want))) if g[j] != want[j]),
                       default=-1)
            bad.append((i, len(m), len(g), len(want), first, last))
    # (stream, chars, got bytes, want bytes, first/last differing byte)
    assert not bad, bad


def _dirty(rng, n):
    """Random bytes encoded, broken into 77-character lines with a '*' every
    ~1,000 characters: blocks cut anywhere leave 0-3 sextets over."""
    chars = orc.encode(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    lines = b"\r\n".join(chars[i:i + 77] for i in range(0, len(chars), 77))
    cut = sorted(rng.integers(0, len(lines), len(lines) // 1000))
    return b"*".join(lines[a:b] for a, b in zip([0] + cut, cut + [len(lines)]))


@pytest.mark.parametrize("cap,read_size", [(200_000, 65536), (300_001, 1 << 20), (1 << 20, 4096)])
def test_decoder_stage_big_blocks_with_carries(monkeypatch, cap, read_size):
    """Streams of many blocks of >= 128 KiB, each decoded by the single-buffer
    pipeline inside its hub batch, with held sextets carried from block to
    block: the stream's bytes equal the oracle's."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(cap))
    rng = np.random.default_rng(cap + read_size)
    dirty = _dirty(rng, 2_500_000 + cap % 7)
    got, err = util.stage_decode(dirty, 0, read_size)
    assert err == 0
    assert got == orc.decode_stream(dirty, 0, 0, 200)


def test_decoder_streams_big_and_small_jobs_in_one_batch(monkeypatch):
    """Long and short decoder streams on one loop share hub batches: the big
    jobs take the pipeline, the rest the batch kernel, and every stream's
    bytes equal the oracle's."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(150_000))
    rng = np.random.default_rng(29)
    msgs = []
    for i in range(48):
        n = int(rng.integers(200_000, 700_000)) if i % 3 == 0 else int(rng.integers(0, 5000))
        msgs.append(_dirty(rng, n) if i % 2 else orc.encode(
            rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
    got, err = util.ingress_stacks(msgs, 65536)
    assert err == 0
    for i, m in enumerate(msgs):
        assert got[i] == orc.decode_stream(m, 0, 0, 200), i


@pytest.mark.parametrize("cap", [4096, 65536])
def test_decoder_stage_chained_blocks(monkeypatch, cap):
    """One long stream in many small blocks: every block after the first is
    committed while its predecessor is still queued or on the GPU, so its
    carried sextets are spelled into its head on the device (k_spell_head,
    chained lane jobs, across batches queued on one lane) -- the stream's
    bytes equal the oracle's, carries at every block edge included."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(cap))
    monkeypatch.setenv("ASYNC_B64_MIN_PULL", str(cap))
    rng = np.random.default_rng(cap)
    dirty = _dirty(rng, 3_000_000)
    for read_size in (1000, 1 << 20):
        got, err = util.stage_decode(dirty, 0, read_size)
        assert err == 0
        assert got == orc.decode_stream(dirty, 0, 0, 200)
