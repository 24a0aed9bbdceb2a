"""Config 5 on the GPU:
queuestream -> GPU base64 encoder stage -> chunkencoder, many stacks on one
loop sharing the batching hub, checked against the oracle's restatement of
the same stack -- including the chunk framing, which follows the encoder's
per-read counts."""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle as orc
from tests import util

pytestmark = pytest.mark.gpu

FX = util.golden("chunk.json")


@pytest.mark.parametrize("case", FX["enc_counts"], ids=lambda c: f"n{c['n']}_c{c['count']}")
@pytest.mark.parametrize("burst", [0, 113])
def test_stage_read_counts_match_reference(case, burst):
    """The GPU stage returns the reference encoder's read counts
    (full count, short only at the end, finalize() on its own)."""
    data = util.splitmix64(0x5EED, case["n"]).tobytes()
    want = [v for v, k in case["counts_rle"] for _ in range(k)]
    got, err = util.encode_counts(data, case["count"], burst, pad=case["pad"])
    assert err == 0
    assert got == want


@pytest.mark.parametrize("grow", [1, 16])
@pytest.mark.parametrize("cap", [64, 4096])
@pytest.mark.parametrize("seed", range(4))
def test_stage_read_counts_small_slots(monkeypatch, cap, seed, grow):
    """Read counts with small blocks, fixed or growing while upstream keeps
    up (ASYNC_B64_STAGE_GROW_MAX): the reference's counts either way."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(cap))
    monkeypatch.setenv("ASYNC_B64_STAGE_GROW_MAX", str(cap * grow))
    monkeypatch.setenv("ASYNC_B64_MIN_PULL", "1")
    rng = np.random.default_rng(seed)
    n = int(rng.integers(0, 50000))
    count = int(rng.choice([4, 8, 200, 1024, 10240]))
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    for burst in (0, 97):
        got, err = util.encode_counts(data, count, burst)
        assert err == 0
        assert got == orc.encode_counts(data, count, burst=burst)


@pytest.mark.parametrize("max_chunk", [4096, 1 << 20])
def test_egress_stacks_vs_oracle(max_chunk):
    lens = util.zipf_lengths()[:300]
    payload = util.splitmix64(0x5EED, int(lens.sum()))
    framed, err = util.egress_stacks(payload, lens, max_chunk, 10240)
    assert err == 0
    off = 0
    for i, L in enumerate(lens.tolist()):
        msg = payload[off:off + L].tobytes()
        off += L
        assert framed[i] == orc.chunked_encode(msg, max_chunk=max_chunk), (i, L)


@pytest.mark.parametrize("cap", [4096, 65536])
def test_egress_stacks_chunks_spanning_blocks(monkeypatch, cap):
    """Small stage blocks (a block still holds one whole read, as the stage
    requires): the chunkencoder's reads often span two blocks, so the lent
    characters come from the stage's spill buffer (the frame holds only
    headers).  Framing stays the oracle's."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(cap))
    lens = util.zipf_lengths()[:200]
    payload = util.splitmix64(0xC0FFEE, int(lens.sum()))
    for max_chunk in (30, 100_000):
        framed, err = util.egress_stacks(payload, lens, max_chunk, 10240)
        assert err == 0
        off = 0
        for i, L in enumerate(lens.tolist()):
            msg = payload[off:off + L].tobytes()
            off += L
            assert framed[i] == orc.chunked_encode(msg, max_chunk=max_chunk), (i, L)


def test_egress_stacks_fixture():
    """The first 24 Zipf messages against the committed framed digests."""
    items = FX["stacks"]["items"]
    lens = [it["len"] for it in items[::2]]
    payload = util.splitmix64(0x5EED, sum(lens))
    for k, mc in enumerate((4096, 1 << 20)):
        framed, err = util.egress_stacks(payload, lens, mc, 10240)
        assert err == 0
        for i, f in enumerate(framed):
            it = items[2 * i + k]
            assert it["max_chunk"] == mc
            assert len(f) == it["framed_len"]
            assert hashlib.sha256(f).hexdigest() == it["framed_sha256"]


def test_egress_stacks_alphabet_and_small_reads():
    lens = [0, 1, 2, 3, 64, 65, 4095, 4096, 4097, 70000]
    payload = util.splitmix64(9, sum(lens))
    framed, err = util.egress_stacks(payload, lens, 1000, 7, ".", "_", False, "-")
    assert err == 0
    off = 0
    for i, L in enumerate(lens):
        msg = payload[off:off + L].tobytes()
        off += L
        assert framed[i] == orc.chunked_encode(msg, max_chunk=1000, pos62=".", pos63="_",
                                               pad=False, padchar="-"), L


@pytest.mark.slow
def test_config5_full():
    """All 16,384 Zipf messages (1.10 GB), max_chunk 1 MiB, tcp-sized reads."""
    lens = util.zipf_lengths()
    payload = util.splitmix64(0x5EED, int(lens.sum()))
    framed, err = util.egress_stacks(payload, lens, 1 << 20, 10240)
    assert err == 0
    off = 0
    for i, L in enumerate(lens.tolist()):
        msg = payload[off:off + L].tobytes()
        off += L
        assert framed[i] == orc.chunked_encode(msg, max_chunk=1 << 20), i


@pytest.mark.parametrize("threads,devices", [(2, 1), (5, 1), (4, 2)])
def test_egress_stacks_threads(threads, devices):
    """Several event loops (one per thread, each with its own hub) sharing
    the messages; devices > 1: each loop pinned to GPU t mod devices (on a
    one-GPU box every loop lands on GPU 0, through the same hipSetDevice
    path a full node takes)."""
    lens = util.zipf_lengths()[:400]
    payload = util.splitmix64(0x5EED, int(lens.sum()))
    framed, err = util.egress_stacks(payload, lens, 1 << 20, 10240, threads=threads,
                                     devices=devices)
    assert err == 0
    off = 0
    for i, L in enumerate(lens.tolist()):
        msg = payload[off:off + L].tobytes()
        off += L
        assert framed[i] == orc.chunked_encode(msg, max_chunk=1 << 20), (i, L)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["1024", "65536", None])
@pytest.mark.parametrize("lend_min", ["1", "4096"])
def test_egress_lent_pieces_gpu(monkeypatch, cap, lend_min):
    """Messages lent from their pinned queue copies on the MI355X: short
    and long messages mixed in one queue, blocks that mix arena bytes and
    lent segments at every alignment (k_gather_host), carries across blocks
    of one message; framed bytes equal the oracle stack's, and every pinned
    reference is released."""
    if cap:
        monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", cap)
    monkeypatch.setenv("ASYNC_B64_LEND_MIN", lend_min)
    L = util.harness()
    rng = np.random.default_rng(0x1E48)
    sizes = [1, 2, 3, 5000, 4095, 4096, 4097, 100001, 7, 65537, 300000, 12, 9000, 3 << 20, 5]
    pieces = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    lent0 = L.b64_hub_lent_total()
    for max_chunk, read_size in ((4096, 1000), (1 << 20, 10240)):
        got, err = util.egress_pieces(pieces, max_chunk, read_size)
        assert err == 0 and got is not None
        data = b"".join(pieces)
        want = orc.chunked_encode(np.frombuffer(data, np.uint8),
                                  piece_lens=[len(p) for p in pieces],
                                  max_chunk=max_chunk, read_size=read_size)
        assert got == want
    assert L.b64_hub_lent_total() > lent0
    assert L.b64_pin_live_refs() == 0
