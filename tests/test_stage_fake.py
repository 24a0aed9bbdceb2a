"""The bytestream_1 stages' slot accounting and completion handling, on CPU.

tests/csrc/libstage_fake.so links the product's host C (event loop,
streams, framing, batching hub and the encoder/decoder stages of
async_amd/csrc/) with a CPU stand-in for the GPU side of the b64x ABI
(tests/csrc/fake_b64x.c).  Its "device" completes queued work in an order a
seeded generator picks (sessions and lanes each in their own order, different
ones interleaved at random), and can run a job's completion callback *before*
publishing its result record and output ("early" jobs) -- the failure that
lost a whole 768-byte block of one decoder stream now and then in round 1
(profiles/r01_v15_stress_ingress.log).  Every stream is compared with the
oracle (the reference's decoder_read, src/base64decoder.c:52-80: no byte is
ever lost).

`raw` mode stands for the round-1 stage, which read the record without
checking it: the same interleavings then lose blocks, which shows the test
has the power to catch the bug.  The product's check
(async_amd/csrc/b64x_result_check.h) is what the non-raw runs exercise.
"""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as orc
from tests import util


def fake():
    return util.fake_harness()


def counters(L):
    out = (ctypes.c_uint64 * 2)()
    L.b64x_diag_counters(out)
    return int(out[0]), int(out[1])


def chained(L):
    L.fake_chained.restype = ctypes.c_uint64
    return int(L.fake_chained())


def stats(L):
    out = (ctypes.c_uint64 * 2)()
    L.fake_stats(out)
    return int(out[0]), int(out[1])


def long_msgs(seed, n=200, junk_every=7):
    rng = np.random.default_rng(seed)
    msgs = [orc.encode(rng.integers(0, 256, int(k), dtype=np.uint8).tobytes())
            for k in rng.integers(1500, 5000, n)]
    for i in range(0, n, junk_every):  # MIME lines: carries at block edges
        msgs[i] = b"\r\n".join(msgs[i][j:j + 76] for j in range(0, len(msgs[i]), 76))
    return msgs


def bad_streams(msgs, got):
    bad = []
    for i, m in enumerate(msgs):
        want = orc.decode(m)
        if got is None or got[i] != want:
            bad.append(i)
    return bad


@pytest.fixture
def small_blocks(monkeypatch):
    # 1 KiB staging: every stream outgrows its first block, 2-7 blocks each
    # (the round-1 stress shape), chained on the lanes while in flight
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", "1024")


@pytest.mark.parametrize("seed,pct", [(1, 30), (2, 60), (3, 100)])
def test_long_decoder_streams_adversarial_orders(small_blocks, seed, pct):
    """Many long decoder streams on one loop (every block a job of a shared
    batch), batches completing in random orders, `pct` % of them calling
    back before their records are published: every stream is the
    oracle's, and the early ones were caught by the check."""
    L = fake()
    L.fake_configure(seed, pct, 0)
    e0 = counters(L)
    j0 = stats(L)
    c0 = chained(L)
    msgs = long_msgs(seed)
    got, err = util.ingress_stacks(msgs, 4096, lib=L)
    assert err == 0
    assert bad_streams(msgs, got) == []
    batches, early = (a - b for a, b in zip(stats(L), j0))
    # blocks 2..7 of a stream are chained to the one before while it is in
    # flight (the device spells the carry), so a stream is not one batch
    # round trip per block
    assert batches >= 2 and chained(L) > c0
    if pct == 100:
        assert early == batches and counters(L)[1] - e0[1] == batches


@pytest.mark.parametrize("seed,pct", [(4, 30), (5, 100)])
def test_long_decoder_streams_growing_blocks(monkeypatch, seed, pct):
    """The same streams with blocks that start at 256 characters and double
    while upstream keeps up (ASYNC_B64_STAGE_GROW_MAX): carries and chains
    across blocks of changing sizes, adversarial completion orders; every
    stream is the oracle's."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", "256")
    monkeypatch.setenv("ASYNC_B64_STAGE_GROW_MAX", str(1 << 16))
    L = fake()
    L.fake_configure(seed, pct, 0)
    msgs = long_msgs(seed, n=120) + [orc.encode(np.random.default_rng(seed).integers(
        0, 256, 300_000, dtype=np.uint8).tobytes())]
    got, err = util.ingress_stacks(msgs, 4096, lib=L)
    assert err == 0
    assert bad_streams(msgs, got) == []


@pytest.mark.parametrize("mode,seed", [(2, 31), (3, 32)])
def test_zero_and_torn_records_are_rejected(small_blocks, mode, seed):
    """Early callbacks that find a well-formed all-zero record (mode 2: what
    round 1's stage served as an empty block, profiles/r02_diag_notes.md) or
    a record whose tail bytes have not landed (mode 3): the record names its
    call (seq, nchars, flags) and its unused tail bytes are checked, so
    every such batch is caught, waited for and read again -- no stream loses
    or corrupts a block."""
    L = fake()
    L.fake_configure(seed, 100, mode)
    try:
        e0 = counters(L)
        j0 = stats(L)
        msgs = long_msgs(seed)
        got, err = util.ingress_stacks(msgs, 4096, lib=L)
        assert err == 0
        assert bad_streams(msgs, got) == []
        batches, early = (a - b for a, b in zip(stats(L), j0))
        assert early == batches and counters(L)[1] - e0[1] == batches
    finally:
        L.fake_configure(1, 0, 0)


def test_record_check_names_the_call():
    """b64x_result_check.h: only this call's finished record passes."""
    L = fake()
    from async_amd._lib import DecResult
    L.fake_result_ok.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint32]
    L.fake_poison.argtypes = [ctypes.c_void_p]

    def rec(valid=10, hold=True, nchars=12, seq=7, tail=None, tail_n=None):
        r = DecResult()
        r.valid, r.nchars, r.seq, r.flags = valid, nchars, seq, int(hold)
        r.tail_n = valid & 3 if tail_n is None else tail_n
        r.out_len = valid // 4 * 3 if hold else valid * 6 // 8
        t = [5, 9, 0, 0][:r.tail_n] + [0] * (4 - r.tail_n) if tail is None else tail
        for k in range(4):
            r.tail[k] = t[k]
        return r

    ok = lambda r, n=12, f=1, q=7: L.fake_result_ok(ctypes.addressof(r), n, f, q)  # noqa: E731
    assert ok(rec())
    assert ok(rec(valid=11, hold=False), f=0)
    assert not ok(rec(seq=6))                     # an earlier call's record
    assert not ok(rec(), q=0)                     # seq 0 is never drawn
    assert not ok(rec(nchars=13))                 # another length
    assert not ok(rec(hold=False))                # another flag
    assert not ok(rec(tail=[5, 64, 0, 0]))        # a held-back byte that is no sextet
    assert not ok(rec(tail=[5, 9, 1, 0]))         # a stray byte past tail_n
    assert not ok(rec(valid=13))                  # more sextets than characters
    zero = DecResult()
    assert not ok(zero, 0, 0, 7) and not ok(zero)
    p = rec()
    L.fake_poison(ctypes.addressof(p))
    assert not ok(p)


def test_round1_raw_read_loses_blocks(small_blocks):
    """The same interleavings with the records read unchecked (round 1):
    blocks are lost -- the test above would have failed before the fix."""
    L = fake()
    L.fake_configure(7, 100, 1)
    try:
        msgs = long_msgs(7)
        got, err = util.ingress_stacks(msgs, 4096, lib=L)
        assert err != 0 or bad_streams(msgs, got)
    finally:
        L.fake_configure(1, 0, 0)


@pytest.mark.parametrize("read_size", [1, 200, 4096])
def test_decoder_stage_every_order(small_blocks, read_size):
    """One stream at a time, many read sizes and carries (junk at block
    edges, '=' mid-stream, ragged tails), completions reordered and early."""
    L = fake()
    L.fake_configure(11 + read_size, 30, 0)
    rng = np.random.default_rng(read_size)
    for n in (0, 1, 2, 700, 766, 767, 768, 769, 3000, 10001):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        chars = orc.encode(data, pad=bool(n % 2))
        dirty = b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76))
        for text in (chars, dirty, b"QQ==" + chars + b"=QU", chars[:max(len(chars) - 1, 0)]):
            got, err = util.stage_decode(text, 0, read_size, lib=L)
            assert err == 0
            assert got == orc.decode(text), (n, len(text))


@pytest.mark.parametrize("seed,pct", [(5, 30), (6, 100)])
def test_short_decoder_streams_through_hub(seed, pct):
    """Short streams are jobs of shared decode batches (lanes): early batch
    callbacks are caught by the lane check (b64x_lane_decode_check)."""
    L = fake()
    L.fake_configure(seed, pct, 0)
    e0 = counters(L)
    rng = np.random.default_rng(seed)
    msgs = []
    for i in range(400):
        data = rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()
        c = orc.encode(data)
        if i % 3 == 1:
            c = b"\r\n".join(c[j:j + 76] for j in range(0, len(c), 76))
        msgs.append(c)
    got, err = util.ingress_stacks(msgs, 200, lib=L)
    assert err == 0
    assert bad_streams(msgs, got) == []
    if pct == 100:  # every batch called back early: each one was caught
        assert counters(L)[1] > e0[1]


def test_egress_stacks_reordered():
    """Encoder stages and the chunkencoder over hub batches completing in
    random orders: framed bytes equal the oracle stack's."""
    L = fake()
    L.fake_configure(9, 0, 0)
    lens = [int(x) for x in util.zipf_lengths(300, seed=0x31, rmax=512)]
    payload = util.splitmix64(0x5EED, sum(lens))
    got, err = util.egress_stacks(payload, lens, 1 << 20, 4096, lib=L)
    assert err == 0
    off = 0
    for i, n in enumerate(lens):
        want = orc.chunked_encode(payload[off:off + n].tobytes(), max_chunk=1 << 20,
                                  read_size=4096)
        off += n
        assert got[i] == want, i


def test_reference_topology_on_fake_device():
    """The reference test's own topology (test/asynctest-base64encoder.c:
    123-151) through the stages with reordered, early completions."""
    L = fake()
    L.fake_configure(3, 20, 0)
    d = util.golden("digests.json")["G1"]
    res, err, eagains = util.stage_reftest(200001, lib=L)
    assert err == 0 and res is not None
    enc, dec = res
    assert dec == util.counting(200001).tobytes()
    assert enc == orc.encode(util.counting(200001).tobytes(), ".", "_", True, "-")
    assert d["out_len"] == 1333336  # the full-size digest stays a GPU test


@pytest.mark.parametrize("cap", ["4096", "100"])
def test_reference_topology_small_blocks(monkeypatch, cap):
    """The decoder gathers its blocks through nice(91) from the encoder, so
    the encoder reserves hub room while the decoder's reservation is open:
    nested reservations must not share or recycle an arena."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", cap)
    monkeypatch.setenv("ASYNC_B64_MIN_PULL", "1")
    L = fake()
    L.fake_configure(4, 30, 0)
    res, err, eagains = util.stage_reftest(100003, lib=L)
    assert err == 0 and res is not None
    enc, dec = res
    assert enc == orc.encode(util.counting(100003).tobytes(), ".", "_", True, "-")
    assert dec == util.counting(100003).tobytes()


# --- ownership: the reference runner's leak check (test/asynctest.c:108-147) --

def test_leak_check_catches_an_outstanding_object():
    """Negative control: an object still live when counting stops is seen."""
    L = fake()
    L.make_async.restype = ctypes.c_void_p
    L.destroy_async.argtypes = [ctypes.c_void_p]
    L.h_count_begin()
    a = L.make_async()
    left = L.h_count_end()
    L.destroy_async(a)
    assert left >= 1


@pytest.mark.parametrize("cap", [None, "4096"])
def test_reference_topology_leak_check(monkeypatch, cap):
    """The reference test's topology (test/asynctest-base64encoder.c:123-151)
    through the stages, with every allocation counted the way the
    reference's runner counts them (fs_set_reallocator, test/asynctest.c:
    276-278): after destroy_async() nothing is outstanding -- every stage,
    hub and stream object was made by fsalloc() and freed by fsfree()
    through async_wound(), the reference's ownership contract
    (src/async.c:127-130, 386-392)."""
    if cap:
        monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", cap)
    L = fake()
    L.fake_configure(21, 30, 0)
    (res, err, _), left = util.counted(util.stage_reftest, 100003, lib=L)
    assert err == 0 and res is not None
    assert res[1] == util.counting(100003).tobytes()
    assert left == 0


def test_egress_and_ingress_stacks_leak_check():
    """Many stacks on one loop (config 5's egress shape and the ingress
    mirror), counted: nothing outstanding after the loop is destroyed."""
    L = fake()
    L.fake_configure(22, 30, 0)
    lens = [int(x) for x in util.zipf_lengths(200, seed=0x33, rmax=256)]
    payload = util.splitmix64(0x5EED, sum(lens))
    (got, err), left = util.counted(util.egress_stacks, payload, lens, 1 << 20, 4096, lib=L)
    assert err == 0 and left == 0
    msgs = long_msgs(23, n=60)
    (got, err), left = util.counted(util.ingress_stacks, msgs, 4096, lib=L)
    assert err == 0 and left == 0
    assert bad_streams(msgs, got) == []


# ---- messages lent from their pinned queue copies (b64_pin.h) ------------

LENT_SIZES = [1, 2, 3, 5000, 4095, 4096, 4097, 100001, 7, 65537, 300000, 12, 9000]


@pytest.mark.parametrize("cap", ["1024", "65536", None])
@pytest.mark.parametrize("lend_min", ["1", "4096", "1000000000"])
@pytest.mark.parametrize("push,late", [(False, False), (True, False), (False, True)])
def test_egress_lent_pieces(monkeypatch, cap, lend_min, push, late):
    """queuestream_enqueue_bytes / _push_bytes of a mix of short and long
    messages -> encoder -> chunkencoder: long messages are encoded from
    their pinned copies (no copy into the arena; carries across blocks of
    one message come from the bytes right before the next block), short
    ones gathered.  The framed stream equals the oracle stack's (late
    termination: the payload, since EAGAIN then shapes the read counts),
    lent jobs happen exactly when a message reaches ASYNC_B64_LEND_MIN, and
    every pinned piece is released once the stack is closed."""
    L = fake()
    L.fake_configure(13, 0, 0)
    if cap:
        monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", cap)
    monkeypatch.setenv("ASYNC_B64_LEND_MIN", lend_min)
    rng = np.random.default_rng(0x1E47)
    pieces = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in LENT_SIZES]
    order = pieces  # push_bytes in reverse order queues them in order
    lent0 = L.b64_hub_lent_total()
    for max_chunk, read_size in ((4096, 1000), (1 << 20, 10240)):
        got, err = util.egress_pieces(pieces, max_chunk, read_size, push=push, late=late, lib=L)
        assert err == 0 and got is not None
        data = b"".join(order)
        if late:
            assert util.dechunk(got) == orc.encode(data)
        else:
            want = orc.chunked_encode(np.frombuffer(data, np.uint8),
                                      piece_lens=[len(p) for p in order],
                                      max_chunk=max_chunk, read_size=read_size)
            assert got == want
    lent = L.b64_hub_lent_total() - lent0
    if int(lend_min) > max(LENT_SIZES):
        assert lent == 0
    else:
        assert lent > 0
    assert L.b64_pin_live_refs() == 0


def test_egress_stacks_lent_and_released():
    """Config 5's shape on the fake device: every message at least
    ASYNC_B64_LEND_MIN long is lent, and no pinned piece outlives its stack."""
    L = fake()
    L.fake_configure(21, 0, 0)
    lens = [int(x) for x in util.zipf_lengths(200, seed=0x77, rmax=256)]
    payload = util.splitmix64(0x5EED, sum(lens))
    lent0 = L.b64_hub_lent_total()
    got, err = util.egress_stacks(payload, lens, 1 << 20, 10240, lib=L)
    assert err == 0
    off = 0
    for i, n in enumerate(lens):
        want = orc.chunked_encode(payload[off:off + n].tobytes(), max_chunk=1 << 20,
                                  read_size=10240)
        off += n
        assert got[i] == want, i
    assert L.b64_hub_lent_total() - lent0 >= sum(1 for n in lens if n >= 4096)
    assert L.b64_pin_live_refs() == 0


def test_egress_lent_fuzz(monkeypatch):
    """Seeded fuzz of lent and gathered messages (scripts/fuzz_lent.py's
    cases, fake device): random queues of 0 B - 1.5 MiB messages, stage
    capacities, lend thresholds, chunk and read sizes, pushes, late
    termination.  Found the gather stopping at min_pull after a lent
    message (smaller blocks than one copying read would fill, so a short
    read count and other chunk sizes than the reference's)."""
    L = fake()
    for seed in range(48):
        rng = np.random.default_rng(0xF0221 + seed)
        k = int(rng.integers(1, 40))
        sizes = [0 if rng.random() < 0.05 else int(np.exp(rng.uniform(0, np.log(1.5 * 2**20))))
                 for _ in range(k)]
        pieces = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
        cap = int(rng.choice([64, 1000, 4096, 65536, 1 << 20]))
        monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(cap))
        # blocks that fill grow (up to 8x or 64x), or stay fixed
        monkeypatch.setenv("ASYNC_B64_STAGE_GROW_MAX", str(cap * int(rng.choice([1, 8, 64]))))
        monkeypatch.setenv("ASYNC_B64_LEND_MIN", str(int(rng.choice([1, 3, 4096, 65536]))))
        max_chunk = int(rng.choice([30, 4096, 65536, 1 << 20]))
        read_size = int(rng.choice([7, 1000, 10240, 1 << 18]))
        push, late = bool(rng.random() < 0.3), bool(rng.random() < 0.3)
        L.fake_configure(seed, 0, 0)
        got, err = util.egress_pieces(pieces, max_chunk, read_size, push=push, late=late, lib=L)
        assert err == 0 and got is not None, seed
        data = b"".join(pieces)
        if late:
            assert util.dechunk(got) == orc.encode(data), seed
        else:
            assert got == orc.chunked_encode(np.frombuffer(data, np.uint8), piece_lens=sizes,
                                             max_chunk=max_chunk, read_size=read_size), seed
    assert L.b64_pin_live_refs() == 0


@pytest.mark.parametrize("decode", [0, 1])
@pytest.mark.parametrize("n,chunk,read_size", [(10_000, 3_000, 400), (200_000, 65_536, 4_096),
                                               (5, 5, 8), (0, 1, 8), (100_000, 0, 8),
                                               (100_000, 0, 4096), (3_000, 0, 200)])
def test_upstream_error_is_returned_not_eagain(small_blocks, decode, n, chunk, read_size):
    """An upstream that gives data and then fails hard (EIO): the stage
    serves what it had (the reference returns each read's output as it
    goes) and then returns -1 with EIO -- not EAGAIN, not a clean EOF
    (ref src/base64encoder.c:127-129, base64decoder.c:58-61)."""
    import errno
    L = fake()
    rng = np.random.default_rng(n + chunk)
    raw = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    data = orc.encode(raw) if decode else raw
    src = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, dtype=np.uint8)
    cap = 2 * len(data) + 64
    out = np.zeros(cap, dtype=np.uint8)
    err = ctypes.c_int(0)
    got = L.h_stage_upstream_error(decode, src.ctypes.data, len(data), chunk, errno.EIO,
                                   read_size, out.ctypes.data, cap, ctypes.byref(err))
    assert err.value == errno.EIO
    assert got >= 0
    want = orc.decode(data) if decode else orc.encode(raw)
    assert out[:got].tobytes() == want[:got]
    if chunk:  # upstream gave every byte before failing
        if decode:
            # whole groups; the reference may also have emitted the bytes
            # of a trailing partial group (at most 2)
            assert len(want) - got <= 2
        else:
            # every full sextet of the bytes (base64encoder.c:132-139)
            assert got == len(raw) * 8 // 6


_PIN_SCRIPT = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from tests import util
L = util.fake_harness()
L.b64_pin_idle_bytes.restype = ctypes.c_size_t
L.fake_host_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
def host():
    o = (ctypes.c_uint64 * 2)()
    L.fake_host_stats(o)
    return int(o[0]), int(o[1])
rng = np.random.default_rng(3)
# a queue alone, before any GPU stage exists: no pinned memory at all
pieces = [rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes() for _ in range(3)]
got, err, _ = util.queue_stream(pieces, read_size=4096, lib=L)
assert err == 0 and got == b"".join(pieces)
assert host() == (0, 0), host()
# with the encoder stage: 20 MiB messages (a slab of their own each, never
# kept idle) and 3 MiB ones (standard 32 MiB slabs, kept within the cap)
slab = 32 << 20
for rnd in range(3):
    pieces = [rng.integers(0, 256, n, dtype=np.uint8).tobytes()
              for n in (20 << 20, 3 << 20, 3 << 20, 21 << 20, 3 << 20)]
    framed, err = util.egress_pieces(pieces, 1 << 20, 10240, lib=L)
    assert err == 0, err
    idle = L.b64_pin_idle_bytes()
    assert idle % slab == 0 and idle <= int(sys.argv[2]), idle
    assert L.b64_pin_live_refs() == 0
print("ok", host(), L.b64_pin_idle_bytes())
"""


@pytest.mark.parametrize("cap", [32 << 20, 2 << 30])
def test_pinned_message_pool_is_bounded(tmp_path, cap):
    """The pinned message pool: nothing is pinned (and no HIP
    runtime started) before the process has a GPU stage; slabs made for one
    oversize message are freed on release; the idle slabs stay within
    ASYNC_B64_PIN_IDLE_BYTES.  A fresh process, since the pool is
    process-wide."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ASYNC_B64_PIN_IDLE_BYTES=str(cap))
    p = subprocess.run([sys.executable, "-c", _PIN_SCRIPT, root, str(cap)], capture_output=True,
                       text=True, env=env, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.startswith("ok"), p.stdout

