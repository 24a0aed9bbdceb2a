"""Host-memory sessions (include/b64x.h b64x_session_*) and the pipelined
stages: asynchronous calls, decode carries kept by
the caller (HOLD_TAIL records, spelled in front of the next block), and
stages forced through many small blocks so every carry length crosses a
block seam."""
import numpy as np
import pytest

from async_amd.session import HOLD_TAIL, Session
from oracle import pyoracle as orc
from tests import util

pytestmark = pytest.mark.gpu


def _dirty(rng, n, pad=True, abc=(-1, -1)):
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    chars = orc.encode(data, abc[0], abc[1], pad)
    sep = b"  " if "\n" in abc else b"\r\n"  # junk for this alphabet
    return sep.join(chars[i:i + 76] for i in range(0, len(chars), 76))


def _spell(tail, abc):
    """Held-back sextets as alphabet characters (what the stage does,
    async_amd/csrc/b64_stages.c spell_sextet)."""
    p62 = "+" if abc[0] == -1 else abc[0]
    p63 = "/" if abc[1] == -1 else abc[1]
    std = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789"
    return "".join(std[v] if v < 62 else (p62 if v == 62 else p63) for v in tail).encode()


def _chained_decode(blocks, abc=(-1, -1), cap=None, drain=False):
    """Decode `blocks` as one stream through two alternating sessions: every
    block but the last with HOLD_TAIL, its held-back sextets spelled in
    front of the next block on the host (the stage's carry).  A block is
    launched once the previous one's record is back; the session it goes to
    may still be busy with the block before (drain=True waits for that one
    first, so the in-place / staged choice sees every result)."""
    cap = (cap or max(64, max((len(b) for b in blocks), default=0))) + 4
    out = []
    head = b""
    with Session(cap) as a, Session(cap) as b:
        ss = (a, b)
        for i, blk in enumerate(blocks + [b""]):
            s = ss[i % 2]
            other = ss[(i + 1) % 2]
            if drain:
                other.wait()
            data = head + blk
            s.host_in[:len(data)] = np.frombuffer(data, np.uint8)
            last = i == len(blocks)
            s.decode_async(len(data), abc + (True, -1), 0 if last else HOLD_TAIL)
            s.wait()
            r = s.result()
            assert r.nchars == len(data) and r.seq != 0
            out.append(bytes(s.host_out[:r.out_len]))
            head = _spell(list(r.tail)[:r.tail_n], abc)
    return b"".join(out)


@pytest.mark.parametrize("seed", range(6))
def test_chained_decode_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    abc = [(-1, -1), ("-", "_"), ("\n", "\r"), (".", "_")][seed % 4]
    stream = _dirty(rng, int(rng.integers(0, 200000)), bool(seed % 2), abc)
    if seed == 3:
        stream = b"QQ=" + stream + b"==Q"
    cuts = np.sort(rng.integers(0, len(stream) + 1, int(rng.integers(1, 40))))
    blocks = [stream[i:j] for i, j in zip([0, *cuts], [*cuts, len(stream)])]
    assert _chained_decode(blocks, abc) == orc.decode(stream, *abc)


def test_chained_decode_every_carry_length():
    """Blocks of 1..7 characters: every tail_n value, empty blocks, and
    carries that pass through blocks holding only junk."""
    rng = np.random.default_rng(7)
    stream = _dirty(rng, 3000)
    pos, blocks = 0, []
    while pos < len(stream):
        k = int(rng.integers(0, 8))
        blocks.append(stream[pos:pos + k])
        pos += k
    blocks.insert(3, b"\r\n\r\n")
    assert _chained_decode(blocks, cap=64) == orc.decode(stream)


def test_encode_async_blocks():
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 500001, dtype=np.uint8).tobytes()
    abc = ("-", "_", True, "#")
    out = []
    with Session(1 << 17) as a, Session(1 << 17) as b:
        ss, pos, i, live = (a, b), 0, 0, []
        while pos < len(data):
            s = ss[i % 2]
            if live and live[0][0] is s:
                _, m = live.pop(0)
                s.wait()
                out.append(bytes(s.host_out[:m]))
            n = min(len(data) - pos, (1 << 17) // 3 * 3)
            s.host_in[:n] = np.frombuffer(data[pos:pos + n], np.uint8)
            s.encode_async(n, abc)
            m = (n + 2) // 3 * 4 if pos + n == len(data) else n // 3 * 4
            live.append((s, m))
            pos += n
            i += 1
        for s, m in live:
            s.wait()
            out.append(bytes(s.host_out[:m]))
    assert b"".join(out) == orc.encode(data, *abc)


def test_session_sync_roundtrip_and_capacity():
    with Session(4096) as s:
        data = bytes(range(256)) * 12
        s.host_in[:3072] = np.frombuffer(data, np.uint8)
        m = s.encode(3072)
        assert bytes(s.host_out[:m]) == orc.encode(data)
        chars = bytes(s.host_out[:m])
        s.host_in[:m] = np.frombuffer(chars, np.uint8)
        r = s.decode(m)
        assert r.out_len == 3072 and bytes(s.host_out[:3072]) == data
        with pytest.raises(Exception):
            s.encode(4097)


@pytest.mark.parametrize("cap", [64, 100, 1000])
@pytest.mark.parametrize("read_size", [1, 7, 200])
def test_stages_many_small_blocks(monkeypatch, cap, read_size):
    """Stages with tiny slots: thousands of chained blocks, both slots in
    flight, carries across every seam."""
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", str(cap))
    monkeypatch.setenv("ASYNC_B64_MIN_PULL", "1")
    rng = np.random.default_rng(cap + read_size)
    data = rng.integers(0, 256, 20011, dtype=np.uint8).tobytes()
    got, err = util.stage_encode(data, 37, read_size, ".", "_", True, "-")
    assert err == 0 and got == orc.encode(data, ".", "_", True, "-")
    dirty = b"\r\n".join(got[i:i + 61] for i in range(0, len(got), 61))
    back, err = util.stage_decode(dirty, 29, read_size, ".", "_")
    assert err == 0 and back == data


def test_reference_topology_small_slots(monkeypatch):
    monkeypatch.setenv("ASYNC_B64_STAGE_CAPACITY", "4096")
    monkeypatch.setenv("ASYNC_B64_MIN_PULL", "1")
    res, err, eagains = util.stage_reftest(100003)
    assert err == 0 and res is not None
    enc, dec = res
    assert enc == orc.encode(util.counting(100003).tobytes(), ".", "_", True, "-")
    assert dec == util.counting(100003).tobytes()


def test_chained_decode_in_place_and_staged_blocks():
    """Clean blocks decode in place over PCIe; a session whose last block
    held junk throughout stages its next one (b64x_session_decode_async).
    Clean and MIME blocks alternate in one chain, so both forms meet at the
    seams, with their carries."""
    rng = np.random.default_rng(21)
    chars = orc.encode(rng.integers(0, 256, 300000, dtype=np.uint8).tobytes(), pad=False)
    blocks = []
    for i, p in enumerate(range(0, len(chars), 19999)):
        blk = chars[p:p + 19999]
        if i % 3 == 1:
            blk = b"\r\n".join(blk[j:j + 76] for j in range(0, len(blk), 76))
        blocks.append(blk)
    stream = b"".join(blocks)
    assert _chained_decode(blocks) == orc.decode(stream)
    # Drained: every result is seen by the in-place / staged choice; ragged
    # cuts give every tail_n.
    assert _chained_decode(blocks, drain=True) == orc.decode(stream)
    cuts = np.sort(rng.integers(0, len(stream) + 1, 30))
    ragged = [stream[i:j] for i, j in zip([0, *cuts], [*cuts, len(stream)])]
    assert _chained_decode(ragged, drain=True) == orc.decode(stream)
