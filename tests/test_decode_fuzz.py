"""Randomised decode parity: the single-buffer decode (probe, lines,
suffix; pass 1 / scan / pass 2 past 2^31 characters is covered elsewhere)
and the uniform-batch row kernels against the oracle, over seeded random
shapes -- stream lengths, line models that hold, break or only look like
lines, junk runs, '=' inside the stream, leading and trailing junk, HOLD_TAIL,
alphabets whose pos62/pos63 are separator bytes, unaligned buffers.  Every
case is bit-exact against oracle/b64_oracle.c (the restatement of
src/base64decoder.c:38-80) including the result record."""
import numpy as np
import pytest
import torch

from async_amd import b64
from oracle import pyoracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
JUNK = [b"\r", b"\n", b" ", b"\t", b"=", b"!", b"\x80", b"\xff", b"\x00", b"-"]
ALPHABETS = [(-1, -1), ("-", "_"), (".", "_"), ("\n", "\r"), ("+", "+"), ("!", "=")]


def _text(rng) -> tuple[bytes, tuple]:
    abc = ALPHABETS[rng.integers(len(ALPHABETS))]
    n = int(rng.choice([rng.integers(0, 64), rng.integers(0, 3000), rng.integers(0, 200_000),
                        rng.integers(0, 3_000_000)], p=[0.25, 0.35, 0.3, 0.1]))
    chars = orc.encode(rng.integers(0, 256, n, dtype=np.uint8).tobytes(), abc[0], abc[1])
    kind = rng.integers(6)
    if kind == 0:  # clean
        text = chars
    elif kind <= 3:  # lines, sometimes broken
        L = int(rng.choice([16, 17, 19, 20, 60, 64, 76, 76, 100, 252, 253, 300]))
        sep = b"".join(JUNK[rng.integers(len(JUNK))] for _ in range(rng.integers(1, 6)))
        lines = [chars[i:i + L] for i in range(0, len(chars), L)]
        if kind == 3 and len(lines) > 4:
            k = int(rng.integers(1, len(lines) - 1))
            lines[k] = lines[k][:int(rng.integers(0, L))]  # a short line
        text = sep.join(lines) + (sep if rng.integers(2) else b"")
    elif kind == 4:  # sprinkled junk
        d = float(rng.choice([1e-4, 1e-2, 0.2]))
        a = np.frombuffer(chars, dtype=np.uint8)
        mask = rng.random(a.size) < d
        junk = np.frombuffer(b"".join(JUNK), dtype=np.uint8)
        ins = junk[rng.integers(0, junk.size, int(mask.sum()))]
        out = np.empty(a.size + ins.size, dtype=np.uint8)
        pos = np.arange(a.size) + np.cumsum(mask)
        out[pos] = a
        jm = np.ones(out.size, bool)
        jm[pos] = False
        out[jm] = ins
        text = out.tobytes()
    else:  # junk runs at the ends and '=' inside
        text = (b"\r\n" * int(rng.integers(0, 40)) + chars[:len(chars) // 2] + b"=" +
                chars[len(chars) // 2:] + b"\n" * int(rng.integers(0, 300)))
    return text, abc


@pytest.mark.parametrize("seed", range(16))
def test_decode_fuzz_vs_oracle(seed):
    rng = np.random.default_rng(1000 + seed)
    for _ in range(60):
        text, abc = _text(rng)
        want = orc.decode(text, abc[0], abc[1])
        off = int(rng.integers(0, 4))
        x = torch.from_numpy(np.frombuffer(bytes(off) + text, dtype=np.uint8).copy()).to(DEV)[off:]
        hold = bool(rng.integers(2))
        out = torch.empty(b64.decoded_cap(len(text)) + 4, dtype=torch.uint8, device=DEV)
        d = b64.decode(x, out=out[off:], abc=(abc[0], abc[1], True, -1), hold_tail=hold)
        info = d.info()
        got = d.bytes().cpu().numpy().tobytes()
        tab = np.array(orc.decode_table(abc[0], abc[1]))
        t = tab[np.frombuffer(text, dtype=np.uint8)] if text else np.zeros(0, int)
        valid = int(((t >= 0) & (t < 64)).sum())
        assert info.valid == valid, (seed, len(text))
        assert info.tail_n == valid % 4
        if hold:
            assert info.out_len == valid // 4 * 3 and got == want[:info.out_len]
        else:
            assert got == want, (seed, len(text), abc)


@pytest.mark.parametrize("seed", range(16))
def test_rows_fuzz_vs_oracle(seed):
    """Uniform batches whose rows share one random format (row 0 sets the
    line model), with random deviant rows."""
    rng = np.random.default_rng(2000 + seed)
    nbuf = int(rng.integers(2, 400))
    n = int(rng.integers(24, 3000))
    L = int(rng.choice([16, 19, 64, 76, 76, 100]))
    sep = b"".join(JUNK[rng.integers(4)] for _ in range(rng.integers(1, 5)))
    rows = []
    for i in range(nbuf):
        c = orc.encode(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        t = sep.join(c[j:j + L] for j in range(0, len(c), L)) + sep
        if rng.random() < 0.05:
            t = t[:5] + b"\x80" + t[5:]
        rows.append(t)
    stride = max(len(r) for r in rows) + int(rng.integers(0, 8)) // 4 * 4
    flat = b"".join(r + b"\n" * (stride - len(r)) for r in rows)
    x = torch.from_numpy(np.frombuffer(flat, dtype=np.uint8).copy()).to(DEV)
    cap = (b64.decoded_cap(stride) + 15) // 16 * 16
    dec = torch.empty(nbuf * cap, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    b64.decode_strided(x, stride, stride, nbuf, dec, cap, outlen)
    ol = outlen.cpu().tolist()
    dh = dec.cpu().numpy()
    for i, r in enumerate(rows):
        want = orc.decode(r + b"\n" * (stride - len(r)))
        assert ol[i] == len(want), (seed, i)
        assert dh[i * cap:i * cap + ol[i]].tobytes() == want, (seed, i)
