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


@pytest.mark.parametrize("seed", range(4))
def test_rows_reuse_fuzz(seed):
    """Row batches of one shape on one stream, one after another (the
    library workspace keeps the line model of the last batch of this shape,
    so only a batch whose first row failed it re-probes): each batch draws
    its own format (line length, separator, clean), deviant rows anywhere
    including row 0; every row exact."""
    rng = np.random.default_rng(3000 + seed)
    nbuf = int(rng.integers(2, 300))
    n = int(rng.integers(24, 2000))
    stride = (n + 2) // 3 * 4 * 2 + 8  # room for any separator density below
    cap = (b64.decoded_cap(stride) + 11) // 12 * 12
    x = torch.empty(nbuf * stride, dtype=torch.uint8, device=DEV)
    dec = torch.empty(nbuf * cap, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    for _ in range(12):
        L = int(rng.choice([0, 16, 19, 64, 76, 76, 100]))
        sep = b"".join(JUNK[rng.integers(4)] for _ in range(rng.integers(1, 5)))
        rows = []
        for i in range(nbuf):
            c = orc.encode(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            t = sep.join(c[j:j + L] for j in range(0, len(c), L)) + sep if L else c
            if rng.random() < 0.05:
                t = t[:5] + b"\x80" + t[5:]
            rows.append(t[:stride])
        flat = b"".join(r + b"\n" * (stride - len(r)) for r in rows)
        x.copy_(torch.from_numpy(np.frombuffer(flat, dtype=np.uint8).copy()).to(DEV))
        b64.decode_strided(x, stride, stride, nbuf, dec, cap, outlen)
        ol = outlen.cpu().tolist()
        dh = dec.cpu().numpy()
        for i, r in enumerate(rows):
            want = orc.decode(r + b"\n" * (stride - len(r)))
            assert ol[i] == len(want), (seed, i)
            assert dh[i * cap:i * cap + ol[i]].tobytes() == want, (seed, i)


def _fit(text: bytes, size: int, rng) -> bytes:
    """text cut or extended (with clean characters) to exactly size bytes."""
    if len(text) >= size:
        return text[:size]
    pad = orc.encode(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
    return (text + pad)[:size]


@pytest.mark.parametrize("seed", range(4))
def test_reuse_fuzz_interleaved(seed):
    """Calls that reuse models: single-buffer decodes drawn from three
    lengths (so the held model is taken whenever the last call of that
    length found nothing past k_decode_lines) with the content kind, the
    alphabet and HOLD_TAIL changing between calls, on the stream's library
    workspace or a caller's, interleaved with row batches of two shapes on
    the same stream (which keep their own model in the library workspace),
    some calls issued back to back without a sync.  Every result exact."""
    rng = np.random.default_rng(5000 + seed)
    sizes = [int(rng.integers(20, 64)), int(rng.integers(3000, 5000)),
             int(rng.integers(150_000, 400_000))]
    ws = torch.zeros(b64.workspace_size(max(sizes)), dtype=torch.uint8, device=DEV)
    pending = []

    def check(p):
        kind, args = p[0], p[1:]
        if kind == "one":
            text, abc, hold, d = args
            want = orc.decode(text, abc[0], abc[1])
            info = d.info()
            got = d.bytes().cpu().numpy().tobytes()
            if hold:
                assert got == want[:info.out_len] and info.out_len == info.valid // 4 * 3
            else:
                assert got == want, (seed, len(text))
        else:
            rows, stride, cap, out, outlen = args
            ol = outlen.cpu().tolist()
            dh = out.cpu().numpy()
            for i, r in enumerate(rows):
                want = orc.decode(r)
                assert ol[i] == len(want), (seed, i)
                assert dh[i * cap:i * cap + ol[i]].tobytes() == want, (seed, i)

    for _ in range(90):
        if rng.random() < 0.2:
            # a row batch: 200 rows of one of two shapes, CRLF-76 or clean,
            # a few deviant rows
            L = int(rng.choice([700, 1024]))
            raws = [orc.encode(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
                    for _ in range(200)]
            if rng.integers(2):
                raws = [b"\r\n".join(r[i:i + 76] for i in range(0, len(r), 76)) + b"\r\n"
                        for r in raws]
            for k in rng.integers(0, 200, int(rng.integers(0, 3))):
                raws[k] = raws[k][:5] + b"\t" + raws[k][6:]
            stride = max(len(r) for r in raws) + 4
            rows = [r + b"\n" * (stride - len(r)) for r in raws]
            cap = (b64.decoded_cap(stride) + 11) // 12 * 12
            out = torch.empty(200 * cap, dtype=torch.uint8, device=DEV)
            outlen = torch.zeros(200, dtype=torch.int64, device=DEV)
            x = torch.from_numpy(np.frombuffer(b"".join(rows), np.uint8).copy()).to(DEV)
            b64.decode_strided(x, stride, stride, 200, out, cap, outlen)
            pending.append(("rows", rows, stride, cap, out, outlen))
        else:
            size = sizes[int(rng.integers(3))]
            text, abc = _text(rng)
            if rng.random() < 0.5:
                abc = (-1, -1)
                text = orc.encode(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
            text = _fit(text, size, rng)
            hold = bool(rng.integers(4) == 0)
            x = torch.from_numpy(np.frombuffer(text, np.uint8).copy()).to(DEV)
            out = torch.empty(b64.decoded_cap(size) + 4, dtype=torch.uint8, device=DEV)
            d = b64.decode(x, out=out, abc=(abc[0], abc[1], True, -1), hold_tail=hold,
                           workspace=ws if rng.integers(2) else None)
            pending.append(("one", text, abc, hold, d))
        if rng.random() < 0.6:  # otherwise leave it in flight behind the next call
            for p in pending:
                check(p)
            pending.clear()
    for p in pending:
        check(p)
