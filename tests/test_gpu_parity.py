"""GPU parity: the HIP kernels, called through the C ABI, against the
oracle and the golden fixtures.  Bit-exact everywhere (integer/byte work).

Sizes: oracle comparisons at sizes the oracle finishes in well under a
second; full BASELINE sizes (1 GiB, 1 M x 1 KiB) through size-independent
properties (digests recorded from the reference, round trips, lengths).
"""
import hashlib

import os

import numpy as np
import pytest
import torch

from async_amd import b64
from oracle import pyoracle as orc
from tests import util

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def dev(data) -> torch.Tensor:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    if a.size == 0:
        return torch.empty(0, dtype=torch.uint8, device=DEV)
    return torch.from_numpy(a.copy()).to(DEV)


def genc(data, pos62=-1, pos63=-1, pad=True, padchar=-1) -> bytes:
    return b64.encode(dev(data), abc=(pos62, pos63, pad, padchar)).cpu().numpy().tobytes()


def _named(info, n, hold):
    """The device record names its call (include/b64x.h b64x_dec_result)."""
    assert info.nchars == n and info.seq != 0 and info.flags == int(hold), \
        (info.nchars, n, info.seq, info.flags)
    for k in range(4):
        assert (info.tail[k] < 64) if k < info.tail_n else info.tail[k] == 0
    return info


def gdec(chars, pos62=-1, pos63=-1, hold=False):
    d = b64.decode(dev(chars), abc=(pos62, pos63, True, -1), hold_tail=hold)
    return d.bytes().cpu().numpy().tobytes(), _named(d.info(), len(chars), hold)


def test_device_and_library():
    b64.device_check()
    assert "gfx950" in b64.build_info()


def test_encode_kat():
    for c in util.golden("kat_encode.json"):
        data = (util.splitmix64(c["seed"], c["n"]).tobytes() if "gen" in c
                else bytes.fromhex(c["in"]))
        got = genc(data, c["pos62"], c["pos63"], c["pad"], c["padchar"])
        if "out" in c:
            assert got.hex() == c["out"], (c["mode"], len(data))
        else:
            assert hashlib.sha256(got).hexdigest() == c["out_sha256"], c["n"]


def test_decode_kat():
    for c in util.golden("kat_decode.json"):
        got, _ = gdec(bytes.fromhex(c["in"]), c["pos62"], c["pos63"])
        assert got.hex() == c["out"], (c["mode"], c["variant"])


def test_leniency_table():
    t = util.golden("leniency.json")
    for c in t["decode"]:
        got, _ = gdec(bytes.fromhex(c["in"]), c["pos62"], c["pos63"])
        assert got.hex() == c["out"], c
    for c in t["encode"]:
        got = genc(bytes.fromhex(c["in"]), c["pos62"], c["pos63"], c["pad"], c["padchar"])
        assert got.decode() == c["out"], c


@pytest.mark.parametrize("abc", [(-1, -1, True, -1), (-1, -1, False, -1),
                                 (".", "_", True, "-"), (0xE9, 0xE8, True, 0x80)])
def test_encode_sizes_vs_oracle(abc):
    rng = np.random.default_rng(1)
    sizes = list(range(0, 100)) + [767, 768, 769, 3071, 3072, 3073, 12 * 1024 + 5,
                                   65535, 65536, 65537, 1 << 20, (1 << 20) + 1]
    sizes += list(rng.integers(100, 300000, 12))
    for n in sizes:
        host = rng.integers(0, 256, int(n), dtype=np.uint8)
        assert genc(host, *abc) == orc.encode(host, *abc), n


def test_encode_misaligned():
    """Input and output views at every offset mod 16 (fallback paths)."""
    rng = np.random.default_rng(2)
    host = rng.integers(0, 256, 50000, dtype=np.uint8)
    big = dev(host)
    for off in range(16):
        for n in (1, 11, 12, 13, 4097, 40000):
            x = big[off:off + n]
            out = torch.zeros(b64.encoded_len(n) + 32, dtype=torch.uint8, device=DEV)
            o = out[(off * 7) % 16:]
            got = b64.encode(x, out=o).cpu().numpy().tobytes()
            assert got == orc.encode(host[off:off + n]), (off, n)


def _junk(rng, chars: bytes, density: float, run_every=0, run_len=0) -> bytes:
    a = np.frombuffer(chars, dtype=np.uint8)
    junk_set = np.array([c for c in range(256) if not (chr(c).isalnum() and c < 128)
                         and c not in b"+/"], dtype=np.uint8)
    if density > 0:
        k = max(1, int(len(a) * density))
        pos = np.sort(rng.integers(0, len(a) + 1, k))
        a = np.insert(a, pos, rng.choice(junk_set, k))
    if run_every:
        pieces = []
        for i in range(0, len(a), run_every):
            pieces.append(a[i:i + run_every])
            pieces.append(rng.choice(junk_set, run_len))
        a = np.concatenate(pieces) if pieces else a
    return a.tobytes()


@pytest.mark.parametrize("density", [0.0, 1e-5, 1e-3, 0.05, 0.5])
def test_decode_dirty_vs_oracle(density):
    """Junk anywhere, including across the kernel's range boundaries."""
    rng = np.random.default_rng(int(density * 1e6) + 3)
    for n in (0, 1, 5, 1000, 4096 * 3 + 17, 300000, 2_000_000):
        host = rng.integers(0, 256, n, dtype=np.uint8)
        chars = orc.encode(host)
        dirty = _junk(rng, chars, density)
        got, info = gdec(dirty)
        want = orc.decode(dirty)
        assert got == want, (n, density)
        if density == 0.0:
            assert got == host.tobytes()


def test_decode_structured_junk():
    rng = np.random.default_rng(4)
    host = rng.integers(0, 256, 1_500_000, dtype=np.uint8)
    chars = orc.encode(host)
    cases = {
        "crlf76": b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76)),
        "pad_mid": chars[:100001] + b"==" + chars[100001:],
        "long_runs": _junk(rng, chars, 0, run_every=700_001, run_len=300_000),
        "lead_trail": b"\n" * 5000 + chars + b"=\n" * 9000,
        "tiny_runs": _junk(rng, chars, 0, run_every=4093, run_len=3),
    }
    for name, dirty in cases.items():
        got, info = gdec(dirty)
        assert got == orc.decode(dirty), name
    # all junk
    junk = bytes(rng.integers(0x80, 0x100, 1_000_000, dtype=np.uint8))
    got, info = gdec(junk)
    assert got == b"" and info.valid == 0 and info.out_len == 0


def test_decode_result_and_hold_tail():
    rng = np.random.default_rng(5)
    for n in (1, 2, 3, 4, 5, 6, 7, 8, 100, 4096 * 5 + 1, 4096 * 5 + 2, 1 << 20):
        host = rng.integers(0, 256, n, dtype=np.uint8)
        chars = orc.encode(host, pad=False)
        dirty = _junk(rng, chars, 0.01)
        table = orc.decode_table()
        alnum = [c for c in dirty if table[c] >= 0]
        valid = len(alnum)
        got, info = gdec(dirty)
        assert info.valid == valid and info.out_len == valid * 6 // 8 == len(got)
        assert info.tail_n == valid % 4
        held, hinfo = gdec(dirty, hold=True)
        assert hinfo.out_len == valid // 4 * 3 and held == got[: hinfo.out_len]
        tail = [table[c] for c in alnum[len(alnum) - valid % 4:]] if valid % 4 else []
        assert list(hinfo.tail[: hinfo.tail_n]) == tail


@pytest.mark.parametrize("abc", [(".", "_"), ("A", "*"), ("*", "*"), (0xE9, 0xE8),
                                 ("=", "\n")])
def test_decode_alphabets_vs_oracle(abc):
    rng = np.random.default_rng(6)
    table = np.array(orc.decode_table(*abc))
    for n in (10, 5000, 400_000):
        # bytes drawn from the whole 0..255 range: alphabet, pos62/63, junk
        raw = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        got, info = gdec(raw, *abc)
        assert got == orc.decode(raw, *abc), (abc, n)
        assert info.valid == int((table[np.frombuffer(raw, np.uint8)] >= 0).sum())


def test_g1_g2_digests():
    d = util.golden("digests.json")
    g1 = genc(util.counting(1000001), ".", "_", True, "-")
    assert hashlib.sha256(g1).hexdigest() == d["G1"]["out_sha256"]
    g2 = genc(util.counting(1 << 20))
    assert hashlib.sha256(g2).hexdigest() == d["G2"]["out_sha256"]


@pytest.mark.slow
def test_g3_1gib_roundtrip():
    """BASELINE config 2 at full size: the recorded reference digest of the
    1 GiB splitmix64 buffer, and decode(encode(x)) == x on the device."""
    d = util.golden("digests.json")["G3"]
    x = torch.empty(d["n"], dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, d["seed"])
    assert hashlib.sha256(x.cpu().numpy()).hexdigest() == d["in_sha256"]
    enc = b64.encode(x)
    assert enc.numel() == d["out_len"]
    assert hashlib.sha256(enc.cpu().numpy()).hexdigest() == d["out_sha256"]
    dd = b64.decode(enc)
    info = dd.info()
    assert info.out_len == d["n"] and info.valid == d["out_len"] - 2
    assert torch.equal(dd.out[: d["n"]], x)


def _strided_check(nbuf, length, sample_idx, g4=None, whole=None):
    qstride_out = b64.encoded_len(length)
    x = torch.empty(nbuf * length, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0x5EED)
    enc = torch.empty(nbuf * qstride_out, dtype=torch.uint8, device=DEV)
    b64.encode_strided(x, length, length, nbuf, enc, qstride_out)
    host = x.cpu().numpy()
    ehost = enc.cpu().numpy()
    for i in sample_idx:
        want = orc.encode(host[i * length:(i + 1) * length])
        assert ehost[i * qstride_out:(i + 1) * qstride_out].tobytes() == want, i
    if g4:
        assert hashlib.sha256(ehost[:qstride_out].tobytes()).hexdigest().startswith(g4)
    if whole:
        # the whole output, not samples: every buffer's characters, laid out
        # back to back (tests/golden/batch_digests.json, make_golden.py)
        assert hashlib.sha256(host).hexdigest() == whole["in_sha256"]
        assert hashlib.sha256(ehost).hexdigest() == whole["out_sha256"]
        per = hashlib.sha256()
        rows = ehost.reshape(nbuf, qstride_out)
        for i in range(nbuf):
            per.update(hashlib.sha256(rows[i]).digest())
        assert per.hexdigest() == whole["per_buffer_sha256_of_sha256"]
    # exact-capacity rows (per-slot kernel) and 16-byte rows (the uniform
    # row kernel needs out_stride >= 12 * ceil(E/16))
    for cap in (b64.decoded_cap(qstride_out), (b64.decoded_cap(qstride_out) + 15) // 16 * 16):
        dec = torch.empty(nbuf * cap, dtype=torch.uint8, device=DEV)
        outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
        b64.decode_strided(enc, qstride_out, qstride_out, nbuf, dec, cap, outlen)
        assert int(outlen.min()) == length and int(outlen.max()) == length
        assert torch.equal(dec.view(nbuf, cap)[:, :length], x.view(nbuf, length))
        if whole:  # the decoded rows, whole, against the input stream's digest
            got = dec.view(nbuf, cap)[:, :length].contiguous().cpu().numpy()
            assert hashlib.sha256(got).hexdigest() == whole["in_sha256"]
            del got
        del dec


def test_strided_small_shapes():
    for nbuf, length in ((1, 1), (3, 2), (7, 3), (64, 12), (100, 1023), (33, 5000)):
        _strided_check(nbuf, length, range(nbuf))


@pytest.mark.parametrize("length", [16, 17, 18, 19, 20, 21, 22, 23, 28, 100, 101, 102, 1000,
                                    1001, 1024, 4096, 4097])
@pytest.mark.parametrize("nbuf", [3, 4, 257])
def test_strided_tight_layout(length, nbuf):
    """in_stride = len, out_stride = E: the output-indexed tight kernel
    (every len mod 3 and E mod 16 seam shape) plus its tail launch."""
    _strided_check(nbuf, length, range(nbuf))


@pytest.mark.parametrize("abc", [("-", "_", True, "#"), (".", "_", False, -1)])
def test_strided_tight_alphabets(abc):
    rng = np.random.default_rng(5)
    for length in (1024, 1026, 31):
        nbuf = 50
        E = b64.encoded_len(length, abc[2])
        host = rng.integers(0, 256, nbuf * length, dtype=np.uint8)
        enc = torch.zeros(nbuf * E, dtype=torch.uint8, device=DEV)
        b64.encode_strided(dev(host), length, length, nbuf, enc, E, abc=abc)
        eh = enc.cpu().numpy()
        for i in range(nbuf):
            assert eh[i * E:(i + 1) * E].tobytes() == orc.encode(
                host[i * length:(i + 1) * length], *abc), (length, i)


@pytest.mark.parametrize("cap_extra", [0, 5, 16])
@pytest.mark.parametrize("length,gap_in,gap_out", [(777, 5, 3), (1024, 0, 0), (4096, 16, 8),
                                                   (13, 1, 0), (100, 0, 7)])
def test_strided_odd_strides_and_junk(length, gap_in, gap_out, cap_extra):
    """Grouped batch kernels with strides that break line alignment, plus
    buffers with junk (exact fix-up path), each buffer vs the oracle."""
    rng = np.random.default_rng(length + gap_in)
    nbuf = 301
    E = b64.encoded_len(length)
    ins, outs = length + gap_in, E + gap_out
    host = rng.integers(0, 256, nbuf * ins, dtype=np.uint8)
    x = dev(host)
    enc = torch.zeros(nbuf * outs, dtype=torch.uint8, device=DEV)
    b64.encode_strided(x, ins, length, nbuf, enc, outs)
    eh = enc.cpu().numpy()
    for i in range(nbuf):
        want = orc.encode(host[i * ins:i * ins + length])
        assert eh[i * outs:i * outs + E].tobytes() == want, i
    # junk in every 7th buffer: a CR, a '=', a run of spaces
    for i in range(0, nbuf, 7):
        j = i * outs + int(rng.integers(0, E))
        eh[j] = (13, 61, 32)[i % 3]
    cap = b64.decoded_cap(E) + cap_extra
    dec = torch.zeros(nbuf * cap, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    b64.decode_strided(dev(eh), outs, E, nbuf, dec, cap, outlen)
    dh, ol = dec.cpu().numpy(), outlen.cpu().numpy()
    for i in range(nbuf):
        want = orc.decode(eh[i * outs:i * outs + E])
        assert int(ol[i]) == len(want), i
        assert dh[i * cap:i * cap + len(want)].tobytes() == want, i


@pytest.mark.parametrize("E", [20, 24, 28, 31, 32, 33, 40, 1368, 1372])
def test_strided_rows_last_slot_shapes(E):
    """Dense rows (out_stride = 12 per 16-character slot, the row kernel):
    every row's last slot gets a different shape -- clean, padded, '='
    inside the prefix, junk after the padding, junk at each position, a
    lone alphabet character after junk -- each row vs the oracle."""
    rng = np.random.default_rng(E)
    nbuf = 1500
    S = (E + 15) // 16
    alpha = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/",
                          dtype=np.uint8)
    rows = rng.choice(alpha, (nbuf, E))
    lo = 16 * (S - 1)
    for i in range(nbuf):
        kind = i % 6
        if kind == 1:  # standard padding
            rows[i, E - 1 - (i // 6) % 2:] = ord("=")
        elif kind == 2:  # one junk byte anywhere in the last slot
            rows[i, lo + int(rng.integers(0, E - lo))] = (10, 13, 61, 32, 0xE9)[i % 5]
        elif kind == 3:  # a junk run to the end of the row
            rows[i, lo + int(rng.integers(0, E - lo)):] = ord("=")
        elif kind == 4:  # junk then one alphabet character at the very end
            if E - lo >= 2:
                rows[i, E - 2] = ord("\n")
        elif kind == 5:  # junk in an interior slot as well
            rows[i, int(rng.integers(0, E))] = ord(" ")
    flat = rows.reshape(-1)
    cap = 12 * S
    dec = torch.zeros(nbuf * cap, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    b64.decode_strided(dev(flat), E, E, nbuf, dec, cap, outlen)
    dh, ol = dec.cpu().numpy(), outlen.cpu().numpy()
    for i in range(nbuf):
        want = orc.decode(rows[i].tobytes())
        assert int(ol[i]) == len(want), (i, i % 6)
        assert dh[i * cap:i * cap + len(want)].tobytes() == want, (i, i % 6)


@pytest.mark.slow
def test_strided_cfg3_full():
    """65,536 x 4 KiB (BASELINE config 3)."""
    d = util.golden("digests.json")
    _strided_check(65536, 4096, [0, 1, 2, 31337, 65535], d["G4_4096"]["out_sha256_prefix"],
                   util.golden("batch_digests.json")["cfg3"])


@pytest.mark.slow
def test_strided_cfg4_full():
    """1,048,576 x 1 KiB (BASELINE config 4, one GPU's worth)."""
    d = util.golden("digests.json")
    _strided_check(1 << 20, 1024, [0, 1, 777777, (1 << 20) - 1],
                   d["G4_1024"]["out_sha256_prefix"], util.golden("batch_digests.json")["cfg4"])


@pytest.mark.slow
def test_strided_cfg4_crlf76_full():
    """Config 4's rows in RFC 2045 lines (18 x (76 + CRLF) = 1,404 bytes per
    row), decoded by the row kernel: the text and the decoded rows, whole,
    against tests/golden/batch_digests.json."""
    g = util.golden("batch_digests.json")["cfg4"]
    nbuf, L, E = g["nbuf"], g["len"], g["out_len"]
    D = g["crlf76"]["row_bytes"]
    x = torch.empty(nbuf * L, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0x5EED)
    enc = torch.empty(nbuf * E, dtype=torch.uint8, device=DEV)
    b64.encode_strided(x, L, L, nbuf, enc, E)
    crlf = torch.tensor([13, 10], dtype=torch.uint8, device=DEV).expand(nbuf, E // 76, 2)
    text = torch.cat([enc.view(nbuf, E // 76, 76), crlf], dim=2).reshape(-1).contiguous()
    del enc
    assert hashlib.sha256(text.cpu().numpy()).hexdigest() == g["crlf76"]["text_sha256"]
    cap = 12 * ((D + 15) // 16)
    dec = torch.empty(nbuf * cap, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    b64.decode_strided(text, D, D, nbuf, dec, cap, outlen)
    assert int(outlen.min()) == L and int(outlen.max()) == L
    got = dec.view(nbuf, cap)[:, :L].contiguous().cpu().numpy()
    assert hashlib.sha256(got).hexdigest() == g["crlf76"]["dec_sha256"]


def test_ragged_batch_vs_oracle():
    rng = np.random.default_rng(7)
    lens = [0, 1, 2, 3, 4, 63, 64, 65, 1000, 4096, 12345, 70000] + \
        list(rng.integers(0, 3000, 200))
    host = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in lens]
    in_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    elens = [b64.encoded_len(int(n)) for n in lens]
    out_off = np.concatenate([[0], np.cumsum(elens)[:-1]]).astype(np.int64)
    x = dev(np.concatenate(host))
    enc = torch.zeros(int(sum(elens)) + 1, dtype=torch.uint8, device=DEV)
    b64.encode_batch(x, torch.from_numpy(in_off).to(DEV), enc,
                     torch.from_numpy(out_off).to(DEV))
    eh = enc.cpu().numpy()
    chunks = []
    for i, h in enumerate(host):
        got = eh[out_off[i]:out_off[i] + elens[i]].tobytes()
        assert got == orc.encode(h), i
        chunks.append(got)
    # decode the same batch back, with junk in every third buffer
    dchunks = [c if i % 3 else _junk(rng, c, 0.02) for i, c in enumerate(chunks)]
    dlens = [len(c) for c in dchunks]
    din_off = np.concatenate([[0], np.cumsum(dlens)]).astype(np.int64)
    caps = [b64.decoded_cap(n) for n in dlens]
    dout_off = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    dec = torch.zeros(int(sum(caps)) + 1, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(len(lens), dtype=torch.int64, device=DEV)
    b64.decode_batch(dev(b"".join(dchunks) or b"\0"), torch.from_numpy(din_off).to(DEV),
                     dec, torch.from_numpy(dout_off).to(DEV), outlen)
    dh = dec.cpu().numpy()
    ol = outlen.cpu().numpy()
    for i, h in enumerate(host):
        assert ol[i] == len(h) and dh[dout_off[i]:dout_off[i] + ol[i]].tobytes() == h.tobytes()


def test_fill_splitmix64():
    d = util.golden("digests.json")
    x = torch.empty(4099, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0x5EED)
    assert np.array_equal(x.cpu().numpy(), util.splitmix64(0x5EED, 4099))
    assert x[:16].cpu().numpy().tobytes().hex() == d["splitmix64_head"]["first16"]


def test_library_workspace_per_stream():
    """d_workspace = NULL on two streams at once: each stream gets its own
    library workspace, so concurrent dirty decodes (pass 1 -> scan -> pass 2
    state lives in the workspace) do not trample each other."""
    import ctypes

    from async_amd import _lib

    lib = _lib.load()
    rng = np.random.default_rng(11)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = []
    for k in range(2):
        raw = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
        chars = orc.encode(raw)
        dirty = _junk(rng, chars, 0.01 * (k + 1))
        x = dev(dirty)
        out = torch.empty(b64.decoded_cap(len(dirty)), dtype=torch.uint8, device=DEV)
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
        jobs.append((x, out, res, raw))
    a = b64._abc(None)
    torch.cuda.synchronize()
    for rep in range(4):  # interleave the two streams' launches
        for (x, out, res, _), st in zip(jobs, streams):
            rc = lib.b64x_decode_dev(ctypes.c_void_p(x.data_ptr()), x.numel(),
                                     ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(res.data_ptr()), ctypes.byref(a), 0,
                                     None, ctypes.c_void_p(st.cuda_stream))
            assert rc == 0
    torch.cuda.synchronize()
    for x, out, res, raw in jobs:
        info = b64.Decoded(out, res).info()
        assert info.out_len == raw.size
        assert np.array_equal(out[: raw.size].cpu().numpy(), raw)


@pytest.mark.parametrize("fmt", ["crlf76", "lf64", "cr_lf_lf60", "crlf76_broken", "lf17",
                                 "lf16", "crlf300"])
def test_decode_line_structured(fmt):
    """Line-wrapped text (MIME CRLF-76, PEM LF-64, odd separators, a line of
    a different length mid-stream, line lengths at the fast path's limits):
    the line-structured ranges of pass 2 and their fall-backs, vs the oracle."""
    rng = np.random.default_rng(len(fmt))
    host = rng.integers(0, 256, 700_001, dtype=np.uint8)
    chars = orc.encode(host)
    Lc, sep = {"crlf76": (76, b"\r\n"), "lf64": (64, b"\n"), "cr_lf_lf60": (60, b"\r\n\n"),
               "crlf76_broken": (76, b"\r\n"), "lf17": (17, b"\n"), "lf16": (16, b"\n"),
               "crlf300": (300, b"\r\n")}[fmt]
    lines = [chars[i:i + Lc] for i in range(0, len(chars), Lc)]
    if fmt == "crlf76_broken":
        lines[5000] = lines[5000][:40]  # one short line mid-stream
    dirty = sep.join(lines) + sep
    got, info = gdec(dirty)
    want = orc.decode(dirty)
    assert got == want, fmt
    if fmt != "crlf76_broken":
        assert got == host.tobytes()


def _windows_match(x, enc, starts, width=3 * 4096):
    """enc[4k/3 ...] against the oracle's encoding of x[k ...] for windows
    starting at the input offsets `starts` (each rounded down to a group)."""
    n = x.numel()
    for s in starts:
        a = max(0, min(s, n - 1)) // 3 * 3
        b = min(n, a + width)
        want = orc.encode(x[a:b].cpu().numpy())
        if b < n:  # an inner window: no padding
            want = want[:(b - a) // 3 * 4]
        got = enc[a // 3 * 4:a // 3 * 4 + len(want)].cpu().numpy().tobytes()
        assert got == want, s


@pytest.mark.slow
def test_beyond_32bit_sizes():
    """Maximum sizes: a 5 GiB + 5 byte buffer (6.7 GB of characters), so
    every 32-bit byte, group and range index wraps.  Windows across the
    2^31/2^32/2^33 offsets match the oracle; the round trip is exact; and
    junk inserted at character offsets around 2^32 leaves the decoded
    bytes unchanged (the decoder skips it, base64decoder.c:48-60)."""
    n = (5 << 30) + 5
    x = torch.empty(n, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0xB16)
    enc = b64.encode(x)
    assert enc.numel() == b64.encoded_len(n)
    marks = [0, (1 << 31) - 7, (1 << 32) - 7, (1 << 32) // 4 * 3 - 7, (1 << 33) // 4 * 3 - 9,
             n - 5000]
    _windows_match(x, enc, marks)
    dd = b64.decode(enc)
    assert dd.info().out_len == n
    assert torch.equal(dd.out[:n], x)
    del dd
    cuts = [(1 << 32) - 3, (1 << 32) + 1, (1 << 33) - 2]
    junk = [torch.tensor(list(b"\r\n"), dtype=torch.uint8, device=DEV),
            torch.full((5000,), ord("*"), dtype=torch.uint8, device=DEV),
            torch.tensor(list(b"\x00\xff="), dtype=torch.uint8, device=DEV)]
    pieces, prev = [], 0
    for c, j in zip(cuts, junk):
        pieces += [enc[prev:c], j]
        prev = c
    pieces.append(enc[prev:])
    dirty = torch.cat(pieces)
    del enc, pieces
    dd = b64.decode(dirty)
    assert dd.info().out_len == n
    assert torch.equal(dd.out[:n], x)
    del dd
    # the single pass over all of it: the held suffix's tile prefixes pass
    # 2^32 characters (64-bit sums) and its tiles 2^16 (round 6: up to
    # kLinesMaxChars on the lines path)
    dd = b64.decode(dirty, expect_junk=True)
    assert dd.info().out_len == n
    assert torch.equal(dd.out[:n], x)


def _gpu_lines(chars: torch.Tensor, L: int, sep: bytes) -> torch.Tensor:
    """chars in lines of L characters, each followed by `sep` (the last
    line short, with its separator), built on the GPU (no boolean masks:
    torch's mask indexing fails past 2^31 elements)."""
    n = chars.numel()
    full = n // L
    sp = torch.tensor(list(sep), dtype=torch.uint8, device=chars.device)
    body = torch.cat([chars[:full * L].view(full, L), sp.expand(full, len(sep))], dim=1).reshape(-1)
    if n % L:
        body = torch.cat([body, chars[full * L:], sp])
    return body.contiguous()


@pytest.mark.parametrize("L,sep", [(76, b"\r\n"), (70, b"\n")])
def test_beyond_31bit_lines(L, sep):
    """MIME-formatted text past 2^31 characters (round 6: the lines path's
    64-bit wave bases, k_decode_lines<true>, both slot forms: L % 4 == 0 and
    not): 1.6 GiB of payload in lines, decoded whole, then with a junk byte
    near the end (the suffix from there, 64-bit prefix); windows across 2^31
    and 2^32 characters against the oracle's decode of the same text."""
    n = 1717986918  # 1.6 GiB: 2.29 G characters, 2.35-2.36 G bytes with separators
    x = torch.empty(n, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0x11E5 + L)
    enc = b64.encode(x)
    text = _gpu_lines(enc, L, sep)
    del enc
    assert text.numel() > (1 << 31)
    dd = b64.decode(text)
    assert dd.info().out_len == n
    assert torch.equal(dd.out[:n], x)
    del dd
    # the oracle on 40-line windows that start on (even) line boundaries,
    # across 2^31 and 2^32 bytes of text
    W = L + len(sep)
    for at in ((1 << 31) - 5000, (1 << 31) + 77, text.numel() - 3 * W * 40):
        a = at // (2 * W) * (2 * W)
        want = orc.decode(text[a:a + 40 * W].cpu().numpy().tobytes())
        o = a // W * L // 4 * 3
        assert x[o:o + len(want)].cpu().numpy().tobytes() == want, at
    # one junk byte inserted late in the stream: the lines pass stops there
    # and the suffix decodes the rest
    k = text.numel() - 1000
    text = torch.cat([text[:k], torch.tensor([ord("*")], dtype=torch.uint8, device=DEV), text[k:]])
    dd = b64.decode(text)
    assert dd.info().out_len == n
    assert torch.equal(dd.out[:n], x)


@pytest.mark.slow
def test_beyond_32bit_strided_batch():
    """A batch whose total input and output pass 4 GiB: 4,194,307 rows of
    1,100 bytes.  Rows around the 2^32 byte offsets match the oracle and
    the row round trip is exact."""
    nbuf, length = (1 << 22) + 3, 1100
    E = b64.encoded_len(length)
    x = torch.empty(nbuf * length, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0x5EED)
    enc = torch.empty(nbuf * E, dtype=torch.uint8, device=DEV)
    b64.encode_strided(x, length, length, nbuf, enc, E)
    for i in (0, (1 << 32) // length - 1, (1 << 32) // length, (1 << 32) // E,
              (1 << 32) // E + 1, nbuf - 1):
        row = x[i * length:(i + 1) * length].cpu().numpy()
        assert enc[i * E:(i + 1) * E].cpu().numpy().tobytes() == orc.encode(row), i
    cap = (b64.decoded_cap(E) + 15) // 16 * 16
    dec = torch.empty(nbuf * cap, dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    b64.decode_strided(enc, E, E, nbuf, dec, cap, outlen)
    assert int(outlen.min()) == length and int(outlen.max()) == length
    assert torch.equal(dec.view(nbuf, cap)[:, :length], x.view(nbuf, length))


@pytest.mark.slow
def test_beyond_32bit_ragged_batch():
    """Ragged batch with a job longer than 4 GiB and offsets past 2^32:
    windows of every job match the oracle, the round trip is exact."""
    lens = [5, (1 << 32) + 100, 7, 3 << 29, 1000]
    in_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    elens = [b64.encoded_len(n) for n in lens]
    out_off = np.concatenate([[0], np.cumsum(elens)[:-1]]).astype(np.int64)
    x = torch.empty(int(in_off[-1]), dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0xACE)
    enc = torch.zeros(int(sum(elens)), dtype=torch.uint8, device=DEV)
    b64.encode_batch(x, torch.from_numpy(in_off).to(DEV), enc,
                     torch.from_numpy(out_off).to(DEV))
    for i, n in enumerate(lens):
        xi = x[int(in_off[i]):int(in_off[i + 1])]
        ei = enc[int(out_off[i]):int(out_off[i]) + elens[i]]
        _windows_match(xi, ei, [0, (1 << 31) - 4, (1 << 32) // 4 * 3 - 5, (1 << 32) - 2,
                                n - 3000])
    caps = [b64.decoded_cap(n) for n in elens]
    dout_off = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    dec = torch.empty(int(sum(caps)), dtype=torch.uint8, device=DEV)
    outlen = torch.zeros(len(lens), dtype=torch.int64, device=DEV)
    ein_off = np.concatenate([[0], np.cumsum(elens)]).astype(np.int64)
    b64.decode_batch(enc, torch.from_numpy(ein_off).to(DEV), dec,
                     torch.from_numpy(dout_off).to(DEV), outlen)
    assert outlen.cpu().tolist() == lens
    for i, n in enumerate(lens):
        assert torch.equal(dec[int(dout_off[i]):int(dout_off[i]) + n],
                           x[int(in_off[i]):int(in_off[i + 1])]), i


@pytest.mark.parametrize("chunks", [3, 8])
def test_decode_long_ranges_vs_oracle(chunks):
    """Ranges longer than one 2,048-character step (what inputs past 2 GiB
    get, since the range count is capped), forced at small sizes through the
    test build's range-size hook (tests/csrc/libb64x_hooks.so): the exact
    pass flushes its window between steps."""
    import ctypes
    from async_amd import _lib
    L = util.hooks()
    old = L.b64x__test_range_chunks(chunks)

    def hdec(chars: bytes, hold: bool):
        x = dev(chars)
        out = torch.empty(max(b64.decoded_cap(len(chars)), 1), dtype=torch.uint8, device=DEV)
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
        ws = torch.zeros(b64.workspace_size(len(chars)), dtype=torch.uint8, device=DEV)
        a = _lib.alphabet()
        _lib.check("b64x_decode_dev", L.b64x_decode_dev(
            x.data_ptr(), len(chars), out.data_ptr(), res.data_ptr(), ctypes.byref(a),
            b64.HOLD_TAIL if hold else 0, ws.data_ptr(),
            torch.cuda.current_stream().cuda_stream))
        info = b64.Decoded(out, res).info()
        return out[:info.out_len].cpu().numpy().tobytes(), info

    try:
        rng = np.random.default_rng(chunks)
        for n in (1, 5000, 3 * 1024 * chunks + 7, 400_000):
            host = rng.integers(0, 256, n, dtype=np.uint8)
            chars = orc.encode(host)
            for dirty in (b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76)),
                          _junk(rng, chars, 0.3),
                          _junk(rng, chars, 0, run_every=5000, run_len=3000)):
                for hold in (False, True):
                    got, info = hdec(dirty, hold)
                    want = orc.decode(dirty)
                    if hold:  # whole groups only; the rest is held back
                        assert info.out_len == 3 * (info.valid // 4)
                        assert got == want[:info.out_len], (n, len(dirty))
                    else:
                        assert got == want, (n, len(dirty))
    finally:
        L.b64x__test_range_chunks(old)


def gdec_j(chars, pos62=-1, pos63=-1, hold=False):
    d = b64.decode(dev(chars), abc=(pos62, pos63, True, -1), hold_tail=hold,
                   expect_junk=True)
    return d.bytes().cpu().numpy().tobytes(), _named(d.info(), len(chars), hold)


@pytest.mark.parametrize("density", [0.0, 1e-3, 0.05, 0.5])
def test_single_pass_decode_vs_oracle(density):
    """B64X_DEC_EXPECT_JUNK (one pass: counts, tile look-back, exact
    decode) gives the oracle's bytes and result record, with and without
    HOLD_TAIL, on clean and dirty input, across tile boundaries (16 ranges
    of 2,048 characters per tile)."""
    rng = np.random.default_rng(int(density * 1e4) + 11)
    for n in (0, 1, 2, 5, 1000, 4096 * 3 + 17, 300000, 2_000_000):
        host = rng.integers(0, 256, n, dtype=np.uint8)
        chars = orc.encode(host)
        dirty = _junk(rng, chars, density)
        want = orc.decode(dirty)
        got, info = gdec_j(dirty)
        assert got == want, (n, density)
        ref, rinfo = gdec(dirty)
        assert (info.out_len, info.valid) == (rinfo.out_len, rinfo.valid)
        hgot, hinfo = gdec_j(dirty, hold=True)
        href, hrinfo = gdec(dirty, hold=True)
        assert hgot == href and hinfo.tail_n == hrinfo.tail_n, n
        assert bytes(hinfo.tail)[:hinfo.tail_n] == bytes(hrinfo.tail)[:hrinfo.tail_n], n


def test_single_pass_decode_repeated_large():
    """Repeated single-pass decodes of one large junk-laden stream in one
    process, every output checked: the form of the stress that found the
    suffix kernel's loop-top barrier not waiting for thread 0's LDS write of
    the next tile's ticket (a wave then decoded another tile; one 1 GiB
    decode in 5 to 60 came out shifted, DESIGN.md §5, scripts/held_stress.py).
    Smaller and shorter here; round trip, so size-independent."""
    n = 192 << 20
    x = torch.empty(n, dtype=torch.uint8, device=DEV)
    b64.fill_splitmix64(x, 0xB10C)
    chars = b64.encode(x)
    g = torch.Generator(device=DEV).manual_seed(3)
    for d in (0.05, 0.001):
        mask = torch.rand(chars.numel(), device=DEV, generator=g) < d
        idx = torch.arange(chars.numel(), device=DEV) + torch.cumsum(mask, 0)
        text = torch.full((chars.numel() + int(mask.sum()),), ord("!"), dtype=torch.uint8,
                          device=DEV)
        text[idx] = chars
        del mask, idx
        out = torch.empty(b64.decoded_cap(text.numel()), dtype=torch.uint8, device=DEV)
        ws = torch.zeros(b64.workspace_size(text.numel()), dtype=torch.uint8, device=DEV)
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
        for it in range(12):
            out.fill_(0xAA)
            b64.decode(text, out=out, workspace=ws, result=res, expect_junk=it % 2 == 0)
            info = b64.Decoded(out, res).info()
            assert info.out_len == n and torch.equal(out[:n], x), (d, it)
        del text, out, ws


def test_single_pass_decode_structured_and_alphabets():
    rng = np.random.default_rng(12)
    host = rng.integers(0, 256, 1_500_000, dtype=np.uint8)
    for abc in ((-1, -1), (".", "_"), ("\n", "\r")):
        chars = orc.encode(host, abc[0], abc[1], True, -1)
        for dirty in (b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76)),
                      chars[:100001] + b"==" + chars[100001:],
                      _junk(rng, chars, 0, run_every=700_001, run_len=300_000),
                      b"\n" * 5000 + chars + b"=\n" * 9000):
            got, info = gdec_j(dirty, *abc)
            assert got == orc.decode(dirty, *abc), abc
    junk = bytes(rng.integers(0x80, 0x100, 1_000_000, dtype=np.uint8))
    got, info = gdec_j(junk)
    assert got == b"" and info.valid == 0 and info.out_len == 0
    # the workspace is left re-armed: the two paths alternate on one stream
    for k in range(4):
        chars = orc.encode(rng.integers(0, 256, 100_000 + k, dtype=np.uint8))
        d = b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76))
        assert (gdec_j(d) if k % 2 else gdec(d))[0] == orc.decode(d)


def _wrap(chars: bytes, L: int, sep: bytes, trailing=True) -> bytes:
    lines = [chars[i:i + L] for i in range(0, len(chars), L)]
    return sep.join(lines) + (sep if trailing and lines else b"")


@pytest.mark.parametrize("L,sep", [(76, b"\r\n"), (64, b"\n"), (16, b"\r\n"), (20, b"\n\n\n\n"),
                                   (17, b"\n"), (19, b"\r\n\n"), (252, b"\n"), (253, b"\n")])
def test_decode_lines_shapes_vs_oracle(L, sep):
    """The line-structured single pass (k_decode_lines) and its suffix decode
    on many stream lengths around slot, line and window boundaries: with and
    without a trailing separator, padded or not, HOLD_TAIL, input and output
    at every alignment, and a stream that breaks the model once (a short
    line, an '=' inside, a junk byte) -- every result against the oracle."""
    rng = np.random.default_rng(L * 7 + len(sep))
    for n in (0, 1, 2, 11, 12, 13, 47, 48, 300, 1001, 4096, 40_000):
        host = rng.integers(0, 256, n, dtype=np.uint8)
        chars = orc.encode(host)
        for trailing in (True, False):
            text = _wrap(chars, L, sep, trailing)
            variants = [text]
            if len(text) > 3 * (L + len(sep)):
                k = (len(text) // (L + len(sep)) // 2) * (L + len(sep))
                variants += [text[:k + 10] + text[k + 11:],          # one short line
                             text[:k + 5] + b"=" + text[k + 6:],     # '=' at a model position
                             text[:k + L] + b"\t" + text[k + L:]]    # one more separator byte
            for v in variants:
                want = orc.decode(v)
                got, info = gdec(v)
                assert got == want, (n, trailing, len(v))
                gh, ih = gdec(v, hold=True)
                assert ih.out_len == 3 * (ih.valid // 4) and ih.valid == info.valid
                assert gh == want[:ih.out_len]
    # alignment of input and output (decode into a slice of a larger buffer)
    host = rng.integers(0, 256, 20_000, dtype=np.uint8)
    text = _wrap(orc.encode(host), L, sep)
    want = orc.decode(text)
    for off in range(4):
        xs = dev(bytes(off) + text)[off:]  # the text at offset `off` of a fresh buffer
        outbuf = torch.empty(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV)
        d = b64.decode(xs, out=outbuf[off:], abc=(-1, -1, True, -1))
        got = d.bytes().cpu().numpy().tobytes()
        assert got == want, off


def _sfx_start(ws: torch.Tensor) -> int:
    """The workspace's record of where the last call's exact suffix decode
    started (header bytes 24..31; 2**64 - 1: it had nothing to do)."""
    torch.cuda.synchronize()
    return int(np.frombuffer(ws[24:32].cpu().numpy().tobytes(), np.uint64)[0])


@pytest.mark.parametrize("aligned", [True, False])
def test_decode_lines_takes_clean_and_mime_whole(aligned):
    """Clean text and MIME/PEM-formatted text are decoded by k_decode_lines
    alone -- the exact suffix decode has nothing to do (a speed property the
    results alone cannot show: the suffix would decode them exactly too) --
    while a stream that breaks the model hands over at its first failing
    slot, at or before the break."""
    rng = np.random.default_rng(41)
    chars = orc.encode(rng.integers(0, 256, 3_000_000, dtype=np.uint8))
    ws = torch.zeros(b64.workspace_size(len(chars) * 2), dtype=torch.uint8, device=DEV)
    off = 0 if aligned else 1
    cases = [(chars, None), (_wrap(chars, 76, b"\r\n"), None), (_wrap(chars, 64, b"\n"), None)]
    k = 2_000_000
    cases.append((chars[:k] + b"!" + chars[k:], k))
    mime = _wrap(chars, 76, b"\r\n")
    cases.append((mime[:k] + b"=" + mime[k + 1:], k))
    for text, brk in cases:
        x = dev(bytes(off) + text)[off:]
        out = torch.empty(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV)
        d = b64.decode(x, out=out, workspace=ws)
        assert d.bytes().cpu().numpy().tobytes() == orc.decode(text)
        start = _sfx_start(ws)
        if brk is None:
            assert start == 2**64 - 1, (len(text), start)
        else:
            assert start <= brk and brk - start < 1 << 12, (brk, start)


def test_repeat_junk_decode_takes_the_hinted_single_pass():
    """A call whose probe cut the line model near the start leaves a hint
    for the next call on the same workspace, input and length: that one
    takes the single pass (no k_decode_lines launch), which runs the probe
    itself in its first block left without a tile.
    Every call is exact; a clean stream in the same buffer goes back to the
    lines pass on the call after the one that finds it clean."""
    rng = np.random.default_rng(47)
    chars = orc.encode(rng.integers(0, 256, 3_000_000, dtype=np.uint8))
    junky = _junk(rng, chars, 0.05)
    clean = orc.encode(rng.integers(0, 256, len(junky), dtype=np.uint8))[:len(junky)]
    buf = torch.empty(len(junky), dtype=torch.uint8, device=DEV)
    out = torch.empty(b64.decoded_cap(len(junky)) + 8, dtype=torch.uint8, device=DEV)
    ws = torch.zeros(b64.workspace_size(len(junky)), dtype=torch.uint8, device=DEV)
    starts = []
    for text in (junky, junky, junky, clean, clean):
        buf.copy_(dev(text))
        d = b64.decode(buf, out=out, workspace=ws)
        assert d.bytes().cpu().numpy().tobytes() == orc.decode(text)
        starts.append(_sfx_start(ws))
    # the first junk call: the lines pass and the suffix from the cut; the
    # hinted ones leave the record of where a suffix started alone
    assert starts[0] < len(junky) // 16 and starts[1] == starts[2] == starts[0]
    # the first clean call still ran on the hint; its probe renewed it
    assert starts[3] == starts[0] and starts[4] == 2**64 - 1


def test_held_model_reused_across_calls_of_one_length():
    """Calls of one length on one workspace reuse the model its last probe
    made (no probe) until a call finds anything past k_decode_lines; the
    data under a held model changes format, gains junk, loses it again, and
    the workspace is zeroed under a held entry (k_decode_lines then finds a
    model of another length and leaves the whole stream to the suffix):
    every call exact, on a caller's workspace and on the library's."""
    rng = np.random.default_rng(53)
    n = 3_000_001
    clean = orc.encode(rng.integers(0, 256, n, dtype=np.uint8))
    size = len(clean)

    def fit(t):
        return (t + clean)[:size]

    texts = {
        "clean": clean,
        "clean2": orc.encode(rng.integers(0, 256, n, dtype=np.uint8)),
        "crlf76": fit(_wrap(orc.encode(rng.integers(0, 256, n, dtype=np.uint8)), 76, b"\r\n")),
        "lf64": fit(_wrap(orc.encode(rng.integers(0, 256, n, dtype=np.uint8)), 64, b"\n")),
        "junk": fit(_junk(rng, clean, 0.05)),
        "sparse": fit(clean[:8192] + _junk(rng, clean[8192:], 1e-3)),
        "tail": clean[:-100] + b"!" + clean[-99:],
        "alljunk": b"\n" * size,
    }
    order = ["clean", "clean2", "clean", "crlf76", "crlf76", "lf64", "clean", "junk", "clean",
             "clean2", "sparse", "clean", "tail", "clean", "alljunk", "clean", "clean2"]
    buf = torch.empty(size, dtype=torch.uint8, device=DEV)
    out = torch.empty(b64.decoded_cap(size) + 8, dtype=torch.uint8, device=DEV)
    for ws in (torch.zeros(b64.workspace_size(size), dtype=torch.uint8, device=DEV), None):
        for i, name in enumerate(order):
            text = texts[name]
            assert len(text) == size
            buf.copy_(dev(text))
            d = b64.decode(buf, out=out, workspace=ws)
            assert d.bytes().cpu().numpy().tobytes() == orc.decode(text), (i, name)
            if ws is not None and name == "clean2" and i > 2:
                ws.zero_()  # a held entry over a zeroed workspace
        # back-to-back calls with no sync between them (the flag a call's
        # suffix raises may land after the next call was issued)
        outs = []
        for name in ("clean", "junk", "clean", "crlf76", "clean"):
            o = torch.empty_like(out)
            b = dev(texts[name])
            outs.append((name, b, o, b64.decode(b, out=o, workspace=ws)))
        for name, _, o, d in outs:
            assert d.bytes().cpu().numpy().tobytes() == orc.decode(texts[name]), name


def test_held_model_tiny_and_hold_tail():
    """Short streams (under one slot) and HOLD_TAIL calls of one length on
    one workspace, content changing between calls."""
    rng = np.random.default_rng(59)
    tab = orc.decode_table()
    ws = torch.zeros(b64.workspace_size(1 << 16), dtype=torch.uint8, device=DEV)
    for size in (5, 15, 16, 17, 100, 4099):
        for k in range(6):
            raw = orc.encode(rng.integers(0, 256, size, dtype=np.uint8))[:size]
            text = raw if k % 3 else bytes(b if rng.random() > 0.2 else 0x0A for b in raw)
            out = torch.empty(b64.decoded_cap(size) + 8, dtype=torch.uint8, device=DEV)
            d = b64.decode(dev(text), out=out, workspace=ws, hold_tail=bool(k & 1))
            want = orc.decode(text)
            got = d.bytes().cpu().numpy().tobytes()
            if k & 1:  # whole groups only
                V = sum(1 for c in text if tab[c] >= 0)
                assert got == want[:V // 4 * 3], (size, k)
            else:
                assert got == want, (size, k)


def _probe_model(ws: torch.Tensor):
    """The line model k_decode_probe left in the workspace (header bytes
    32..63): (L, s, T, skip)."""
    torch.cuda.synchronize()
    m = np.frombuffer(ws[32:64].cpu().numpy().tobytes(), np.uint32)
    return int(m[0]), int(m[1]), int(m[3]), int(m[7])


def test_probe_samples_cut_sparse_junk():
    """k_decode_probe checks samples past its first window against the
    model: sparse junk the window does not show cuts k_decode_lines' slots
    near the first sampled junk (so the exact suffix does not redo them),
    while clean and MIME text, and junk only in the stream's last bytes, keep
    every slot with k_decode_lines."""
    rng = np.random.default_rng(43)
    chars = orc.encode(rng.integers(0, 256, 3_000_000, dtype=np.uint8))
    n = len(chars)
    ws = torch.zeros(b64.workspace_size(n * 2), dtype=torch.uint8, device=DEV)
    sparse = chars[:4096] + _junk(rng, chars[4096:], 1e-3)
    tail = chars[:-1000] + b"!" + chars[-1000:]
    mime = _wrap(chars, 76, b"\r\n")
    mime_sparse = mime[:8192] + _junk(rng, mime[8192:], 1e-3)
    for name, text, cut in (("clean", chars, False), ("mime", mime, False), ("tail", tail, False),
                            ("sparse", sparse, True), ("mime_sparse", mime_sparse, True)):
        out = torch.empty(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV)
        d = b64.decode(dev(text), out=out, workspace=ws)
        assert d.bytes().cpu().numpy().tobytes() == orc.decode(text), name
        L, s, T, skip = _probe_model(ws)
        assert L == (76 if name.startswith("mime") else 0), name
        if cut:
            # 256 samples, dense near the start: at 0.1 % junk the first one
            # that finds junk lies within the first few percent of the stream
            assert skip == 1 and 16 * T < len(text) // 20, (name, T)
        else:
            assert skip == 0, name


def _mime_batch(nbuf, n, L, sep, rng, deviants=()):
    rows = []
    for i in range(nbuf):
        c = orc.encode(rng.integers(0, 256, n, dtype=np.uint8))
        t = _wrap(c, L, sep)
        if i in deviants:
            t = t[:7] + b"\t" + t[7:] if deviants[i] == "junk" else _wrap(c, L + 4, sep)
        rows.append(t)
    return rows


@pytest.mark.parametrize("n,L,sep", [(1024, 76, b"\r\n"), (4096, 76, b"\r\n"), (1000, 64, b"\n"),
                                     (777, 76, b"\r\n"), (3000, 19, b"\n"), (100, 16, b"\n\n"),
                                     (22, 16, b"\n\n"), (40, 16, b"\r\n")])
def test_strided_mime_rows_vs_oracle(n, L, sep):
    """MIME-formatted uniform batches (k_rows_prep's line model from row 0,
    k_decode_rows_lines): every row against the oracle, including rows that
    do not follow row 0's model (a junk byte, other line lengths) and so go
    to the exact fix-up."""
    rng = np.random.default_rng(n + L)
    nbuf = 300
    rows = _mime_batch(nbuf, n, L, sep, rng, deviants={3: "junk", 150: "len", nbuf - 1: "junk"})
    stride = max(len(r) for r in rows)
    flat = b"".join(r + b"\n" * (stride - len(r)) for r in rows)
    x = dev(flat)
    dcap = b64.decoded_cap(stride)
    # output strides: rounded to 16; whole 12-byte slots (the MIME hot path
    # then fills each row's slack); whole slots with room to spare
    for cap in ((dcap + 15) // 16 * 16, (dcap + 11) // 12 * 12, (dcap + 11) // 12 * 12 + 48):
        # the last row gets exactly its capacity, then a guard band that no
        # store may touch (no slack filler past the last row)
        size = (nbuf - 1) * cap + dcap
        dec = torch.full((size + 64,), 0xA5, dtype=torch.uint8, device=DEV)
        outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
        b64.decode_strided(x, stride, stride, nbuf, dec, cap, outlen)
        ol = outlen.cpu().tolist()
        dh = dec.cpu().numpy()
        assert (dh[size:] == 0xA5).all(), cap
        for i, r in enumerate(rows):
            want = orc.decode(r + b"\n" * (stride - len(r)))
            assert ol[i] == len(want), (cap, i)
            assert dh[i * cap:i * cap + ol[i]].tobytes() == want, (cap, i)


@pytest.mark.parametrize("n,L,sep,nbuf", [(1024, 76, b"\r\n", 2600), (1000, 64, b"\n", 1100),
                                          (3000, 76, b"\r\n", 700)])
def test_strided_mime_rows_bands_vs_oracle(n, L, sep, nbuf):
    """The row-group mapping of the MIME rows kernel (RowModel::nb/ru: a
    lane's U slots share one row slot q, U bands of Ru rows apart) over
    batches with whole bands and a partial last one, deviant rows inside
    whole bands and in the last, and a guard band after the output."""
    rng = np.random.default_rng(n + nbuf)
    dv = {5: "junk", nbuf // 3: "len", nbuf // 2: "junk", nbuf - 2: "len", nbuf - 1: "junk"}
    rows = _mime_batch(nbuf, n, L, sep, rng, deviants=dv)
    stride = max(len(r) for r in rows)
    flat = b"".join(r + b"\n" * (stride - len(r)) for r in rows)
    x = dev(flat)
    dcap = b64.decoded_cap(stride)
    for cap in ((dcap + 11) // 12 * 12, (dcap + 15) // 16 * 16):
        size = (nbuf - 1) * cap + dcap
        dec = torch.full((size + 64,), 0xA5, dtype=torch.uint8, device=DEV)
        outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
        b64.decode_strided(x, stride, stride, nbuf, dec, cap, outlen)
        ol = outlen.cpu().tolist()
        dh = dec.cpu().numpy()
        assert (dh[size:] == 0xA5).all(), cap
        for i, r in enumerate(rows):
            want = orc.decode(r + b"\n" * (stride - len(r)))
            assert ol[i] == len(want), (cap, i)
            assert dh[i * cap:i * cap + ol[i]].tobytes() == want, (cap, i)


def test_strided_rows_model_reuse_across_batches():
    """Row batches of one shape on one stream reuse the workspace's model
    (k_rows_prep runs only when the shape changes, another call used the
    workspace, or the last batch's first row failed the model): batches
    whose format changes under a held model, a first row that fails, a
    contiguous decode in between and another alphabet all stay exact."""
    rng = np.random.default_rng(77)
    nbuf, n = 900, 1024
    fmts = {"crlf76": (76, b"\r\n"), "lf64": (64, b"\n"), "clean": (0, b"")}

    def batch(fmt, deviants=()):
        L, sep = fmts[fmt]
        if L:
            return _mime_batch(nbuf, n, L, sep, rng, deviants=dict(deviants))
        return [orc.encode(rng.integers(0, 256, n, dtype=np.uint8)) for _ in range(nbuf)]

    stride = 1404 + 36  # room for every format's rows, padded with LF
    dcap = b64.decoded_cap(stride)
    cap = (dcap + 11) // 12 * 12

    def run(rows, abc=None):
        assert max(len(r) for r in rows) <= stride
        flat = b"".join(r + b"\n" * (stride - len(r)) for r in rows)
        x = dev(flat)
        size = (nbuf - 1) * cap + dcap
        dec = torch.full((size + 64,), 0xA5, dtype=torch.uint8, device=DEV)
        outlen = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
        b64.decode_strided(x, stride, stride, nbuf, dec, cap, outlen, abc=abc)
        ol = outlen.cpu().tolist()
        dh = dec.cpu().numpy()
        assert (dh[size:] == 0xA5).all()
        for i, r in enumerate(rows):
            want = orc.decode(r + b"\n" * (stride - len(r)), *(abc or ()))
            assert ol[i] == len(want), i
            assert dh[i * cap:i * cap + ol[i]].tobytes() == want, i

    for step in ("crlf76", "crlf76", "lf64", "lf64", "crlf76", "clean", "clean", "crlf76"):
        run(batch(step, deviants={7: "junk"}))
    run(batch("crlf76", deviants={0: "junk", 9: "len"}))  # first row fails the model
    run(batch("crlf76"))
    z = dev(orc.encode(rng.integers(0, 256, 1 << 20, dtype=np.uint8)))
    b64.decode(z)  # another call on the stream's workspace
    run(batch("crlf76", deviants={nbuf - 1: "junk"}))
    rows = [r.replace(b"+", b"-").replace(b"/", b"_") for r in batch("crlf76")]
    run(rows, abc=("-", "_"))
    run(batch("crlf76"))


def test_strided_rows_graph_replay_after_another_shape():
    """A row batch captured in a HIP graph while its workspace held the
    model of its shape (no prep captured), replayed after a batch of
    another shape re-probed that workspace: the row kernel finds the model
    made for another shape, takes no slot, and the exact fix-up decodes
    every row."""
    rng = np.random.default_rng(81)
    s = torch.cuda.Stream()

    def batch(n, nbuf):
        rows = _mime_batch(nbuf, n, 76, b"\r\n", rng)
        stride = max(len(r) for r in rows)
        flat = b"".join(r + b"\n" * (stride - len(r)) for r in rows)
        cap = (b64.decoded_cap(stride) + 11) // 12 * 12
        out = torch.zeros(nbuf * cap, dtype=torch.uint8, device=DEV)
        ol = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
        return rows, stride, dev(flat), cap, out, ol

    def check(rows, stride, cap, out, ol):
        olh = ol.cpu().tolist()
        dh = out.cpu().numpy()
        for i, r in enumerate(rows):
            want = orc.decode(r + b"\n" * (stride - len(r)))
            assert olh[i] == len(want), i
            assert dh[i * cap:i * cap + olh[i]].tobytes() == want, i

    rows, stride, x, cap, out, ol = batch(1024, 500)
    rows2, stride2, x2, cap2, out2, ol2 = batch(700, 300)
    with torch.cuda.stream(s):
        for _ in range(2):  # the stream's workspace, holding this shape's model
            b64.decode_strided(x, stride, stride, 500, out, cap, ol, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            b64.decode_strided(x, stride, stride, 500, out, cap, ol, stream=s)
        # another shape on the same stream's workspace replaces the model
        b64.decode_strided(x2, stride2, stride2, 300, out2, cap2, ol2, stream=s)
        out.zero_()
        ol.zero_()
        g.replay()
    s.synchronize()
    check(rows, stride, cap, out, ol)
    check(rows2, stride2, cap2, out2, ol2)


def test_decode_graph_replay_after_other_lengths():
    """A decode captured in a HIP graph (after calls of its length left a
    held model, which a capture does not reuse), replayed after decodes of
    other lengths and other content on the same workspace: exact."""
    rng = np.random.default_rng(83)
    s = torch.cuda.Stream()
    text = _wrap(orc.encode(rng.integers(0, 256, 1_000_000, dtype=np.uint8)), 76, b"\r\n")
    other = orc.encode(rng.integers(0, 256, 700_000, dtype=np.uint8))
    ws = torch.zeros(b64.workspace_size(len(text)), dtype=torch.uint8, device=DEV)
    x, y = dev(text), dev(other)
    out = torch.zeros(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV)
    out2 = torch.zeros(b64.decoded_cap(len(other)) + 8, dtype=torch.uint8, device=DEV)
    res = torch.zeros(256, dtype=torch.uint8, device=DEV)
    with torch.cuda.stream(s):
        for _ in range(2):
            d = b64.decode(x, out=out, workspace=ws, result=res, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            b64.decode(x, out=out, workspace=ws, result=res, stream=s)
        d2 = b64.decode(y, out=out2, workspace=ws, stream=s)
        assert d2.bytes().cpu().numpy().tobytes() == orc.decode(other)
        out.zero_()
        g.replay()
    s.synchronize()
    want = orc.decode(text)
    assert out[:len(want)].cpu().numpy().tobytes() == want


def _paths():
    import ctypes

    from async_amd import _lib
    out = (ctypes.c_uint64 * 5)()
    _lib.load().b64x_diag_paths(out)
    return [int(v) for v in out]


def test_new_content_at_a_held_address_and_length():
    """The held model and the probe's hint are keyed on workspace, input
    address and length, never on content.  Different
    content written into the same buffer, decoded right after a junk-laden
    call and right after a clean one, on a caller's workspace and on the
    library's: every decode is exact, and each takes the path the state
    predicts (b64x_diag_paths: probes, held-model skips, hinted single
    passes)."""
    rng = np.random.default_rng(89)
    n = (3 << 20) + 7  # a length no other test decodes (hints and held models)
    raw = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)]
    clean = [orc.encode(r) for r in raw]
    m = len(clean[0])
    # junk-laden text of exactly the clean length: the first m characters of
    # a 5 %-junk text, and what they decode to
    junky = [_junk(rng, c, 0.05)[:m] for c in clean]
    want_j = [orc.decode(t) for t in junky]
    # clean for its first half, 5 % junk after: a probe cuts its model past
    # the stream's first sixteenth (no hint)
    mid = (clean[0][:m // 2] + _junk(rng, clean[0][m // 2:], 0.05))[:m]
    want_mid = orc.decode(mid)
    x = torch.empty(m, dtype=torch.uint8, device=DEV)
    out = torch.zeros(b64.decoded_cap(m) + 8, dtype=torch.uint8, device=DEV)
    res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
    PROBE, HELD, HINT = 0, 1, 2

    for ws in (torch.zeros(b64.workspace_size(m), dtype=torch.uint8, device=DEV), None):
        s = torch.cuda.Stream()

        def run(text, want, expect):
            x.copy_(torch.from_numpy(np.frombuffer(text, dtype=np.uint8).copy()))
            torch.cuda.synchronize()
            before = _paths()
            d = b64.decode(x, out=out, workspace=ws, result=res, stream=s)
            s.synchronize()
            after = _paths()
            assert d.info().out_len == len(want)
            assert out[:len(want)].cpu().numpy().tobytes() == want
            took = [after[k] - before[k] for k in (PROBE, HELD, HINT)]
            assert took == expect, (took, expect)

        # a call of another length on the workspace: whatever an earlier
        # test left there, nothing is held for this length now
        x.copy_(torch.from_numpy(np.frombuffer(clean[0], dtype=np.uint8).copy()))
        b64.decode(x[:m - 4], workspace=ws, stream=s).info()
        # a clean call probes (nothing held for this length)...
        run(clean[0], raw[0].tobytes(), [1, 0, 0])
        # ...and the next clean content at the same address and length reuses
        # the model without a probe
        run(clean[1], raw[1].tobytes(), [0, 1, 0])
        # junk right after a clean call: held model (the hint is clean), the
        # lines pass fails at the first junk byte and the suffix raises the flag
        run(junky[0], want_j[0], [0, 1, 0])
        # the same junk again: the flag forces a probe, which cuts the model
        # near the start and sets the hint
        run(junky[0], want_j[0], [1, 0, 0])
        # different junk: the hint picks the probe + single pass
        run(junky[1], want_j[1], [1, 0, 1])
        # clean content right after a junk-laden call: the hint still says
        # junk (single pass, exact), and its probe renews the hint as clean
        run(clean[2], raw[2].tobytes(), [1, 0, 1])
        # then the lines pass on the held clean model, no probe
        run(clean[3], raw[3].tobytes(), [0, 1, 0])
        # junk under the held clean model, then the probe that sets the hint
        run(junky[2], want_j[2], [0, 1, 0])
        run(junky[2], want_j[2], [1, 0, 0])
        # the hinted single pass on content its probe (run inside it) cuts
        # past the first sixteenth: the hint turns clean and the cut model is
        # held, its cut not published (that probe runs with the decode)...
        run(mid, want_mid, [1, 0, 1])
        # ...so the next call takes the held cut model without a probe and
        # k_decode_lines publishes the cut itself; the suffix had work, so
        # the call after that probes again
        run(mid, want_mid, [0, 1, 0])
        run(mid, want_mid, [1, 0, 0])
        if ws is None:
            import ctypes

            from async_amd import _lib
            _lib.load().b64x_release_stream(ctypes.c_void_p(s.cuda_stream))


def test_capture_on_a_fresh_stream():
    """Graph capture on a stream that never decoded: the
    library does not allocate or rebind a workspace inside a capture.
    b64.decode() then captures with a torch-allocated workspace,
    decode_strided takes the general batch path, and the C call with
    d_workspace NULL answers -EBUSY without enqueuing anything; every replay
    is exact."""
    import ctypes

    from async_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(85)
    raw = rng.integers(0, 256, 300_000, dtype=np.uint8)
    text = _wrap(orc.encode(raw), 76, b"\r\n")
    x = dev(text)
    out = torch.zeros(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV)
    res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
    nbuf = 300
    rows = _mime_batch(nbuf, 1024, 76, b"\r\n", rng)
    stride = max(len(r) for r in rows)
    flat = dev(b"".join(r + b"\n" * (stride - len(r)) for r in rows))
    cap = (b64.decoded_cap(stride) + 11) // 12 * 12
    rout = torch.zeros(nbuf * cap, dtype=torch.uint8, device=DEV)
    ol = torch.zeros(nbuf, dtype=torch.int64, device=DEV)
    a = b64._abc(None)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        b64.decode(x, out=out, result=res, stream=s)
        b64.decode_strided(flat, stride, stride, nbuf, rout, cap, ol, stream=s)
        rc = lib.b64x_decode_dev(ctypes.c_void_p(x.data_ptr()), x.numel(),
                                 ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.data_ptr()),
                                 ctypes.byref(a), 0, None, ctypes.c_void_p(s.cuda_stream))
    assert rc == -16  # -EBUSY
    for _ in range(2):
        out.zero_()
        rout.zero_()
        ol.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out[:raw.size].cpu().numpy(), raw)
        olh = ol.cpu().tolist()
        dh = rout.cpu().numpy()
        for i, r in enumerate(rows):
            want = orc.decode(r + b"\n" * (stride - len(r)))
            assert olh[i] == len(want), i
            assert dh[i * cap:i * cap + olh[i]].tobytes() == want, i
    lib.b64x_release_stream(ctypes.c_void_p(s.cuda_stream))


def test_workspace_taken_over_while_its_stream_is_busy():
    """No event is recorded per call: a workspace stays with its stream and
    the event that guards it is recorded when another stream takes it over.
    Nine streams (one more than the cache) decode in turn with the library
    workspace while each stream's earlier work is still queued behind a long
    decode, so every take-over must wait for the old stream on the device;
    every result is exact."""
    import ctypes

    from async_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(87)
    big = rng.integers(0, 256, 30 << 20, dtype=np.uint8)
    bx = dev(orc.encode(big))
    bout = torch.empty(b64.decoded_cap(bx.numel()), dtype=torch.uint8, device=DEV)
    a = b64._abc(None)
    streams = [torch.cuda.Stream() for _ in range(9)]
    jobs = []
    for k in range(27):
        raw = rng.integers(0, 256, 100_000 + 4099 * k, dtype=np.uint8)
        text = _wrap(orc.encode(raw), 76, b"\r\n") if k % 3 == 0 else \
            _junk(rng, orc.encode(raw), 0.01) if k % 3 == 1 else orc.encode(raw)
        jobs.append((raw, dev(text),
                     torch.zeros(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV),
                     torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)))
    bres = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
    torch.cuda.synchronize()
    for k, (raw, x, out, res) in enumerate(jobs):
        st = streams[k % 9]
        if k % 9 == 0:  # keep the streams busy while their workspaces move
            for s2 in streams[::2]:
                assert lib.b64x_decode_dev(ctypes.c_void_p(bx.data_ptr()), bx.numel(),
                                           ctypes.c_void_p(bout.data_ptr()),
                                           ctypes.c_void_p(bres.data_ptr()), ctypes.byref(a), 0,
                                           None, ctypes.c_void_p(s2.cuda_stream)) == 0
        assert lib.b64x_decode_dev(ctypes.c_void_p(x.data_ptr()), x.numel(),
                                   ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.data_ptr()),
                                   ctypes.byref(a), 0, None, ctypes.c_void_p(st.cuda_stream)) == 0
    torch.cuda.synchronize()
    for raw, x, out, res in jobs:
        assert np.array_equal(out[:raw.size].cpu().numpy(), raw)
    assert np.array_equal(bout[:big.size].cpu().numpy(), big)
    for st in streams:
        lib.b64x_release_stream(ctypes.c_void_p(st.cuda_stream))


def test_workspace_taken_over_from_the_null_stream():
    """the NULL stream (torch's default stream, cuda_stream == 0)
    holds a library workspace like any other stream.  Its handle is 0, which
    the workspace cache once also used to mean "idle": a side stream taking
    the NULL stream's workspace over then recorded no event on it and did not
    wait for the NULL stream's queued decode, so two junk-laden decodes ran
    on one set of tickets and tile words at once.  Here the NULL stream's
    decode is queued behind a GPU sleep, the side stream's behind one as long,
    and the side stream takes the NULL stream's workspace over (it is the
    least recently used); both outputs must be exact."""
    import ctypes

    from async_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(1234)
    a = b64._abc(None)

    def job(n, seed):
        raw = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
        text = _junk(rng, orc.encode(raw), 0.05)
        x = dev(text)
        out = torch.zeros(b64.decoded_cap(len(text)) + 8, dtype=torch.uint8, device=DEV)
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
        return raw, x, out, res

    def decode(j, st, flags=0):
        raw, x, out, res = j
        assert lib.b64x_decode_dev(ctypes.c_void_p(x.data_ptr()), x.numel(),
                                   ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.data_ptr()),
                                   ctypes.byref(a), flags, None,
                                   ctypes.c_void_p(st)) == 0

    side = [torch.cuda.Stream() for _ in range(8)]
    small = job(50_000, 1)
    big0 = job(48 << 20, 2)
    big1 = job(48 << 20, 3)
    torch.cuda.synchronize()
    for st in side:  # start from no side stream holding a workspace
        lib.b64x_release_stream(ctypes.c_void_p(st.cuda_stream))
    lib.b64x_release_stream(ctypes.c_void_p(0))
    decode(small, 0)                       # the NULL stream binds one
    for st in side[:7]:                    # seven more, used after it
        decode(small, st.cuda_stream)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    assert cur.cuda_stream == 0, "torch's default stream is the NULL stream"
    torch.cuda._sleep(40_000_000)          # ~20 ms on the NULL stream
    decode(big0, 0, b64.EXPECT_JUNK)       # queued behind it
    for st in side[:7]:                    # the seven become more recent
        decode(small, st.cuda_stream)
    with torch.cuda.stream(side[7]):
        torch.cuda._sleep(40_000_000)      # as long on the taking stream
    decode(big1, side[7].cuda_stream, b64.EXPECT_JUNK)  # takes the NULL stream's over
    torch.cuda.synchronize()
    for raw, x, out, res in (small, big0, big1):
        assert np.array_equal(out[:raw.size].cpu().numpy(), raw)
    for st in side:
        lib.b64x_release_stream(ctypes.c_void_p(st.cuda_stream))
    lib.b64x_release_stream(ctypes.c_void_p(0))


def test_bind_thread_puts_the_thread_on_the_gpus_node():
    """b64x_bind_thread: the calling thread's CPU mask afterwards lies inside
    the GPU's NUMA node (sysfs), within what it was allowed before; a thread
    already inside one node is left as it is.  Run on threads of their own,
    so the test process keeps its mask."""
    import threading

    from async_amd import placement as pl
    node = b64.device_numa_node(0)
    if node < 0:
        pytest.skip("no NUMA node for the GPU on this box")
    on_node = pl.node_cpus(node)
    out = {}

    def run():
        before = os.sched_getaffinity(0)
        out["rc"] = b64.bind_thread(0)
        out["after"] = os.sched_getaffinity(0)
        out["before"] = before
    t = threading.Thread(target=run)
    t.start()
    t.join()
    if not (out["before"] & on_node):
        assert out["rc"] < 0 and out["after"] == out["before"]
        return
    assert out["rc"] == node
    assert out["after"] <= on_node and out["after"] <= out["before"]
    other = out["before"] - on_node
    if other:
        def run2():
            os.sched_setaffinity(0, other)
            out["rc2"] = b64.bind_thread(0)
            out["after2"] = os.sched_getaffinity(0)
        t = threading.Thread(target=run2)
        t.start()
        t.join()
        assert out["after2"] == other and out["rc2"] != node


def test_library_workspace_is_bounded():
    """Decodes with d_workspace == NULL on 100 fresh streams keep at most 8
    library workspaces (~14 MiB of HBM each), not one per stream forever;
    b64x_release_stream unbinds a stream's one for the next; every result
    stays exact."""
    import ctypes

    from async_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(31)
    raw = rng.integers(0, 256, 30000, dtype=np.uint8)
    text = dev(b"\r\n".join(orc.encode(raw)[i:i + 76] for i in range(0, 40000, 76)))
    a = b64._abc(None)
    ws_bytes = b64.workspace_size(0)

    def run(st):
        out = torch.empty(b64.decoded_cap(text.numel()), dtype=torch.uint8, device=DEV)
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
        rc = lib.b64x_decode_dev(ctypes.c_void_p(text.data_ptr()), text.numel(),
                                 ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.data_ptr()),
                                 ctypes.byref(a), 0, None, ctypes.c_void_p(st.cuda_stream))
        assert rc == 0
        st.synchronize()
        assert np.array_equal(out[:raw.size].cpu().numpy(), raw)

    keep = [torch.cuda.Stream() for _ in range(100)]
    run(keep[0])  # first use of the path (code objects, one workspace)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for st in keep[1:]:
        run(st)
    torch.cuda.synchronize()
    grew = free0 - torch.cuda.mem_get_info()[0]
    assert grew < 8 * ws_bytes + (64 << 20), grew  # unbounded: 99 x 14 MiB
    for st in keep:
        lib.b64x_release_stream(ctypes.c_void_p(st.cuda_stream))
    run(keep[5])  # a released stream gets a fresh workspace
    lib.b64x_release_stream(ctypes.c_void_p(keep[5].cuda_stream))


def test_release_stream_from_python():
    """b64.release_stream(): a stream that decoded with the
    library workspace hands it back while its decode may still be queued;
    the next decode on the stream binds one again; every result is exact."""
    rng = np.random.default_rng(91)
    s = torch.cuda.Stream()
    raws = [rng.integers(0, 256, 200_000 + 777 * k, dtype=np.uint8) for k in range(4)]
    texts = [dev(orc.encode(r)) if k % 2 else dev(_junk(rng, orc.encode(r), 0.02))
             for k, r in enumerate(raws)]
    outs = [torch.zeros(b64.decoded_cap(t.numel()) + 8, dtype=torch.uint8, device=DEV)
            for t in texts]
    ress = [torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV) for _ in texts]
    torch.cuda.synchronize()
    for t, o, r in zip(texts, outs, ress):
        b64.decode(t, out=o, result=r, stream=s)
        b64.release_stream(s)
    torch.cuda.synchronize()
    for raw, o, r in zip(raws, outs, ress):
        assert b64.Decoded(o, r).info().out_len == raw.size
        assert np.array_equal(o[:raw.size].cpu().numpy(), raw)
    b64.release_stream(s)  # nothing bound: a no-op


def test_library_workspace_threads_past_the_cache():
    """12 threads, each decoding on its own stream with d_workspace == NULL
    (more streams than the 8 cached workspaces, so entries are evicted while
    other threads are enqueuing): an entry handed out is pinned until its
    call's kernels are queued and an event is recorded behind them, and
    eviction waits on that event, not the device -- every decode stays
    exact (the unpinned LRU could free a workspace between its
    lookup and the launches that use it).  The threads make only C calls
    (the library, hipStreamSynchronize, hipMemcpyAsync); buffers, streams
    and the checks are the main thread's."""
    import ctypes
    import threading

    from async_amd import _lib
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
    rng = np.random.default_rng(41)
    jobs = []
    for k in range(12):
        raw = rng.integers(0, 256, 200000 + 977 * k, dtype=np.uint8)
        text = _junk(rng, orc.encode(raw), 0.003) if k % 2 else \
            b"\r\n".join(orc.encode(raw)[i:i + 76] for i in range(0, 300000, 76))
        x = dev(text)
        out = torch.zeros(b64.decoded_cap(x.numel()), dtype=torch.uint8, device=DEV)
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device=DEV)
        jobs.append({"raw": raw, "x": x, "out": out, "res": res, "st": torch.cuda.Stream(),
                     "pinned": lib.b64x_host_alloc(b64.RES_BYTES), "ok": 0, "err": None})
    torch.cuda.synchronize()
    a = b64._abc(None)

    def worker(j):
        try:
            st = ctypes.c_void_p(j["st"].cuda_stream)
            rec = b64.DecResult.from_address(j["pinned"])  # pinned: an async D2H
            for rep in range(6):
                seq = ctypes.c_uint32(0)
                rc = lib.b64x_decode_dev_seq(ctypes.c_void_p(j["x"].data_ptr()), j["x"].numel(),
                                             ctypes.c_void_p(j["out"].data_ptr()),
                                             ctypes.c_void_p(j["res"].data_ptr()),
                                             ctypes.byref(a), 0, None, st, ctypes.byref(seq))
                if rc == -16:  # -EBUSY: every cached entry mid-enqueue
                    continue
                assert rc == 0, rc
                assert hip.hipMemcpyAsync(j["pinned"], j["res"].data_ptr(),
                                          b64.RES_BYTES, 2, st) == 0
                assert hip.hipStreamSynchronize(st) == 0
                assert lib.b64x_result_check(ctypes.byref(rec), j["x"].numel(), 0,
                                             seq.value) == 0
                assert rec.out_len == j["raw"].size
                j["ok"] += 1
            lib.b64x_release_stream(st)
        except BaseException as e:  # noqa: BLE001 -- reported below
            j["err"] = e

    th = [threading.Thread(target=worker, args=(j,), daemon=True) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th)
    for j in jobs:
        assert j["err"] is None, j["err"]
        assert j["ok"] >= 1
        assert np.array_equal(j["out"][:j["raw"].size].cpu().numpy(), j["raw"])
        lib.b64x_host_free(j["pinned"])


def test_decoded_info_checks_the_record():
    """Decoded.info() waits for the decode's own stream and refuses a record
    that does not name the call."""
    raw = np.arange(3000, dtype=np.uint8)
    x = dev(orc.encode(raw))
    st = torch.cuda.Stream()
    d = b64.decode(x, stream=st)
    assert d.seq != 0 and d.nchars == x.numel()
    assert d.info().out_len == raw.size
    stale = b64.Decoded(d.out, d.result, d.nchars, d.flags, d.seq + 1, st)
    with pytest.raises(b64.B64xError):
        stale.info()
