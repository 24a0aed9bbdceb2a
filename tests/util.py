"""Shared test helpers (test infrastructure only)."""
from __future__ import annotations

import ctypes
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "tests", "csrc", "libstage_harness.so")


def golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """The synthetic byte stream of SURVEY.md §8(c) (numpy, vectorised)."""
    n8 = (n + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(1, n8 + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n]


def counting(n: int) -> np.ndarray:
    return (np.arange(n, dtype=np.uint64) & 0xFF).astype(np.uint8)


FAKE_HARNESS = os.path.join(ROOT, "tests", "csrc", "libstage_fake.so")

_harness = None
_fake = None


def harness() -> ctypes.CDLL:
    """tests/csrc/libstage_harness.so (links the product library)."""
    global _harness
    if _harness is None:
        try:
            import torch  # noqa: F401  (one HIP runtime: see async_amd/_lib.py)
        except ImportError:
            pass
        _harness = _bind(ctypes.CDLL(HARNESS))
    return _harness


def fake_harness() -> ctypes.CDLL:
    """tests/csrc/libstage_fake.so: the same harness and the product's host
    C (loop, streams, framing, hub, stages) over the CPU stand-in for the
    GPU side (tests/csrc/fake_b64x.c).  No GPU, no HIP runtime."""
    global _fake
    if _fake is None:
        L = _bind(ctypes.CDLL(FAKE_HARNESS))
        L.fake_configure.argtypes = [ctypes.c_uint64, ctypes.c_uint, ctypes.c_int]
        L.fake_configure.restype = None
        L.fake_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
        L.fake_stats.restype = None
        L.b64x_diag_counters.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
        L.b64x_diag_counters.restype = None
        _fake = L
    return _fake


HOOKS = os.path.join(ROOT, "tests", "csrc", "libb64x_hooks.so")
_hooks = None


def hooks() -> ctypes.CDLL:
    """tests/csrc/libb64x_hooks.so: the kernels built with B64X_TEST_HOOKS
    (b64x__test_range_chunks); the product library has no such knob."""
    global _hooks
    if _hooks is None:
        import torch  # noqa: F401  (one HIP runtime: see async_amd/_lib.py)
        from async_amd import _lib
        L = ctypes.CDLL(HOOKS)
        for name, (res, args) in _lib.SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        L.b64x__test_range_chunks.argtypes = [ctypes.c_uint64]
        L.b64x__test_range_chunks.restype = ctypes.c_uint64
        _hooks = L
    return _hooks


def _lib_or_default(lib):
    return lib if lib is not None else harness()


def _bind(L: ctypes.CDLL) -> ctypes.CDLL:
    """Argument types of the harness entry points (both builds)."""
    sz, ssz, vp, ch, ip = (ctypes.c_size_t, ctypes.c_ssize_t, ctypes.c_void_p,
                           ctypes.c_char, ctypes.POINTER(ctypes.c_int))
    L.h_reftest.argtypes = [sz, vp, sz, ctypes.POINTER(sz), vp, sz, ip,
                            ctypes.POINTER(sz)]
    L.h_reftest.restype = ssz
    L.h_encode_stream.argtypes = [vp, sz, sz, sz, ch, ch, ctypes.c_int, ch, vp, sz, ip]
    L.h_encode_stream.restype = ssz
    L.h_decode_stream.argtypes = [vp, sz, sz, sz, ch, ch, vp, sz, ip]
    L.h_decode_stream.restype = ssz
    L.h_copy_stream.argtypes = [vp, sz, sz, sz, vp, sz, ip, ctypes.POINTER(sz)]
    L.h_copy_stream.restype = ssz
    L.h_stage_upstream_error.argtypes = [ctypes.c_int, vp, sz, sz, ctypes.c_int, sz, vp, sz, ip]
    L.h_stage_upstream_error.restype = ssz
    L.h_fdsink_unwatchable.argtypes = [ctypes.c_int, ip]
    L.h_fdsink_unwatchable.restype = ctypes.c_int
    L.h_encode_counts.argtypes = [vp, sz, sz, sz, sz, ch, ch, ctypes.c_int, ch, vp, sz, ip]
    L.h_encode_counts.restype = ssz
    L.h_chunk_stream.argtypes = [vp, sz, sz, sz, ctypes.c_int, sz, vp, sz, ip]
    L.h_chunk_stream.restype = ssz
    L.h_queue_stream.argtypes = [vp, vp, sz, ctypes.c_int, sz, sz, vp, sz, ip,
                                 ctypes.POINTER(sz)]
    L.h_queue_stream.restype = ssz
    L.h_egress_stacks.argtypes = [vp, vp, sz, sz, sz, ch, ch, ctypes.c_int, ch, vp, vp,
                                  vp, ip, vp]
    L.h_egress_stacks.restype = ctypes.c_int
    L.h_egress_stacks_mt.argtypes = L.h_egress_stacks.argtypes + [sz]
    L.h_egress_stacks_mt.restype = ctypes.c_int
    L.h_egress_stacks_mt_dev.argtypes = L.h_egress_stacks.argtypes + [sz, ctypes.c_int]
    L.h_egress_stacks_mt_on.argtypes = L.h_egress_stacks.argtypes + [sz, ctypes.c_int]
    L.h_egress_stacks_mt_dev.restype = ctypes.c_int
    L.h_ingress_stacks.argtypes = [vp, vp, sz, sz, ch, ch, vp, vp, vp, ip, vp]
    L.h_ingress_stacks.restype = ctypes.c_int
    L.h_count_begin.argtypes = []
    L.h_count_begin.restype = None
    L.h_count_end.argtypes = []
    L.h_count_end.restype = ctypes.c_int
    L.h_prof_start.argtypes = [ctypes.c_int]
    L.h_prof_stop.argtypes = [ctypes.c_char_p]
    L.h_device_count.argtypes = []
    L.h_device_count.restype = ctypes.c_int
    L.h_egress_pieces.argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_int, sz, sz, vp, sz, ip]
    L.h_egress_pieces.restype = ssz
    L.b64_pin_live_refs.argtypes = []
    L.b64_pin_live_refs.restype = ctypes.c_long
    L.b64_hub_lent_total.argtypes = []
    L.b64_hub_lent_total.restype = ctypes.c_ulong
    L.h_take_read_seconds.argtypes = [ctypes.POINTER(ctypes.c_ulong)]
    L.h_take_read_seconds.restype = ctypes.c_double
    dp = ctypes.POINTER(ctypes.c_double)
    L.h_fd_decode.argtypes = [vp, sz, sz, sz, ch, ch, vp, sz, ctypes.c_int, ip, dp]
    L.h_fd_decode.restype = ssz
    L.h_fd_encode.argtypes = [vp, vp, sz, sz, ch, ch, ctypes.c_int, ch, vp, sz, ctypes.c_int,
                              ip, dp]
    L.h_fd_encode.restype = ssz
    L.h_fd_raw.argtypes = [vp, sz, sz, sz, vp, sz, ctypes.c_int, ip, dp]
    L.h_fd_raw.restype = ssz
    return L


def cch(v) -> bytes:
    if isinstance(v, str):
        v = v.encode("latin-1")
    if isinstance(v, (bytes, bytearray)):
        return bytes(v[:1])
    return bytes([v & 0xFF])


def _buf(data: bytes):
    a = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    return a, a.ctypes.data


def stage_encode(data: bytes, burst=0, read_size=200, pos62=-1, pos63=-1, pad=True,
                 padchar=-1, lib=None):
    """Product encoder stage on the product loop; returns (bytes|None, errno)."""
    a, p = _buf(data)
    cap = (len(data) + 2) // 3 * 4 + 16
    out = np.empty(cap, np.uint8)
    err = ctypes.c_int(0)
    n = _lib_or_default(lib).h_encode_stream(p, len(data), burst, read_size, cch(pos62), cch(pos63),
                                  int(bool(pad)), cch(padchar), out.ctypes.data, cap,
                                  ctypes.byref(err))
    return (None if n < 0 else out[:n].tobytes()), err.value


def stage_decode(data: bytes, burst=0, read_size=200, pos62=-1, pos63=-1, lib=None):
    a, p = _buf(data)
    cap = (len(data) + 3) // 4 * 3 + 16
    out = np.empty(cap, np.uint8)
    err = ctypes.c_int(0)
    n = _lib_or_default(lib).h_decode_stream(p, len(data), burst, read_size, cch(pos62), cch(pos63),
                                  out.ctypes.data, cap, ctypes.byref(err))
    return (None if n < 0 else out[:n].tobytes()), err.value


def stage_reftest(length=1000001, lib=None):
    ecap = (length + 2) // 3 * 4 + 16
    enc = np.empty(ecap, np.uint8)
    dec = np.empty(length + 16, np.uint8)
    elen = ctypes.c_size_t(0)
    err = ctypes.c_int(0)
    eag = ctypes.c_size_t(0)
    n = _lib_or_default(lib).h_reftest(length, enc.ctypes.data, ecap, ctypes.byref(elen),
                            dec.ctypes.data, dec.size, ctypes.byref(err), ctypes.byref(eag))
    return (None if n < 0 else (enc[: elen.value].tobytes(), dec[:n].tobytes())), \
        err.value, eag.value


def counted(fn, *args, lib=None, **kw):
    """Run fn(*args, lib=..., **kw) with the reference runner's counting
    allocator wired in (test/asynctest.c:111-147, 276-278); returns
    (fn's result, objects still outstanding afterwards)."""
    L = _lib_or_default(lib)
    L.h_count_begin()
    try:
        r = fn(*args, lib=L, **kw)
    finally:
        left = L.h_count_end()
    return r, left


def zipf_lengths(n_msgs=16384, seed=0x2F, rmax=16384, s=1.1) -> np.ndarray:
    """SURVEY.md §8(d) config 5 message lengths (same definition as
    tests/golden/make_golden.py:zipf_lengths, vectorised)."""
    r = np.arange(1, rmax + 1, dtype=np.float64)
    w = r ** -s
    cdf = np.cumsum(w) / w.sum()
    words = splitmix64(seed, 8 * n_msgs).view("<u8")
    u = (words >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    idx = np.minimum(np.searchsorted(cdf, u, side="right"), rmax - 1)
    return (64 * (idx + 1)).astype(np.int64)


def encode_counts(data: bytes, read_size: int, burst=0, pos62=-1, pos63=-1, pad=True,
                  padchar=-1, lib=None):
    """The GPU encoder stage's positive read returns; (list|None, errno)."""
    a, p = _buf(data)
    cap = len(data) // 2 + 64
    counts = np.empty(cap, dtype=np.intp)
    err = ctypes.c_int(0)
    n = _lib_or_default(lib).h_encode_counts(p, len(data), 0, burst, read_size, cch(pos62), cch(pos63),
                                  int(bool(pad)), cch(padchar), counts.ctypes.data, cap,
                                  ctypes.byref(err))
    return (None if n < 0 else counts[:min(n, cap)].tolist()), err.value


def chunk_stream(data: bytes, max_chunk: int, termination=0, read_size=100, burst=0, lib=None):
    a, p = _buf(data)
    cap = len(data) + (len(data) // max(max_chunk, 2) + 2) * 16 + 16
    out = np.empty(cap, np.uint8)
    err = ctypes.c_int(0)
    n = _lib_or_default(lib).h_chunk_stream(p, len(data), burst, max_chunk, termination, read_size,
                                 out.ctypes.data, cap, ctypes.byref(err))
    return (None if n < 0 else out[:n].tobytes()), err.value


def queue_stream(pieces, push=False, burst=0, read_size=100, lib=None):
    data = b"".join(pieces)
    a, p = _buf(data)
    lens = np.asarray([len(x) for x in pieces] or [0], dtype=np.uintp)
    out = np.empty(len(data) + 16, np.uint8)
    err = ctypes.c_int(0)
    eag = ctypes.c_size_t(0)
    n = _lib_or_default(lib).h_queue_stream(p, lens.ctypes.data, len(pieces), int(push), burst,
                                 read_size, out.ctypes.data, out.size, ctypes.byref(err),
                                 ctypes.byref(eag))
    return (None if n < 0 else out[:n].tobytes()), err.value, eag.value


def framed_cap(n: int, max_chunk: int) -> int:
    chars = (n + 2) // 3 * 4
    return chars + (chars // max(max_chunk, 2) + 3) * 16 + 16


def device_count() -> int:
    return int(harness().h_device_count())


def egress_stacks(payload: np.ndarray, lens, max_chunk: int, read_size: int, pos62=-1,
                  pos63=-1, pad=True, padchar=-1, times=None, raw=False, threads=1,
                  devices=1, device=None, lib=None):
    """Run len(lens) GPU egress stacks on `threads` loops (loop t on GPU
    t mod `devices` when devices > 1, every loop on GPU `device` when it is
    given); returns
    (list of framed bytes | None, errno).  `times` (a float64[2] array)
    receives the C-side setup and loop seconds; raw=True returns
    (out, out_off, out_len) instead of a list."""
    lens = np.asarray(lens, dtype=np.uint64)
    in_off = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(lens, out=in_off[1:])
    caps = np.array([framed_cap(int(n), max_chunk) for n in lens], np.uint64)
    out_off = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(caps, out=out_off[1:])
    out = np.empty(int(out_off[-1]) or 1, np.uint8)
    out.fill(0)  # fault the pages in outside the measured call
    out_len = np.zeros(max(lens.size, 1), np.uint64)
    err = ctypes.c_int(0)
    src = np.ascontiguousarray(payload, dtype=np.uint8)
    tp = times.ctypes.data if times is not None else None
    args = (src.ctypes.data, in_off.ctypes.data, lens.size, max_chunk, read_size, cch(pos62),
            cch(pos63), int(bool(pad)), cch(padchar), out.ctypes.data, out_off.ctypes.data,
            out_len.ctypes.data, ctypes.byref(err), tp)
    if device is not None:
        rc = _lib_or_default(lib).h_egress_stacks_mt_on(*args, max(threads, 1), int(device))
    elif devices > 1:
        rc = _lib_or_default(lib).h_egress_stacks_mt_dev(*args, max(threads, 1), devices)
    elif threads > 1:
        rc = _lib_or_default(lib).h_egress_stacks_mt(*args, threads)
    else:
        rc = _lib_or_default(lib).h_egress_stacks(*args)
    if rc != 0:
        return None, err.value
    if raw:
        return (out, out_off, out_len), 0
    return [out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes()
            for i in range(lens.size)], 0


def ingress_stacks(msgs, read_size: int, pos62=-1, pos63=-1, times=None, lib=None):
    """Run len(msgs) GPU decoder stacks (queuestream -> base64_decode) on one
    loop; returns (list of decoded bytes | None, errno)."""
    lens = np.array([len(m) for m in msgs], np.uint64)
    in_off = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(lens, out=in_off[1:])
    src = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
    caps = lens // 4 * 3 + 3
    out_off = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(caps, out=out_off[1:])
    out = np.zeros(int(out_off[-1]) or 1, np.uint8)
    out_len = np.zeros(max(lens.size, 1), np.uint64)
    err = ctypes.c_int(0)
    tp = times.ctypes.data if times is not None else None
    rc = _lib_or_default(lib).h_ingress_stacks(src.ctypes.data, in_off.ctypes.data, lens.size, read_size,
                                    cch(pos62), cch(pos63), out.ctypes.data,
                                    out_off.ctypes.data, out_len.ctypes.data,
                                    ctypes.byref(err), tp)
    if rc != 0:
        return None, err.value
    return [out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes()
            for i in range(lens.size)], 0


def fd_decode(chars, write_chunk=1 << 20, read_size=1 << 18, pos62=-1, pos63=-1, sock=False,
              out=None, lib=None):
    """Ingress through a real fd: a peer thread writes `chars` into a pipe
    (or AF_UNIX socketpair) -> pipestream -> base64_decode stage -> consumer.
    Returns (decoded bytes as a numpy view | None, errno, seconds)."""
    src = np.frombuffer(chars, np.uint8) if isinstance(chars, (bytes, bytearray)) else \
        np.ascontiguousarray(chars, dtype=np.uint8)
    cap = src.size // 4 * 3 + 16
    if out is None:
        out = np.empty(cap, np.uint8)
    err = ctypes.c_int(0)
    t = (ctypes.c_double * 1)()
    n = _lib_or_default(lib).h_fd_decode(src.ctypes.data if src.size else None, src.size,
                                         write_chunk, read_size, cch(pos62), cch(pos63),
                                         out.ctypes.data, out.size, int(bool(sock)),
                                         ctypes.byref(err), t)
    return (None if n < 0 else out[:n]), err.value, t[0]


def fd_encode(data, pieces=None, max_chunk=1 << 20, pos62=-1, pos63=-1, pad=True, padchar=-1,
              sock=False, out=None, lib=None):
    """Egress through a real fd: `data` (split into `pieces` lengths) on a
    queuestream -> base64_encode stage -> chunk_encode(max_chunk) -> fdsink
    (10,240-byte pulls, write(2)) -> a pipe a peer thread drains
    (max_chunk 0: no framing, the sink reads the encoder).  Returns
    (framed bytes as a numpy view | None, errno, seconds)."""
    src = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else \
        np.ascontiguousarray(data, dtype=np.uint8)
    lens = np.asarray(pieces if pieces is not None else [src.size], dtype=np.uintp)
    cap = framed_cap(src.size, max_chunk) if max_chunk else (src.size + 2) // 3 * 4 + 16
    if out is None:
        out = np.empty(cap, np.uint8)
    err = ctypes.c_int(0)
    t = (ctypes.c_double * 1)()
    n = _lib_or_default(lib).h_fd_encode(src.ctypes.data if src.size else None,
                                         lens.ctypes.data, lens.size, max_chunk, cch(pos62),
                                         cch(pos63), int(bool(pad)), cch(padchar),
                                         out.ctypes.data, out.size, int(bool(sock)),
                                         ctypes.byref(err), t)
    return (None if n < 0 else out[:n]), err.value, t[0]


def egress_pieces(pieces, max_chunk: int, read_size: int, push=False, late=False, lib=None):
    """queuestream_enqueue_bytes (or _push_bytes) of every piece ->
    base64_encode -> chunk_encode(max_chunk), drained read_size at a time:
    (framed bytes, errno)."""
    data = b"".join(pieces)
    src = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    lens = np.array([len(p) for p in pieces] or [0], dtype=np.uint64)
    cap = framed_cap(len(data), max_chunk) + 64
    out = np.zeros(cap, dtype=np.uint8)
    err = ctypes.c_int(0)
    n = _lib_or_default(lib).h_egress_pieces(src.ctypes.data, lens.ctypes.data, len(pieces),
                                             int(push), int(late), max_chunk, read_size,
                                             out.ctypes.data, cap, ctypes.byref(err))
    return (out[:n].tobytes() if n >= 0 else None), err.value


def fd_raw(data, write_chunk=1 << 20, read_size=1 << 18, sock=False, out=None, lib=None):
    """The pipe or socket alone: a peer thread writes `data`, this thread
    read(2)s it into `out`.  Returns (bytes array, errno, seconds)."""
    src = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data
    if out is None:
        out = np.empty(src.size + 1, np.uint8)
    err = ctypes.c_int(0)
    t = np.zeros(1)
    n = _lib_or_default(lib).h_fd_raw(src.ctypes.data if src.size else None, src.size, write_chunk,
                                      read_size, out.ctypes.data, out.size, int(sock),
                                      ctypes.byref(err), t.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return (out[:n] if n >= 0 else None), err.value, float(t[0])


def dechunk(framed: bytes) -> bytes:
    """The payload of an HTTP/1.1 chunked body (chunkencoder's framing)."""
    out, pos = bytearray(), 0
    while True:
        eol = framed.index(b"\r\n", pos)
        size = int(framed[pos:eol], 16)
        pos = eol + 2
        if size == 0:
            return bytes(out)
        out += framed[pos:pos + size]
        pos += size + 2
