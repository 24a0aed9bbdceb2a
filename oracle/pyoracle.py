"""TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/liboracle.so.

The oracle is the CPU restatement of the reference's base64 stages
(oracle/b64_oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it, and only as the checker / the timed CPU
baseline -- never as a product code path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_sz = ctypes.c_size_t
_ssz = ctypes.c_ssize_t
_vp = ctypes.c_void_p
_ch = ctypes.c_char


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make`")
        L = ctypes.CDLL(LIB_PATH)
        L.orc_decode_table.argtypes = [_ch, _ch, _vp]
        L.orc_decode_table.restype = None
        L.orc_encode.argtypes = [_vp, _sz, _ch, _ch, ctypes.c_int, _ch, _vp]
        L.orc_encode.restype = _sz
        L.orc_decode.argtypes = [_vp, _sz, _ch, _ch, _vp]
        L.orc_decode.restype = _sz
        L.orc_encode_stream.argtypes = [_vp, _sz, _sz, _sz, _sz, _ch, _ch,
                                        ctypes.c_int, _ch, _vp, _sz,
                                        ctypes.POINTER(_sz)]
        L.orc_encode_stream.restype = _ssz
        L.orc_decode_stream.argtypes = [_vp, _sz, _sz, _sz, _sz, _ch, _ch, _vp, _sz]
        L.orc_decode_stream.restype = _ssz
        L.orc_reftest.argtypes = [_sz, _vp, _sz, ctypes.POINTER(_sz), _vp, _sz]
        L.orc_reftest.restype = _ssz
        L.orc_chunked_encode.argtypes = [_vp, _vp, _sz, _sz, ctypes.c_int, _sz, _ch, _ch,
                                         ctypes.c_int, _ch, _vp, _sz]
        L.orc_chunked_encode.restype = _ssz
        L.orc_encode_counts.argtypes = [_vp, _sz, _sz, _sz, _sz, _ch, _ch, ctypes.c_int, _ch,
                                        _vp, _sz]
        L.orc_encode_counts.restype = _ssz
        L.orc_encode_rows.argtypes = [_vp, _sz, _sz, _vp, _sz]
        L.orc_encode_rows.restype = _sz
        L.orc_decode_rows.argtypes = [_vp, _sz, _sz, _vp, _sz]
        L.orc_decode_rows.restype = _sz
        _lib = L
    return _lib


def _c(v) -> bytes:
    if isinstance(v, str):
        v = v.encode("latin-1")
    if isinstance(v, (bytes, bytearray)):
        return bytes(v[:1])
    return bytes([v & 0xFF])


def _arr(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8)
    return np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)[:0]


def _p(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def encode(data, pos62=-1, pos63=-1, pad=True, padchar=-1, as_array=False):
    a = _arr(data)
    out = np.empty((a.size + 2) // 3 * 4 + 1, dtype=np.uint8)
    n = lib().orc_encode(_p(a), a.size, _c(pos62), _c(pos63), int(bool(pad)),
                         _c(padchar), out.ctypes.data)
    return out[:n] if as_array else out[:n].tobytes()


def encode_rows(rows: np.ndarray, out: np.ndarray) -> int:
    """Encode each row of `rows` (nbuf x len, uint8, C-contiguous) into the
    matching row of `out` (nbuf x >= E); default alphabet, padding.  Runs
    without the GIL (ctypes), so threads over row slices run in parallel."""
    return lib().orc_encode_rows(_p(rows), rows.shape[1], rows.shape[0], _p(out), out.shape[1])


def decode_rows(rows: np.ndarray, out: np.ndarray) -> int:
    return lib().orc_decode_rows(_p(rows), rows.shape[1], rows.shape[0], _p(out), out.shape[1])


def decode(data, pos62=-1, pos63=-1, as_array=False):
    a = _arr(data)
    out = np.empty((a.size + 3) // 4 * 3 + 1, dtype=np.uint8)
    n = lib().orc_decode(_p(a), a.size, _c(pos62), _c(pos63), out.ctypes.data)
    return out[:n] if as_array else out[:n].tobytes()


class AssertDomain(Exception):
    """The reference would have tripped its assert (base64encoder.c:140)."""


def encode_stream(data, src_chunk=0, burst=0, read_size=200, pos62=-1, pos63=-1,
                  pad=True, padchar=-1) -> bytes:
    a = _arr(data)
    cap = (a.size + 2) // 3 * 4 + 8
    out = np.empty(cap, dtype=np.uint8)
    ov = _sz(0)
    n = lib().orc_encode_stream(_p(a), a.size, src_chunk, burst, read_size,
                                _c(pos62), _c(pos63), int(bool(pad)), _c(padchar),
                                out.ctypes.data, cap, ctypes.byref(ov))
    if n < 0:
        if ov.value:
            raise AssertDomain(f"{ov.value} overrunning reads")
        raise RuntimeError("oracle encode_stream failed")
    return out[:n].tobytes()


def decode_stream(data, src_chunk=0, burst=0, read_size=200, pos62=-1, pos63=-1) -> bytes:
    a = _arr(data)
    cap = (a.size + 3) // 4 * 3 + 8
    out = np.empty(cap, dtype=np.uint8)
    n = lib().orc_decode_stream(_p(a), a.size, src_chunk, burst, read_size,
                                _c(pos62), _c(pos63), out.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("oracle decode_stream failed")
    return out[:n].tobytes()


def decode_table(pos62=-1, pos63=-1) -> list[int]:
    t = (ctypes.c_int8 * 256)()
    lib().orc_decode_table(_c(pos62), _c(pos63), t)
    return list(t)


def reftest(length: int = 1000001):
    """The reference test topology; returns (encoded chars, decoded bytes)."""
    ecap = (length + 2) // 3 * 4 + 16
    enc = np.empty(ecap, dtype=np.uint8)
    dec = np.empty(length + 16, dtype=np.uint8)
    elen = _sz(0)
    n = lib().orc_reftest(length, enc.ctypes.data, ecap, ctypes.byref(elen),
                          dec.ctypes.data, dec.size)
    if n < 0:
        raise RuntimeError("oracle reftest failed")
    return enc[: elen.value].tobytes(), dec[:n].tobytes()


def chunked_encode(data, piece_lens=None, max_chunk=1 << 20, termination=0, read_size=None,
                   pos62=-1, pos63=-1, pad=True, padchar=-1) -> bytes:
    """The config-5 egress stack: terminated queuestream of pieces ->
    encoder -> chunkencoder(max_chunk), drained read_size at a time."""
    a = _arr(data)
    lens = np.asarray(piece_lens if piece_lens is not None else [a.size], dtype=np.uintp)
    rs = read_size or max(max_chunk, 16)
    chars = (a.size + 2) // 3 * 4
    cap = chars + (chars // max(max_chunk, 2) + 2) * 16 + 16
    out = np.empty(cap, dtype=np.uint8)
    n = lib().orc_chunked_encode(_p(a), lens.ctypes.data, lens.size, max_chunk, termination,
                                 rs, _c(pos62), _c(pos63), int(bool(pad)), _c(padchar),
                                 out.ctypes.data, cap)
    if n < 0:
        raise AssertDomain("chunked stack failed (assert domain?)")
    return out[:n].tobytes()


def encode_counts(data, read_size, src_chunk=0, burst=0, pos62=-1, pos63=-1, pad=True,
                  padchar=-1) -> list[int]:
    """The reference encoder's positive read returns for this read pattern."""
    a = _arr(data)
    cap = a.size // 2 + 64
    counts = np.empty(cap, dtype=np.intp)
    n = lib().orc_encode_counts(_p(a), a.size, src_chunk, burst, read_size, _c(pos62),
                                _c(pos63), int(bool(pad)), _c(padchar), counts.ctypes.data, cap)
    if n < 0:
        raise AssertDomain("encode_counts failed (assert domain?)")
    return counts[:min(n, cap)].tolist()
