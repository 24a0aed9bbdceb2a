"""ctypes binding of the b64x C ABI (include/b64x.h) in libasync_b64.so.

The library is built in-tree (``make`` / ``__graft_entry__.build()``) and is
the only compute path: if it is missing, or no gfx950 device is usable, the
calls below raise -- there is no CPU fallback.

PyTorch bundles its own HIP runtime (torch/lib/libamdhip64.so, soname
libamdhip64.so.7).  It is imported *before* the library is loaded so that
libasync_b64.so's dependency on libamdhip64.so.7 resolves to that same,
already-loaded runtime: one HIP runtime per process, so device pointers and
streams from torch are valid in our kernels.
"""
from __future__ import annotations

import ctypes
import errno
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libasync_b64.so")

_lock = threading.Lock()
_lib = None


class B64xError(RuntimeError):
    """A b64x entry point returned a negative errno value."""

    def __init__(self, func: str, code: int):
        self.code = code
        name = errno.errorcode.get(-code, str(code))
        super().__init__(f"{func} failed: {name} ({code})")


class Alphabet(ctypes.Structure):
    """b64x_alphabet: (char) -1 selects the reference's defaults."""

    _fields_ = [
        ("pos62", ctypes.c_char),
        ("pos63", ctypes.c_char),
        ("padchar", ctypes.c_char),
        ("pad", ctypes.c_bool),
    ]


class DecResult(ctypes.Structure):
    """b64x_dec_result, 40 bytes, written by the device; nchars, seq and
    flags name the call that wrote it (include/b64x.h)."""

    _fields_ = [
        ("out_len", ctypes.c_uint64),
        ("valid", ctypes.c_uint64),
        ("tail_n", ctypes.c_uint32),
        ("tail", ctypes.c_uint8 * 4),
        ("nchars", ctypes.c_uint64),
        ("seq", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
    ]


assert ctypes.sizeof(DecResult) == 40
RES_BYTES = ctypes.sizeof(DecResult)  # device buffers for one record

_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_vp = ctypes.c_void_p
_int = ctypes.c_int
_ap = ctypes.POINTER(Alphabet)

# name -> (restype, argtypes); every symbol include/b64x.h declares.
SIGNATURES = {
    "b64x_encoded_len": (_u64, [_u64, ctypes.c_bool]),
    "b64x_decoded_cap": (_u64, [_u64]),
    "b64x_decode_workspace_size": (_u64, [_u64]),
    "b64x_encode_dev": (_int, [_vp, _u64, _vp, _ap, _vp]),
    "b64x_decode_dev": (_int, [_vp, _u64, _vp, _vp, _ap, ctypes.c_uint, _vp, _vp]),
    "b64x_decode_dev_seq": (_int, [_vp, _u64, _vp, _vp, _ap, ctypes.c_uint, _vp, _vp,
                                   ctypes.POINTER(_u32)]),
    "b64x_result_check": (_int, [ctypes.POINTER(DecResult), _u64, ctypes.c_uint, _u32]),
    "b64x_encode_strided": (_int, [_vp, _u64, _u64, _u32, _vp, _u64, _ap, _vp]),
    "b64x_decode_strided": (_int, [_vp, _u64, _u64, _u32, _vp, _u64, _vp, _ap, _vp]),
    "b64x_encode_batch": (_int, [_vp, _vp, _u32, _vp, _vp, _ap, _vp]),
    "b64x_decode_batch": (_int, [_vp, _vp, _u32, _vp, _vp, _vp, _ap, _vp]),
    "b64x_session_open": (_vp, [_u64]),
    "b64x_session_close": (None, [_vp]),
    "b64x_session_acquire": (_vp, [_u64]),
    "b64x_session_release": (None, [_vp]),
    "b64x_session_capacity": (_u64, [_vp]),
    "b64x_session_host_in": (_vp, [_vp]),
    "b64x_session_host_out": (_vp, [_vp]),
    "b64x_session_encode": (_int, [_vp, _u64, _ap, ctypes.POINTER(_u64)]),
    "b64x_release_stream": (None, [_vp]),
    "b64x_session_decode": (_int, [_vp, _u64, _ap, ctypes.c_uint, ctypes.POINTER(DecResult)]),
    "b64x_session_encode_async": (_int, [_vp, _u64, _ap, _vp, _vp]),
    "b64x_session_decode_async": (_int, [_vp, _u64, _ap, ctypes.c_uint, _vp, _vp]),
    "b64x_session_result": (ctypes.POINTER(DecResult), [_vp]),
    "b64x_session_decode_result": (_int, [_vp, ctypes.POINTER(DecResult)]),
    "b64x_session_wait": (_int, [_vp]),
    "b64x_host_alloc": (_vp, [_u64]),
    "b64x_host_free": (None, [_vp]),
    "b64x_lane_open": (_vp, []),
    "b64x_lane_close": (None, [_vp]),
    "b64x_lane_acquire": (_vp, []),
    "b64x_lane_release": (None, [_vp]),
    "b64x_lane_encode_async": (_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32, _ap, _vp, _vp]),
    "b64x_lane_encode_check": (_int, [_vp]),
    "b64x_lane_decode_async": (_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _ap,
                                      _vp, _vp, ctypes.POINTER(_u32)]),
    "b64x_lane_decode_check": (_int, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32]),
    "b64x_lane_wait": (_int, [_vp]),
    "b64x_diag_counters": (None, [ctypes.POINTER(_u64)]),
    "b64x_diag_paths": (None, [ctypes.POINTER(_u64)]),
    "b64x_fill_splitmix64": (_int, [_vp, _u64, _u64, _vp]),
    "b64x_device_check": (_int, []),
    "b64x_device_numa_node": (_int, [_int]),
    "b64x_bind_thread": (_int, [_int]),
    "b64x_build_info": (ctypes.c_char_p, []),
    "b64x_strerror": (ctypes.c_char_p, [_int]),
}

# The bytestream_1 stages and loop pieces the library also exports (C ABI of
# include/base64encoder.h, base64decoder.h, async.h, blobstream.h,
# nicestream.h); checked for presence, not called from Python.
STAGE_SYMBOLS = [
    "base64_encode", "base64encoder_as_bytestream_1", "base64encoder_read",
    "base64encoder_close", "base64encoder_register_callback",
    "base64encoder_unregister_callback",
    "base64_decode", "base64decoder_as_bytestream_1", "base64decoder_read",
    "base64decoder_close", "base64decoder_register_callback",
    "base64decoder_unregister_callback",
    "make_async", "destroy_async", "async_now", "async_timer_start",
    "async_timer_cancel", "async_execute", "async_wound", "async_loop",
    "async_quit_loop", "async_register", "async_unregister",
    "NULL_ACTION_1", "bytestream_1_close_relaxed",
    "open_blobstream", "copy_blobstream", "adopt_blobstream",
    "blobstream_as_bytestream_1", "blobstream_remaining", "blobstream_read",
    "blobstream_close", "blobstream_register_callback",
    "blobstream_unregister_callback",
    "make_nice", "nicestream_as_bytestream_1", "nicestream_read",
    "nicestream_close", "nicestream_register_callback",
    "nicestream_unregister_callback",
]


def _import_torch_first() -> None:
    try:
        import torch  # noqa: F401  (loads torch's libamdhip64.so.7)
    except ImportError:  # a torch-less process uses /opt/rocm's runtime
        pass


# Diagnostics an A/B timing may load an older library without
# (tests/test_abi.py checks that the product exports them).
_DIAG_ONLY = {"b64x_diag_paths"}


def load() -> ctypes.CDLL:
    """Load libasync_b64.so (raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make` or "
                "__graft_entry__.build(); there is no CPU fallback")
        _import_torch_first()
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if name in _DIAG_ONLY and not hasattr(lib, name):
                continue  # an older build under A/B (scripts/ab_*.py): no diagnostics
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(func: str, rc: int) -> None:
    if rc != 0:
        raise B64xError(func, rc)


def alphabet(pos62=-1, pos63=-1, pad=True, padchar=-1) -> Alphabet:
    """Build a b64x_alphabet; ints, 1-char str/bytes; -1 = default."""

    def ch(v):
        if isinstance(v, str):
            v = v.encode("latin-1")
        if isinstance(v, (bytes, bytearray)):
            if len(v) != 1:
                raise ValueError("alphabet characters are single bytes")
            v = v[0]
        return bytes([v & 0xFF])

    return Alphabet(ch(pos62), ch(pos63), ch(padchar), bool(pad))
