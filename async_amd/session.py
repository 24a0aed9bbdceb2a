"""Host-memory sessions: pinned staging + H2D + GPU kernels + D2H.

Python view of the ``b64x_session_*`` entry points (include/b64x.h), the
host-memory leg the bytestream_1 stages in async_amd/csrc/b64_stages.c are
built on.  Used by the tests and by
scripts/bench_host_pipeline.py, which measures the PCIe-inclusive rate.

    s = Session(1 << 20)
    s.host_in[:n] = data
    s.encode_async(n); s.wait(); chars = s.host_out[:encoded_len(n)]

A stream decoded in blocks uses HOLD_TAIL for every block but the last and
spells the record's held-back sextets (``result().tail``) in front of the
next block, as the bytestream_1 decoder stage does.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import B64xError, DecResult, alphabet

HOLD_TAIL = 1


def _abc(abc) -> _lib.Alphabet:
    return abc if isinstance(abc, _lib.Alphabet) else alphabet(*abc) if abc else alphabet()


class Session:
    """One b64x_session: a HIP stream, pinned host_in/host_out, device
    buffers and a decode workspace, all sized for ``capacity``."""

    def __init__(self, capacity: int):
        self._L = _lib.load()
        ctypes.set_errno(0)
        h = self._L.b64x_session_open(capacity)
        if not h:
            raise B64xError("b64x_session_open", -(ctypes.get_errno() or 19))
        self._h = ctypes.c_void_p(h)
        self.capacity = int(self._L.b64x_session_capacity(self._h))
        out_cap = max(4 * ((self.capacity + 16 + 2) // 3), 3 * ((self.capacity + 16 + 3) // 4))
        self.host_in = np.ctypeslib.as_array(
            ctypes.cast(self._L.b64x_session_host_in(self._h),
                        ctypes.POINTER(ctypes.c_uint8)), (self.capacity,))
        self.host_out = np.ctypeslib.as_array(
            ctypes.cast(self._L.b64x_session_host_out(self._h),
                        ctypes.POINTER(ctypes.c_uint8)), (out_cap,))

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def close(self) -> None:
        if self._h:
            self._L.b64x_session_close(self._h)
            self._h = None
            self.host_in = self.host_out = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- synchronous ------------------------------------------------------
    def encode(self, n: int, abc=None) -> int:
        out = ctypes.c_uint64(0)
        _lib.check("b64x_session_encode",
                   self._L.b64x_session_encode(self._h, n, ctypes.byref(_abc(abc)),
                                               ctypes.byref(out)))
        return int(out.value)

    def decode(self, n: int, abc=None, flags: int = 0) -> DecResult:
        res = DecResult()
        _lib.check("b64x_session_decode",
                   self._L.b64x_session_decode(self._h, n, ctypes.byref(_abc(abc)), flags,
                                               ctypes.byref(res)))
        return res

    # -- asynchronous -----------------------------------------------------
    def encode_async(self, n: int, abc=None) -> None:
        _lib.check("b64x_session_encode_async",
                   self._L.b64x_session_encode_async(self._h, n, ctypes.byref(_abc(abc)),
                                                     None, None))

    def decode_async(self, n: int, abc=None, flags: int = 0) -> None:
        _lib.check("b64x_session_decode_async",
                   self._L.b64x_session_decode_async(self._h, n, ctypes.byref(_abc(abc)),
                                                     flags, None, None))

    def wait(self) -> None:
        _lib.check("b64x_session_wait", self._L.b64x_session_wait(self._h))

    def result(self) -> DecResult:
        """Checked copy of the last completed decode's result (call after
        wait()); raises if the record is not a finished, consistent one."""
        res = DecResult()
        _lib.check("b64x_session_decode_result",
                   self._L.b64x_session_decode_result(self._h, ctypes.byref(res)))
        return res


def diag_counters() -> tuple[int, int]:
    """(session records, lane batches) found unfinished when their
    completion callback had already run (see b64x_diag_counters)."""
    out = (ctypes.c_uint64 * 2)()
    _lib.load().b64x_diag_counters(out)
    return int(out[0]), int(out[1])
