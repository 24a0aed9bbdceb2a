"""Host-side mirror of the base64 byte-stream engine over device tensors.

Thin wrappers over the b64x C ABI (include/b64x.h): torch provides device
memory and the stream, libasync_b64.so does the work.  The names follow the
reference's operations (src/base64encoder.c ``base64_encode`` /
src/base64decoder.c ``base64_decode``), applied to whole device-resident
buffers and batches instead of a pull-model stream:

    encode(x)                  one buffer      (b64x_encode_dev)
    decode(x)                  one buffer      (b64x_decode_dev)
    encode_strided / decode_strided            uniform batches
    encode_batch / decode_batch                ragged batches (offsets)

Every function raises (B64xError / RuntimeError) if the HIP library is
missing or a call fails; nothing here computes base64 on the CPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import RES_BYTES, B64xError, DecResult, alphabet  # noqa: F401

HOLD_TAIL = 1  # B64X_DEC_HOLD_TAIL
EXPECT_JUNK = 2  # B64X_DEC_EXPECT_JUNK


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def _u8(t: torch.Tensor, what: str) -> torch.Tensor:
    if t.dtype != torch.uint8 or not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{what} must be a contiguous uint8 CUDA tensor")
    return t


def encoded_len(n: int, pad: bool = True) -> int:
    return int(_lib.load().b64x_encoded_len(n, pad))


def decoded_cap(nchars: int) -> int:
    return int(_lib.load().b64x_decoded_cap(nchars))


def workspace_size(nchars: int = 0) -> int:
    return int(_lib.load().b64x_decode_workspace_size(nchars))


_DEFAULT_ABC: list = []  # the reference's alphabet, built once (read-only to the library)


def _abc(abc) -> _lib.Alphabet:
    if abc is None:
        if not _DEFAULT_ABC:
            _DEFAULT_ABC.append(alphabet())
        return _DEFAULT_ABC[0]
    return abc if isinstance(abc, _lib.Alphabet) else alphabet(*abc) if abc else alphabet()


def encode(x: torch.Tensor, out: torch.Tensor | None = None, abc=None,
           stream=None) -> torch.Tensor:
    """Base64-encode a device buffer; returns the character tensor."""
    lib = _lib.load()
    a = _abc(abc)
    _u8(x, "input")
    n = x.numel()
    m = encoded_len(n, a.pad)
    if out is None:
        out = torch.empty(max(m, 1), dtype=torch.uint8, device=x.device)
    _u8(out, "output")
    if out.numel() < m:
        raise ValueError("output too small")
    _lib.check("b64x_encode_dev", lib.b64x_encode_dev(
        _ptr(x), n, _ptr(out), ctypes.byref(a), _stream(stream)))
    return out[:m]


@dataclass
class Decoded:
    out: torch.Tensor          # capacity-sized output buffer
    result: torch.Tensor       # b64x_dec_result (RES_BYTES) on the device
    nchars: int = 0            # the call's character count, flags and the
    flags: int = 0             # sequence number it drew: what its record
    seq: int = 0               # must echo (b64x_result_check)
    stream: object = None      # the stream the decode ran on

    def info(self) -> DecResult:
        """The call's result record, checked: waits for the decode's own
        stream, copies the record back and refuses one that is not this
        call's or is inconsistent (b64x_result_check)."""
        s = self.stream if self.stream is not None else torch.cuda.current_stream()
        s.synchronize()
        host = self.result[:RES_BYTES].cpu().numpy()  # keep alive across the copy
        r = DecResult.from_buffer_copy(host.tobytes())
        if self.seq:
            _lib.check("b64x_result_check", _lib.load().b64x_result_check(
                ctypes.byref(r), self.nchars, self.flags, self.seq))
        return r

    def bytes(self) -> torch.Tensor:
        """The decoded bytes (synchronises to read the length)."""
        return self.out[: self.info().out_len]


def decode(x: torch.Tensor, out: torch.Tensor | None = None, abc=None,
           hold_tail: bool = False, workspace: torch.Tensor | None = None,
           result: torch.Tensor | None = None, stream=None,
           expect_junk: bool = False) -> Decoded:
    """Leniently decode a device buffer of base64 characters.
    expect_junk: the input holds non-alphabet bytes throughout (MIME line
    breaks) -- decode in one pass (B64X_DEC_EXPECT_JUNK); same result."""
    lib = _lib.load()
    a = _abc(abc)
    _u8(x, "input")
    n = x.numel()
    cap = decoded_cap(n)
    if out is None:
        out = torch.empty(max(cap, 1), dtype=torch.uint8, device=x.device)
    _u8(out, "output")
    if out.numel() < cap:
        raise ValueError("output too small")
    if result is None:
        result = torch.zeros(RES_BYTES, dtype=torch.uint8, device=x.device)
    # workspace: a caller's (zeroed before its first use; the library keeps
    # it re-armed), else the library's own for the stream (NULL), which also
    # keeps the line model of its last probe for the next call of a length
    # Under graph capture with no workspace given, a torch-allocated one (the
    # library will not allocate or rebind one inside a capture: -EBUSY).
    if workspace is None and torch.cuda.is_current_stream_capturing():
        workspace = torch.zeros(workspace_size(n), dtype=torch.uint8, device=x.device)
    flags = (HOLD_TAIL if hold_tail else 0) | (EXPECT_JUNK if expect_junk else 0)
    seq = ctypes.c_uint32(0)
    # the stream looked up once (torch.cuda.current_stream() costs ~3 us of
    # the call's host time, and a junk-laden or small decode is timed with it)
    s = stream if stream is not None else torch.cuda.current_stream()
    _lib.check("b64x_decode_dev_seq", lib.b64x_decode_dev_seq(
        _ptr(x), n, _ptr(out), _ptr(result), ctypes.byref(a), flags,
        _ptr(workspace) if workspace is not None else None, s.cuda_stream,
        ctypes.byref(seq)))
    return Decoded(out, result, n, flags & HOLD_TAIL, seq.value, s)


def encode_strided(x: torch.Tensor, in_stride: int, length: int, nbuf: int,
                   out: torch.Tensor, out_stride: int, abc=None, stream=None) -> None:
    lib = _lib.load()
    a = _abc(abc)
    _u8(x, "input")
    _u8(out, "output")
    if nbuf and (x.numel() < (nbuf - 1) * in_stride + length or
                 out.numel() < (nbuf - 1) * out_stride + encoded_len(length, a.pad)):
        raise ValueError("buffers too small for the batch")
    _lib.check("b64x_encode_strided", lib.b64x_encode_strided(
        _ptr(x), in_stride, length, nbuf, _ptr(out), out_stride, ctypes.byref(a),
        _stream(stream)))


def decode_strided(x: torch.Tensor, in_stride: int, length: int, nbuf: int,
                   out: torch.Tensor, out_stride: int, outlen: torch.Tensor,
                   abc=None, stream=None) -> None:
    lib = _lib.load()
    a = _abc(abc)
    _u8(x, "input")
    _u8(out, "output")
    if outlen.dtype != torch.int64 or outlen.numel() < nbuf or not outlen.is_cuda:
        raise ValueError("outlen must be an int64 CUDA tensor with nbuf entries")
    if nbuf and (x.numel() < (nbuf - 1) * in_stride + length or
                 out.numel() < (nbuf - 1) * out_stride + decoded_cap(length)):
        raise ValueError("buffers too small for the batch")
    _lib.check("b64x_decode_strided", lib.b64x_decode_strided(
        _ptr(x), in_stride, length, nbuf, _ptr(out), out_stride, _ptr(outlen),
        ctypes.byref(a), _stream(stream)))


def _offsets(t: torch.Tensor, n: int, what: str) -> torch.Tensor:
    if t.dtype != torch.int64 or not t.is_cuda or t.numel() < n:
        raise ValueError(f"{what} must be an int64 CUDA tensor of {n} entries")
    return t


def encode_batch(x: torch.Tensor, in_off: torch.Tensor, out: torch.Tensor,
                 out_off: torch.Tensor, abc=None, stream=None) -> None:
    """Ragged batch: buffer i = x[in_off[i]:in_off[i+1]] -> out[out_off[i]:]."""
    lib = _lib.load()
    a = _abc(abc)
    nbuf = in_off.numel() - 1
    _offsets(in_off, nbuf + 1, "in_off")
    _offsets(out_off, nbuf, "out_off")
    _lib.check("b64x_encode_batch", lib.b64x_encode_batch(
        _ptr(_u8(x, "input")), _ptr(in_off), nbuf, _ptr(_u8(out, "output")),
        _ptr(out_off), ctypes.byref(a), _stream(stream)))


def decode_batch(x: torch.Tensor, in_off: torch.Tensor, out: torch.Tensor,
                 out_off: torch.Tensor, outlen: torch.Tensor, abc=None,
                 stream=None) -> None:
    lib = _lib.load()
    a = _abc(abc)
    nbuf = in_off.numel() - 1
    _offsets(in_off, nbuf + 1, "in_off")
    _offsets(out_off, nbuf, "out_off")
    _offsets(outlen, nbuf, "outlen")
    _lib.check("b64x_decode_batch", lib.b64x_decode_batch(
        _ptr(_u8(x, "input")), _ptr(in_off), nbuf, _ptr(_u8(out, "output")),
        _ptr(out_off), _ptr(outlen), ctypes.byref(a), _stream(stream)))


def release_stream(stream=None) -> None:
    """Hand back the library decode workspace bound to `stream`
    (b64x_release_stream).  Required before the stream's handle is destroyed
    if it decoded without a workspace of its own: a later takeover of the
    workspace records an event on the handle it is bound to.  torch's own
    streams (torch.cuda.Stream(), the default stream) come from pools that
    live as long as the process, so this matters for handles wrapped with
    torch.cuda.ExternalStream whose owner destroys them; for the others it
    only frees the workspace at once instead of when the least recently used
    one is taken over.  The next decode on the stream binds one again; work
    already queued is not affected."""
    _lib.load().b64x_release_stream(_stream(stream))


def fill_splitmix64(x: torch.Tensor, seed: int, stream=None) -> torch.Tensor:
    """Fill a device buffer with the synthetic splitmix64 byte stream."""
    lib = _lib.load()
    _u8(x, "buffer")
    _lib.check("b64x_fill_splitmix64", lib.b64x_fill_splitmix64(
        _ptr(x), x.numel(), seed, _stream(stream)))
    return x


def device_numa_node(device: int = -1) -> int:
    """The NUMA node the GPU hangs off (b64x_device_numa_node); negative
    errno when unknown."""
    return _lib.load().b64x_device_numa_node(device)


def bind_thread(device: int = -1) -> int:
    """Bind the calling thread to the GPU's NUMA node (b64x_bind_thread):
    threads it starts afterwards inherit the mask.  Returns the node or a
    negative errno (the thread unchanged)."""
    return _lib.load().b64x_bind_thread(device)


def device_check() -> None:
    """Raise unless a gfx950 device is usable by the library."""
    _lib.check("b64x_device_check", _lib.load().b64x_device_check())


def build_info() -> str:
    return _lib.load().b64x_build_info().decode()
