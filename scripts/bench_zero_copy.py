#!/usr/bin/env python3
"""Host-memory encode: the session way (H2D, kernel, D2H on one stream)
against the kernel reading and writing pinned host memory directly over
PCIe (zero-copy), for several block sizes.  Output checked.  JSON lines."""
import base64
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import _lib, b64  # noqa: E402

lib = _lib.load()
ABC = b64._abc(None)


def timed(fn, k=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(k):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / k


for mib in (4, 32, 256):
    n = mib << 20
    E = b64.encoded_len(n)
    h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_in.copy_(torch.randint(0, 256, (n,), dtype=torch.uint8))
    h_out = torch.empty(E, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(E, dtype=torch.uint8, device="cuda")

    def staged():
        d_in.copy_(h_in, non_blocking=True)
        b64.encode(d_in, out=d_out)
        h_out.copy_(d_out, non_blocking=True)

    def zero_copy():  # the kernel on the pinned host pointers themselves
        _lib.check("b64x_encode_dev", lib.b64x_encode_dev(
            h_in.data_ptr(), n, h_out.data_ptr(), b64.ctypes.byref(ABC),
            torch.cuda.current_stream().cuda_stream))

    t_s = timed(staged)
    ref = h_out.clone()
    t_z = timed(zero_copy)
    ok = torch.equal(h_out, ref)
    print(json.dumps({"measure": "host_encode", "mib": mib, "staged_ms": t_s, "zero_copy_ms": t_z,
                      "staged_GiBps": n / t_s / 1e-3 / 2**30, "zero_copy_GiBps": n / t_z / 1e-3 / 2**30,
                      "same_output": ok}), flush=True)


# Decode: staged (H2D, kernels, D2H of the capacity bound) against the
# kernels reading the pinned input and writing the pinned output in place,
# on clean text and on MIME text (CRLF every 76 characters, which pass 2
# re-reads).
def mime(text: bytes) -> bytes:
    return b"".join(text[i:i + 76] + b"\r\n" for i in range(0, len(text), 76))


for mib in (4, 32, 256):
    n = mib << 20
    raw = torch.randint(0, 256, (n,), dtype=torch.uint8).numpy().tobytes()
    clean = base64.b64encode(raw)
    for kind, text in (("clean", clean), ("crlf76", mime(clean))):
        m = len(text)
        cap = b64.decoded_cap(m)
        h_in = torch.frombuffer(bytearray(text), dtype=torch.uint8).pin_memory()
        h_out = torch.empty(cap, dtype=torch.uint8).pin_memory()
        d_in = torch.empty(m, dtype=torch.uint8, device="cuda")
        d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        res = torch.zeros(_lib.RES_BYTES, dtype=torch.uint8, device="cuda")
        ws = torch.zeros(b64.workspace_size(m), dtype=torch.uint8, device="cuda")

        def dec(src, dst):
            _lib.check("b64x_decode_dev", lib.b64x_decode_dev(
                src, m, dst, res.data_ptr(), b64.ctypes.byref(ABC), 0, ws.data_ptr(),
                torch.cuda.current_stream().cuda_stream))

        def staged():
            d_in.copy_(h_in, non_blocking=True)
            dec(d_in.data_ptr(), d_out.data_ptr())
            h_out.copy_(d_out, non_blocking=True)

        def zero_copy():
            dec(h_in.data_ptr(), h_out.data_ptr())

        t_s = timed(staged)
        ok_s = bytes(h_out[:n].numpy()) == raw
        h_out.zero_()
        t_z = timed(zero_copy)
        ok_z = bytes(h_out[:n].numpy()) == raw
        print(json.dumps({"measure": "host_decode", "input": kind, "mib": mib, "chars": m,
                          "staged_ms": t_s, "zero_copy_ms": t_z,
                          "staged_GiBps": n / t_s / 1e-3 / 2**30,
                          "zero_copy_GiBps": n / t_z / 1e-3 / 2**30,
                          "staged_exact": ok_s, "zero_copy_exact": ok_z}), flush=True)
