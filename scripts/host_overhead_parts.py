#!/usr/bin/env python3
"""Where a decode call's host time goes: b64.decode against the bare C-ABI
call with its arguments prepared once (1 GiB at junk density 0.05, EXPECT_JUNK
and the hinted path; the GPU synced before each call)."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import _lib, b64  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "scripts"))
from bench_dirty import sprinkle  # noqa: E402

n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
b64.fill_splitmix64(x, 0x5EED)
junk = sprinkle(b64.encode(x), 0.05)
out = torch.empty(b64.decoded_cap(junk.numel()), dtype=torch.uint8, device="cuda")
rr = torch.zeros(_lib.RES_BYTES, dtype=torch.uint8, device="cuda")
ws = torch.zeros(b64.workspace_size(junk.numel()), dtype=torch.uint8, device="cuda")
lib = _lib.load()
a = b64.alphabet()
st = torch.cuda.current_stream().cuda_stream
seq = ctypes.c_uint32(0)
args = lambda f: (junk.data_ptr(), junk.numel(), out.data_ptr(), rr.data_ptr(), ctypes.byref(a),  # noqa: E731
                  f, ws.data_ptr(), st, ctypes.byref(seq))
pre = {f: args(f) for f in (0, b64.EXPECT_JUNK)}


def run(name, fn):
    fn()
    torch.cuda.synchronize()
    host = []
    for _ in range(30):
        t0 = time.perf_counter()
        fn()
        host.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    print(json.dumps({"call": name, "host_us_median": round(statistics.median(host), 2)}), flush=True)


run("b64.decode hinted", lambda: b64.decode(junk, out=out, workspace=ws, result=rr))
run("b64.decode expect_junk", lambda: b64.decode(junk, out=out, workspace=ws, result=rr,
                                                 expect_junk=True))
run("C-ABI hinted", lambda: lib.b64x_decode_dev_seq(*pre[0]))
run("C-ABI expect_junk", lambda: lib.b64x_decode_dev_seq(*pre[b64.EXPECT_JUNK]))
run("torch.cuda.is_current_stream_capturing", torch.cuda.is_current_stream_capturing)
run("torch.cuda.current_stream", torch.cuda.current_stream)
run("b64.alphabet", b64.alphabet)
run("b64.decoded_cap", lambda: b64.decoded_cap(n))
