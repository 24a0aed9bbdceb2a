#!/usr/bin/env python3
"""Copy-kernel shapes on the GPU (tests/csrc/libb64x_hooks.so,
b64x__test_copy_mode): 2.5 GB moved per launch like config 2's encode or
decode, median of 20 after 3 warm-ups, HIP events.  One JSON line per mode."""
import ctypes
import json
import os
import statistics

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = {0: "U4 TH256 nt", 1: "U1 TH256 nt", 2: "U2 TH256 nt", 3: "U8 TH256 nt",
         4: "U4 TH512 nt", 5: "U4 TH1024 nt", 6: "U4 TH256 cached", 7: "U2 TH1024 nt",
         8: "U1 TH1024 nt"}
lib = ctypes.CDLL(os.path.join(ROOT, "tests", "csrc", "libb64x_hooks.so"))
lib.b64x__test_copy_mode.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p,
                                                             ctypes.c_int]
half = (2505397592 // 2) // (1 << 16) * (1 << 16)
src = torch.full((half,), 7, dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
st = torch.cuda.current_stream().cuda_stream
for rnd in range(2):
    for m, name in MODES.items():
        ts = []
        for i in range(23):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            rc = lib.b64x__test_copy_mode(src.data_ptr(), dst.data_ptr(), half, st, m)
            b.record()
            b.synchronize()
            assert rc == 0, rc
            if i >= 3:
                ts.append(a.elapsed_time(b))
        ms = statistics.median(ts)
        print(json.dumps({"round": rnd, "mode": m, "shape": name, "ms": ms,
                          "TB_s": 2 * half / ms / 1e9}), flush=True)
