#!/usr/bin/env python3
"""Host-side cost of one decode call (the time b64.decode takes to return,
the GPU idle and synced before each call) and the GPU gap it leaves: 1 GiB
at junk density 0.05 on the hinted path, with EXPECT_JUNK, and clean.
    python scripts/host_overhead.py [LIB]"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
from async_amd import b64  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "scripts"))
from bench_dirty import sprinkle  # noqa: E402

n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
b64.fill_splitmix64(x, 0x5EED)
enc = b64.encode(x)
junk = sprinkle(enc, 0.05)
out = torch.empty(b64.decoded_cap(junk.numel()), dtype=torch.uint8, device="cuda")
rr = torch.zeros(_lib.RES_BYTES, dtype=torch.uint8, device="cuda")
ws = torch.zeros(b64.workspace_size(junk.numel()), dtype=torch.uint8, device="cuda")
legs = {
    "junk_hinted": lambda: b64.decode(junk, out=out, workspace=ws, result=rr),
    "junk_ej": lambda: b64.decode(junk, out=out, workspace=ws, result=rr, expect_junk=True),
    "clean": lambda: b64.decode(enc, out=out, workspace=ws, result=rr),
}
# ORDER=ej,hinted,... runs the legs in that order, twice (the first leg after
# the setup may run on a GPU whose clocks are still ramping); REPS calls a leg
order = os.environ.get("ORDER", "junk_hinted,junk_ej,clean").split(",")
for name in order:
    fn = legs[name]
    fn()
    torch.cuda.synchronize()
    host, gpu = [], []
    for _ in range(int(os.environ.get("REPS", "20"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        b.record()
        b.synchronize()
        host.append((t1 - t0) * 1e6)
        gpu.append(a.elapsed_time(b) * 1e3)
    print(json.dumps({"leg": name, "host_us_median": statistics.median(host),
                      "event_us_median": statistics.median(gpu)}), flush=True)
