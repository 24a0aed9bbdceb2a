#!/usr/bin/env python3
"""Where one decoder stream's loop thread spends its time (VERDICT r04 item
6): config 2's 1 GiB of characters, blob -> base64_decode stage (GPU) ->
consumer reading 256 KiB at a time, on one loop, timed, then again under
the harness's SIGPROF sampler (process CPU time by function; the loop
thread's idle waits are not sampled, so samples x period against the wall
time gives how busy the threads were).

    python scripts/ingress_profile.py OUTDIR
"""
import ctypes
import json
import os
import resource
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from async_amd import b64  # noqa: E402
from tests import util  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ingress_prof"
    os.makedirs(out, exist_ok=True)
    N = 1 << 30
    x = torch.empty(N, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    ch = b64.encode(x).cpu().numpy()
    xh = x.cpu().numpy()
    dst = np.empty(N + 16, np.uint8)
    dst.fill(0)
    H = util.harness()
    if os.environ.get("ASYNC_B64_HUB_TRACE") == "1":
        # phase rows: the consumer's reads (everything a read triggers) and
        # the hub's own counters, printed to stderr when the hub goes
        for _ in range(3):
            err = ctypes.c_int(0)
            H.h_take_read_seconds(None)
            t0 = time.perf_counter()
            n = H.h_decode_stream(ch.ctypes.data, ch.size, 0, 1 << 18, util.cch(-1),
                                  util.cch(-1), dst.ctypes.data, dst.size, ctypes.byref(err))
            dt = time.perf_counter() - t0
            reads = ctypes.c_ulong()
            read_s = H.h_take_read_seconds(ctypes.byref(reads))
            print(json.dumps({"traced": True, "GiB_s": N / dt / 2**30, "wall_s": dt,
                              "read_s": read_s, "reads": reads.value, "ok": n == N}), flush=True)
        return
    rows = []
    for prof in (False, False, True):
        err = ctypes.c_int(0)
        if prof:
            H.h_prof_start(4000)
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        n = H.h_decode_stream(ch.ctypes.data, ch.size, 0, 1 << 18, util.cch(-1), util.cch(-1),
                              dst.ctypes.data, dst.size, ctypes.byref(err))
        dt = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        if prof:
            path = os.path.join(out, "ingress_blob_prof.txt")
            H.h_prof_stop(path.encode())
        ok = n == N and np.array_equal(dst[:N], xh)
        row = {"profiled": prof, "GiB_s": N / dt / 2**30, "wall_s": dt, "ok": bool(ok),
               "user_s": r1.ru_utime - r0.ru_utime, "sys_s": r1.ru_stime - r0.ru_stime}
        rows.append(row)
        print(json.dumps(row), flush=True)
    with open(os.path.join(out, "ingress_blob_rows.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_resolve.py"),
                        os.path.join(out, "ingress_blob_prof.txt"), "40"],
                       capture_output=True, text=True)
    with open(os.path.join(out, "ingress_blob_prof_resolved.txt"), "w") as f:
        f.write(r.stdout)
    print(r.stdout, flush=True)


if __name__ == "__main__":
    main()
