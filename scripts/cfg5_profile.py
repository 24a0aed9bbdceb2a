#!/usr/bin/env python3
"""Config 5 (16,384 Zipf messages through queuestream -> GPU encoder ->
chunkencoder, 10,240-byte reads) on ONE loop, where the time goes: three
timed passes (setup = building the stacks, the queuestream copies
included; loop = pulls, batches, framing, reads), then one pass under the
harness's SIGPROF sampler (tests/csrc/stage_harness.c h_prof_start/stop:
the loop thread's CPU time by function) with the hub's own counters
(ASYNC_B64_HUB_TRACE: batches, launches, wake-ups).

    python scripts/cfg5_profile.py OUTDIR
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ASYNC_B64_HUB_TRACE"] = "1"

import torch  # noqa: E402,F401  (one HIP runtime, see async_amd/_lib.py)

from tests import util  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cfg5prof"
    os.makedirs(out, exist_ok=True)
    lens = util.zipf_lengths()
    payload = util.splitmix64(0x5EED, int(lens.sum()))
    util.egress_stacks(payload[:4096], [64] * 64, 1 << 20, 10240)  # warm-up
    util.egress_stacks(payload, lens, 1 << 20, 10240, raw=True)    # pools filled
    rows = []
    for _ in range(3):
        t = np.zeros(2)
        t0 = time.perf_counter()
        res, err = util.egress_stacks(payload, lens, 1 << 20, 10240, times=t, raw=True)
        wall = time.perf_counter() - t0
        assert res is not None, err
        rows.append({"setup_s": t[0], "loop_s": t[1], "GiB_s": lens.sum() / t.sum() / 2**30,
                     "py_wall_s": wall})
        print(json.dumps(rows[-1]), flush=True)
    H = util.harness()
    H.h_prof_start(2000)
    t = np.zeros(2)
    util.egress_stacks(payload, lens, 1 << 20, 10240, times=t, raw=True)
    prof = os.path.join(out, "cfg5_1loop_prof.txt")
    H.h_prof_stop(prof.encode())
    print(json.dumps({"profiled_pass": {"setup_s": t[0], "loop_s": t[1]}}), flush=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_resolve.py"), prof,
                        "40"], capture_output=True, text=True)
    with open(os.path.join(out, "cfg5_1loop_prof_resolved.txt"), "w") as f:
        f.write(r.stdout)
    print(r.stdout, flush=True)


if __name__ == "__main__":
    main()
