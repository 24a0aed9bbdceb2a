#!/usr/bin/env python3
"""Config 5 (16,384 Zipf messages through queuestream -> GPU encoder ->
chunkencoder, 10,240-byte reads) on ONE loop, where the time goes.

Three timed passes under ASYNC_B64_HUB_TRACE=1, each broken into phases:
  setup_s    building the stacks (queuestream_enqueue_bytes copies every
             message, as the reference's does: src/queuestream.c:117-122)
  loop_s     the event loop, of which
    read_s     inside the consumers' reads (everything below that a read
               triggers, plus chunkencoder framing and the copy out)
    gather_s   the encoder stages' upstream reads: queuestream -> arena
    reserve_s  arena reservations (with the launches of the batches they seal)
    launch_s   batch launches (H2D, kernel, D2H enqueue)
    wake_s     completion processing (hub wake-ups)
    gpu_span_s first batch launched to last batch completed (the GPU side:
               gather kernels reading the lent messages over the host link,
               encode kernels writing the characters into pinned memory)
    other_s    loop_s minus read_s minus wake_s: the loop itself, waiting
               for the GPU, callbacks
then one pass under the harness's SIGPROF sampler (the loop thread's CPU
time by function).

    python scripts/cfg5_profile.py OUTDIR [--passes K] [--threads T] [--no-prof]
           [--no-trace]

--threads T runs the stacks on T loops (one hub each; the hub rows are
summed over them); --no-trace times the passes without the hub trace (the
bench's own conditions), so only setup_s / loop_s are reported.
"""
import ctypes
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--no-trace" not in sys.argv:
    os.environ["ASYNC_B64_HUB_TRACE"] = "1"

import torch  # noqa: E402,F401  (one HIP runtime, see async_amd/_lib.py)

from tests import util  # noqa: E402


def hub_lines(fn):
    """Run fn() with fd 2 captured; return its result and the b64_hub lines."""
    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile(mode="w+b") as f:
        os.dup2(f.fileno(), 2)
        try:
            r = fn()
        finally:
            os.dup2(saved, 2)
            os.close(saved)
        f.seek(0)
        text = f.read().decode(errors="replace")
    return r, [ln for ln in text.splitlines() if ln.startswith("b64_hub:")]


def parse(line):
    toks = line.split()[1:]
    return {toks[i]: float(toks[i + 1]) for i in range(0, len(toks) - 1, 2)
            if re.match(r"^-?[0-9.]+$", toks[i + 1])}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?", default="gpurun_out/cfg5prof")
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--no-trace", action="store_true")
    a = ap.parse_args()
    out = a.out
    os.makedirs(out, exist_ok=True)
    lens = util.zipf_lengths()
    payload = util.splitmix64(0x5EED, int(lens.sum()))
    H = util.harness()
    T = a.threads
    util.egress_stacks(payload[:4096], [64] * 64, 1 << 20, 10240)  # warm-up
    util.egress_stacks(payload, lens, 1 << 20, 10240, raw=True, threads=T)  # pools filled
    H.b64_hub_pooled.restype = ctypes.c_ulong
    rows = []
    for _ in range(a.passes):
        pooled0 = H.b64_hub_pooled()
        t = np.zeros(2)
        H.h_take_read_seconds(None)
        t0 = time.perf_counter()
        (res, err), lines = hub_lines(
            lambda: util.egress_stacks(payload, lens, 1 << 20, 10240, times=t, raw=True,
                                       threads=T))
        wall = time.perf_counter() - t0
        assert res is not None, err
        nreads = ctypes.c_ulong()
        read_s = H.h_take_read_seconds(ctypes.byref(nreads))
        hub = {}
        for ln in lines:  # one hub per loop; sum in case of several
            for k, v in parse(ln).items():
                hub[k] = hub.get(k, 0.0) + v
        row = {"setup_s": t[0], "loop_s": t[1], "GiB_s": lens.sum() / t.sum() / 2**30,
               "loop_GiB_s": lens.sum() / t[1] / 2**30, "py_wall_s": wall,
               "read_s": read_s, "reads": nreads.value,
               "gather_s": hub.get("gather_s"), "gather_GiB_s":
                   hub.get("gather_bytes", 0) / max(hub.get("gather_s", 0), 1e-9) / 2**30,
               "reserve_s": hub.get("reserve_s"), "launch_s": hub.get("launch_s"),
               "wake_s": hub.get("wake_s"), "batches": hub.get("batches"),
               "gpu_span_s": hub.get("span_s"), "lent_bytes": hub.get("lent_bytes"),
               "arena_allocs": hub.get("allocs"), "hubs": len(lines),
               "arenas_live_max_sum": hub.get("max_live"),
               "pooled_before": pooled0, "pooled_after": H.b64_hub_pooled(),
               "other_s": t[1] - read_s - hub.get("wake_s", 0.0)}
        row["threads"] = T
        rows.append(row)
        print(json.dumps(row), flush=True)
        del res
    with open(os.path.join(out, f"cfg5_phases_t{T}.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    if a.no_prof:
        return
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
