#!/usr/bin/env python3
"""Many short streams on ONE event loop: N decoder stacks (queuestream ->
GPU decoder, the ingress mirror of config 5) or N egress stacks
(queuestream -> GPU encoder -> chunkencoder), 100-4,000-byte messages,
drained with 64 KiB reads.  Prints one JSON line per run; the decoded
bytes are checked against the originals.

    python scripts/bench_ingress.py [--kind dec|enc] [--msgs 1000 16384]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as orc  # noqa: E402  (encodes the inputs)
from tests import util  # noqa: E402


def run(kind: str, nmsg: int) -> dict:
    rng = np.random.default_rng(1)
    raw = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
           for n in rng.integers(100, 4000, nmsg)]
    times = np.zeros(2)
    if kind == "dec":
        enc = [orc.encode(m) for m in raw]
        util.ingress_stacks(enc[:10], 65536)  # warm-up (lanes, arenas)
        got, err = util.ingress_stacks(enc, 65536, times=times)
        assert err == 0 and got == raw
        nbytes = sum(len(m) for m in enc)
    else:
        payload = np.frombuffer(b"".join(raw), np.uint8)
        lens = [len(m) for m in raw]
        util.egress_stacks(payload[:sum(lens[:10])], lens[:10], 1 << 20, 65536)
        got, err = util.egress_stacks(payload, lens, 1 << 20, 65536, times=times)
        assert err == 0
        nbytes = payload.size
    return {"measure": f"{kind}_stacks_one_loop", "messages": nmsg, "in_bytes": nbytes,
            "setup_s": float(times[0]), "loop_s": float(times[1]),
            "us_per_message_loop": float(times[1]) / nmsg * 1e6,
            "GBps_in_loop": nbytes / float(times[1]) / 1e9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", nargs="*", default=["dec", "enc"])
    ap.add_argument("--msgs", type=int, nargs="*", default=[1000, 16384, 65536])
    a = ap.parse_args()
    for k in a.kind:
        for n in a.msgs:
            print(json.dumps(run(k, n)), flush=True)


if __name__ == "__main__":
    main()
