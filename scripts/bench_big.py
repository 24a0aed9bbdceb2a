#!/usr/bin/env python3
"""Past 2^31 characters (DESIGN.md §5 "Larger inputs"): the clean decode of
one buffer of 3 x 2^30 characters (2.25 GiB of payload) and of 4.5 GiB of
payload (6 x 2^30 characters, past 2^32).  Since round 6 both take the probe
/ lines / suffix pipeline (up to 2^33 characters); rounds 1-5 sent anything
past 2^31 to pass 1, the scan and pass 2.  Encode and decode timed with HIP
events (median of 10 after 2 warm-ups), bit-checked, one JSON line; the
1 GiB decode beside it for comparison.

    python scripts/bench_big.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from async_amd import b64  # noqa: E402


def timed(fn, steps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts), min(ts), max(ts)


def main():
    out = {}
    for name, n in (("1GiB", 1 << 30), ("2.25GiB", 9 << 28), ("4.5GiB", 9 << 29)):
        x = torch.empty(n, dtype=torch.uint8, device="cuda")
        b64.fill_splitmix64(x, 0x5EED)
        enc = b64.encode(x)
        dec = torch.empty(b64.decoded_cap(enc.numel()), dtype=torch.uint8, device="cuda")
        ws = torch.zeros(b64.workspace_size(enc.numel()), dtype=torch.uint8, device="cuda")
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device="cuda")
        e_ms = timed(lambda: b64.encode(x, out=enc))
        d_ms = timed(lambda: b64.decode(enc, out=dec, workspace=ws, result=res))
        d = b64.decode(enc, out=dec, workspace=ws, result=res)
        ok = d.info().out_len == n and torch.equal(dec[:n], x)
        alg = n + enc.numel()
        out[name] = {"chars": enc.numel(), "bytes": n, "exact": ok,
                     "encode_ms": e_ms, "decode_ms": d_ms,
                     "encode_TBps": alg / (e_ms[0] * 1e-3) / 1e12,
                     "decode_TBps": alg / (d_ms[0] * 1e-3) / 1e12,
                     "decode_frac_of_8TBps": alg / (d_ms[0] * 1e-3) / 8e12}
        del x, enc, dec, ws
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
