#!/usr/bin/env python3
"""Why does bench.py's config-4 encode read ~9 % above the flat encode when
scripts/ab_batch.py and scripts/placement_probe.py see ~3 %?  Runs bench.py's
own legs in different orders in one process and prints each batch leg's
encode/decode kernel ms:  batch first (fresh process), then the single leg +
copy ceilings, then the batch leg again, then once more after emptying the
allocator's cache.

    python scripts/bench_order_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sys.argv = [sys.argv[0], "--no-cpu"]
    import torch
    import bench
    from async_amd import b64
    args = bench.parse()

    def leg(tag):
        r = bench.bench_batch(args, 1, 0, b64)
        print(json.dumps({"order": tag, "enc_ms": round(r["encode_kernel_ms"], 4),
                          "dec_ms": round(r["decode_kernel_ms"], 4)}), flush=True)

    leg("batch first")
    r = bench.bench_single(args, 1, 0, b64)
    print(json.dumps({"order": "single", "enc_ms": round(r["enc_ms"], 4),
                      "dec_ms": round(r["dec_ms"], 4)}), flush=True)
    leg("after single")
    bench.copy_ceilings(r["N"], r["E"])
    leg("after single + ceilings")
    del r
    torch.cuda.empty_cache()
    leg("after empty_cache")


if __name__ == "__main__":
    main()
