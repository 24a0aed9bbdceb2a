#!/usr/bin/env python3
"""Does the batch encode trail the flat encode on the same bytes, or on the
same buffers?  Allocates --sets pairs of (1 GiB input, config-4 output) and,
on each pair, times K back-to-back calls between two HIP events of
  flat:  b64x_encode_dev of the whole 1 GiB into the output buffer
         (k_encode_flat, 1,431,655,768 characters), and
  tight: b64x_encode_strided of the 1 M x 1 KiB batch into the same buffer
         (k_encode_tight2, 1,434,451,968 characters),
alternating, median of --reps.  Prints one JSON line per set with the
buffers' addresses (mod 2 MiB and 1 GiB) so placement effects show.

    python scripts/placement_probe.py [--sets 4] [--steps 20] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from async_amd import b64
    st = torch.cuda.current_stream()
    L, nbuf = 1024, 1 << 20
    Es = b64.encoded_len(L)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(args.steps):
                fn()
            b.record(st)
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / args.steps)
        return statistics.median(ts)

    keep = []
    for s in range(args.sets):
        x = torch.empty(nbuf * L, dtype=torch.uint8, device="cuda")
        b64.fill_splitmix64(x, 0x5EED + s)
        enc = torch.empty(nbuf * Es, dtype=torch.uint8, device="cuda")
        enc.fill_(0)
        keep.append((x, enc))
        row = {"set": s, "x_mod2M": x.data_ptr() % (2 << 20), "enc_mod2M": enc.data_ptr() % (2 << 20),
               "x_GiB": x.data_ptr() >> 30, "enc_GiB": enc.data_ptr() >> 30}
        for rnd in range(2):
            row[f"flat{rnd}"] = round(timed(lambda: b64.encode(x, out=enc, stream=st)), 2)
            row[f"tight{rnd}"] = round(timed(
                lambda: b64.encode_strided(x, L, L, nbuf, enc, Es, stream=st)), 2)
        torch.cuda.synchronize()
        # the batch output is the flat output's bytes regrouped: spot-check a buffer
        ref = b64.encode(x[L * 5:L * 6].clone())
        assert torch.equal(enc[Es * 5:Es * 6], ref), "tight encode mismatch"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
