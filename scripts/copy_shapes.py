#!/usr/bin/env python3
"""Copy kernels in the encode's shapes, one process, alternating (test-hooks
build, tests/csrc/libb64x_hooks.so): 12-byte loads at a 12-byte stride ->
16 stored (k_encode_flat's mix) and 16-byte loads at a 12-byte stride -> 16
stored (k_encode_tight2's), 1, 2 or 4 per lane, over config 2's 1 GiB; with
k_encode_flat and k_encode_tight2 (config 4) on the same bytes beside them.
Median of --reps timings of --steps calls between two events, --rounds
rounds.  Prints one JSON line per round and a summary.

    python scripts/copy_shapes.py [--rounds 3] [--steps 20] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from async_amd import b64
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "csrc", "libb64x_hooks.so"))
    lib.b64x__test_copy_mix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.b64x__test_copy_mix.restype = ctypes.c_int
    st = torch.cuda.current_stream()
    N = 1 << 30
    L, nb = 1024, 1 << 20
    Es = b64.encoded_len(L)
    src = torch.empty(N + 4096, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(src, 0x5EED)
    dst = torch.empty(nb * Es + 4096, dtype=torch.uint8, device="cuda")
    x = src[:N]

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                fn()
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / a.steps)
        return round(statistics.median(ts), 1)

    legs = {}
    for mix, name in ((0, "12@12"), (2, "16@12")):
        for shape, U in enumerate((1, 2, 4)):
            units = N // 12 // (256 * U) * (256 * U)
            legs[f"{name} U{U}"] = (lambda mix=mix, shape=shape, units=units:
                                    lib.b64x__test_copy_mix(src.data_ptr(), dst.data_ptr(), units,
                                                            st.cuda_stream, mix, shape))
    legs["k_encode_flat"] = lambda: b64.encode(x, out=dst, stream=st)
    legs["k_encode_tight2"] = lambda: b64.encode_strided(x, L, L, nb, dst, Es, stream=st)
    agg = {k: [] for k in legs}
    scratch = torch.empty(2, 256 << 20, dtype=torch.uint8, device="cuda")
    for r in range(a.rounds):
        for _ in range(300):  # clock pre-heat
            scratch[0].copy_(scratch[1])
        row = {"round": r}
        for k, fn in legs.items():
            row[k] = timed(fn)
            agg[k].append(row[k])
        print(json.dumps(row), flush=True)
    print(json.dumps({"summary": {k: statistics.median(v) for k, v in agg.items()}}), flush=True)


if __name__ == "__main__":
    main()
