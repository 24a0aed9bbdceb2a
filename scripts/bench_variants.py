#!/usr/bin/env python3
"""A/B the kernel variants behind the b64x__tune hook, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24), plus the copy-kernel
calibration of the reachable HBM rate for each traffic mix.

Every variant's output is compared with variant 0's (bit-exact) before its
time counts.  Prints one JSON object.
"""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import _lib, b64  # noqa: E402

lib = _lib.load()
lib.b64x__tune.argtypes = [ctypes.c_int, ctypes.c_int]
lib.b64x__tune.restype = ctypes.c_int
lib.b64x__probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_int, ctypes.c_void_p]
lib.b64x__probe_copy.restype = ctypes.c_int

N = int(os.environ.get("N", 1 << 30))
ROUNDS = int(os.environ.get("ROUNDS", 5))
K = int(os.environ.get("K", 10))
ENC_V = [int(v) for v in os.environ.get("ENC_V", "0,1,2,3,4,5,6").split(",")]
DEC_V = [int(v) for v in os.environ.get("DEC_V", "0,1,2,3,4,5").split(",")]
# decode range length in chunks (b64x__tune slot 2); 0 = library default
RANGES = [int(v) for v in os.environ.get("RANGES", "0").split(",")]

s = torch.cuda.current_stream()
x = torch.empty(N, dtype=torch.uint8, device="cuda")
b64.fill_splitmix64(x, 0x5EED)
E = b64.encoded_len(N)
enc = torch.empty(E, dtype=torch.uint8, device="cuda")
enc_ref = torch.empty(E, dtype=torch.uint8, device="cuda")
dec = torch.empty(b64.decoded_cap(E), dtype=torch.uint8, device="cuda")
ws = torch.zeros(b64.workspace_size(E), dtype=torch.uint8, device="cuda")
res = torch.zeros(24, dtype=torch.uint8, device="cuda")


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record(s)
    for _ in range(K):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / K


out = {"N": N, "E": E, "rounds": ROUNDS, "K": K, "encode": {}, "decode": {}, "copy": {}}
lib.b64x__tune(0, ENC_V[0])
b64.encode(x, out=enc_ref)
torch.cuda.synchronize()
times = {("e", v): [] for v in ENC_V}
times.update({("d", v, rg): [] for v in DEC_V for rg in RANGES})
for r in range(ROUNDS):
    for v in ENC_V:
        lib.b64x__tune(0, v)
        enc.zero_()
        t = timed(lambda: b64.encode(x, out=enc))
        if r == 0 and not torch.equal(enc, enc_ref):
            raise SystemExit(f"encode variant {v} differs")
        times[("e", v)].append(t)
    lib.b64x__tune(0, ENC_V[0])
    for v in DEC_V:
        for rg in RANGES:
            lib.b64x__tune(1, v)
            lib.b64x__tune(2, rg)
            dec.zero_()
            t = timed(lambda: b64.decode(enc_ref, out=dec, workspace=ws, result=res))
            if r == 0 and not torch.equal(dec[:N], x):
                raise SystemExit(f"decode variant {v} range {rg} differs")
            times[("d", v, rg)].append(t)
    lib.b64x__tune(2, 0)
per = N + E
for key_t, ts in times.items():
    kind, v = key_t[0], key_t[1]
    key = "encode" if kind == "e" else "decode"
    med = statistics.median(ts)
    name = str(v) if kind == "e" else f"{v}/r{key_t[2]}"
    out[key][name] = {"median_ms": med, "min_ms": min(ts), "GBps": per / med / 1e6,
                        "hbm_frac": per / med / 1e6 / 8000}

# copy calibration: the encode shape (12 B in / 16 B out per lane), the
# decode shape (16 in / 12 out) and a plain 16/16 copy, over the same slot
# count as the 1 GiB encode (N/12 slots).
big_in = torch.empty(max(N, E) + 65536, dtype=torch.uint8, device="cuda")
big_out = torch.empty(max(N, E) + 65536, dtype=torch.uint8, device="cuda")
slots = N // 12
for name, kind, rd, wr in (("copy16_16", 0, 16, 16), ("enc_shape_12_16", 1, 12, 16),
                           ("dec_shape_16_12", 2, 16, 12)):
    for nt in (0, 8):
        ts = [timed(lambda: lib.b64x__probe_copy(big_in.data_ptr(), big_out.data_ptr(),
                                                   slots, kind + nt, s.cuda_stream))
              for _ in range(ROUNDS)]
        med = statistics.median(ts)
        out["copy"][f"{name}_nt{nt // 8}"] = {"median_ms": med,
                                             "GBps": slots * (rd + wr) / med / 1e6}
print(json.dumps(out, indent=1))
