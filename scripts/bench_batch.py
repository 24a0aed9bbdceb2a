#!/usr/bin/env python3
"""Time the uniform-stride batch kernels (BASELINE configs 3 and 4) under
the b64x__tune knobs, interleaved in one process; outputs checked."""
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
K = int(os.environ.get("K", 10))
KNOBS = [tuple(int(x) for x in kv.split(":")) for kv in
         os.environ.get("KNOBS", "3:0,3:1").split(",")]
s = torch.cuda.current_stream()
res = {}
CAPS = [int(c) for c in os.environ.get("CAPS", "0").split(",")]
CFGS = os.environ.get("CFGS", "cfg4,cfg3").split(",")
for name, nbuf, L, capr in [(n, nb, L, c) for n, nb, L in (("cfg4", 1 << 20, 1024),
                                                              ("cfg3", 1 << 16, 4096))
                            if n in CFGS for c in CAPS]:
    Es = b64.encoded_len(L)
    # decode row stride: capacity rounded up to `capr` bytes (0: 12 per slot)
    cap = (b64.decoded_cap(Es) + capr - 1) // capr * capr if capr else 12 * ((Es + 15) // 16)
    x = torch.empty(nbuf * L, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    enc = torch.empty(nbuf * Es, dtype=torch.uint8, device="cuda")
    dec = torch.empty(nbuf * cap, dtype=torch.uint8, device="cuda")
    outlen = torch.zeros(nbuf, dtype=torch.int64, device="cuda")
    b64.encode_strided(x, L, L, nbuf, enc, Es)
    for idx, val in KNOBS:
        old = lib.b64x__tune(idx, val)
        ts = {"enc": [], "dec": []}
        for _ in range(3):
            for kind in ("enc", "dec"):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fn = (lambda: b64.encode_strided(x, L, L, nbuf, enc, Es)) if kind == "enc" else \
                     (lambda: b64.decode_strided(enc, Es, Es, nbuf, dec, cap, outlen))
                fn()
                a.record(s)
                for _ in range(K):
                    fn()
                b.record(s)
                b.synchronize()
                ts[kind].append(a.elapsed_time(b) / K)
        ok = bool((outlen == L).all()) and torch.equal(dec.view(nbuf, cap)[:, :L], x.view(nbuf, L))
        lib.b64x__tune(idx, old)
        per = nbuf * (L + Es)
        res[f"{name} cap{capr} knob{idx}={val}"] = {
            "ok": ok, "enc_ms": statistics.median(ts["enc"]), "dec_ms": statistics.median(ts["dec"]),
            "enc_GBps": per / statistics.median(ts["enc"]) / 1e6,
            "dec_GBps": per / statistics.median(ts["dec"]) / 1e6}
print(json.dumps(res, indent=1))
