#!/usr/bin/env python3
"""Stress the junk suffix kernel of a library build: 1 GiB of config-2
characters with junk at density 0.05 and 0.001, decoded --iters times each
in one pass (B64X_DEC_EXPECT_JUNK) and on the automatic path, every output
compared with the payload.  On a mismatch prints the differing runs of
output bytes (offset, length) and where they fall in 1,536-byte range
outputs, then goes on.

    python scripts/held_stress.py LIB [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def runs(mask, limit=12, window=1 << 16):
    first = int(torch.argmax(mask.to(torch.uint8)))
    idx = torch.nonzero(mask[first:first + window]).flatten().cpu() + first
    out = []
    if idx.numel() == 0:
        return out
    start = prev = int(idx[0])
    for v in idx[1:].tolist():
        if v != prev + 1:
            out.append((start, prev - start + 1))
            if len(out) >= limit:
                return out
            start = v
        prev = v
    out.append((start, prev - start + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from async_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    from async_amd import b64
    from bench_dirty import sprinkle
    n = 1 << 30
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    enc = b64.encode(x)
    import ctypes
    dbg = None
    try:
        dbg = ctypes.CDLL(os.path.abspath(a.lib)).b64x__sfx_debug
        dbg.argtypes = [ctypes.POINTER(ctypes.c_uint * 4), ctypes.c_int]
    except AttributeError:
        pass

    def dbg_read():
        if dbg is None:
            return None
        v = (ctypes.c_uint * 4)()
        dbg(ctypes.byref(v), 1)
        return list(v)

    bad = 0
    for d in (0.05, 0.001):
        junk = sprinkle(enc, d)
        out = torch.empty(b64.decoded_cap(junk.numel()), dtype=torch.uint8, device="cuda")
        ws = torch.zeros(b64.workspace_size(junk.numel()), dtype=torch.uint8, device="cuda")
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device="cuda")
        for it in range(a.iters):
            for ej in (True, False):
                out.fill_(0xAA)
                b64.decode(junk, out=out, workspace=ws, result=res, expect_junk=ej)
                torch.cuda.synchronize()
                info = b64.Decoded(out, res).info()
                ok = info.out_len == n and torch.equal(out[:n], x)
                dv = dbg_read()
                if dv is not None and (dv[0] or dv[1] or not ok):
                    print(json.dumps({"density": d, "iter": it, "expect_junk": ej, "ok": ok,
                                      "lds_copy_differs_readahead": dv[0],
                                      "lds_copy_differs_direct": dv[1], "max_j": dv[2],
                                      "ranges": dv[3]}), flush=True)
                if not ok:
                    bad += 1
                    m = out[:n] != x
                    rr = runs(m)
                    print(json.dumps({"density": d, "iter": it, "expect_junk": ej,
                                      "out_len": info.out_len, "bytes_bad": int(m.sum()),
                                      "runs": rr, "runs_mod1536": [(o % 1536, l) for o, l in rr]}),
                          flush=True)
        print(json.dumps({"density": d, "iters": a.iters, "bad_so_far": bad}), flush=True)
        del junk, out, ws
    print(json.dumps({"done": True, "bad": bad}), flush=True)


if __name__ == "__main__":
    main()
