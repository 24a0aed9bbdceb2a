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
        # each 2,048-character range's alphabet count and its output start
        # (ceil(B/4)*3 for B alphabet characters before it), for locating a
        # wrong run
        tn = junk.cpu().numpy()
        import numpy as np
        valid = np.zeros(256, dtype=np.uint8)
        for c in b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/":
            valid[c] = 1
        nr = (tn.size + 2047) // 2048
        v = np.zeros(nr * 2048, dtype=np.uint8)
        v[:tn.size] = valid[tn]
        cnt = v.reshape(nr, 2048).sum(axis=1, dtype=np.int64)
        B = np.concatenate([[0], np.cumsum(cnt)])
        starts = (B[:-1] + 3) // 4 * 3
        del tn, v
        out = torch.empty(b64.decoded_cap(junk.numel()), dtype=torch.uint8, device="cuda")
        ws = torch.zeros(b64.workspace_size(junk.numel()), dtype=torch.uint8, device="cuda")
        res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device="cuda")
        for it in range(a.iters):
            if it % 10 == 0:
                print(json.dumps({"density": d, "iter": it, "bad_so_far": bad}), flush=True)
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
                    first = rr[0][0] if rr else -1
                    r = int(np.searchsorted(starts, first, side="right") - 1)
                    where = {"range": r, "tile12": r // 12, "tile16": r // 16,
                             "offset_in_range_output": int(first - starts[r]),
                             "range_count": int(cnt[r]), "range_B_mod4": int(B[r] % 4)}
                    print(json.dumps({"density": d, "iter": it, "expect_junk": ej, "where": where,
                                      "out_len": info.out_len, "bytes_bad": int(m.sum()),
                                      "runs": rr, "runs_mod1536": [(o % 1536, l) for o, l in rr]}),
                          flush=True)
        print(json.dumps({"density": d, "iters": a.iters, "bad_so_far": bad}), flush=True)
        del junk, out, ws
    print(json.dumps({"done": True, "bad": bad}), flush=True)


if __name__ == "__main__":
    main()
