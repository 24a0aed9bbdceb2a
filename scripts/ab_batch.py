#!/usr/bin/env python3
"""Interleaved A/B of library builds on the batch legs, timed the way
bench.py's batch_cfg3 / batch_cfg4 time them: K strided encodes back to back
between two HIP events, then K strided decodes between two more (no event
between calls).  One child process per (round, library) so that the
libraries alternate on one box; each child reports the median of --reps
such timings per leg, and the summary the median over rounds.

    python scripts/ab_batch.py [--rounds 3] [--steps 20] [--reps 5] LIB [LIB ...]

Legs: cfg2 (one 1 GiB buffer, the single-buffer kernels on the same bytes),
cfg3 (65,536 x 4 KiB) and cfg4 (1,048,576 x 1 KiB) clean rows, and cfg4 in
CRLF-76 lines (the MIME rows).  Every leg is bit-checked.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGS = ("cfg2_enc", "cfg2_dec", "cfg3_enc", "cfg3_dec", "cfg4_enc", "cfg4_dec", "cfg4_crlf_dec")


def child(lib, steps, reps):
    sys.path.insert(0, ROOT)
    import torch
    from async_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    from async_amd import b64
    st = torch.cuda.current_stream()
    res, bad = {}, []

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(steps):
                fn()
            b.record(st)
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / steps)
        return statistics.median(ts)

    # config 2 beside them: the single-buffer kernels on the same bytes
    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    e = torch.empty(b64.encoded_len(x.numel()), dtype=torch.uint8, device="cuda")
    d = torch.empty(b64.decoded_cap(e.numel()), dtype=torch.uint8, device="cuda")
    ws = torch.zeros(b64.workspace_size(e.numel()), dtype=torch.uint8, device="cuda")
    rr = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device="cuda")
    res["cfg2_enc"] = timed(lambda: b64.encode(x, out=e, stream=st))
    res["cfg2_dec"] = timed(lambda: b64.decode(e, out=d, workspace=ws, result=rr, stream=st))
    torch.cuda.synchronize()
    if not torch.equal(d[:x.numel()], x):
        bad.append("cfg2")
    del x, e, d, ws
    for name, nb, L in (("cfg3", 1 << 16, 4096), ("cfg4", 1 << 20, 1024)):
        Es = b64.encoded_len(L)
        cap = 12 * ((Es + 15) // 16)
        x = torch.empty(nb * L, dtype=torch.uint8, device="cuda")
        b64.fill_splitmix64(x, 0x5EED)
        e = torch.empty(nb * Es, dtype=torch.uint8, device="cuda")
        d = torch.empty(nb * cap, dtype=torch.uint8, device="cuda")
        ol = torch.zeros(nb, dtype=torch.int64, device="cuda")
        res[name + "_enc"] = timed(lambda: b64.encode_strided(x, L, L, nb, e, Es, stream=st))
        res[name + "_dec"] = timed(lambda: b64.decode_strided(e, Es, Es, nb, d, cap, ol, stream=st))
        torch.cuda.synchronize()
        if not (bool((ol == L).all()) and torch.equal(d.view(nb, cap)[:, :L], x.view(nb, L))):
            bad.append(name)
        if name == "cfg4":
            lines = (Es + 75) // 76
            rows = e.view(nb, Es)
            if lines * 76 > Es:
                rows = torch.cat([rows, torch.full((nb, lines * 76 - Es), 10, dtype=torch.uint8,
                                                   device="cuda")], dim=1)
            crlf = torch.tensor([13, 10], dtype=torch.uint8, device="cuda").expand(nb, lines, 2)
            D = lines * 78
            mb = torch.cat([rows.reshape(nb, lines, 76), crlf], dim=2).reshape(-1).contiguous()
            del rows, crlf
            cap2 = 12 * ((D + 15) // 16)
            d2 = torch.empty(nb * cap2, dtype=torch.uint8, device="cuda")
            res["cfg4_crlf_dec"] = timed(lambda: b64.decode_strided(mb, D, D, nb, d2, cap2, ol,
                                                                     stream=st))
            torch.cuda.synchronize()
            if not (bool((ol == L).all()) and torch.equal(d2.view(nb, cap2)[:, :L], x.view(nb, L))):
                bad.append("cfg4_crlf")
            del mb, d2
        del x, e, d, ol
    print(json.dumps({"lib": lib, "ok": not bad, "bad": bad, **res}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--price", action="store_true",
                    help="pricing builds that skip work: report wrong output, do not stop")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    if a.child:
        return child(a.libs[0], a.steps, a.reps)
    agg = {lib: {} for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            p = subprocess.run([sys.executable, __file__, "--child", "--steps", str(a.steps),
                                "--reps", str(a.reps), lib],
                               capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode or not line:
                print(p.stdout, p.stderr, file=sys.stderr)
                sys.exit(p.returncode or 1)
            d = json.loads(line[-1])
            print(json.dumps(d), flush=True)
            if not d["ok"] and not a.price:
                sys.exit(1)
            for k in LEGS:
                agg[lib].setdefault(k, []).append(d[k])
    for lib in a.libs:
        print(json.dumps({"summary": lib, **{k: round(statistics.median(v), 2)
                                             for k, v in agg[lib].items()}}), flush=True)


if __name__ == "__main__":
    main()
