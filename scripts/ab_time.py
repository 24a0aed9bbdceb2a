#!/usr/bin/env python3
"""Interleaved A/B timing of library builds (scripts/ab_variants.sh):
config 2's encode and clean decode, and the 1 GiB CRLF-76 decode, K steps
each with HIP events, in a child process per (round, variant) so that the
variants alternate on the same box.

    python scripts/ab_time.py [--rounds 3] [--steps 20] LIB [LIB ...]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, steps, only=()):
    sys.path.insert(0, ROOT)
    import torch
    from async_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    from async_amd import b64
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from bench_dirty import crlf76, sprinkle
    n = 1 << 30
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    enc = b64.encode(x)
    dirty = crlf76(enc)
    junk = sprinkle(enc, 0.05)
    junk1 = sprinkle(enc, 0.001)
    out = torch.empty(b64.decoded_cap(junk.numel()), dtype=torch.uint8, device="cuda")
    rr = torch.zeros(_lib.RES_BYTES, dtype=torch.uint8, device="cuda")
    ws = torch.zeros(b64.workspace_size(junk.numel()), dtype=torch.uint8, device="cuda")
    res = {}

    def timeit(name, fn):
        if only and name not in only:
            res[name] = (0.0, 0.0, 0.0)
            return
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(steps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[name] = (statistics.median(ts), statistics.mean(ts), min(ts))

    # the copy ceiling beside the kernels, same process and box: one 16-byte
    # (or 12-byte) non-temporal load and store per lane with the leg's own
    # read/write mix (tests/csrc/libb64x_hooks.so, bench.py copy_ceilings)
    import ctypes
    hooks = ctypes.CDLL(os.path.join(ROOT, "tests", "csrc", "libb64x_hooks.so"))
    hooks.b64x__test_copy_mix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    st = torch.cuda.current_stream().cuda_stream
    ue, ud = n // 12 // 256 * 256, enc.numel() // 16 // 256 * 256
    timeit("copy_enc", lambda: hooks.b64x__test_copy_mix(x.data_ptr(), enc.data_ptr(), ue, st,
                                                         0, 0))
    timeit("copy_dec", lambda: hooks.b64x__test_copy_mix(enc.data_ptr(), out.data_ptr(), ud, st,
                                                         1, 0))
    timeit("encode", lambda: b64.encode(x, out=enc))
    ran = lambda k: not only or k in only  # noqa: E731 -- checks only for legs that ran
    bad = []

    def chk(name, good):
        if ran(name) and not good:
            bad.append(name)
        return True
    timeit("decode", lambda: b64.decode(enc, out=out, workspace=ws, result=rr))
    ok = chk("decode", torch.equal(out[:n], x))
    timeit("crlf", lambda: b64.decode(dirty, out=out, workspace=ws, result=rr))
    ok = chk("crlf", torch.equal(out[:n], x))
    timeit("junk", lambda: b64.decode(junk, out=out, workspace=ws, result=rr))
    ok = chk("junk", torch.equal(out[:n], x))
    timeit("junk1", lambda: b64.decode(junk1, out=out, workspace=ws, result=rr))
    ok = chk("junk1", torch.equal(out[:n], x))
    timeit("junk_ej", lambda: b64.decode(junk, out=out, workspace=ws, result=rr,
                                         expect_junk=True))
    ok = chk("junk_ej", torch.equal(out[:n], x))
    timeit("crlf_ej", lambda: b64.decode(dirty, out=out, workspace=ws, result=rr,
                                         expect_junk=True))
    ok = chk("crlf_ej", torch.equal(out[:n], x))
    timeit("clean_ej", lambda: b64.decode(enc, out=out, workspace=ws, result=rr,
                                          expect_junk=True))
    ok = chk("clean_ej", torch.equal(out[:n], x))
    # config 4: 1 M x 1 KiB rows, strided decode (clean)
    del dirty, junk, junk1, enc, out, x
    if only and not ({"rows_enc", "rows_dec", "rows_crlf", "ragged_dec"} & set(only)):
        for k in ("rows_enc", "rows_dec", "rows_crlf", "ragged_dec"):
            res[k] = (0.0, 0.0, 0.0)
        print(json.dumps({"lib": lib, "ok": not bad, "bad": bad, **res}), flush=True)
        return
    nb, L = 1 << 20, 1024
    Es = b64.encoded_len(L)
    cap = 12 * ((Es + 15) // 16)
    xb = torch.empty(nb * L, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(xb, 0x5EED)
    eb = torch.empty(nb * Es, dtype=torch.uint8, device="cuda")
    db = torch.empty(nb * cap, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(nb, dtype=torch.int64, device="cuda")
    b64.encode_strided(xb, L, L, nb, eb, Es)  # the rows the decode legs read
    timeit("rows_enc", lambda: b64.encode_strided(xb, L, L, nb, eb, Es))
    timeit("rows_dec", lambda: b64.decode_strided(eb, Es, Es, nb, db, cap, ol))
    ok = chk("rows_dec", bool((ol == L).all()) and torch.equal(db.view(nb, cap)[:, :L], xb.view(nb, L)))
    # the same rows MIME-formatted (76-character lines, CRLF)
    lines = (Es + 75) // 76
    rows = eb.view(nb, Es)
    if lines * 76 > Es:
        rows = torch.cat([rows, torch.full((nb, lines * 76 - Es), 10, dtype=torch.uint8,
                                           device="cuda")], dim=1)
    crlf = torch.tensor([13, 10], dtype=torch.uint8, device="cuda").expand(nb, lines, 2)
    D = lines * 78
    mb = torch.cat([rows.reshape(nb, lines, 76), crlf], dim=2).reshape(-1).contiguous()
    del rows, crlf
    cap2 = 12 * ((D + 15) // 16)
    db2 = torch.empty(nb * cap2, dtype=torch.uint8, device="cuda")
    timeit("rows_crlf", lambda: b64.decode_strided(mb, D, D, nb, db2, cap2, ol))
    ok = chk("rows_crlf", bool((ol == L).all()) and
             torch.equal(db2.view(nb, cap2)[:, :L], xb.view(nb, L)))
    # a ragged batch of 65,536 messages of 100-4,000 bytes (the hub's shape)
    del mb, db2, db, eb, xb
    g = torch.Generator().manual_seed(5)
    lens = torch.randint(100, 4000, (65536,), generator=g, dtype=torch.int64)
    ioff = torch.zeros(65537, dtype=torch.int64)
    ioff[1:] = torch.cumsum(lens, 0)
    elen = (lens + 2) // 3 * 4
    eoff = torch.zeros(65537, dtype=torch.int64)
    eoff[1:] = torch.cumsum(elen, 0)
    xr = torch.empty(int(ioff[-1]), dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(xr, 7)
    er = torch.empty(int(eoff[-1]), dtype=torch.uint8, device="cuda")
    ioff_d, eoff_d = ioff.cuda(), eoff.cuda()
    b64.encode_batch(xr, ioff_d, er, eoff_d)
    cap = (elen + 3) // 4 * 3
    doff = torch.zeros(65537, dtype=torch.int64)
    doff[1:] = torch.cumsum(cap, 0)
    dr = torch.empty(int(doff[-1]) + 16, dtype=torch.uint8, device="cuda")
    doff_d = doff.cuda()
    olr = torch.zeros(65536, dtype=torch.int64, device="cuda")
    timeit("ragged_dec", lambda: b64.decode_batch(er, eoff_d, dr, doff_d[:-1], olr))
    ok = chk("ragged_dec", bool((olr.cpu() == lens).all()))
    for i in (0, 1, 777, 65535):
        a0, d0 = int(ioff[i]), int(doff[i])
        ok = chk("ragged_dec", torch.equal(dr[d0:d0 + int(lens[i])], xr[a0:a0 + int(lens[i])]))
    print(json.dumps({"lib": lib, "ok": not bad, "bad": bad, **res}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated legs (default: all)")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    if a.child:
        return child(a.libs[0], a.steps, tuple(x for x in a.only.split(",") if x))
    agg = {lib: {} for lib in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            p = subprocess.run([sys.executable, __file__, "--child", "--steps", str(a.steps), "--only", a.only, lib],
                               capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode or not line:
                print(p.stdout, p.stderr, file=sys.stderr)
                sys.exit(p.returncode or 1)
            d = json.loads(line[-1])
            print(json.dumps(d), flush=True)
            for k in ("copy_enc", "copy_dec", "encode", "decode", "crlf", "junk", "junk1", "junk_ej", "crlf_ej", "clean_ej", "rows_enc", "rows_dec", "rows_crlf", "ragged_dec"):
                agg[lib].setdefault(k, []).append(d[k][0])
    for lib in a.libs:
        print(json.dumps({"summary": lib, **{k: round(statistics.median(v), 1)
                                             for k, v in agg[lib].items()}}), flush=True)


if __name__ == "__main__":
    main()
