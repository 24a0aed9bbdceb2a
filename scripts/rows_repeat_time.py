"""Per-call times of the MIME rows decode (config 4 rows, CRLF-76), one
library per process: HIP events around each call (synchronized after each),
and K back-to-back calls timed as one span.  Used to A/B the row model's
reuse across batches.   rows_repeat_time.py LIB [steps]"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lib, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
    sys.path.insert(0, ROOT)
    import torch
    from async_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    from async_amd import b64
    nb, L = 1 << 20, 1024
    Es = b64.encoded_len(L)
    xb = torch.empty(nb * L, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(xb, 0x5EED)
    eb = torch.empty(nb * Es, dtype=torch.uint8, device="cuda")
    b64.encode_strided(xb, L, L, nb, eb, Es)
    lines = (Es + 75) // 76
    rows = eb.view(nb, Es)
    if lines * 76 > Es:
        rows = torch.cat([rows, torch.full((nb, lines * 76 - Es), 10, dtype=torch.uint8,
                                           device="cuda")], dim=1)
    crlf = torch.tensor([13, 10], dtype=torch.uint8, device="cuda").expand(nb, lines, 2)
    D = lines * 78
    mb = torch.cat([rows.reshape(nb, lines, 76), crlf], dim=2).reshape(-1).contiguous()
    del rows, crlf, eb
    cap = 12 * ((D + 15) // 16)
    db = torch.empty(nb * cap, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(nb, dtype=torch.int64, device="cuda")
    call = lambda: b64.decode_strided(mb, D, D, nb, db, cap, ol)  # noqa: E731
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    ok = bool((ol == L).all()) and torch.equal(db.view(nb, cap)[:, :L], xb.view(nb, L))
    per = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        call()
        b.record()
        b.synchronize()
        per.append(a.elapsed_time(b) * 1e3)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        call()
    b.record()
    b.synchronize()
    span = a.elapsed_time(b) * 1e3 / steps
    print(json.dumps({"lib": lib, "ok": ok, "median_us": statistics.median(per),
                      "min_us": min(per), "max_us": max(per), "back_to_back_us": span,
                      "per_call_us": [round(t, 1) for t in per]}), flush=True)


if __name__ == "__main__":
    main()
