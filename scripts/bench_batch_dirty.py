#!/usr/bin/env python3
"""Batch decode of MIME-formatted buffers: config 4's shape (1 M x 1 KiB)
and config 3's (64 Ki x 4 KiB), every buffer's characters broken into
76-character lines with CRLF, so every buffer needs the exact path.  Times
decode_strided against the clean rows; output checked.  One JSON line."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import b64  # noqa: E402

K = int(os.environ.get("K", 10))


def crlf_rows(enc: torch.Tensor, nbuf: int, E: int) -> tuple[torch.Tensor, int]:
    """Each E-character row -> lines of 76 joined by CRLF (and a final CRLF
    after a short last line), as a uniform-stride batch of D bytes."""
    lines = (E + 75) // 76
    pad = lines * 76 - E
    rows = enc.view(nbuf, E)
    if pad:
        rows = torch.cat([rows, torch.full((nbuf, pad), ord("\n"), dtype=torch.uint8,
                                           device=enc.device)], dim=1)
    rows = rows.view(nbuf, lines, 76)
    crlf = torch.tensor([13, 10], dtype=torch.uint8, device=enc.device).expand(nbuf, lines, 2)
    out = torch.cat([rows, crlf], dim=2).reshape(nbuf, lines * 78)
    return out.contiguous().view(-1), lines * 78


def timed(fn) -> float:
    s = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(K):
            fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b) / K)
    return statistics.median(ts)


res = {}
for name, nbuf, L in (("cfg4", 1 << 20, 1024), ("cfg3", 1 << 16, 4096)):
    E = b64.encoded_len(L)
    x = torch.empty(nbuf * L, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    enc = torch.empty(nbuf * E, dtype=torch.uint8, device="cuda")
    b64.encode_strided(x, L, L, nbuf, enc, E)
    dirty, D = crlf_rows(enc, nbuf, E)
    cap = (b64.decoded_cap(D) + 15) // 16 * 16
    dec = torch.empty(nbuf * cap, dtype=torch.uint8, device="cuda")
    outlen = torch.zeros(nbuf, dtype=torch.int64, device="cuda")
    t_clean = timed(lambda: b64.decode_strided(enc, E, E, nbuf, dec, cap, outlen))
    t_dirty = timed(lambda: b64.decode_strided(dirty, D, D, nbuf, dec, cap, outlen))
    ok = bool((outlen == L).all()) and torch.equal(dec.view(nbuf, cap)[:, :L], x.view(nbuf, L))
    res[name] = {"ok": ok, "row_chars_clean": E, "row_chars_crlf": D,
                 "clean_ms": t_clean, "crlf_ms": t_dirty,
                 "crlf_alg_GBps": nbuf * (D + L) / t_dirty / 1e6}
print(json.dumps({"measure": "batch_decode_crlf76", **res}))
