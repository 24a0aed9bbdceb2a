#!/usr/bin/env python3
"""Diagnose bench.py's host_fd egress leg: config 2's bytes (or SIZE) ->
queuestream -> base64_encode -> chunk_encode(1 MiB) -> fdsink -> pipe,
de-chunked and compared with b64.encode of the same bytes; prints the
chunk sizes seen and the first differing character.
    python scripts/egress_fd_check.py [SIZE]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import b64  # noqa: E402
from tests import util  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
x = torch.empty(N, dtype=torch.uint8, device="cuda")
b64.fill_splitmix64(x, 0x5EED)
want = b64.encode(x).cpu().numpy().tobytes()
xh = x.cpu().numpy()
chunk = 1 << 20
framed = np.zeros(util.framed_cap(N, chunk), np.uint8)
for rep in range(2):
    got, err, dt = util.fd_encode(xh, max_chunk=chunk, out=framed)
    body = got.tobytes() if got is not None else b""
    pos, sizes, parts = 0, [], []
    while pos < len(body):
        eol = body.index(b"\r\n", pos)
        size = int(body[pos:eol], 16)
        pos = eol + 2
        if size == 0:
            break
        sizes.append(size)
        parts.append(body[pos:pos + size])
        pos += size + 2
    dec = b"".join(parts)
    first = next((i for i in range(0, min(len(dec), len(want)), 1 << 16)
                  if dec[i:i + (1 << 16)] != want[i:i + (1 << 16)]), None)
    short = [(i, s) for i, s in enumerate(sizes[:-1]) if s != chunk]
    print(json.dumps({"rep": rep, "err": err, "seconds": dt, "chunks": len(sizes),
                      "short_chunks": short[:10], "n_short": len(short), "len": len(dec),
                      "want_len": len(want), "first_bad_64k_block": first}), flush=True)
