#!/usr/bin/env python3
"""PMC workload: 1 GiB of config-2 characters with junk at density 0.05
(a '!' before a character with that probability), decoded 3 times on the
automatic path and 3 times with B64X_DEC_EXPECT_JUNK, bit-checked.
    python scripts/junk_decode_once.py [LIB]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    lib = sys.argv[1]
    _lib.LIB_PATH = lib if os.path.isabs(lib) else os.path.join(ROOT, lib)
from async_amd import b64  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "scripts"))
from bench_dirty import sprinkle  # noqa: E402

n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
b64.fill_splitmix64(x, 0x5EED)
junk = sprinkle(b64.encode(x), 0.05)
out = torch.empty(b64.decoded_cap(junk.numel()), dtype=torch.uint8, device="cuda")
ws = torch.zeros(b64.workspace_size(junk.numel()), dtype=torch.uint8, device="cuda")
for ej in (False, True):
    for _ in range(3):
        d = b64.decode(junk, out=out, workspace=ws, expect_junk=ej)
    # (PRICING=1: a timing build whose output is wrong on purpose)
    assert os.environ.get("PRICING") or (d.info().out_len == n and torch.equal(out[:n], x))
print("ok")
