#!/usr/bin/env python3
"""Seeded fuzz of the lent-message egress path on the MI355X: random queues
of messages (0 B - 1.5 MiB, log-uniform, some empty), random stage
capacities, lend thresholds, chunk sizes and read sizes, pushes and late
termination; every framed stream against the oracle stack (late
termination: the de-chunked payload), and no pinned reference left.
    python -u scripts/fuzz_lent.py SEEDS"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime)

from oracle import pyoracle as orc  # noqa: E402
from tests import util  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L = util.harness()
t0 = time.time()
for seed in range(n):
    rng = np.random.default_rng(0xF0221 + seed)
    k = int(rng.integers(1, 40))
    sizes = [0 if rng.random() < 0.05 else int(np.exp(rng.uniform(0, np.log(1.5 * 2**20))))
             for _ in range(k)]
    pieces = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
    cap = str(int(rng.choice([64, 1000, 4096, 65536, 1 << 20])))
    lend_min = str(int(rng.choice([1, 3, 4096, 65536])))
    max_chunk = int(rng.choice([30, 4096, 65536, 1 << 20]))
    read_size = int(rng.choice([7, 1000, 10240, 1 << 18]))
    push = bool(rng.random() < 0.3)
    late = bool(rng.random() < 0.3)
    os.environ["ASYNC_B64_STAGE_CAPACITY"] = cap
    os.environ["ASYNC_B64_LEND_MIN"] = lend_min
    got, err = util.egress_pieces(pieces, max_chunk, read_size, push=push, late=late)
    data = b"".join(pieces)
    ok = err == 0 and got is not None
    if ok and late:
        ok = util.dechunk(got) == orc.encode(data)
    elif ok:
        ok = got == orc.chunked_encode(np.frombuffer(data, np.uint8), piece_lens=sizes,
                                       max_chunk=max_chunk, read_size=read_size)
    if not ok:
        print(f"MISMATCH seed {seed}: sizes {sizes} cap {cap} lend_min {lend_min} "
              f"max_chunk {max_chunk} read_size {read_size} push {push} late {late} err {err}",
              flush=True)
        sys.exit(1)
    if seed % 25 == 0:
        print(f"seed {seed} {time.time() - t0:.1f}", flush=True)
refs = L.b64_pin_live_refs()
print(f"FUZZ OK lent egress {n} seeds, pinned refs left {refs}, {time.time() - t0:.1f} s", flush=True)
sys.exit(0 if refs == 0 else 1)
