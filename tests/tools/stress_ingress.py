"""Repeat the 600-stream decoder ingress scenario; count mismatching
streams per iteration (test infrastructure: checks against the oracle).

A GPU tool: `python -u tests/tools/stress_ingress.py 30` (one loop, 600
stacks, 1 KiB staging).  It caught a stale completion result on
coarse-grained pinned session memory (b64x_session_open)."""
import ctypes
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["ASYNC_B64_STAGE_CAPACITY"] = "1024"
from tests import util  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
util.harness()
# the b64x library the harness resolved (LD_LIBRARY_PATH may point at a
# diagnostic build): its counters of completions that came before their result
_core = ctypes.CDLL("libasync_b64.so")
_core.b64x_diag_counters.argtypes = [ctypes.POINTER(ctypes.c_uint64)]


def counters():
    out = (ctypes.c_uint64 * 2)()
    _core.b64x_diag_counters(out)
    return int(out[0]), int(out[1])


tot = 0
for it in range(iters):
    rng = np.random.default_rng(23 + it)
    msgs = [orc.encode(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes())
            for n in rng.integers(1500, 5000, 600)]
    msgs[7] = b"\r\n".join(msgs[7][i:i + 76] for i in range(0, len(msgs[7]), 76))
    got, err = util.ingress_stacks(msgs, 4096)
    bad = []
    for i, m in enumerate(msgs):
        w = orc.decode(m)
        g = got[i] or b""
        if g != w:
            d = [j for j in range(min(len(g), len(w))) if g[j] != w[j]]
            bad.append((i, len(m), len(g), len(w), d[0] if d else -1, d[-1] if d else -1))
    tot += len(bad)
    print(f"it={it} err={err} bad={len(bad)} {bad[:4]} early={counters()}", flush=True)
print(f"TOTAL bad={tot} early={counters()}", flush=True)
