#!/usr/bin/env python3
"""bench.py's host_fd leg alone (pipe/socket ingress, blob ingress, pipe
egress, the channel calibration), for A/B of host-side changes: one JSON
line.  python scripts/host_fd_only.py [--size BYTES]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (one HIP runtime, see async_amd/_lib.py)

import bench  # noqa: E402
from async_amd import b64  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=1 << 30)
a = ap.parse_args()
res = bench.bench_host_fd(argparse.Namespace(size=a.size), b64)
print(json.dumps({k: (v.get("GiB_s", v.get("GiB_s_payload_equiv")) if isinstance(v, dict) else v)
                  for k, v in res.items()}), flush=True)
