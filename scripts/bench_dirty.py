#!/usr/bin/env python3
"""Decode throughput on "dirty" input (CRLF every 76
characters, MIME style), which leaves the fast path at the first CR and
runs the exact path (scan + pass 2) over the rest.  Checked bit-exact
against the original bytes.  Prints one JSON line per size.

    python scripts/bench_dirty.py [--mib 1024] [--steps 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from async_amd import b64  # noqa: E402


def crlf76(chars: torch.Tensor) -> torch.Tensor:
    n = chars.numel()
    rows = (n + 75) // 76
    pad = rows * 76 - n
    body = torch.cat([chars, torch.zeros(pad, dtype=torch.uint8, device=chars.device)])
    body = body.view(rows, 76)
    crlf = torch.tensor([13, 10], dtype=torch.uint8, device=chars.device).expand(rows, 2)
    out = torch.cat([body, crlf], dim=1).reshape(-1)
    # drop the zero padding of the last row (keep its CRLF)
    if pad:
        keep = torch.ones(out.numel(), dtype=torch.bool, device=chars.device)
        start = (rows - 1) * 78 + (76 - pad)
        keep[start:start + pad] = False
        out = out[keep]
    return out.contiguous()


def sprinkle(chars: torch.Tensor, density: float, seed=7) -> torch.Tensor:
    """Unstructured junk: a byte outside the alphabet ('!') before each
    character with probability `density`."""
    g = torch.Generator(device=chars.device).manual_seed(seed)
    mask = (torch.rand(chars.numel(), device=chars.device, generator=g) < density)
    idx = torch.arange(chars.numel(), device=chars.device) + torch.cumsum(mask, 0)
    out = torch.full((chars.numel() + int(mask.sum()),), ord("!"), dtype=torch.uint8,
                     device=chars.device)
    out[idx] = chars
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, nargs="*", default=[64, 1024])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--junk", type=float, default=0.0,
                    help="unstructured junk density instead of CRLF-76 lines")
    ap.add_argument("--expect-junk", action="store_true",
                    help="B64X_DEC_EXPECT_JUNK: the single-pass decode")
    args = ap.parse_args()
    for mib in args.mib:
        n = mib << 20
        x = torch.empty(n, dtype=torch.uint8, device="cuda")
        b64.fill_splitmix64(x, 0x5EED)
        enc = b64.encode(x)
        dirty = sprinkle(enc, args.junk) if args.junk else crlf76(enc)
        del enc
        ws = torch.zeros(b64.workspace_size(dirty.numel()), dtype=torch.uint8, device="cuda")
        out = torch.empty(b64.decoded_cap(dirty.numel()), dtype=torch.uint8, device="cuda")
        d = b64.decode(dirty, out=out, workspace=ws, expect_junk=args.expect_junk)
        ok = d.info().out_len == n and torch.equal(out[:n], x)
        times = []
        for _ in range(args.steps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            b64.decode(dirty, out=out, workspace=ws, expect_junk=args.expect_junk)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        ms = sorted(times)[len(times) // 2]
        alg = dirty.numel() + n
        print(json.dumps({"measure": f"decode_junk{args.junk:g}" if args.junk else "decode_crlf76",
                          "expect_junk": args.expect_junk,
                          "payload_bytes": n, "chars": dirty.numel(),
                          "ms": ms, "GiB_s_payload": n / ms / 1e-3 / 2**30,
                          "alg_TB_s": alg / ms / 1e-3 / 1e12, "exact": bool(ok)}), flush=True)
        del x, dirty, ws, out


if __name__ == "__main__":
    main()
