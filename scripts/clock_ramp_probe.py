#!/usr/bin/env python3
"""Clock ramp after idle: the first milliseconds of GPU work after the GPU
has idled (or run only short bursts) run slower.  Times bench.py's headline
step (1 GiB encode + decode) K times between two events after
  warm:   a pre-heat of --heat steps right before the barrier,
  bench:  bench.py's sequence (W warmup steps, sync, the bit check, sync),
  idle:   --idle seconds of sleep,
  copyN:  --idle seconds of sleep, then N ms of torch copies (a pre-heat
          that is not the measured work),
interleaved over --rounds; also the batch (config-4) encode the same ways.

    python scripts/clock_ramp_probe.py [--rounds 3] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--heat", type=int, default=60)
    ap.add_argument("--idle", type=float, default=0.2)
    ap.add_argument("--modes", default="idle,bench,warm,copy10,copy25,copy50,copy100")
    a = ap.parse_args()
    import torch
    from async_amd import b64
    st = torch.cuda.current_stream()
    N = 1 << 30
    E = b64.encoded_len(N)
    x = torch.empty(N, dtype=torch.uint8, device="cuda")
    b64.fill_splitmix64(x, 0x5EED)
    enc = torch.empty(E, dtype=torch.uint8, device="cuda")
    dec = torch.empty(b64.decoded_cap(E), dtype=torch.uint8, device="cuda")
    ws = torch.zeros(b64.workspace_size(E), dtype=torch.uint8, device="cuda")
    res = torch.zeros(b64.RES_BYTES, dtype=torch.uint8, device="cuda")
    L, nb = 1024, 1 << 20
    Es = b64.encoded_len(L)
    e4 = torch.empty(nb * Es, dtype=torch.uint8, device="cuda")

    def step():
        b64.encode(x, out=enc, stream=st)
        b64.decode(enc, out=dec, workspace=ws, result=res, stream=st)

    def enc4():
        b64.encode_strided(x, L, L, nb, e4, Es, stream=st)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(a.steps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / a.steps, 1)

    def prep(mode, fn):
        if mode == "warm":
            for _ in range(a.heat):
                fn()
        elif mode.startswith("copy"):
            # torch copies of 256 MiB for the given ms (~0.08 ms each)
            ms = int(mode[4:])
            torch.cuda.synchronize()
            time.sleep(a.idle)
            for _ in range(int(ms / 0.085)):
                scratch[0].copy_(scratch[1])
        elif mode == "bench":
            for _ in range(a.warmup):
                fn()
            torch.cuda.synchronize()
            assert torch.equal(dec[:N], x)
        else:
            torch.cuda.synchronize()
            time.sleep(a.idle)

    scratch = torch.empty(2, 256 << 20, dtype=torch.uint8, device="cuda")
    step()
    enc4()
    for r in range(a.rounds):
        row = {"round": r}
        for mode in a.modes.split(","):
            prep(mode, step)
            row["step_" + mode] = timed(step)
            prep(mode, enc4)
            row["enc4_" + mode] = timed(enc4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
