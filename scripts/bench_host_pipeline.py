"""PCIe-inclusive rates of the host-memory path.

Two measurements, both bit-checked against the device-resident result:

  sessions  K sessions round-robin over a host buffer of TOTAL bytes:
            memcpy into pinned host_in, H2D, kernels, D2H into pinned
            host_out (+ memcpy out), with up to K blocks in flight.  This is
            what a caller holding host buffers gets per GPU.
  stages    the drop-in bytestream_1 stages on the product event loop:
            blobstream -> base64 encoder stage -> consumer (1 MiB reads), and
            blobstream -> decoder stage -> consumer, timed end to end.

Prints one JSON line per measurement.  Usage:
    python scripts/bench_host_pipeline.py [--total MiB] [--block MiB] [--k K]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from async_amd.session import HOLD_TAIL, Session  # noqa: E402


def splitmix(n, seed=1):
    k = np.arange(1, (n + 7) // 8 + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:n]


def run_resident(src: np.ndarray, block: int, k: int, op: str, total: int):
    """PCIe-inclusive rate without host memcpy: each session's pinned host_in
    already holds its block (as if upstream had read into it); results stay
    in pinned host_out.  Returns seconds for `total` input units."""
    sess = [Session(block) for _ in range(k)]
    step = block // 3 * 3 if op == "encode" else block // 4 * 4
    try:
        for s in sess:
            s.host_in[:step] = src[:step]
            s.encode(step) if op == "encode" else s.decode(step)
        nblk = (total + step - 1) // step
        t0 = time.perf_counter()
        for i in range(nblk):
            s = sess[i % k]
            if i >= k:
                s.wait()
            n = min(step, total - i * step)
            if op == "encode":
                s.encode_async(n)
            else:  # whole groups of clean text: blocks need no carry
                s.decode_async(n, None, 0)
        for s in sess:
            s.wait()
        return time.perf_counter() - t0
    finally:
        for s in sess:
            s.close()


def pcie_calibration(nbytes: int):
    """Plain pinned<->device copies (torch), each direction and both at once."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h2 = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        res["h2d_GB_s"] = nbytes / (time.perf_counter() - t0) / 1e9
        t0 = time.perf_counter()
        h.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        res["d2h_GB_s"] = nbytes / (time.perf_counter() - t0) / 1e9
        t0 = time.perf_counter()
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()
        res["duplex_GB_s_each"] = nbytes / (time.perf_counter() - t0) / 1e9
    return res


def run_sessions(src: np.ndarray, block: int, k: int, op: str, out: np.ndarray):
    """Stream src through k sessions; returns (seconds, out_len)."""
    sess = [Session(block) for _ in range(k)]
    step = block // 3 * 3 if op == "encode" else block // 4 * 4
    try:
        # warm up every session once (allocations, code objects)
        for s in sess:
            s.host_in[:step] = src[:step]
            if op == "encode":
                s.encode(step)
            else:
                s.decode(step)
        live = []  # (session, out_len or None)
        opos = 0
        t0 = time.perf_counter()
        pos, i = 0, 0
        while pos < len(src) or live:
            if pos < len(src) and len(live) < k:
                s = sess[i % k]
                n = min(step, len(src) - pos)
                s.host_in[:n] = src[pos:pos + n]
                last = pos + n == len(src)
                if op == "encode":
                    s.encode_async(n)
                    m = (n + 2) // 3 * 4 if last else n // 3 * 4
                else:
                    # blocks are whole 4-character groups of clean text, so no
                    # block holds a carry for the next one
                    s.decode_async(n, None, 0)
                    m = None
                live.append((s, m))
                pos += n
                i += 1
                continue
            s, m = live.pop(0)
            s.wait()
            if m is None:
                m = s.result().out_len
            out[opos:opos + m] = s.host_out[:m]
            opos += m
        dt = time.perf_counter() - t0
    finally:
        for s in sess:
            s.close()
    return dt, opos


def _oracle_stack_rate(payload, lens, threads):
    """The oracle's restatement of the same stack (queuestream -> encoder ->
    chunkencoder(1 MiB), 10,240-byte reads) over all messages, `threads`
    Python threads (ctypes drops the GIL inside the C oracle)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import pyoracle as orc
    offs = np.concatenate([[0], np.cumsum(lens)])
    n = len(lens)
    bounds = np.linspace(0, offs[-1], threads + 1)
    cuts = np.searchsorted(offs, bounds)

    def work(t):
        for i in range(cuts[t], cuts[t + 1]):
            orc.chunked_encode(payload[offs[i]:offs[i + 1]], max_chunk=1 << 20,
                               read_size=10240)
    t0 = time.perf_counter()
    if threads == 1:
        work(0)
    else:
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(work, range(threads)))
    dt = time.perf_counter() - t0
    assert cuts[-1] == n
    return dt


def run_egress(n_msgs: int, thread_counts=(1, 4, 8, 16)):
    """Config 5: n_msgs Zipf messages, each its own queuestream -> GPU
    encoder stage -> chunkencoder(1 MiB) stack, drained 10,240 bytes per
    read (tcp_connection.c:22); host memory in, framed host memory out.
    T event loops (threads, one hub each) share the messages by bytes.
    The oracle stack is timed with the same thread counts beside it."""
    from oracle import pyoracle as orc
    from tests import util
    lens = util.zipf_lengths()[:n_msgs]
    payload = util.splitmix64(0x5EED, int(lens.sum()))
    nbytes = int(lens.sum())
    offs = np.concatenate([[0], np.cumsum(lens)])
    util.egress_stacks(payload[:4096], [64] * 64, 1 << 20, 10240)  # warm-up
    ndev = util.device_count()
    for T in thread_counts:
        times = np.zeros(2)
        gpus = min(T, ndev)  # loop t on GPU t mod gpus (8 on a full node)
        # one untimed pass: T loops' arenas (pinned), lanes and the
        # queuestream buffers' pages come from process-wide pools / the heap
        util.egress_stacks(payload, lens, 1 << 20, 10240, raw=True, threads=T, devices=gpus)
        res, err = util.egress_stacks(payload, lens, 1 << 20, 10240, times=times, raw=True,
                                      threads=T, devices=gpus)
        dt = float(times.sum())
        out, out_off, out_len = res
        idx = list(range(0, n_msgs, max(1, n_msgs // 64)))
        ok = err == 0 and all(
            out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes() ==
            orc.chunked_encode(payload[offs[i]:offs[i + 1]].tobytes(), max_chunk=1 << 20)
            for i in idx)
        framed_total = int(out_len.sum())
        del out, res
        cpu_dt = _oracle_stack_rate(payload, lens, T)
        print(json.dumps({"measure": "egress_config5", "threads": T, "gpus": gpus,
                          "messages": n_msgs,
                          "bytes": nbytes, "framed_bytes": framed_total, "seconds": dt,
                          "setup_s": float(times[0]), "loop_s": float(times[1]),
                          "GiB_s": nbytes / dt / 2**30, "msgs_per_s": n_msgs / dt,
                          "exact_sampled": bool(ok),
                          "cpu_oracle": {"threads": T, "seconds": cpu_dt,
                                         "GiB_s": nbytes / cpu_dt / 2**30}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=1024, help="MiB of input bytes")
    ap.add_argument("--block", type=int, default=32, help="MiB per session block")
    ap.add_argument("--k", type=int, default=4, help="sessions in flight")
    ap.add_argument("--stage-total", type=int, default=256, help="MiB through the stages")
    ap.add_argument("--only", default="", help="comma list: sessions,resident,stages,egress")
    ap.add_argument("--egress-msgs", type=int, default=16384, help="config-5 messages")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    want = (lambda k: not only or k in only)

    import torch
    from async_amd import b64

    if want("egress"):
        run_egress(args.egress_msgs)
    if only == {"egress"}:
        return
    total = args.total << 20
    block = args.block << 20
    src = splitmix(total)
    # Device-resident reference result for the bit check.
    ref_chars = b64.encode(torch.from_numpy(src).cuda()).cpu().numpy()
    if want("sessions"):
        chars = np.empty(len(ref_chars), np.uint8)
        dt, m = run_sessions(src, block, args.k, "encode", chars)
        ok = m == len(ref_chars) and np.array_equal(chars, ref_chars)
        print(json.dumps({"measure": "sessions_encode", "bytes": total, "block": block,
                          "k": args.k, "seconds": dt, "GiB_s": total / dt / 2**30,
                          "exact": bool(ok)}), flush=True)
        back = np.empty(total + 16, np.uint8)
        dt, m = run_sessions(ref_chars, block, args.k, "decode", back)
        ok = m == total and np.array_equal(back[:m], src)
        print(json.dumps({"measure": "sessions_decode", "chars": len(ref_chars), "bytes": m,
                          "block": block, "k": args.k, "seconds": dt,
                          "GiB_s": m / dt / 2**30, "exact": bool(ok)}), flush=True)
        del chars, back

    if want("resident"):
        print(json.dumps({"measure": "pcie_calibration", "bytes": 256 << 20,
                          **pcie_calibration(256 << 20)}), flush=True)
    for kk in ((2, 4, 8) if want("resident") else ()):
        dt = run_resident(src, block, kk, "encode", total)
        print(json.dumps({"measure": "resident_encode", "bytes": total, "block": block,
                          "k": kk, "seconds": dt, "GiB_s": total / dt / 2**30,
                          "pcie_GB_s": (total + len(ref_chars)) / dt / 1e9}), flush=True)
        dt = run_resident(ref_chars, block, kk, "decode", len(ref_chars))
        print(json.dumps({"measure": "resident_decode", "bytes": total, "block": block,
                          "k": kk, "seconds": dt, "GiB_s": total / dt / 2**30,
                          "pcie_GB_s": (total + len(ref_chars)) / dt / 1e9}), flush=True)
        # the same blocks decoded without carries (each holds whole groups):
        # clean input with no carry head reads and writes in place
        dt = run_resident(ref_chars, block, kk, "decode_blocks", len(ref_chars))
        print(json.dumps({"measure": "resident_decode_blocks", "bytes": total, "block": block,
                          "k": kk, "seconds": dt, "GiB_s": total / dt / 2**30,
                          "pcie_GB_s": (total + len(ref_chars)) / dt / 1e9}), flush=True)

    # The bytestream_1 stages on the product loop (tests/csrc harness).
    if not want("stages"):
        return
    from tests import util
    st_total = args.stage_total << 20
    data = src[:st_total]
    raw = data.tobytes()
    st_chars = b64.encode(torch.from_numpy(data).cuda()).cpu().numpy()
    L = util.harness()
    ecap = (st_total + 2) // 3 * 4 + 16
    out = np.empty(ecap, np.uint8)
    err = ctypes.c_int(0)
    for rs in (1 << 20, 64 << 10):
        t0 = time.perf_counter()
        n = L.h_encode_stream(raw, st_total, 0, rs, b"\xff", b"\xff", 1, b"\xff",
                              out.ctypes.data, ecap, ctypes.byref(err))
        dt = time.perf_counter() - t0
        ok = n == len(st_chars) and np.array_equal(out[:n], st_chars)
        print(json.dumps({"measure": "stage_encode", "bytes": st_total, "read_size": rs,
                          "capacity": int(os.environ.get("ASYNC_B64_STAGE_CAPACITY", 1 << 20)),
                          "seconds": dt, "GiB_s": st_total / dt / 2**30,
                          "exact": bool(ok), "err": err.value}), flush=True)
        enc = out[:n].tobytes()
        dout = np.empty(st_total + 16, np.uint8)
        t0 = time.perf_counter()
        n2 = L.h_decode_stream(enc, len(enc), 0, rs, b"\xff", b"\xff",
                               dout.ctypes.data, dout.size, ctypes.byref(err))
        dt = time.perf_counter() - t0
        ok = n2 == st_total and np.array_equal(dout[:n2], data)
        print(json.dumps({"measure": "stage_decode", "bytes": st_total, "read_size": rs,
                          "seconds": dt, "GiB_s": st_total / dt / 2**30,
                          "exact": bool(ok), "err": err.value}), flush=True)


if __name__ == "__main__":
    main()
