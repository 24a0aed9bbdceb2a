#!/usr/bin/env python3
"""Where config 5's host side runs, and what placement does to it (GPU box).

Prints one JSON line per variant: the machine's NUMA layout as this process
sees it (the GPU's node from sysfs, the PCIe link, the CPUs and memory nodes
the process may use, per node), then config 5 on one loop (the bench's
stack: 16,384 Zipf messages, queuestream -> encoder -> chunkencoder, host
memory in and out) with the calling thread -- and so the loop thread the
harness starts, which inherits its mask -- bound to:
  all      the process's whole CPU mask (what bench.py did through round 5)
  gpu      the allowed CPUs on the GPU's node
  other    the allowed CPUs on another node (when there are any)
each after an untimed pass, 5 timed passes, plus where the big anonymous
mappings' pages sit (/proc/self/numa_maps).

    python scripts/numa_probe.py [--passes 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from async_amd import placement
    from tests import util

    dev = torch.cuda.current_device()
    topo = placement.topology(dev)
    print(json.dumps({"topology": topo}), flush=True)
    lens = util.zipf_lengths()
    nbytes = int(lens.sum())
    payload = util.splitmix64(0x5EED, nbytes)
    allowed = sorted(os.sched_getaffinity(0))
    gpu_cpus = placement.node_cpus(topo.get("gpu_node", -1)) & set(allowed)
    other = sorted(set(allowed) - gpu_cpus)
    variants = [("all", set(allowed))]
    if gpu_cpus:
        variants.append(("gpu", gpu_cpus))
    if other and gpu_cpus:
        variants.append(("other", set(other)))
    util.egress_stacks(payload[:4096], [64] * 64, 1 << 20, 10240, device=dev)
    for name, cpus in variants + variants[:1]:
        os.sched_setaffinity(0, cpus)
        util.egress_stacks(payload, lens, 1 << 20, 10240, raw=True, threads=1, device=dev)
        rates, setup, loop = [], [], []
        for _ in range(args.passes):
            times = np.zeros(2)
            res, err = util.egress_stacks(payload, lens, 1 << 20, 10240, raw=True, threads=1,
                                          device=dev, times=times)
            assert res is not None, err
            rates.append(nbytes / times.sum() / 2**30)
            setup.append(float(times[0]))
            loop.append(float(times[1]))
            del res
        print(json.dumps({"variant": name, "cpus": placement.cpulist(cpus),
                          "nodes_of_cpus": sorted({placement.cpu_node(c) for c in cpus}),
                          "GiB_s": [round(r, 3) for r in rates],
                          "setup_s": [round(s, 4) for s in setup],
                          "loop_s": [round(s, 4) for s in loop],
                          "pages_by_node": placement.pages_by_node(min_bytes=16 << 20)}),
              flush=True)
    os.sched_setaffinity(0, set(allowed))


if __name__ == "__main__":
    main()
