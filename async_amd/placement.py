"""NUMA placement of the host side: which node the GPU hangs off, which CPUs
and memory nodes this process may use, and where memory pages sit.

Host plumbing for the bench and the probes (Linux sysfs and procfs only; no
libnuma in the image).  The C side binds loop threads itself
(b64x_bind_thread, include/b64x.h); this module reads the same facts for
reporting them on the bench line."""
from __future__ import annotations

import glob
import os
import re


def _read(path: str, default: str = "") -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def parse_cpulist(s: str) -> set:
    out = set()
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def cpulist(cpus) -> str:
    """{0,1,2,5} -> '0-2,5'"""
    cpus = sorted(cpus)
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def node_cpus(node: int) -> set:
    if node is None or node < 0:
        return set()
    return parse_cpulist(_read(f"/sys/devices/system/node/node{node}/cpulist"))


def cpu_node(cpu: int) -> int:
    for p in glob.glob(f"/sys/devices/system/cpu/cpu{cpu}/node*"):
        m = re.search(r"node(\d+)$", p)
        if m:
            return int(m.group(1))
    return -1


def pci_path(device: int) -> str | None:
    import torch
    p = torch.cuda.get_device_properties(device)
    dom = getattr(p, "pci_domain_id", 0)
    bus = getattr(p, "pci_bus_id", None)
    slot = getattr(p, "pci_device_id", None)
    if bus is None or slot is None:
        return None
    path = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{slot:02x}.0"
    return path if os.path.isdir(path) else None


def topology(device: int) -> dict:
    """The GPU's node and link, and this process's CPUs and memory nodes."""
    path = pci_path(device)
    node = int(_read(os.path.join(path, "numa_node"), "-1")) if path else -1
    allowed = sorted(os.sched_getaffinity(0))
    status = _read("/proc/self/status")
    mems = re.search(r"Mems_allowed_list:\s*(\S+)", status)
    nodes = sorted(int(re.search(r"node(\d+)$", p).group(1))
                   for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
    by_node = {}
    for n in nodes:
        c = node_cpus(n) & set(allowed)
        if c:
            by_node[str(n)] = cpulist(c)
    return {
        "gpu_pci": os.path.basename(path) if path else None,
        "gpu_node": node,
        "link": {k: _read(os.path.join(path, k)) for k in
                 ("current_link_speed", "current_link_width", "max_link_speed",
                  "max_link_width")} if path else None,
        "nodes": len(nodes),
        "allowed_cpus": cpulist(allowed),
        "allowed_cpus_by_node": by_node,
        "mems_allowed": mems.group(1) if mems else None,
    }


def pages_by_node(min_bytes: int = 16 << 20) -> dict:
    """Resident pages per NUMA node, summed over this process's mappings of
    at least min_bytes (the pinned arenas, the payload, the bench's arrays)
    from /proc/self/numa_maps, in MiB."""
    tot = {}
    page = os.sysconf("SC_PAGE_SIZE")
    maps = {}
    for line in _read("/proc/self/maps").splitlines():
        a, _, rest = line.partition(" ")
        lo, hi = a.split("-")
        maps[int(lo, 16)] = int(hi, 16) - int(lo, 16)
    for line in _read("/proc/self/numa_maps").splitlines():
        f = line.split()
        if not f:
            continue
        start = int(f[0], 16)
        if maps.get(start, 0) < min_bytes:
            continue
        kp = page
        for x in f:
            if x.startswith("kernelpagesize_kB="):
                kp = int(x.split("=")[1]) * 1024
        for x in f:
            m = re.match(r"N(\d+)=(\d+)$", x)
            if m:
                tot[m.group(1)] = tot.get(m.group(1), 0) + int(m.group(2)) * kp
    return {k: round(v / 2**20, 1) for k, v in sorted(tot.items())}
