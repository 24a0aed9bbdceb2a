"""Static checks on the gfx950 code object of a built library (test tooling).

The code object is taken out of the shared library's `.hip_fatbin` section
with clang-offload-bundler and disassembled with llvm-objdump.  Each kernel
is split into basic blocks (branch targets and the instruction after a
branch start one), and two facts are propagated forward over the control-flow
graph, joined by OR at block entries:

  lds   an LDS write (ds_write*, ds_or*, ds_add*, ...) may still be in
        flight: lgkmcnt counts it until an `s_waitcnt lgkmcnt(0)`;
  dma   a global -> LDS copy (global_load_lds_*) may still be in flight:
        vmcnt counts it until an `s_waitcnt vmcnt(0)`.

`barrier_report()` lists every `s_barrier` reached with either fact set on
some path.  On gfx950 (back-off barrier) the hardware barrier does not wait
for them, and the compiler's waitcnt pass does not add a wait for its own
sake; the only wait comes from the fence of __syncthreads(), a soft wait the
pass may drop.  In round 5's first k_decode_suffix_held (commit d2beeb5) it
was dropped at the loop-top barrier, whose back edge carries thread 0's
write of the next tile's ticket: `ds_write_b32 ... offset:23176` then
`s_branch` to the loop header, `s_barrier`, `ds_read_b32 ... offset:23176`
with no wait in between.  block_sync() puts an explicit
`s_waitcnt lgkmcnt(0)` in front of every barrier since.

`dma_reads()` lists, per kernel that copies into LDS, the LDS reads reached
while a copy may be in flight, so that a test can pin that the copies'
buffers are read only after a vmcnt(0).
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_LDS_WRITE = re.compile(
    r"^ds_(write|wrxchg|or|and|xor|add|sub|inc|dec|min|max|cmpst|mskor|rsub|store)")
_DMA = re.compile(r"^(global|buffer)_load_lds|^buffer_load_\w+.*\blds\b")
_BRANCH = re.compile(r"^s_(c?branch\w*|cbranch\w*)\b")
_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")


def _section(path: str, name: bytes) -> bytes:
    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    strtab = sh(shstrndx)
    for i in range(shnum):
        s = sh(i)
        nm = data[strtab[4] + s[0]:data.index(b"\0", strtab[4] + s[0])]
        if nm == name:
            return data[s[4]:s[4] + s[5]]
    raise KeyError(name)


def disassemble(so_path: str) -> str:
    """llvm-objdump -d of the gfx950 code object inside `so_path`."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        co = os.path.join(d, "k.co")
        with open(fat, "wb") as f:
            f.write(_section(so_path, b".hip_fatbin"))
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        "--input=" + fat, "--targets=" + TARGET, "--output=" + co],
                       check=True, capture_output=True)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True,
                              capture_output=True, text=True).stdout


def functions(dis: str) -> dict:
    """{symbol: [(offset, instruction text, branch target offset or None)]}"""
    out, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            base = int(m.group(1), 16)
            cur = out.setdefault(m.group(2), [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        text, _, comment = line.strip().partition("//")
        text = text.strip()
        if not text:
            continue
        am = re.match(r"\s*([0-9A-F]+):", comment)
        if not am:
            continue
        off = int(am.group(1), 16) - base
        tm = _TARGET.search(comment)
        cur.append((off, text, int(tm.group(2), 16) if tm and _BRANCH.match(text) else None))
    return out


def _flow(insns):
    """Per instruction index: (lds, dma) in flight before it, joined over
    every path from the kernel's entry."""
    n = len(insns)
    index = {off: i for i, (off, _, _) in enumerate(insns)}
    leaders = {0}
    for i, (_, text, tgt) in enumerate(insns):
        if tgt is not None:
            leaders.add(index.get(tgt, n))
            leaders.add(i + 1)
        elif text.startswith("s_endpgm"):
            leaders.add(i + 1)
    starts = sorted(x for x in leaders if x < n)
    ends = {s: (starts[k + 1] if k + 1 < len(starts) else n) for k, s in enumerate(starts)}
    succ = {}
    for s in starts:
        e = ends[s]
        last = insns[e - 1][1]
        tgt = insns[e - 1][2]
        nxt = []
        if tgt is not None:
            nxt.append(index[tgt])
        if not (last.startswith("s_branch") or last.startswith("s_endpgm")) and e < n:
            nxt.append(e)
        succ[s] = nxt
    state_in = {s: None for s in starts}
    state_in[0] = (False, False)
    before = [None] * n
    work = [0]
    while work:
        s = work.pop()
        lds, dma = state_in[s]
        for i in range(s, ends[s]):
            prev = before[i]
            before[i] = (lds, dma) if prev is None else (prev[0] or lds, prev[1] or dma)
            text = insns[i][1]
            if text.startswith("s_waitcnt"):
                if "lgkmcnt(0)" in text:
                    lds = False
                if "vmcnt(0)" in text:
                    dma = False
            elif _LDS_WRITE.match(text):
                lds = True
            elif _DMA.match(text):
                dma = True
        for t in succ[s]:
            old = state_in[t]
            new = (lds, dma) if old is None else (old[0] or lds, old[1] or dma)
            if new != old:
                state_in[t] = new
                work.append(t)
    return before


def barrier_report(dis: str) -> list:
    """[(kernel, offset, 'lds'|'dma', instruction before)] for every barrier
    some path reaches with an LDS write or an LDS copy still in flight."""
    bad = []
    for name, insns in functions(dis).items():
        if not insns:
            continue
        st = _flow(insns)
        for i, (off, text, _) in enumerate(insns):
            if not text.startswith("s_barrier") or st[i] is None:
                continue
            lds, dma = st[i]
            prev = insns[i - 1][1] if i else ""
            if lds:
                bad.append((name, off, "lds", prev))
            if dma:
                bad.append((name, off, "dma", prev))
    return bad


def barrier_count(dis: str) -> int:
    return sum(1 for insns in functions(dis).values() for _, t, _ in insns
               if t.startswith("s_barrier"))


def dma_reads(dis: str) -> dict:
    """{kernel: [(offset, instruction)]}: the LDS reads of kernels that copy
    global -> LDS, reached while such a copy may still be in flight."""
    out = {}
    for name, insns in functions(dis).items():
        if not any(_DMA.match(t) for _, t, _ in insns):
            continue
        st = _flow(insns)
        out[name] = [(off, t) for i, (off, t, _) in enumerate(insns)
                     if t.startswith("ds_read") and st[i] is not None and st[i][1]]
    return out


def kernel_symbols(dis: str) -> set:
    return set(functions(dis))


if __name__ == "__main__":
    import sys
    d = disassemble(sys.argv[1])
    print("barriers:", barrier_count(d))
    for row in barrier_report(d):
        print("barrier in flight:", row)
    for k, v in dma_reads(d).items():
        print(k[:70], "reads while a copy is in flight:", len(v))
        for off, t in v:
            print("   ", hex(off), t)
