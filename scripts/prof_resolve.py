"""Fold the harness's SIGPROF histogram (tests/csrc/stage_harness.c
h_prof_stop) into per-function counts, naming static functions of objects
built here with `nm` (the dynamic symbol table has only exported ones).
Usage: python scripts/prof_resolve.py prof.txt [top]"""
import bisect
import os
import subprocess
import sys
from collections import Counter

_nm = {}


def symbols(obj):
    """Sorted (addr, name) of an object's text symbols, or None."""
    if obj not in _nm:
        root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
        base = os.path.basename(obj)
        local = [os.path.join(root, d, base) for d in ("async_amd", "tests/csrc", "oracle")]
        tab = []
        for path in local + [obj]:
            if not os.path.exists(path):
                continue
            out = subprocess.run(["nm", "-n", "--defined-only", path], capture_output=True,
                                 text=True).stdout
            for line in out.splitlines():
                parts = line.split()
                if len(parts) == 3 and parts[1] in "tTwW":
                    tab.append((int(parts[0], 16), parts[2]))
            if tab:
                break
        _nm[obj] = sorted(tab) or None
    return _nm[obj]


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = Counter()
    total = 0
    with open(path) as f:
        next(f)
        for line in f:
            n, obj, sym, off = line.split()
            n = int(n)
            total += n
            base = os.path.basename(obj)
            if sym == "?":
                tab = symbols(obj)
                if tab:
                    i = bisect.bisect_right(tab, (int(off, 16), "￿")) - 1
                    sym = tab[i][1] if i >= 0 else "?"
            c[f"{base} {sym}"] += n
    for k, n in c.most_common(top):
        print(f"{n:8d} {100 * n / max(total, 1):5.1f}%  {k}")
    print(f"{total:8d} total")


if __name__ == "__main__":
    main()
