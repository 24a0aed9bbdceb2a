"""More seeds of tests/test_decode_fuzz.py's reuse fuzz (single buffers and
row batches) and its plain decode and row fuzz than the suite runs (GPU box):
    python scripts/fuzz_reuse_more.py FIRST COUNT"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import test_decode_fuzz as f  # noqa: E402


def main():
    first, count = int(sys.argv[1]), int(sys.argv[2])
    t0 = time.time()
    for seed in range(first, first + count):
        f.test_reuse_fuzz_interleaved(seed)
        f.test_decode_fuzz_vs_oracle(seed)
        f.test_rows_reuse_fuzz(seed)
        f.test_rows_fuzz_vs_oracle(seed)
        print(f"seed {seed} ok ({time.time() - t0:.0f} s)", flush=True)
    print("ALL OK", flush=True)


if __name__ == "__main__":
    main()
