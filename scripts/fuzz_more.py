"""More seeds of the GPU decode fuzz (tests/test_decode_fuzz.py) than the
suite runs: the row-batch fuzz and the single-buffer decode fuzz for seeds
16 .. 16+N, each case bit-exact against the oracle.  GPU box only:
    python -u scripts/fuzz_more.py ROWS_SEEDS DECODE_SEEDS"""
import sys, time
sys.path.insert(0, ".")
import tests.test_decode_fuzz as t
t0 = time.time()
n1, n2 = int(sys.argv[1]), int(sys.argv[2])
for s in range(16, 16 + n1):
    t.test_rows_fuzz_vs_oracle(s)
    if s % 50 == 0: print("rows seed", s, round(time.time() - t0, 1), flush=True)
for s in range(16, 16 + n2):
    t.test_decode_fuzz_vs_oracle(s)
    if s % 25 == 0: print("decode seed", s, round(time.time() - t0, 1), flush=True)
print("FUZZ OK rows", n1, "decode", n2, "extra seeds", round(time.time() - t0, 1), "s", flush=True)
