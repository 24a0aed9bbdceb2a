#!/bin/bash
# HBM traffic of the bench's kernels: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (TCC slots: FETCH_SIZE needs 3 of 4, WRITE_SIZE 2), each
# with --kernel-trace only.  Output: gpurun_out/pmc_traffic/{fetch,write}.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_traffic"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/$c" -o run \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-host --no-mime --batch-steps 3 > "$OUT/$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
