#!/bin/bash
# GPU box: parity tests, the dirty-decode benchmark (CRLF-76, plain and
# EXPECT_JUNK), a short bench.py, and rocprofv3 kernel traces of the dirty
# decode and of the bench.  Each step has its own limit; a crash/timeout
# ends the script.  Output: gpurun_out/<TAG>_*.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dec}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$ROOT/gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 6 "$ROOT/gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$NO_TESTS" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"}
fi
step dirty 300 python scripts/bench_dirty.py --mib 64 1024 --steps 7
step dirty_junk 300 python scripts/bench_dirty.py --mib 64 1024 --steps 7 --expect-junk
step batch_dirty 300 python scripts/bench_batch_dirty.py
step bench 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-host
cd /tmp && export TMPDIR=/tmp
step prof_dirty 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_prof_dirty" -o run --output-format csv -- python3 "$ROOT/scripts/bench_dirty.py" --mib 1024 --steps 5
step prof_bench 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_prof_bench" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-host
echo ALLDONE
