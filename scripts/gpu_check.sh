#!/bin/bash
# GPU box driver: smoke, GPU tests, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout (exit code
# other than 0 or 1) ends the script -- nothing more runs on the GPU.
# Usage: scripts/gpu_check.sh [pytest -k expr] [bench args...]
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
K="${1-not slow}"; shift || true
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "$ROOT/gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/device.txt
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -q -m gpu -k "$K" --timeout 600 -p no:cacheprovider
step bench 600 python bench.py --steps 20 --warmup 3 "$@"
cd /tmp && export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu
echo ALLDONE
