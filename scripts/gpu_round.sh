#!/bin/bash
# GPU box: smoke + GPU tests (scripts/gpu_tests.sh), then one bench.py run
# and its rocprofv3 kernel-trace summary; each step under its own limit,
# stopping at the first failure.  TAG names the outputs under gpurun_out/.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${TAG:-r}
TAG=$TAG bash scripts/gpu_tests.sh || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 600 gpurun_out/${TAG}_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-host --no-cfg5 > "$ROOT/gpurun_out/${TAG}_prof.log" 2>&1
rc=$?; tail -3 "$ROOT/gpurun_out/${TAG}_prof.log"; exit $rc
