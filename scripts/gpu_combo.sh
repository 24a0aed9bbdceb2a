#!/bin/bash
# GPU box: the GPU tests of the files named in $TESTS, the junk-decode A/B
# of the libraries given, PMC passes of the first NPMC of them, then the
# config-5 phase profile -- each step under its own limit, stopping at the
# first failure.   TAG=x TESTS="tests/a.py tests/b.py" scripts/gpu_combo.sh LIB...
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
TAG=${TAG:-combo}
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ $# -gt 0 ]; then
  timeout -k 10 700 python scripts/ab_time.py --rounds ${ROUNDS:-3} --steps ${STEPS:-10} \
      --only "${ONLY:-decode,crlf,junk,junk1,junk_ej}" "$@" > gpurun_out/${TAG}_ab.jsonl 2>&1
  rc=$?; grep summary gpurun_out/${TAG}_ab.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_ab.jsonl; exit $rc; }
  i=0
  for lib in "${@:1:${NPMC:-0}}"; do
    i=$((i+1))
    timeout -k 10 400 bash scripts/pmc_passes.sh ${TAG}_lib$i scripts/junk_decode_once.py "$lib" || exit $?
  done
fi
if [ -n "$CFG5" ]; then
  timeout -k 10 300 python -u scripts/cfg5_profile.py gpurun_out/${TAG}_cfg5 > gpurun_out/${TAG}_cfg5.log 2>&1
  rc=$?; head -5 gpurun_out/${TAG}_cfg5.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_cfg5.log; exit $rc; }
fi
echo ALLDONE
