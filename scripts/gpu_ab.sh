#!/bin/bash
# GPU box: the GPU tests, then interleaved A/B (scripts/ab_time.py) of variant
# builds (scripts/ab_variants.sh), optionally the PMC passes of the MIME rows
# and lines decodes.  Usage: TAG=x [ROUNDS=3] [PMC=1] scripts/gpu_ab.sh LIB...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python scripts/ab_time.py --rounds ${ROUNDS:-3} "$@" > gpurun_out/${TAG}_ab.jsonl 2>&1
rc=$?; grep summary gpurun_out/${TAG}_ab.jsonl; [ $rc -ne 0 ] && exit $rc
if [ -n "$PMC" ]; then
  K=3 bash scripts/pmc_passes.sh ${TAG}_rows scripts/bench_batch_dirty.py || exit $?
  bash scripts/pmc_passes.sh ${TAG}_lines scripts/bench_dirty.py --mib 1024 --steps 3 || exit $?
fi
echo ALLDONE
