#!/bin/bash
# GPU box: selected GPU tests (PYTEST_K, default the workspace/capture ones),
# then the batch-leg A/B (scripts/ab_batch.py) of the given library builds.
# Usage: TAG=x [ROUNDS=3] [PYTEST_K=expr] scripts/gpu_batch_ab.sh LIB...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-bab}
K=${PYTEST_K:-"workspace or capture or graph or strided"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python scripts/ab_batch.py --rounds ${ROUNDS:-3} ${ABARGS} "$@" > gpurun_out/${TAG}_ab.jsonl 2>&1
rc=$?; grep summary gpurun_out/${TAG}_ab.jsonl; [ $rc -ne 0 ] && exit $rc
echo ALLDONE
