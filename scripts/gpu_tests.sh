#!/bin/bash
# GPU box: smoke, then the GPU test suite, each under its own time limit;
# stops at the first step that crashes or times out.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
TAG=${TAG:-t}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.log; exit $rc
