#!/bin/bash
# GPU box: the GPU test suite, then the 600-stream decoder ingress stress
# (tests/tools/stress_ingress.py, ITERS repetitions).  Each step has its own
# time limit; a step that times out, crashes or is killed ends the script (a
# plain test failure, exit 1, does not).
mkdir -p gpurun_out
step() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
TAG=${TAG:-r02}
if [ -z "$NO_TESTS" ]; then
    step "${TAG}_pytest_gpu" 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
fi
step "${TAG}_stress_ingress" 600 python -u tests/tools/stress_ingress.py "${ITERS:-30}"
