#!/bin/bash
# GPU box: the GPU tests (unless NOTEST), then interleaved A/B timing of the
# junk-decode legs of variant builds.  TAG=x [ONLY=legs] scripts/gpu_junk_ab.sh LIB...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-jab}
if [ -z "$NOTEST" ]; then
  TAG=$TAG bash scripts/gpu_tests.sh || exit $?
fi
timeout -k 10 900 python scripts/ab_time.py --rounds ${ROUNDS:-3} --steps ${STEPS:-10} --only "${ONLY:-decode,junk,junk1,junk_ej,crlf_ej}" "$@" > gpurun_out/${TAG}_ab.jsonl 2>&1
rc=$?; grep summary gpurun_out/${TAG}_ab.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_ab.jsonl; exit $rc; }
echo ALLDONE
