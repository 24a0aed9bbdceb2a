#!/bin/bash
# GPU box: the decode parity tests, the junk-decode A/B of variant builds,
# then PMC passes of the junk workload on the first NPMC (2) libraries
# (PMC_SETS: which counter sets, scripts/pmc_passes.sh).
#   TAG=x scripts/gpu_sfx_round.sh LIB_A LIB_B [LIB ...]
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
TAG=${TAG:-sfx}
if [ -z "$NOTEST" ]; then  # NOTEST=1: variants only, the product unchanged
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_decode_fuzz.py tests/test_stages_gpu.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 700 python scripts/ab_time.py --rounds ${ROUNDS:-3} --steps ${STEPS:-10} \
    --only "${ONLY:-decode,crlf,junk,junk1,junk_ej,crlf_ej,clean_ej}" "$@" > gpurun_out/${TAG}_ab.jsonl 2>&1
rc=$?; grep summary gpurun_out/${TAG}_ab.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_ab.jsonl; exit $rc; }
[ -n "$NOPMC" ] && exit 0
i=0
NPMC=${NPMC:-2}
for lib in "${@:1:$NPMC}"; do
  i=$((i+1))
  timeout -k 10 400 bash scripts/pmc_passes.sh ${TAG}_lib$i scripts/junk_decode_once.py "$lib" || exit $?
done
echo ALLDONE
