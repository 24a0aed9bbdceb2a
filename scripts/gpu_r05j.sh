#!/bin/bash
# GPU box: the decode tests that cover the MIME rows and the junk suffix,
# then the batch A/B and the junk legs of scripts/ab_time.py for two builds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-j}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "mime or rows or strided or fuzz or junk or suffix or single_pass or oracle" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/ab_batch.py --rounds 3 "$@" > gpurun_out/${TAG}_ab.jsonl 2>&1
rc=$?; grep summary gpurun_out/${TAG}_ab.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/ab_time.py --rounds 3 --only decode,crlf,junk,junk1,junk_ej "$@" > gpurun_out/${TAG}_junk.jsonl 2>&1
rc=$?; grep summary gpurun_out/${TAG}_junk.jsonl; exit $rc
