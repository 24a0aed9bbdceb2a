#!/bin/bash
# GPU box: host copy rates (tests/tools/host_copy_rate), then the host_fd leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-k}
timeout -k 10 200 ./tests/tools/host_copy_rate > gpurun_out/${TAG}_copy_rate.jsonl 2>&1
rc=$?; cat gpurun_out/${TAG}_copy_rate.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/host_fd_only.py > gpurun_out/${TAG}_fd.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_fd.log; exit $rc
