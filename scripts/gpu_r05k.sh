#!/bin/bash
# GPU box: host copy rates, then the host_fd leg with the split copy on and off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-k}
timeout -k 10 200 ./tests/tools/host_copy_rate > gpurun_out/${TAG}_copy_rate.jsonl 2>&1
rc=$?; cat gpurun_out/${TAG}_copy_rate.jsonl; [ $rc -ne 0 ] && exit $rc
for t in 2 0 2 0; do
  ASYNC_B64_COPY_THREADS=$t timeout -k 10 300 python -u scripts/host_fd_only.py > gpurun_out/${TAG}_fd_t$t.log 2>&1
  rc=$?; echo "threads $t: $(tail -1 gpurun_out/${TAG}_fd_t$t.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
