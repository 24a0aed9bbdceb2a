#!/bin/bash
# GPU box: the host_fd leg at several stage block sizes (ASYNC_B64_STAGE_CAPACITY).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-cap}
for c in ${CAPS:-1048576 4194304 8388608}; do
  ASYNC_B64_STAGE_CAPACITY=$c timeout -k 10 300 python -u scripts/host_fd_only.py > gpurun_out/${TAG}_$c.log 2>&1
  rc=$?; echo "cap $c: $(tail -1 gpurun_out/${TAG}_$c.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
