#!/bin/bash
# GPU box: config 5's pass-to-pass spread: K passes
# back to back at 1 and 16 loops without the hub trace (the bench's
# conditions), then 1 loop with the phase rows.  TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-c5}
K=${K:-6}
for T in 1 16; do
  timeout -k 10 400 python -u scripts/cfg5_profile.py gpurun_out/${TAG} --passes $K --threads $T --no-prof --no-trace > gpurun_out/${TAG}_t${T}.log 2>&1
  rc=$?; tail -n $K gpurun_out/${TAG}_t${T}.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u scripts/cfg5_profile.py gpurun_out/${TAG}_trace --passes $K --threads 1 --no-prof > gpurun_out/${TAG}_trace.log 2>&1
rc=$?; tail -n $K gpurun_out/${TAG}_trace.log | cut -c1-400; exit $rc
