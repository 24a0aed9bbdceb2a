#!/bin/bash
# GPU box: the fd ingress junk test with the split copy off and on, then on
# the kernel variants (swapped in for the in-tree library, restored after).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-l}
run() {
  timeout -k 10 300 python -u -m pytest tests/test_fd_streams.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fd_decode_gpu" > gpurun_out/${TAG}_$1.log 2>&1
  rc=$?; echo "$1 rc $rc: $(tail -1 gpurun_out/${TAG}_$1.log)"
  return $rc
}
ASYNC_B64_COPY_THREADS=0 run cur_t0; [ $? -gt 1 ] && exit 1
ASYNC_B64_COPY_THREADS=2 run cur_t2; [ $? -gt 1 ] && exit 1
cp async_amd/libasync_b64.so /tmp/cur_lib.so
for v in cnt base; do
  cp build/variants/$v/libasync_b64.so async_amd/libasync_b64.so
  run $v; rc=$?
  cp /tmp/cur_lib.so async_amd/libasync_b64.so
  [ $rc -gt 1 ] && exit 1
done
ASYNC_B64_COPY_THREADS=0 run cur_t0b; [ $? -gt 1 ] && exit 1
exit 0
