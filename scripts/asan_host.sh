#!/bin/bash
# Host-side AddressSanitizer + UBSan run of the C code (event loop, streams,
# framing, stages, batching hub; the HIP kernels are built as usual -- GPU
# sanitizers are not available).  Builds an instrumented copy under
# build_asan/ and runs the CPU tests there; with `gpu` also the GPU stage,
# session and egress tests (host sanitizers only; LD_PRELOAD of gcc's
# libasan/libubsan, leak checking off: the HIP runtime keeps its mappings).
#   scripts/asan_host.sh [gpu]
set -e
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
B="$ROOT/build_asan"
if [ ! -f "$B/async_amd/libasync_b64.so" ] || [ -n "$(find "$ROOT/async_amd/csrc" "$ROOT/include" "$ROOT/tests/csrc" -newer "$B/async_amd/libasync_b64.so" -name '*.[ch]*' | head -1)" ]; then
  rm -rf "$B" && mkdir -p "$B"
  cp -r "$ROOT/include" "$ROOT/async_amd" "$ROOT/tests" "$ROOT/oracle" "$ROOT/Makefile" "$ROOT/INTEGRATION.md" "$ROOT/bench.py" "$B/"
  rm -rf "$B/build" "$B"/async_amd/*.so "$B"/oracle/*.so "$B"/tests/csrc/*.so
  sed -i 's/^CFLAGS    = -O2 /CFLAGS    = -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer /' "$B/Makefile"
  make -C "$B" -j8 >/dev/null
fi
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:protect_shadow_gap=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
# prepended to any preload already in the environment, which stays in place
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+:$LD_PRELOAD}"
cd "$B"
if [ "$1" = gpu ]; then
  LD_PRELOAD="$PRE" timeout -k 10 600 python -u -m pytest tests/test_stages_gpu.py \
      tests/test_session_gpu.py tests/test_egress_gpu.py -x -q -m gpu --timeout 300 \
      --timeout-method thread -p no:cacheprovider
else
  LD_PRELOAD="$PRE" timeout -k 10 900 python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider
fi
