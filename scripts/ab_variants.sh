#!/bin/bash
# A/B builds of the product library with compile-time tuning constants
# (never the shipped defaults' replacement until measured):
#   scripts/ab_variants.sh NAME "-DB64X_LINES_U=4 ..."  ->  build/variants/NAME/libasync_b64.so
# scripts/ab_time.py times them against each other on the GPU box.
set -e
cd "$(dirname "$0")/.."
make -s async_amd/libasync_b64.so
name=$1; shift
d=build/variants/$name
mkdir -p "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC \
    -Iasync_amd/csrc -Iinclude -Wno-pass-failed -mllvm -amdgpu-kernarg-preload-count=16 $* -c async_amd/csrc/b64x_kernels.hip -o "$d/k.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$d/libasync_b64.so" "$d/k.o" \
    build/fsalloc.o build/loop.o build/streams.o build/framing.o build/fdstreams.o build/b64_hub.o \
    build/b64_stages.o build/b64_pin.o \
    -Wl,-soname,libasync_b64.so
rm -f "$d/k.o"
echo "$d/libasync_b64.so"
