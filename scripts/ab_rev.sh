#!/bin/bash
# A/B build of the product library with b64x_kernels.hip taken from a git
# revision (the host objects are the working tree's):
#   scripts/ab_rev.sh NAME REV  ->  build/variants/NAME/libasync_b64.so
# scripts/ab_time.py times it against the working tree's library.
set -e
cd "$(dirname "$0")/.."
make -s async_amd/libasync_b64.so
name=$1; rev=$2
d=build/variants/$name
mkdir -p "$d"
git show "$rev":async_amd/csrc/b64x_kernels.hip > "$d/k.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC \
    -Iasync_amd/csrc -Iinclude -Wno-pass-failed -mllvm -amdgpu-kernarg-preload-count=16 -c "$d/k.hip" -o "$d/k.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$d/libasync_b64.so" "$d/k.o" \
    build/fsalloc.o build/loop.o build/streams.o build/framing.o build/fdstreams.o build/b64_hub.o \
    build/b64_stages.o build/b64_pin.o \
    -Wl,-soname,libasync_b64.so
rm -f "$d/k.o" "$d/k.hip"
echo "$d/libasync_b64.so"
