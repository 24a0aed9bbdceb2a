#!/bin/bash
# A/B build of the product library from a patched copy of b64x_kernels.hip
# (pricing and experiment forms stay out of the product source):
#   scripts/ab_src.sh NAME FILE.hip  ->  build/variants/NAME/libasync_b64.so
set -e
cd "$(dirname "$0")/.."
make -s async_amd/libasync_b64.so
name=$1; src=$2
d=build/variants/$name
mkdir -p "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC \
    -Iasync_amd/csrc -Iinclude -Wno-pass-failed -mllvm -amdgpu-kernarg-preload-count=16 -c "$src" -o "$d/k.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$d/libasync_b64.so" "$d/k.o" \
    build/fsalloc.o build/loop.o build/streams.o build/framing.o build/fdstreams.o build/b64_hub.o \
    build/b64_stages.o build/b64_pin.o \
    -Wl,-soname,libasync_b64.so
rm -f "$d/k.o"
echo "$d/libasync_b64.so"
