#!/bin/bash
# Rebuilds round 5's first k_decode_suffix_held (commit d2beeb5, plain
# __syncthreads()) and the shipped kernels for gfx950 on the CPU, and prints
# what profiles/r06_isa_barrier_evidence.txt quotes: the loop-header block of
# k_decode_suffix_held<false> in the MIR before and after SIInsertWaitcnts,
# and tests/tools/isa_check.py's control-flow report on both code objects.
# No GPU; about a minute.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
trap 'rm -rf "$W"' EXIT
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -Wno-pass-failed -mllvm -amdgpu-kernarg-preload-count=16"
F=_ZN12_GLOBAL__N_120k_decode_suffix_heldILb0EEEvPKhmPhjNS_8DecAlphaEPvjP15b64x_dec_resultS7_jPj
git -C "$ROOT" show d2beeb5:async_amd/csrc/b64x_kernels.hip > "$W/b64x_kernels.hip"
git -C "$ROOT" show d2beeb5:include/b64x.h > "$W/b64x.h"
git -C "$ROOT" show d2beeb5:async_amd/csrc/b64x_result_check.h > "$W/b64x_result_check.h"
$HIPCC $FLAGS -I"$W" --offload-device-only -S -o /dev/null "$W/b64x_kernels.hip" \
    -mllvm -print-before=si-insert-waitcnts -mllvm -print-after=si-insert-waitcnts \
    -mllvm -filter-print-funcs=$F > "$W/mir.txt" 2>&1
$HIPCC $FLAGS -I"$W" -shared -o "$W/pre.so" "$W/b64x_kernels.hip" 2>/dev/null
python3 - "$W/mir.txt" <<'EOF'
import re, sys
txt = open(sys.argv[1]).read()
dumps = re.split(r"# \*\*\* IR Dump (Before|After) SI insert wait instructions.*\n", txt)
# dumps: ['', 'Before', body, 'After', body]
for tag, body in zip(dumps[1::2], dumps[2::2]):
    blocks = re.split(r"\n(?=bb\.\d+)", body)
    for b in blocks:
        # the loop header: the block whose barrier is followed by the ticket read
        if "S_BARRIER" in b and re.search(r"S_BARRIER\n(\s*S_WAITCNT_soft \d+\n)?\s*renamable \$vgpr\d+ = DS_READ_B32_gfx9 killed renamable \$vgpr\d+, 23176", b):
            lines = [l for l in b.split("\n") if not l.lstrip().startswith("liveins")]
            print(f"## MIR {tag.lower()} si-insert-waitcnts")
            print("\n".join(l[:150] for l in lines[:9]))
            break
EOF
echo
echo "## isa_check.py on the d2beeb5 build"
python3 "$ROOT/tests/tools/isa_check.py" "$W/pre.so" | grep -E "^barrier|^barriers"
echo
echo "## isa_check.py on the shipped library"
python3 "$ROOT/tests/tools/isa_check.py" "$ROOT/async_amd/libasync_b64.so" | grep -E "^barrier|^barriers|in flight"
