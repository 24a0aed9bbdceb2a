#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run, kernel-trace
# only) over the batch benchmark and a short bench.py, for per-kernel
# instruction / wait / traffic comparisons.  Output: gpurun_out/pmck/.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmck"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export K=2 KNOBS="${KNOBS:-4:0}"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SMEM" \
           "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/b$i" -o run -- python3 "$ROOT/scripts/bench_batch.py" > "$OUT/b$i.log" 2>&1
  rc=$?; echo "batch pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/f$i" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --batch-steps 1 > "$OUT/f$i.log" 2>&1
  rc=$?; echo "flat pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
