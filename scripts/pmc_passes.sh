#!/bin/bash
# PMC counter passes over one Python workload: one counter group per
# rocprofv3 run (the per-block limits of MI355X_MICROARCH.md: at most 8 SQ_,
# 4 TCC_ -- FETCH_SIZE takes 3, WRITE_SIZE 2), --kernel-trace only, each pass
# under its own time limit; a failing pass ends the script.
#   scripts/pmc_passes.sh TAG script.py [args...]
# Output: gpurun_out/pmc_TAG/p<i>/ (summarise with scripts/summarize_pmc_sets.py).
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
SCRIPT="$ROOT/$1"; shift
cd /tmp && export TMPDIR=/tmp
# PMC_SETS="FETCH_SIZE;SQ_INSTS_VALU SQ_WAVES" runs only those sets
SETS=${PMC_SETS:-"SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SMEM;SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC;FETCH_SIZE;WRITE_SIZE"}
i=0
IFS=';' read -ra SETLIST <<< "$SETS"
for set in "${SETLIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$SCRIPT" "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc $TAG pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
