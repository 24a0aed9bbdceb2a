#!/bin/bash
# GPU box: config 5 at 16 loops with the hub trace: K passes, arena
# allocations per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-c5t}
K=${K:-8}
timeout -k 10 400 python -u scripts/cfg5_profile.py gpurun_out/${TAG} --passes $K --threads 16 --no-prof > gpurun_out/${TAG}.log 2>&1
rc=$?; tail -n $K gpurun_out/${TAG}.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l[:200]); continue
    print({k: (round(v,4) if isinstance(v,float) else v) for k,v in d.items() if k in ('setup_s','loop_s','GiB_s','arena_allocs','hubs','batches','wake_s','gpu_span_s','launch_s','reserve_s','arenas_live_max_sum','pooled_before','pooled_after')})
"; exit $rc
