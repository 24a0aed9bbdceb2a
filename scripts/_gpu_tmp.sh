cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t29_pytest.log 2>&1
rc=$?; tail -12 gpurun_out/t29_pytest.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for tn in 5:0 5:4; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dprof29_$tn -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_dirty.py --mib 1024 --tune $tn > $GRAFT_REPO_ROOT/gpurun_out/dprof29_$tn.log 2>&1 || exit $?
grep '^{' $GRAFT_REPO_ROOT/gpurun_out/dprof29_$tn.log
done
python3 - <<'P'
import csv,glob
for f in sorted(glob.glob('/root/repo/gpurun_out/dprof29_*/**/run_kernel_stats.csv',recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        if 'k_decode' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
P
