cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x --timeout 300 -p no:cacheprovider > gpurun_out/t13_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/t13_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-batch > gpurun_out/t13_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/t13_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('clean', d['value'], d['encode_ms'], d['decode_ms'])"
timeout -k 10 300 python scripts/bench_dirty.py --mib 1024 > gpurun_out/t13_dirty.log 2>&1 || exit $?
grep '^{' gpurun_out/t13_dirty.log
