cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t25_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/t25_pytest.log; exit $rc
