cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --size 268435456 > gpurun_out/t14_mr.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/t14_mr.log | tail -5; exit $rc
