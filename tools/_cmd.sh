set -o pipefail
O=gpurun_out/r02z; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_dist_prof.log 2>&1 || exit $?
GNN_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/rehearse2_prof.log 2>&1 || exit $?
