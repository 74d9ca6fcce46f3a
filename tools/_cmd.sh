mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k sage > gpurun_out/t_sage_dist.log 2>&1 && \
GNN_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --backend gloo --workload cfg4 --steps 5 --warmup 2 > gpurun_out/rehearse2_cfg4.log 2>&1
