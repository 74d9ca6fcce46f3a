mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
GNN_BENCH_STACKS=60 NP=8 RT=400 BENCH_ARGS="--scale 0.02" bash tools/gpu_check.sh rehearse && \
GNN_BENCH_STACKS=60 NP=4 RT=400 BENCH_ARGS="--scale 0.1" bash tools/gpu_check.sh rehearse
