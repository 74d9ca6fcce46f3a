mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
GNN_BENCH_STACKS=90 NP=8 RT=560 bash tools/gpu_check.sh rehearse
