mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TT=600 bash tools/gpu_check.sh tests smoke bench
