mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PTAG=_final bash tools/gpu_check.sh prof
