set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/sage_gemm_forward_ab.py > gpurun_out/sage_gemm_fwd_ab.log 2>&1
