set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_gpu_suite.log 2>&1 && \
TAG=r5a SQ=1 bash tools/profile_round.sh > gpurun_out/profile_round_r5a.log 2>&1
