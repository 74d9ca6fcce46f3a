# round-5 first GPU pass: the GPU suite, the profile round (per-instance PMC + SQ) and the
# default bench line (tools/profile_round.sh); stops at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5a_gpu_suite.log 2>&1 && \
TAG=r5a SQ=1 bash tools/profile_round.sh > gpurun_out/profile_round_r5a.log 2>&1
