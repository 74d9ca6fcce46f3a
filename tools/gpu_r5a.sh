# round-5 GPU pass: the GPU suite (up to 10 failures reported), then the profile round
# (per-instance PMC + SQ) with the default bench line, the GAT schedule / pipeline A/B and the
# sampler probe; a failing GPU step ends the script
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
  > gpurun_out/r5a_gpu_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r5a_gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # a crash / timeout ends the call; test failures do not
TAG=r5a SQ=1 bash tools/profile_round.sh > gpurun_out/profile_round_r5a.log 2>&1 && \
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 30 --libs gatpipe2 > gpurun_out/r5b_gat_tasks_ab.log 2>&1 && \
timeout -k 10 300 python3 -u tools/sample_probe.py --reps 30 > gpurun_out/r5b_sample_probe.log 2>&1
