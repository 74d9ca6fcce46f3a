# round-5 second GPU pass: the GAT schedule / pipeline A/B, the sampler probe (eager timing and a
# rocprofv3 kernel trace of the 3-launch batch); stops at the first failure
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 30 --libs gatpipe2 > gpurun_out/r5b_gat_tasks_ab.log 2>&1 && \
timeout -k 10 300 python3 -u tools/sample_probe.py --reps 30 > gpurun_out/r5b_sample_probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r5b_sample -o run -- \
  python3 -u tools/sample_probe.py --reps 10 > gpurun_out/r5b_sample_probe_prof.log 2>&1
find gpurun_out/prof/r5b_sample -type f ! -name '*kernel_stats.csv' -delete 2>/dev/null
exit 0
