# round-5 GPU pass s: scan tile size A/B (words per thread 4 / 2 / 1) on the cfg4 sampler
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/sample_probe.py --reps 30 --libs wpt2,wpt1 > gpurun_out/r5s_scan_wpt_ab.log 2>&1
