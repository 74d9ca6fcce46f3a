# round-5 GPU pass r: GAT backward row pass without the mask code, edges in flight per lane
# (row / node pass) A/B; GAT GPU tests first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gat_gpu.py tests/test_training_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5r_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/gat_bwd_probe.py --reps 15 --short 8 --libs nodropt,rowu4,nodeu8,nodeu2 > gpurun_out/r5r_gat_bwd_ab.log 2>&1
