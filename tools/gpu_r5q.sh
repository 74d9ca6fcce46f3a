# round-5 GPU pass q: GAT er one chunk ahead of the rows (tests, A/B against the pre-change
# kernels in one process)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gat_gpu.py tests/test_training_gpu.py tests/test_fullsize_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5q_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 40 --libs gatr5j > gpurun_out/r5q_gat_ab.log 2>&1
