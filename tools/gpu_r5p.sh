# round-5 GPU pass p: the er-recomputing GAT kernels as their own instances (tests, A/B against
# the pre-change kernels and the chunk-slot / pipelining variants)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gat_gpu.py tests/test_training_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5p_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 40 --libs gatr5j,recslots4+rec,recpipe+rec > gpurun_out/r5p_gat_ab.log 2>&1
