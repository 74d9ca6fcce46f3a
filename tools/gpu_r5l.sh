# round-5 GPU pass l: the er-recomputing GAT loop with two row buffers (tests, A/B), the scan
# probes, the cfg3 training step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gat_gpu.py tests/test_training_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5l_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 40 > gpurun_out/r5l_gat_er_ab.log 2>&1 && \
timeout -k 10 300 python3 -u tools/sample_probe.py --libs noticket,noemit > gpurun_out/r5l_sample_probe.log 2>&1 && \
timeout -k 10 300 python3 -u tools/train_step_probe.py --model gat > gpurun_out/r5l_train_gat.log 2>&1
