# round-5 GPU pass u: GAT backward node pass with dropout as a template flag (tests; A/B against
# the committed node kernel; the GAT and GCN training steps)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gat_gpu.py tests/test_training_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5u_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/gat_bwd_probe.py --reps 15 --short 8 --libs dropold > gpurun_out/r5u_gat_bwd_ab.log 2>&1 &&
timeout -k 10 300 python3 -u tools/train_step_probe.py --model gat --steps 20 > gpurun_out/r5u_train.log 2>&1 &&
timeout -k 10 300 python3 -u tools/train_step_probe.py --model gcn --steps 20 >> gpurun_out/r5u_train.log 2>&1
