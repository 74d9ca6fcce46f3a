# round-5 GPU pass f: fp32-MFMA weight gradients and the leaner row / node passes of the GAT
# backward: their tests, then the A/B probes; a failing GPU step ends the script
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_gat_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5f_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gemm_tn_ab.py --reps 30 > gpurun_out/r5f_gemm_tn_ab.log 2>&1 && \
timeout -k 10 300 python3 -u tools/gat_bwd_probe.py --reps 15 --short 4,8,16 > gpurun_out/r5f_gat_bwd_probe.log 2>&1
