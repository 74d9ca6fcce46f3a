# round-5 GPU pass i: parallel gemm_tn partial reduction, GAT projection on the MFMA transform,
# 8192-word scan tiles; tests, the sampler probe, train-step probes, the default bench
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_gat_gpu.py tests/test_sampler_gpu.py tests/test_sage_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5i_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5i_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sample_probe.py > gpurun_out/r5i_sample_probe.log 2>&1 && \
timeout -k 10 300 python3 -u tools/train_step_probe.py --model gcn > gpurun_out/r5i_train_gcn.log 2>&1 && \
timeout -k 10 300 python3 -u tools/train_step_probe.py --model gat > gpurun_out/r5i_train_gat.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err
