# round-5 GPU pass g: LDS-staged MFMA weight gradients, sampler host path; tests, the weight-
# gradient A/B, the GAT backward probe with SQ counters; a failing GPU step ends the script
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_gat_gpu.py tests/test_sampler_gpu.py tests/test_sage_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5g_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gemm_tn_ab.py --reps 30 > gpurun_out/r5g_gemm_tn_ab.log 2>&1 && \
timeout -k 10 300 python3 -u tools/sample_probe.py > gpurun_out/r5g_sample_probe.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --output-format csv -d gpurun_out/prof/r5g_sq -o run -- python3 -u tools/gat_bwd_probe.py --reps 3 > gpurun_out/r5g_sq.log 2>&1
rc=$?
find gpurun_out/prof/r5g_* -type f ! -name '*counter_collection.csv' -delete 2>/dev/null
exit $rc
