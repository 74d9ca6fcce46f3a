# round-5 GPU pass v: the GAT backward passes' counters on the final tree (FETCH / WRITE / L2,
# SQ) via tools/gat_bwd_probe.py
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r5v_stats -o run -- python3 -u tools/gat_bwd_probe.py --reps 3 > gpurun_out/r5v_stats.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/r5v_fetch -o run -- python3 -u tools/gat_bwd_probe.py --reps 3 > gpurun_out/r5v_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/prof/r5v_write -o run -- python3 -u tools/gat_bwd_probe.py --reps 3 > gpurun_out/r5v_write.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --output-format csv -d gpurun_out/prof/r5v_sq -o run -- python3 -u tools/gat_bwd_probe.py --reps 3 > gpurun_out/r5v_sq.log 2>&1
rc=$?
find gpurun_out/prof/r5v_* -type f ! -name '*kernel_stats.csv' ! -name '*counter_collection.csv' -delete 2>/dev/null
exit $rc
