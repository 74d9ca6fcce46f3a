mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq_gat -o run -- python bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq_gat.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq_spmm -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-layer > gpurun_out/pmc_sq_spmm.log 2>&1
