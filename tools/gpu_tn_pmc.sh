# counters of the weight-gradient kernel alone (tools/tn_probe.py), one rocprofv3 pass each
set -eo pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6u}
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/tools/tn_probe.py > $O/stats.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/sq -o run --output-format csv -- python3 $R/tools/tn_probe.py > $O/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/tools/tn_probe.py > $O/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $R/tools/tn_probe.py > $O/sq2.log 2>&1
find $O -type f ! -name '*kernel_stats.csv' ! -name '*counter_collection.csv' ! -name '*.log' -delete
