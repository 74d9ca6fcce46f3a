# round-5 GPU pass r: GAT aggregation traffic per variant (FETCH_SIZE, WRITE_SIZE, L2 hits):
# er gathered (main), er from the rows (--rec), the no-er probe library
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for v in "main:" "rec:--rec" "noer:--lib noer"; do
  name=${v%%:*}; args=${v#*:}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/r5r_${name}_fetch -o run -- python3 -u tools/gat_variant_run.py $args > gpurun_out/r5r_${name}_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/prof/r5r_${name}_write -o run -- python3 -u tools/gat_variant_run.py $args > gpurun_out/r5r_${name}_write.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r5r_${name}_stats -o run -- python3 -u tools/gat_variant_run.py $args > gpurun_out/r5r_${name}_stats.log 2>&1 || exit 1
done
find gpurun_out/prof/r5r_* -type f ! -name '*kernel_stats.csv' ! -name '*counter_collection.csv' -delete 2>/dev/null
exit 0
