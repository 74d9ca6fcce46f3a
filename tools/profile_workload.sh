#!/bin/bash
# rocprofv3 passes for one bench workload on the GPU box (run from the repo root):
#   1. --kernel-trace --stats            -> <out>/<tag>_stats/run_kernel_stats.csv
#   2. --pmc FETCH_SIZE                  -> <out>/<tag>_fetch/run_counter_collection.csv
#   3. --pmc WRITE_SIZE                  -> <out>/<tag>_write/run_counter_collection.csv
#   4. --pmc TCC_HIT_sum TCC_MISS_sum    -> <out>/<tag>_l2/run_counter_collection.csv
#   5. (SQ=1) --pmc 8 SQ counters        -> <out>/<tag>_sq/run_counter_collection.csv
#      (wave cycles split into waiting / issue-stalled / issuing, VALU / VMEM-read / SALU
#      instructions, waves: tools/summarize_profiles.py)
# Each counter pass is its own run (no trace domains beside --pmc), each under its own
# time limit; the script stops at the first failure.
#   tools/profile_workload.sh <tag> <bench args...>
set -eo pipefail
tag=$1
shift
out=gpurun_out/prof
mkdir -p "$out"
export TMPDIR=/tmp
bench=(python3 -u bench.py --steps 5 --warmup 2 --no-extras --no-cold --no-cpu-baseline --no-cpu-reference --no-layer --no-train --no-variants --no-replay "$@")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${tag}_stats" -o run -- "${bench[@]}" \
  > "$out/${tag}_stats.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/${tag}_fetch" -o run -- "${bench[@]}" \
  > "$out/${tag}_fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/${tag}_write" -o run -- "${bench[@]}" \
  > "$out/${tag}_write.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/${tag}_l2" -o run -- "${bench[@]}" \
  > "$out/${tag}_l2.log" 2>&1
if [ -n "${SQ:-}" ]; then
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --output-format csv -d "$out/${tag}_sq" -o run \
    -- "${bench[@]}" > "$out/${tag}_sq.log" 2>&1
fi
# keep only the summaries (the 64 MiB merge-back limit): stats + counter CSVs
find "$out" -path "*${tag}_*" -type f ! -name '*kernel_stats.csv' ! -name '*counter_collection.csv' \
  ! -name '*.log' -delete
find "$out" -path "*${tag}_*" -type f | sort | xargs ls -la
