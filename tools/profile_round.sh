#!/bin/bash
# Round-end profiles: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE / L2 hit passes of the
# bench command of every single-GPU workload (tools/profile_workload.sh), then the default
# bench line. Stops at the first failure.
set -eo pipefail
mkdir -p gpurun_out
for wl in cfg2 ns cfg3 cfg4; do
  echo "== profile $wl ($(date +%T))"
  bash tools/profile_workload.sh "r3_$wl" --workload "$wl"
done
echo "== default bench ($(date +%T))"
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo "== done ($(date +%T))"
