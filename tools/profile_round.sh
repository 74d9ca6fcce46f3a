#!/bin/bash
# Round-end profiles: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE / L2 hit passes of the
# bench command of every single-GPU workload (tools/profile_workload.sh), then the default
# bench line. Stops at the first failure. TAG (default r4) prefixes the output directories.
set -eo pipefail
mkdir -p gpurun_out
TAG=${TAG:-r4}
for wl in ${WORKLOADS:-cfg2 ns cfg3 cfg4}; do
  echo "== profile $wl ($(date +%T))"
  bash tools/profile_workload.sh "${TAG}_$wl" --workload "$wl"
done
if [ -z "${NO_BENCH:-}" ]; then
  echo "== default bench ($(date +%T))"
  timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
fi
echo "== done ($(date +%T))"
