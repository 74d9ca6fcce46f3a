#!/bin/bash
# Round-end profiles: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE / L2 hit passes (and,
# with SQ=1, an SQ wave-cycle pass) of the bench command of every single-GPU workload
# (tools/profile_workload.sh), then the default bench line. Stops at the first failure. TAG
# (default r5) prefixes the output directories; <TAG>_stamp.txt records bench.source_stamp()
# of the profiled tree (tools/summarize_profiles.py copies it into profiles/traffic_*.json).
set -eo pipefail
mkdir -p gpurun_out/prof
TAG=${TAG:-r5}
python3 -c "import bench; print(bench.source_stamp())" > "gpurun_out/prof/${TAG}_stamp.txt"
echo "== source stamp $(cat gpurun_out/prof/${TAG}_stamp.txt)"
for wl in ${WORKLOADS:-cfg2 ns cfg3 cfg4}; do
  echo "== profile $wl ($(date +%T))"
  bash tools/profile_workload.sh "${TAG}_$wl" --workload "$wl"
done
if [ -z "${NO_BENCH:-}" ]; then
  echo "== default bench ($(date +%T))"
  timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
fi
echo "== done ($(date +%T))"
