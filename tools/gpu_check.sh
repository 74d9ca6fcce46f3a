#!/bin/bash
# One GPU-box session: gpu tests, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout (exit >1) ends the script.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -gt 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 20 --warmup 5
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline
fi
