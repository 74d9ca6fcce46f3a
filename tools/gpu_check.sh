#!/bin/bash
# One GPU-box session. Usage: tools/gpu_check.sh <mode>...   modes: tests bench bench_ns prof pmc
# Each GPU step has its own time limit; a crash/timeout (exit >1) ends the script.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n ${TAILN:-25} "$OUT/$name.log"
  if [ $rc -gt 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for MODE in "$@"; do
  case $MODE in
    tests) step pytest_gpu ${TT:-1200} python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    testsk) step pytest_gpu_k 900 python -m pytest tests -m gpu -v -p no:cacheprovider -k "${K:-spmm}" ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 5 ;;
    gat_ab) step gat_ab 900 python tools/gat_ab.py ${GAT_AB_ARGS:-} ;;
    ab) step spmm_ab 900 python tools/spmm_ab.py --workload ${AB_WL:-cfg2} ${AB_ARGS:-} ;;
    bench_gat) step bench_gat 600 python bench.py --steps 20 --warmup 5 --workload cfg3 ;;
    bench_sage) step bench_sage 900 python bench.py --steps 20 --warmup 5 --workload cfg4 ;;
    bench_ns) step bench_ns 900 python bench.py --steps 20 --warmup 5 --workload ns ;;
    prof) step rocprof${PTAG:-} 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof${PTAG:-}" -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    pmc) step pmc_fetch${PTAG:-} 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch${PTAG:-}" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}
         step pmc_write${PTAG:-} 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write${PTAG:-}" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    rehearse2) GNN_BENCH_DEVICE=0 step rehearse2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 ;;
    rehearse) GNN_BENCH_DEVICE=0 step rehearse${NP:-4} ${RT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-4} --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${NP:-4} --backend gloo --steps 3 --warmup 1 ${BENCH_ARGS:-} ;;
    *) echo "unknown mode $MODE"; exit 2 ;;
  esac
done
