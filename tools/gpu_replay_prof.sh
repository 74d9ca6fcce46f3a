# per-kernel times of each SpMM replay variant (rocprofv3 --kernel-trace --stats, one run each)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6e
cd /tmp
for wl in cfg2 ns; do
  for v in a_as_built b_hub_to_L2_table c_hub_to_one_row d_all_to_L2_table; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6e/prof_${wl}_$v -o run --output-format csv -- python3 $R/tools/spmm_replay.py --workload $wl --reps 5 --only $v > $R/gpurun_out/r6e/replay_${wl}_$v.log 2>&1 || exit $?
  done
done
