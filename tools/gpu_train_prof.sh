# kernel stats of the benchmarked training steps (cfg2 GCN layer, cfg3 GAT block):
# rocprofv3 --kernel-trace --stats of tools/train_step_probe.py, one run per model
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for m in gcn gat; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/train_prof_$m -o run --output-format csv -- python3 $R/tools/train_step_probe.py --model $m --steps 10 > $R/gpurun_out/train_prof_$m.log 2>&1 || exit $?
done
