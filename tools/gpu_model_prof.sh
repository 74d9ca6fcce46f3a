# kernel traces of the whole-model training steps (GCN_Model / GAT at cfg2 / cfg3 sizes)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/${TAG:-r6i}
cd /tmp
for m in ${MODELS:-gcn_model gat_model}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG:-r6i}/prof_$m -o run --output-format csv -- python3 $R/tools/train_step_probe.py --model $m --steps 10 > $R/gpurun_out/${TAG:-r6i}/$m.log 2>&1 || exit $?
  grep median $R/gpurun_out/${TAG:-r6i}/$m.log
done
