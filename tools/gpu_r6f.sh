# training-step kernel traces (degree order) + gemm_tn tests after the M = 16 shape
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6f
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_training_gpu.py tests/test_gat_gpu.py -p no:cacheprovider > $R/gpurun_out/r6f/pytest.log 2>&1 || { tail -30 $R/gpurun_out/r6f/pytest.log; exit 1; }
tail -2 $R/gpurun_out/r6f/pytest.log
cd /tmp
for m in gcn gat; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f/train_prof_$m -o run --output-format csv -- python3 $R/tools/train_step_probe.py --model $m --steps 10 > $R/gpurun_out/r6f/train_prof_$m.log 2>&1 || exit $?
  grep median $R/gpurun_out/r6f/train_prof_$m.log
done
