# narrow gemm_tn / padded out_att / own-gather permutes: tests + whole-model kernel traces
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_training_gpu.py tests/test_gat_gpu.py -p no:cacheprovider > $R/gpurun_out/r6j/pytest.log 2>&1 || { tail -40 $R/gpurun_out/r6j/pytest.log; exit 1; }
tail -1 $R/gpurun_out/r6j/pytest.log
cd /tmp
for m in gcn_model gat_model; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6j/prof_$m -o run --output-format csv -- python3 $R/tools/train_step_probe.py --model $m --steps 10 > $R/gpurun_out/r6j/$m.log 2>&1 || exit $?
  grep median $R/gpurun_out/r6j/$m.log
done
