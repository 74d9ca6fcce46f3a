# round 6 (late): hashed GAT model dropout -- its tests, then the GAT / GCN model steps A/B
set -o pipefail
mkdir -p gpurun_out/r6x
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dropout_gpu.py tests/test_gat_gpu.py tests/test_training_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r6x/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6x/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  timeout -k 10 200 python3 -u tools/train_step_probe.py --model gat_model --steps 20 --set HASHED_DROPOUT=$v >> gpurun_out/r6x/ab.log 2>&1 || exit $?
  tail -1 gpurun_out/r6x/ab.log
done
timeout -k 10 200 python3 -u tools/train_step_probe.py --model gcn_model --steps 20 >> gpurun_out/r6x/ab.log 2>&1 || exit $?
tail -1 gpurun_out/r6x/ab.log
