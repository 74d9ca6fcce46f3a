# round 6 (late): the hidden GAT dropout fused into the heads' op -- the whole GPU suite (torch
# seeded per test now), then the model A/B
set -o pipefail
mkdir -p gpurun_out/r6y
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6y/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r6y/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  timeout -k 10 200 python3 -u -c "
import sys, runpy
from graphneuralnetwork_amd import gat
gat.GAT_FUSE_OUT_DROPOUT = bool($v)
sys.argv = ['train_step_probe.py', '--model', 'gat_model', '--steps', '20']
runpy.run_path('tools/train_step_probe.py', run_name='__main__')
" >> gpurun_out/r6y/ab.log 2>&1 || exit $?
  echo "fuse=$v $(tail -1 gpurun_out/r6y/ab.log)"
done
