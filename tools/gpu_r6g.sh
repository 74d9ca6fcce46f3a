# full GPU suite + smoke + a 2-rank gloo rehearsal of the N-rank bench line (one GPU)
set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6g/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6g/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r6g/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6g/smoke.log 2>&1 || { cat gpurun_out/r6g/smoke.log; exit 1; }
grep smoke gpurun_out/r6g/smoke.log
GNN_BENCH_DEVICE=0 GNN_BENCH_DETAIL=gpurun_out/r6g/bench_detail_n2.json timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --scale 0.25 > gpurun_out/r6g/rehearse2.json 2> gpurun_out/r6g/rehearse2.err || { tail -30 gpurun_out/r6g/rehearse2.err; exit 1; }
wc -c gpurun_out/r6g/rehearse2.json
python -c "import json; d=json.load(open('gpurun_out/r6g/rehearse2.json')); print(d['n_gpus'], d['value'], d.get('phases_ms_max'))"
