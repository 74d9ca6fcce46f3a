set -e
# 2-rank gloo rehearsals of the N-GPU bench flows on one GPU (times are host-staged and meaningless)
mkdir -p gpurun_out
for wl in cfg2 cfg3 cfg4; do
  GNN_BENCH_DEVICE=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951${#wl} bench.py --gpus 2 --backend gloo --scale 0.05 --steps 3 --warmup 1 --workload $wl > gpurun_out/${TAG:-r03v}_rehearse2_$wl.json 2> gpurun_out/${TAG:-r03v}_rehearse2_$wl.log
done
