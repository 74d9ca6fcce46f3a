"""Probe: can N torch.distributed 'nccl' (RCCL) ranks share ONE GPU on this box?

If yes, the bench's RCCL path (bench.py --gpus N, backend nccl) can be rehearsed on a one-GPU
box with GNN_BENCH_DEVICE=0. Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29541 tools/rccl_probe.py
Prints one line per rank: the all-to-all-v result check and the all_reduce result.
"""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", int(os.environ.get("GNN_BENCH_DEVICE", "0")))
torch.cuda.set_device(dev)
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
dist.init_process_group("nccl", device_id=dev)
t = torch.full((1,), float(rank + 1), device=dev)
dist.all_reduce(t)
# all-to-all-v: rank r sends (p + 1) rows of width 4 to peer p, valued 100 r + p
send_counts = [p + 1 for p in range(world)]
recv_counts = [rank + 1] * world
inp = torch.cat([torch.full((p + 1, 4), 100.0 * rank + p, device=dev) for p in range(world)])
out = torch.empty(sum(recv_counts), 4, device=dev)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    dist.all_to_all_single(out, inp, output_split_sizes=recv_counts, input_split_sizes=send_counts)
torch.cuda.current_stream(dev).wait_stream(s)
exp = torch.cat([torch.full((rank + 1, 4), 100.0 * q + rank, device=dev) for q in range(world)])
ok = bool(torch.equal(out, exp))
print(f"rank {rank}/{world}: all_reduce {t.item()} (expect {world * (world + 1) / 2}), "
      f"all_to_all_v ok={ok}", flush=True)
dist.barrier()
dist.destroy_process_group()
