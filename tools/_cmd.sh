set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gat_ab.py --variants base,c16u2,c32u2,c32u4,c64u4 --rounds 6 > gpurun_out/gat_chunk_slow.log 2>&1
timeout -k 10 400 python -u tools/hub_ab.py --op gat --workload cfg2 --feat 64 --ks 0,16384,65536,131072,262144 > gpurun_out/gat_hub_slow.log 2>&1
timeout -k 10 300 python -c "
import torch, time
x = torch.empty(2**28, device='cuda'); y = torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); t=time.time()
for _ in range(20): y.copy_(x)
torch.cuda.synchronize(); dt=(time.time()-t)/20; print('copy 1 GiB -> GB/s', 2*2**30/dt/1e9)
" > gpurun_out/copy_slow.log 2>&1
