"""One SageLayer-shaped transform (relu(X W^T), X [M, 256] -> 128, the cfg4 layer-0 GEMM) run
REPS times, for rocprofv3 --pmc passes on gcn_transform_kernel alone.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... -- python3 tools/transform_pmc.py [M K N]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from graphneuralnetwork_amd.ops import gcn_transform
    m, k, n = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (61771, 256, 128)))
    dev = torch.device("cuda:0")
    x = torch.randn(m, k, device=dev)
    w = torch.randn(n, k, device=dev) / k ** 0.5
    for _ in range(20):
        gcn_transform(x, w, relu=True)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
