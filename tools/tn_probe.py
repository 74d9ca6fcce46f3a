"""The weight-gradient pass alone, for counter collection: gemm_tn over (Z, dY) with the column
sums of dY from its own loads (the x6 DB kernel of a GCN layer trained as (A X) W^T + b) at cfg2
size (1M x 128 x 128), --reps launches after one warm-up.

    python tools/tn_probe.py [--reps 10] [--masked]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--masked", action="store_true")
    a = ap.parse_args()
    import torch
    from graphneuralnetwork_amd.ops import gemm_tn, gemm_tn_masked
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    z = torch.randn(1_000_000, 128, device=dev, generator=gen)
    dy = torch.randn(1_000_000, 128, device=dev, generator=gen)
    h = torch.relu(torch.randn(1_000_000, 128, device=dev, generator=gen))
    run = (lambda: gemm_tn_masked(z, dy, h, 2.0, True, trans=True)) if a.masked else \
        (lambda: gemm_tn(z, dy, dy, trans=True))
    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        run()
    e.record()
    torch.cuda.synchronize()
    print(f"gemm_tn {'masked' if a.masked else 'DB'}: {s.elapsed_time(e) / a.reps:.4f} ms/launch")


if __name__ == "__main__":
    main()
