"""Fused GAT projection (gnn_gat_project_f32) vs torch.mm + gnn_gat_logits_f32 at cfg3 shape.

    python tools/project_probe.py [--n 1000000] [--k 64] [--heads 8] [--fh 8]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--fh", type=int, default=8)
    a = ap.parse_args()
    from graphneuralnetwork_amd.ops import gat_logits, gat_project
    dev = torch.device("cuda:0")
    F = a.heads * a.fh
    x = torch.randn(a.n, a.k, device=dev)
    w = torch.randn(a.k, F, device=dev) / a.k ** 0.5
    s, d = torch.randn(F, device=dev), torch.randn(F, device=dev)
    wh = torch.mm(x, w)
    res = {"fused_ms": timeit(lambda: gat_project(x, w, a.heads, a.fh, s, d)),
           "mm_ms": timeit(lambda: torch.mm(x, w)),
           "logits_ms": timeit(lambda: gat_logits(wh, a.heads, a.fh, s, d))}
    res["bytes_min"] = a.n * (a.k + F + 2 * a.heads) * 4
    res["fused_GBps"] = res["bytes_min"] / res["fused_ms"] / 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    main()
