"""A/B in one process: the GCN transform in row order vs with its output rows scattered
(gnn_gcn_transform_rows_f32, out_rows = a random permutation, as a degree order's inv).

    python tools/transform_rows_ab.py [--shapes 1000000x128x128,10000000x128x128]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timed(fn, reps=10, rounds=5):
    out = []
    for _ in range(rounds):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / reps)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1000000x128x128,10000000x128x128,1000000x64x128")
    a = ap.parse_args()
    from graphneuralnetwork_amd.ops import gcn_transform
    dev = torch.device("cuda:0")
    for sh in a.shapes.split(","):
        m, k, f = (int(v) for v in sh.split("x"))
        x = torch.randn(m, k, device=dev)
        w = torch.randn(f, k, device=dev)
        y = torch.empty(m, f, device=dev)
        perm = torch.randperm(m, device=dev)
        r = {"shape": sh,
             "in_order_ms": timed(lambda: gcn_transform(x, w, out=y)),
             "scattered_ms": timed(lambda: gcn_transform(x, w, out=y, out_rows=perm,
                                                         check_rows=False)),
             "index_select_after_ms": timed(lambda: gcn_transform(x, w, out=y)[perm])}
        print(json.dumps(r), flush=True)
        del x, y, perm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
