"""Interleaved A/B of the inference SageLayer GEMM relu(buf @ W^T), buf = [M, 2F] (the
[self | mean of neighbours] cat buffer, GraphSAGE/GraphSAGE.py:18-20): hipBLASLt
(torch._addmm_activation) vs the hand-written fp32-MFMA kernel (gnn_linear_relu_f32),
and the plain GCN transform shapes as a regression check.

    python tools/sage_gemm_ab.py [--rows 8192,32768,62479,200000]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="8192,32768,62479,200000")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--big", action="store_true", help="also 10M x 128 -> 128 and 10M x 256 -> 256")
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gcn_transform
    _lib.load()
    dev = torch.device("cuda:0")
    shapes = [(m, 256, 128, True) for m in (int(v) for v in args.rows.split(","))]
    shapes += [(1_000_000, 128, 128, False), (1_000_000, 256, 128, False)]
    if args.big:
        shapes += [(10_000_000, 128, 128, False), (10_000_000, 256, 256, False)]
    for M, K, N, relu in shapes:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) / K ** 0.5
        zero = torch.zeros(N, device=dev)
        y_lib = torch.empty(M, N, device=dev)
        y_mf = torch.empty(M, N, device=dev)
        if relu:
            lib = lambda: torch._addmm_activation(zero, x, W.t())  # noqa: E731
        else:
            lib = lambda: torch.mm(x, W.t(), out=y_lib)  # noqa: E731
        mf = lambda: gcn_transform(x, W, relu=relu, out=y_mf)  # noqa: E731
        ref = lib()
        err = float((mf() - ref).abs().max() / ref.abs().max())
        times = {"hipblaslt": [], "mfma": []}
        for _ in range(args.rounds):
            for name, fn in (("hipblaslt", lib), ("mfma", mf)):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fn()
                a.record()
                for _ in range(5):
                    fn()
                b.record()
                torch.cuda.synchronize()
                times[name].append(a.elapsed_time(b) / 5)
        flop = 2.0 * M * K * N
        print(json.dumps({"M": M, "K": K, "N": N, "relu": relu, "max_rel_err": err,
                          **{f"{k}_us": round(statistics.median(v) * 1e3, 2)
                             for k, v in times.items()},
                          **{f"{k}_TFs": round(flop / (statistics.median(v) / 1e3) / 1e12, 1)
                             for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
