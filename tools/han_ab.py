"""A/B of HAN inference: the per-metapath GATConv path (one projection + one aggregation
launch per metapath) against HANLayer's block-diagonal batch (one of each for all
metapaths), on random dense metapath adjacencies (HAN/utils.py loads them dense).

    python tools/han_ab.py [--n 4000] [--deg 16] [--m 3] [--heads 8,8] [--rounds 20]
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
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--deg", type=int, default=16)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--fin", type=int, default=1870)
    ap.add_argument("--hidden", type=int, default=8)
    ap.add_argument("--heads", default="8,8")
    ap.add_argument("--rounds", type=int, default=20)
    args = ap.parse_args()
    from graphneuralnetwork_amd import han
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    n = args.n
    gs = []
    for _ in range(args.m):
        A = (torch.rand(n, n, device=dev) < args.deg / n).float()
        A.fill_diagonal_(1.0)  # metapath graphs keep the self-loop, so no row is edgeless
        gs.append(A)
    heads = [int(x) for x in args.heads.split(",")]
    net = han.HANModel(args.m, args.fin, args.hidden, 3, heads, dropout=0.6).to(dev).eval()
    h = torch.randn(n, args.fin, device=dev)
    res = {}
    with torch.no_grad():
        outs = {}
        for name, flag in (("batched", True), ("per_metapath", False)):
            han.BATCH_METAPATHS = flag
            for _ in range(3):
                outs[name] = net(gs, h)
            torch.cuda.synchronize()
            t = []
            for _ in range(args.rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                net(gs, h)
                e1.record()
                torch.cuda.synchronize()
                t.append(e0.elapsed_time(e1))
            res[name] = round(statistics.median(t), 4)
        han.BATCH_METAPATHS = True
        diff = float((outs["batched"] - outs["per_metapath"]).abs().max()
                     / outs["per_metapath"].abs().max())
    print(json.dumps({"n": n, "metapaths": args.m, "deg": args.deg, "heads": heads,
                      "forward_ms_median": res, "max_rel_diff": diff}), flush=True)


if __name__ == "__main__":
    main()
