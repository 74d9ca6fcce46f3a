"""Order of the packed row tasks of pass 2 (the XCD-sliced SpMM's rest pass, bench.py's path).

The tasks are [begin, end) row ranges in row order; wave i of the task class takes task i and
workgroup w runs on XCD w % 8, so consecutive row ranges go to different XCDs. Each task is
independent, so the list can be permuted without changing any result. Variants:

  row      the builder's order
  blocked  XCD x gets the x-th eighth of the rows (consecutive ranges on one XCD)
  shuffle  a random permutation

    python tools/task_order_probe.py [--workload cfg2|ns] [--rounds 6]
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
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import seg_len_for
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, m = (1_000_000, 10_000_000) if a.workload == "cfg2" else (10_000_000, 100_000_000)
    F = 128
    s, d = rmat_edges(n, m, 0)
    ga = ops.column_order(gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev),
                                        n), F).graph
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    ref = ops.spmm_forward(ga, X).clone()
    seg = seg_len_for(F)
    xp = ga.xcd_hub_plan(ops.xcd_hub_rows_for(n, F), ops.XCD_MIN_DEG, min(ops.XCD_CHUNK, seg),
                         ops.XCD_PHASES, ops.XCD_ITEM_ROWS, ops.XCD_SMALL_ITEM)
    _, rest = xp.direct()
    tp = rest.task_plan(seg, ops.TASK_MAX_DEG, ops.TASK_COST)
    orig = tp.task_row.view(-1, 2).clone()
    T = orig.shape[0]
    p = torch.arange(T, device=dev)
    per = -(-T // 32) * 4                                    # tasks per XCD block, 4 | per
    chunks = [list(range(x * per, min(T, (x + 1) * per))) for x in range(8)]
    order = []
    for j in range(0, per, 4):                                # 4 tasks (one workgroup) per XCD
        for x in range(8):
            order += chunks[x][j:j + 4]
    blocked = torch.tensor(order, dtype=torch.int64, device=dev)
    assert blocked.numel() == T and int(torch.unique(blocked).numel()) == T
    g = torch.Generator(device="cpu").manual_seed(0)
    orders = {"row": p, "blocked": blocked, "shuffle": torch.randperm(T, generator=g).to(dev)}
    print(json.dumps({"workload": a.workload, "tasks": T, "mid_rows": tp.n_mid}), flush=True)
    times = {k: [] for k in orders}
    for r in range(a.rounds):
        for k, perm in orders.items():
            tp.task_row.view(-1, 2).copy_(orig[perm])
            ops.spmm_forward(ga, X, out=Y)
            torch.cuda.synchronize()
            if r == 0:
                print(json.dumps({k: "check", "bit_equal": bool(torch.equal(Y, ref))}), flush=True)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(5):
                ops.spmm_forward(ga, X, out=Y)
            ev[1].record()
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]) / 5)
    tp.task_row.view(-1, 2).copy_(orig)
    print(json.dumps({"median_ms": {k: round(statistics.median(t), 4) for k, t in times.items()}}))


if __name__ == "__main__":
    main()
