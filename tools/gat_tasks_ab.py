"""A/B of the GAT aggregation at cfg3 (8 x 8 heads over the 1M / 10M R-MAT graph in the
column-degree order, as bench.py run_gat): the row classes (packed small rows + gat_short_kernel)
with er gathered or recomputed from the gathered Wh rows (a_dst, gnn_gat_csr_ex_f32), and with
--tasks the packed row tasks (gnn_gat_csr_tasks_f32, task cost 64 / 128 / 256 edges + rows,
degree threshold 16 / 32), interleaved in one process, HIP events per launch; outputs compared
with the row-class path.

    python tools/gat_tasks_ab.py [--reps 30] [--tasks] [--libs <variant tags>]

--libs: variant libraries (lib/variants/libgnn_<tag>.so, build.build_variant) timed with the
row-class schedule beside the main library (round 5: gatpipe2 = a depth-2 chunk pipeline, since
removed, profiles/r05b_gat_tasks_ab.log; the round-5 "noer" traffic probe, a wrong-result
switch, was removed from the product sources in round 6).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--libs", default="")
    ap.add_argument("--tasks", action="store_true", help="also the packed-task schedules")
    a = ap.parse_args()
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    s, d = rmat_edges(1_000_000, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), 1_000_000, device=dev)
    H, Fh, Fin = 8, 8, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(g.n_rows, Fin, device=dev, generator=gen)
    W = torch.randn(Fin, H * Fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    order = ops.gat_column_order(g, H, Fh)
    ga = order.graph
    wh, el, er = ops.gat_project(X, W, H, Fh, a_s, a_d, col_rows=order.inv)
    out = torch.empty_like(wh)
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.build import LIB_DIR
    variants = [("rowclass", False, 128, 16, None, False),
                ("rowclass_er_from_rows", False, 128, 16, None, True)]
    if a.tasks:
        variants += [("tasks_c64", True, 64, 16, None, False),
                     ("tasks_c128", True, 128, 16, None, False),
                     ("tasks_c256", True, 256, 16, None, False),
                     ("tasks_c128_d32", True, 128, 32, None, False)]
    for t in a.libs.split(","):  # "<tag>" or "<tag>+rec" (with a_dst: er from the rows)
        if t:
            tag, rec = t.split("+")[0], t.endswith("+rec")
            variants.append((f"rowclass_{t}", False, 128, 16,
                             LIB_DIR / "variants" / f"libgnn_{tag}.so", rec))

    current = {"lib": "unset"}

    def prep(v):  # outside the timed region: a library switch rebinds every symbol
        _, tasks, cost, deg, lib, rec = v
        ops.GAT_TASKS, ops.GAT_TASK_COST, ops.GAT_SHORT_MAX_DEG = tasks, cost, deg
        ops.GAT_ER_RECOMPUTE = rec
        if current["lib"] != lib:
            _lib.use_variant(lib)
            current["lib"] = lib

    def run(v):
        prep(v)
        return ops.gat_aggregate(ga, wh, el, er, H, Fh, 0.2, ops.GAT_DENSE, "elu", out=out,
                                 a_dst=a_d if v[5] else None)

    ref = run(variants[0]).clone()
    times = {v[0]: [] for v in variants}
    err = {}
    for v in variants:  # warm-up (plans) and the comparison
        y = run(v)
        torch.cuda.synchronize()
        err[v[0]] = float(((y - ref).abs().max() / ref.abs().max()).item())
    for _ in range(a.reps):
        for v in variants:
            prep(v)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v[0]].append(e0.elapsed_time(e1))
    print(json.dumps({k: {"median_ms": round(statistics.median(t), 4),
                          "max_rel_diff_vs_rowclass": err[k]} for k, t in times.items()}),
          flush=True)


if __name__ == "__main__":
    main()
