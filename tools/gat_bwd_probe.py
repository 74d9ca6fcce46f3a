"""GAT backward passes at cfg3 (8 x 8 heads over the 1M / 10M R-MAT graph, symmetric normalised
adjacency, natural order as bench.py's gat_train_step): per-pass HIP-event medians of the two-pass
backward (row pass, recomputing node pass) for short-row degree bounds, and of the three-pass
backward, interleaved in one process.

    python tools/gat_bwd_probe.py [--reps 20] [--short 0,4,8,16] [--three] [--libs tags]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--short", default="8")
    ap.add_argument("--three", action="store_true")
    ap.add_argument("--libs", default="", help="variant library tags (lib/variants/libgnn_<tag>"
                    ".so) timed with the two-pass backward beside the main library")
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.build import LIB_DIR
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    s, d = rmat_edges(1_000_000, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), 1_000_000, device=dev)
    H, Fh = 8, 8
    gen = torch.Generator(device=dev).manual_seed(0)
    wh = torch.randn(g.n_rows, H * Fh, device=dev, generator=gen)
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    el, er = ops.gat_logits(wh, H, Fh, a_s, a_d)
    stats = torch.empty((g.n_rows, H), device=dev)
    y = ops.gat_aggregate(g, wh, el, er, H, Fh, 0.2, ops.GAT_DENSE, "elu", stats=stats)
    dy = torch.randn(g.n_rows, H * Fh, device=dev, generator=gen)
    variants = [(f"two_pass_short{k}", True, int(k), None) for k in a.short.split(",") if k != ""]
    if a.three:
        variants.append(("three_pass", False, 8, None))
    variants += [(f"two_pass_{t}", True, 8, LIB_DIR / "variants" / f"libgnn_{t}.so")
                 for t in a.libs.split(",") if t]

    def run(v, tl=None):
        _, rc, k, lib = v
        _lib.use_variant(lib)
        ops.GAT_BWD_RECOMPUTE, ops.GAT_BWD_SHORT_DEG = rc, k
        return ops.gat_backward(g, wh, el, er, stats, y, dy, a_s, a_d, H, Fh, 0.2,
                                ops.GAT_DENSE, True, timings=tl)

    ref = [t.clone() for t in run(variants[0])]
    err = {}
    for v in variants:
        out = run(v)
        torch.cuda.synchronize()
        err[v[0]] = max(float((o - r).abs().max() / r.abs().max().clamp_min(1e-30))
                        for o, r in zip(out, ref))
    per = {v[0]: {} for v in variants}
    for _ in range(a.reps):
        for v in variants:
            tl = []
            run(v, tl)
            torch.cuda.synchronize()
            for name, e0, e1 in tl:
                per[v[0]].setdefault(name, []).append(e0.elapsed_time(e1))
    print(json.dumps({k: {"per_pass_median_ms": {n: round(statistics.median(t), 4)
                                                  for n, t in p.items()},
                          "sum_ms": round(sum(statistics.median(t) for t in p.values()), 4),
                          "max_rel_diff_vs_first": err[k]} for k, p in per.items()}, indent=1),
          flush=True)


if __name__ == "__main__":
    main()
