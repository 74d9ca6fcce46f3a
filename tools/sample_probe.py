"""Time the cfg4 mini-batch sampler alone (8192 seeds, [25, 10], 10M-node R-MAT adjacency in
degree order, as bench.py run_sage): the fused sample_batch and the hop-by-hop path, HIP events
around each call, plus the host wall time per call. Run under rocprofv3 --kernel-trace --stats
for the per-kernel split.

    python tools/sample_probe.py [--reps 20] [--libs wpt1,wpt2]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--libs", default="", help="variant library tags timed beside the main "
                    "library (fused path only; lib/variants/libgnn_<tag>.so)")
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.build import LIB_DIR
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import (degree_ordered, sample_batch,
                                                sample_batch_stepwise, symmetric_adjacency)
    dev = torch.device("cuda:0")
    n = 10_000_000
    s, d = rmat_edges(n, 100_000_000, 0)
    adj = symmetric_adjacency(s, d, n, device=dev)
    del s, d
    adj, _, _ = degree_ordered(adj)
    gen = torch.Generator(device=dev).manual_seed(0)
    cand = torch.nonzero(adj.rowptr[1:] > adj.rowptr[:-1]).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    out = {}
    from graphneuralnetwork_amd import sampler as S

    def pending(*args, **kw):  # the sizes left on the device: the kernels' own time
        return sample_batch(*args, sync=False, **kw)

    runs = [("fused", sample_batch, None), ("stepwise", sample_batch_stepwise, None),
            ("fused_pending", pending, None)]
    for t in a.libs.split(","):
        if t:
            lib = LIB_DIR / "variants" / f"libgnn_{t}.so"
            runs += [(f"fused_{t}", sample_batch, lib), (f"fused_pending_{t}", pending, lib)]
    ref = sample_batch(adj, seeds, (25, 10), seed=0)
    for name, fn, lib in runs:
        _lib.use_variant(lib)
        S._SAMPLE_WS.clear()  # a variant's scan may size its workspace differently
        b = fn(adj, seeds, (25, 10), seed=0).sync()
        assert torch.equal(b.frontier, ref.frontier) and torch.equal(b.neigh_map, ref.neigh_map)
        for _ in range(3):
            fn(adj, seeds, (25, 10), seed=0)
        torch.cuda.synchronize()
        ev, wall = [], []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            fn(adj, seeds, (25, 10), seed=0)
            e1.record()
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e3)
            ev.append(e0.elapsed_time(e1))
        out[name] = {"event_ms": round(statistics.median(ev), 4),
                     "wall_ms": round(statistics.median(wall), 4)}
    _lib.use_variant(None)
    S._SAMPLE_WS.clear()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
