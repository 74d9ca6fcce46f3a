"""Probe: do the memory-bound SpMM and the MFMA-bound transform overlap when launched on two
streams at once? (timing only -- independent data, no dependency between them)

If the pair takes about max(SpMM, GEMM) rather than their sum, a Graph_conv_layer whose
SpMM row blocks feed the transform of finished blocks ((A X) W^T, F_in <= F_out) can hide the
GEMM behind the aggregation.

    python tools/layer_overlap_probe.py --workload cfg5     (GPU)
Variants of the transform: the main library's, plus lib/variants/libgnn_ovl_<tag>.so built with
    python tools/layer_overlap_probe.py --build
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
VARIANTS = {"two128": ["GNN_TF_ONE256=0"]}


def ev_time(fn, reps=5):
    import torch
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--workload", default="cfg5")
    ap.add_argument("--chunks", default="1,4")
    a = ap.parse_args()
    if a.build:
        from graphneuralnetwork_amd.build import build_variant
        for n, d in VARIANTS.items():
            print(build_variant("ovl_" + n, d, only=["transform.hip"]))
        return
    import torch
    import bench
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.ops import column_order, gcn_transform, spmm_forward
    dev = torch.device("cuda:0")
    _lib.load()
    wl = bench.WORKLOADS[a.workload]
    F = wl.get("feat", 128)
    g = bench.build_graph(wl["nodes"], wl["edges"], dev, 0, 1)
    order = column_order(g, F)
    ga = g if order is None else order.graph
    X = torch.randn(g.n_cols, F, device=dev)
    Y = torch.empty(g.n_rows, F, device=dev)
    W = torch.randn(F, F, device=dev) / F ** 0.5
    S = torch.empty(g.n_rows, F, device=dev)
    spmm = lambda: spmm_forward(ga, X, None, out=Y)  # noqa: E731
    spmm()
    torch.cuda.synchronize()
    s1 = torch.cuda.Stream(dev)
    libs = {"main": None}
    vdir = ROOT / "graphneuralnetwork_amd" / "lib" / "variants"
    for n in VARIANTS:
        p = vdir / f"libgnn_ovl_{n}.so"
        if p.exists():
            libs[n] = p
    res = {"workload": a.workload, "F": F, "nnz": g.nnz}
    res["spmm_ms"] = ev_time(spmm)
    for name, path in libs.items():
        if path is not None:
            _lib.use_variant(path)
        else:
            _lib.use_variant(None)
        for nch in [int(c) for c in a.chunks.split(",")]:
            bounds = [g.n_rows * i // nch for i in range(nch + 1)]

            def gemm():
                for i in range(nch):
                    r0, r1 = bounds[i], bounds[i + 1]
                    y = gcn_transform(X[r0:r1], W, out=S[r0:r1])
                    assert y is not None

            gemm()
            t_gemm = ev_time(gemm)

            def both():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                with torch.cuda.stream(s1):
                    gemm()
                spmm()
                cur.wait_stream(s1)

            t_both = ev_time(both)

            def both_rev():  # the GEMM enqueued first
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                spmm_done = torch.cuda.Event()
                with torch.cuda.stream(s1):
                    spmm()
                    spmm_done.record(s1)
                gemm()
                cur.wait_event(spmm_done)

            t_rev = ev_time(both_rev)
            res[f"{name}_chunks{nch}"] = {"gemm_ms": round(t_gemm, 3), "both_ms": round(t_both, 3),
                                          "both_gemm_first_ms": round(t_rev, 3),
                                          "sum_ms": round(t_gemm + res["spmm_ms"], 3)}
            print(json.dumps(res), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
