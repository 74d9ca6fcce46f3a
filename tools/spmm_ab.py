"""Interleaved A/B of SpMM kernel variants and long-row split sizes at one shape (one process).

    python tools/spmm_ab.py [--workload cfg2|ns] [--rounds 8]
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
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--variants", default="0,1,7")
    ap.add_argument("--seg-lens", default="")
    ap.add_argument("--seg-len", type=int, default=192)
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.ops import spmm_forward
    lib = _lib.load()
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if args.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = gcn_normalized_csr(s, d, n, device=dev)
    F = 128
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    ref = spmm_forward(g, X).clone()
    stream = torch.cuda.current_stream(dev)
    nbytes = g.nnz * (8 + 4 * F) + n * (8 + 4 * F)

    def run(variant, seg_len):
        p = g.plan(seg_len)
        partial = torch.empty((max(p.n_seg, 1), F), device=dev)
        rc = lib.gnn_dev_spmm_variant_f32(
            g.rowptr.data_ptr(), g.col.data_ptr(), g.val.data_ptr(), n, X.data_ptr(), F, F, None,
            Y.data_ptr(), F, p.seg_len, *p.args(), partial.data_ptr(), variant,
            stream.cuda_stream)
        _lib.check(rc, "variant")

    configs = [(v, args.seg_len) for v in map(int, args.variants.split(","))] + \
              [(0, int(sl)) for sl in args.seg_lens.split(",") if sl and int(sl) != args.seg_len]
    times = {c: [] for c in configs}
    for c in configs:  # correctness + warm-up
        run(*c)
        torch.cuda.synchronize()
        err = float((Y - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, (c, err)
    for _ in range(args.rounds):
        for c in configs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(3):
                run(*c)
            b.record(stream)
            torch.cuda.synchronize()
            times[c].append(a.elapsed_time(b) / 3)
    out = []
    for c, t in times.items():
        m = statistics.median(t)
        out.append({"variant": c[0], "seg_len": c[1], "median_ms": m, "min_ms": min(t),
                    "GBps": nbytes / (m / 1e3) / 1e9})
    for r in sorted(out, key=lambda r: r["median_ms"]):
        print(json.dumps(r))


if __name__ == "__main__":
    main()
