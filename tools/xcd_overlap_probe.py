"""Would the two passes of the XCD-sliced hub SpMM overlap if run on two streams?

Timing-only probe (the outputs are not used): pass 1 (items, L2-bound) and pass 2 (rest,
HBM-bound cold gathers) launched back-to-back on one stream vs. concurrently on two
streams, dependency ignored. If the concurrent time is well below the sum, splitting
pass 2 into rows without partial refs (run beside pass 1) and rows with refs (after it)
would pay.

    python tools/xcd_overlap_probe.py [--workload cfg2|ns]
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
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.graph import seg_len_for
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if args.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    del s, d
    F = 128
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    seg = seg_len_for(F)
    xp = g.xcd_hub_plan(ops.xcd_hub_rows_for(n, F), ops.XCD_MIN_DEG, min(ops.XCD_CHUNK, seg))
    lib = _lib.load()
    buf = torch.empty(xp.k + xp.n_pos, F, device=dev)
    p1, p2 = xp.items.plan(seg), xp.rest.plan(seg)
    part = torch.empty(max(p2.n_seg, 1), F, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def pass1(st):
        ops._spmm_hub_call(lib, xp.items, xp.items.col, p1, p1.args(), X, buf, F, None,
                           buf[xp.k:], F, None, 0, st.cuda_stream, "p1")

    def pass2(st):
        ops._spmm_hub_call(lib, xp.rest, xp.rest.col, p2, p2.args(), X, buf, F, None, Y, F,
                           part, 0, st.cuda_stream, "p2")

    def seq():
        with torch.cuda.stream(s1):
            pass1(s1)
            pass2(s1)

    def conc():
        pass1(s1)
        pass2(s2)

    def tm(fn, reps=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s1)
            s2.wait_event(a)
            for _ in range(reps):
                fn()
                s1.wait_stream(s2)
                s2.wait_stream(s1)
            b.record(s1)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / reps)
        return statistics.median(ts)

    t1 = tm(lambda: pass1(s1))
    t2 = tm(lambda: pass2(s1))
    ts = tm(seq)
    tc = tm(conc)
    print(json.dumps({"workload": args.workload, "pass1_ms": round(t1, 4), "pass2_ms": round(t2, 4),
                      "sequential_ms": round(ts, 4), "concurrent_ms": round(tc, 4)}), flush=True)


if __name__ == "__main__":
    main()
