"""A/B in one process of the MFMA transform's two arithmetics (ops.set_transform_precision:
'fp32-mfma' = v_mfma_f32_16x16x4_f32, 'split-bf16' = fp32 products from bf16 MFMAs) against
hipBLASLt (F.linear / addmm), on the transform shapes of the bench workloads:

    python tools/transform_prec_ab.py                (GPU)
Prints one JSON line: microseconds per launch (median of 5 x 20) and the max error relative to
sum_k |x w| against a float64 product on a row sample.
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
SHAPES = ("8192:256:128:1,61771:256:128:1,200000:256:128:1,1000000:128:128:0,"
          "1000000:128:128:2,10000000:128:128:2,1000000:256:256:0,10000000:256:256:2")


def timed(fn, reps=20, rounds=5):
    out = []
    for _ in range(rounds):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / reps * 1e3)
    return round(statistics.median(out), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8192:256:128:1,61771:256:128:1,1000000:128:128:0",
                    help="rows:k:fout:mode, mode 0 = plain, 1 = ReLU, 2 = scattered rows")
    a = ap.parse_args()
    from graphneuralnetwork_amd.ops import gcn_transform, set_transform_precision
    dev = torch.device("cuda:0")
    res = {}
    for sh in a.shapes.split(","):
        m, k, f, mode = (int(v) for v in sh.split(":"))
        x = torch.randn(m, k, device=dev)
        w = torch.randn(f, k, device=dev) / k ** 0.5
        out = torch.empty(m, f, device=dev)
        perm = torch.randperm(m, device=dev) if mode == 2 else None
        zero = torch.zeros(f, device=dev)
        r = {}
        idx = torch.randint(0, m, (2048,), device=dev)
        ref = x[idx].double() @ w.double().T
        mag = x[idx].abs().double() @ w.abs().double().T
        for prec in ("fp32-mfma", "split-bf16"):
            set_transform_precision(prec)
            fn = lambda: gcn_transform(x, w, relu=mode == 1, out=out, out_rows=perm,  # noqa: E731
                                       check_rows=False)
            r[prec] = timed(fn)
            y = fn()
            yy = y[perm[idx]] if perm is not None else y[idx]
            if mode == 1:
                yy = yy  # ReLU: compare where the reference is positive
                err = ((yy.double() - ref.clamp_min(0)).abs() / mag).max()
            else:
                err = ((yy.double() - ref).abs() / mag).max()
            r[prec + "_err"] = float(err)
        set_transform_precision("split-bf16")
        if mode == 1:
            r["hipblaslt"] = timed(lambda: torch._addmm_activation(zero, x, w.t()))
        else:
            r["hipblaslt"] = timed(lambda: torch.nn.functional.linear(x, w))
        res[sh] = r
        print(json.dumps({sh: r}), flush=True)
        del x, out, perm
        torch.cuda.empty_cache()
    print(json.dumps({"us": res}), flush=True)
    # the GAT projection (gnn_gat_project_f32 / _rows_f32): cfg3's 1M x 64 -> 8 heads x 8
    from graphneuralnetwork_amd.ops import gat_project
    for n, k, H, fh in ((1_000_000, 64, 8, 8), (1_000_000, 128, 4, 8)):
        x = torch.randn(n, k, device=dev)
        w = torch.randn(k, H * fh, device=dev) / k ** 0.5
        a_s, a_d = torch.randn(H * fh, device=dev), torch.randn(H * fh, device=dev)
        perm = torch.randperm(n, device=dev)
        idx = torch.randint(0, n, (2048,), device=dev)
        ref = x[idx].double() @ w.double()
        mag = x[idx].abs().double() @ w.abs().double()
        r = {}
        for prec in ("fp32-mfma", "split-bf16"):
            set_transform_precision(prec)
            r[prec] = timed(lambda: gat_project(x, w, H, fh, a_s, a_d))
            r[prec + "_rows"] = timed(lambda: gat_project(x, w, H, fh, a_s, a_d, col_rows=perm))
            wh = gat_project(x, w, H, fh, a_s, a_d)[0]
            r[prec + "_err"] = float(((wh[idx].double() - ref).abs() / mag).max())
        set_transform_precision("split-bf16")
        tag = f"project {n}x{k}->{H}x{fh}"
        res[tag] = r
        print(json.dumps({tag: r}), flush=True)
        del x, perm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
