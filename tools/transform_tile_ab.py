"""A/B of transform tile-height variants (lib/variants, built with tools/transform_tile_ab.py
--build) on the SageLayer GEMM relu(buf @ W^T), buf [M, 256] -> 128, vs hipBLASLt.

    python tools/transform_tile_ab.py --build     (CPU)
    python tools/transform_tile_ab.py             (GPU)
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
VARIANTS = {"base": [], "tr32_1m": ["GNN_TF_TR32_ROWS=1000000"],
            "tr32": ["GNN_TF_TR32_ROWS=(1LL<<40)"],
            "tr16": ["GNN_TF_TR32_ROWS=(1LL<<40)", "GNN_TF_TR16_ROWS=(1LL<<40)"],
            "grid1024": ["GNN_TF_GRID=1024"],
            "one256": ["GNN_TF_ONE256=1"], "cb2": ["GNN_TF_K256_CB2=1"],
            "pf2": ["GNN_TF_PREFETCH=2"], "pf3": ["GNN_TF_PREFETCH=3"],
            "mt32": ["GNN_TF_MIN_TR=32"], "mt32pf2": ["GNN_TF_MIN_TR=32", "GNN_TF_PREFETCH=2"],
            "old": None}  # "old": lib/variants/libgnn_tf_old.so, built from another tree


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default="base,tr32,tr16")
    ap.add_argument("--shapes", default="8192:256:128:1,62479:256:128:1,200000:256:128:1,"
                    "1000000:256:128:1,1000000:128:128:0,10000000:128:128:0,1000000:64:64:0")
    a = ap.parse_args()
    names = a.variants.split(",")
    if a.build:
        from graphneuralnetwork_amd.build import build_variant
        for n in names:
            if VARIANTS[n] is not None:
                print(build_variant("tf_" + n, VARIANTS[n], only=["transform.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import gcn_transform
    ops.TRANSFORM_WIDE_MFMA = True  # time the 256-column MFMA paths too (off by policy)
    dev = torch.device("cuda:0")
    res = {}
    for sh in a.shapes.split(","):
        m, k, f, relu = (int(v) for v in sh.split(":"))
        x = torch.randn(m, k, device=dev)
        w = torch.randn(f, k, device=dev) / k ** 0.5
        zero = torch.zeros(f, device=dev)
        t = {n: [] for n in names + ["hipblaslt"]}
        for _ in range(5):
            for n in names:
                _lib.use_variant(ROOT / "graphneuralnetwork_amd" / "lib" / "variants" /
                                 f"libgnn_tf_{n}.so")
                fn = lambda: gcn_transform(x, w, relu=bool(relu))  # noqa: E731
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                t[n].append(e0.elapsed_time(e1) / 20 * 1e3)
            fn = lambda: torch._addmm_activation(zero, x, w.t())  # noqa: E731
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t["hipblaslt"].append(e0.elapsed_time(e1) / 20 * 1e3)
        res[sh] = {n: round(statistics.median(v), 2) for n, v in t.items()}
        del x
        torch.cuda.empty_cache()
    print(json.dumps({"us": res}), flush=True)


if __name__ == "__main__":
    main()
