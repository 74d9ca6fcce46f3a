"""A/B of the narrow-side linear kernels (gnn_linear_small_f32) at GCN_Model's classifier shapes
(cfg2: 1M rows, 128 -> 8 and 8 -> 128): broadcast-kernel variants (-DGNN_SMALL_IN_R,
-DGNN_SMALL_IN_NT) against the main library and hipBLASLt's torch.mm, HIP-event medians,
interleaved in one process.

    python tools/small_ab.py --build             (CPU side: the variant libraries)
    python tools/small_ab.py [--reps 30]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

VARIANTS = {"r8": ["GNN_SMALL_IN_R=8"], "r2": ["GNN_SMALL_IN_R=2"], "plain": ["GNN_SMALL_IN_NT=0"],
            "r8plain": ["GNN_SMALL_IN_R=8", "GNN_SMALL_IN_NT=0"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    from graphneuralnetwork_amd.build import LIB_DIR, build_variant
    if a.build:
        for tag, d in VARIANTS.items():
            print(build_variant("small_" + tag, d, only=["narrow.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import linear_small
    dev = torch.device("cuda:0")
    libs = {"main": None}
    libs.update({t: LIB_DIR / "variants" / f"libgnn_small_{t}.so" for t in VARIANTS})
    out = {}
    for n, k, fo in ((1_000_000, 8, 128), (1_000_000, 128, 8)):
        gen = torch.Generator(device=dev).manual_seed(n + k)
        x = torch.randn(n, k, device=dev, generator=gen)
        w = torch.randn(fo, k, device=dev, generator=gen)
        times = {name: [] for name in list(libs) + ["torch_mm"]}
        ref = torch.mm(x, w.t())
        for name, lib in libs.items():
            _lib.use_variant(lib)
            y = linear_small(x, w)
            assert float((y - ref).abs().max()) < 1e-3 * float(ref.abs().max())
        for _ in range(a.reps):
            for name, lib in list(libs.items()) + [("torch_mm", None)]:
                if name != "torch_mm":
                    _lib.use_variant(lib)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                if name == "torch_mm":
                    torch.mm(x, w.t())
                else:
                    linear_small(x, w)
                e.record()
                torch.cuda.synchronize()
                times[name].append(s.elapsed_time(e))
        _lib.use_variant(None)
        out[f"{n}x{k}->{fo}"] = {name: round(statistics.median(t), 4) for name, t in times.items()}
        print(json.dumps({f"{n}x{k}->{fo}": out[f"{n}x{k}->{fo}"]}), flush=True)


if __name__ == "__main__":
    main()
