"""A/B of gemm_tn x6 build variants at the cfg2 training shapes (1M x 128 x 128): the DB form
(dW = dY^T Z with db from dY's loads) and the masked form (ReLU / dropout folded in), main
library against variants built with -D defines, HIP-event medians, interleaved in one process.

    python tools/tn_ab.py --build   (CPU side)
    python tools/tn_ab.py [--reps 30]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
VARIANTS = {"tn14": ["GNN_TN_X6_2X2=0"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    from graphneuralnetwork_amd.build import LIB_DIR, build_variant
    if a.build:
        for tag, d in VARIANTS.items():
            print(build_variant(tag, d, only=["gemm_tn.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gemm_tn, gemm_tn_masked
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    z = torch.randn(1_000_000, 128, device=dev, generator=gen)
    dy = torch.randn(1_000_000, 128, device=dev, generator=gen)
    h = torch.relu(torch.randn(1_000_000, 128, device=dev, generator=gen))
    libs = {"main": None}
    libs.update({t: LIB_DIR / "variants" / f"libgnn_{t}.so" for t in VARIANTS})
    forms = {"DB": lambda: gemm_tn(z, dy, dy, trans=True),
             "masked": lambda: gemm_tn_masked(z, dy, h, 2.0, True, trans=True)}
    ref = {}
    for name, lib in libs.items():
        _lib.use_variant(lib)
        for f, fn in forms.items():
            c, d = fn()
            if f in ref:
                assert torch.equal(c, ref[f][0]) or float((c - ref[f][0]).abs().max()) < 1e-3
            else:
                ref[f] = (c, d)
    times = {(n, f): [] for n in libs for f in forms}
    for _ in range(a.reps):
        for name, lib in libs.items():
            _lib.use_variant(lib)
            for f, fn in forms.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                torch.cuda.synchronize()
                times[(name, f)].append(s.elapsed_time(e))
    _lib.use_variant(None)
    print(json.dumps({f"{n}/{f}": round(statistics.median(t), 4) for (n, f), t in times.items()}))


if __name__ == "__main__":
    main()
