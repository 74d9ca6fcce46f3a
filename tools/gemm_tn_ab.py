"""A/B of the weight-gradient kernel (gnn_gemm_tn_f32) at the training shapes: the split-bf16
MFMA partials (main library, the default arithmetic), the fp32-MFMA partials (main library under
ops.set_transform_precision("fp32-mfma")), the FMA partials (variant library ``tnfma``,
-DGNN_TN_FMA, when built) and hipBLASLt's torch.mm, HIP-event medians, interleaved in one
process.

    python tools/gemm_tn_ab.py --build           (CPU side: the variant library)
    python tools/gemm_tn_ab.py [--reps 30]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

SHAPES = [(1_000_000, 128, 128, True), (1_000_000, 64, 64, False), (10_000_000, 128, 128, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    if a.build:
        from graphneuralnetwork_amd.build import build_variant
        print(build_variant("tnfma", ["GNN_TN_FMA"], only=["gemm_tn.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.build import LIB_DIR
    from graphneuralnetwork_amd.ops import gemm_tn, set_transform_precision
    dev = torch.device("cuda:0")
    libs = {"x6": (None, "split-bf16"), "f32mfma": (None, "fp32-mfma")}
    if (LIB_DIR / "variants" / "libgnn_tnfma.so").exists():
        libs["fma"] = (LIB_DIR / "variants" / "libgnn_tnfma.so", "split-bf16")
    out = {}
    for n, m, k, dsum in SHAPES:
        gen = torch.Generator(device=dev).manual_seed(n + m)
        x = torch.randn(n, m, device=dev, generator=gen)
        y = torch.randn(n, k, device=dev, generator=gen)
        d = torch.randn(n, k, device=dev, generator=gen) if dsum else None
        ref = None
        times = {name: [] for name in list(libs) + ["torch_mm"]}
        diffs = {}
        for name, (lib, prec) in libs.items():
            _lib.use_variant(lib)
            set_transform_precision(prec)
            c = gemm_tn(x, y, d, trans=True)[0]
            torch.cuda.synchronize()
            if ref is None:
                ref = (x.double().t() @ y.double()).t().float()
            diffs[name] = float(((c - ref).abs().max() / ref.abs().max()).item())
        for _ in range(a.reps):
            for name in times:
                if name != "torch_mm":
                    _lib.use_variant(libs[name][0])
                    set_transform_precision(libs[name][1])
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if name == "torch_mm":
                    torch.mm(y.t(), x)
                else:
                    gemm_tn(x, y, d, trans=True)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1))
        _lib.use_variant(None)
        set_transform_precision("split-bf16")
        nbytes = 4 * n * (m + k + (k if dsum else 0))
        out[f"n{n}_m{m}_k{k}_dsum{int(dsum)}"] = {
            nm: {"median_ms": round(statistics.median(t), 4),
                 "GBps": round(nbytes / (statistics.median(t) / 1e3) / 1e9, 1),
                 "TFLOPs": round(2 * n * m * k / (statistics.median(t) / 1e3) / 1e12, 1)}
            for nm, t in times.items()}
        out[f"n{n}_m{m}_k{k}_dsum{int(dsum)}"]["max_rel_err_vs_float64"] = diffs
        del x, y, d
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
