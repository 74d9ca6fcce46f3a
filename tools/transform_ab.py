"""GCN feature transform: gnn_gcn_transform_f32 (fp32 MFMA) vs torch.nn.functional.linear
(hipBLASLt), interleaved, at the bench shapes.

    python tools/transform_ab.py [--variants tag,...]   (lib/variants/libgnn_<tag>.so, built
                                                          with tools/lib_ab.py --build)
"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="")
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gcn_transform
    root = Path(__file__).resolve().parent.parent / "graphneuralnetwork_amd" / "lib" / "variants"
    variants = [v for v in args.variants.split(",") if v]
    dev = torch.device("cuda:0")
    for n, k, fo in ((1_000_000, 128, 128), (10_000_000, 128, 128), (1_000_000, 64, 64),
                     (2708, 128, 64)):
        x = torch.randn(n, k, device=dev)
        w = torch.randn(fo, k, device=dev) / k ** 0.5
        ref = torch.nn.functional.linear(x.double(), w.double()).float() if n <= 1_000_000 else None
        y = gcn_transform(x, w)
        if ref is not None:
            err = float((y - ref).abs().max() / ref.abs().max())
            assert err < 1e-5, err
        fns = {"mfma": lambda: gcn_transform(x, w),
               "hipblaslt": lambda: torch.nn.functional.linear(x, w)}
        for v in variants:
            def fv(v=v):
                _lib.use_variant(root / f"libgnn_{v}.so")
                try:
                    return gcn_transform(x, w)
                finally:
                    _lib.use_variant(None)
            fns[v] = fv
            if ref is not None:  # every variant must compute the same product
                yv = fv()
                errv = float((yv - ref).abs().max() / ref.abs().max())
                assert errv < 1e-5, (v, errv)
        t = {k_: [] for k_ in fns}
        for _ in range(5):
            for name, f in fns.items():
                f()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    f()
                b.record()
                torch.cuda.synchronize()
                t[name].append(a.elapsed_time(b) / 5)
        flop = 2.0 * n * k * fo
        print(json.dumps({"n": n, "k": k, "fout": fo,
                          **{f"{name}_ms": statistics.median(v) for name, v in t.items()},
                          **{f"{name}_TFs": flop / statistics.median(v) / 1e9
                             for name, v in t.items()}}), flush=True)
        del x, y, ref


if __name__ == "__main__":
    main()
