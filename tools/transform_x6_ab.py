"""A/B of split-bf16 (X6) transform builds (lib/variants/libgnn_x6_<tag>.so) in one process.

    python tools/transform_x6_ab.py --build        (CPU)
    python tools/transform_x6_ab.py                (GPU)
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
VARIANTS = {"base": [], "pipe": ["GNN_TF_X6_PIPE=1"],
            "tr16": ["GNN_TF_TR32_ROWS=(1LL<<40)", "GNN_TF_TR16_ROWS=(1LL<<40)"]}
SHAPES = "61771:256:128:1,200000:256:128:1,1000000:128:128:0,10000000:128:128:0,1000000:256:256:0"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--shapes", default=SHAPES)
    a = ap.parse_args()
    names = a.variants.split(",")
    if a.build:
        from graphneuralnetwork_amd.build import build_variant
        for n in names:
            print(build_variant("x6_" + n, VARIANTS[n], only=["transform.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gcn_transform
    dev = torch.device("cuda:0")
    res = {}
    for sh in a.shapes.split(","):
        m, k, f, relu = (int(v) for v in sh.split(":"))
        x = torch.randn(m, k, device=dev)
        w = torch.randn(f, k, device=dev) / k ** 0.5
        out = torch.empty(m, f, device=dev)
        t = {n: [] for n in names}
        ref = None
        for _ in range(5):
            for n in names:
                _lib.use_variant(ROOT / "graphneuralnetwork_amd" / "lib" / "variants" /
                                 f"libgnn_x6_{n}.so")
                fn = lambda: gcn_transform(x, w, relu=bool(relu), out=out)  # noqa: E731
                fn()
                if ref is None:
                    ref = out.clone()
                elif not torch.equal(out, ref):
                    t[n + "_differs"] = True
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                t[n].append(e0.elapsed_time(e1) / 20 * 1e3)
        res[sh] = {n: (round(statistics.median(v), 2) if isinstance(v, list) else v)
                   for n, v in t.items()}
        print(json.dumps({sh: res[sh]}), flush=True)
        del x, out
        torch.cuda.empty_cache()
    print(json.dumps({"us": res}), flush=True)


if __name__ == "__main__":
    main()
