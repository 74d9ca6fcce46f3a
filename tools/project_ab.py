"""A/B of gnn_gat_project_f32 builds (lib/variants) at the cfg3 shape.

    python tools/project_ab.py --build      (CPU side)
    python tools/project_ab.py              (GPU)
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
VARIANTS = {"base": [], "blds": ["GNN_PROJ_B_LDS"], "nowh": ["GNN_PROJ_NO_WH"],
            "g256": ["GNN_PROJ_GRID=256"], "g512": ["GNN_PROJ_GRID=512"],
            "g1024": ["GNN_PROJ_GRID=1024"], "g4096": ["GNN_PROJ_GRID=4096"],
            "g8192": ["GNN_PROJ_GRID=8192"], "blds_g4096": ["GNN_PROJ_B_LDS", "GNN_PROJ_GRID=4096"],
            "nomfma": ["GNN_PROJ_NO_MFMA"], "nomfma_nowh": ["GNN_PROJ_NO_MFMA", "GNN_PROJ_NO_WH"],
            "g2": ["GNN_PROJ_G=2"], "g2_512": ["GNN_PROJ_G=2", "GNN_PROJ_GRID=512"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        from graphneuralnetwork_amd.build import build_variant
        for n in names:
            print(build_variant("proj_" + n, VARIANTS[n], only=["project.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gat_project
    dev = torch.device("cuda:0")
    n, k, H, fh = 1_000_000, 64, 8, 8
    x = torch.randn(n, k, device=dev)
    w = torch.randn(k, H * fh, device=dev)
    s, d = torch.randn(H * fh, device=dev), torch.randn(H * fh, device=dev)
    res = {}
    for v in names:
        _lib.use_variant(ROOT / "graphneuralnetwork_amd" / "lib" / "variants" / f"libgnn_proj_{v}.so")
        for _ in range(3):
            gat_project(x, w, H, fh, s, d)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            gat_project(x, w, H, fh, s, d)
        b.record()
        torch.cuda.synchronize()
        res[v] = a.elapsed_time(b) / 20
    print(json.dumps(res))


if __name__ == "__main__":
    main()
