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
VARIANTS = {"base": [], "d1": ["GNN_PROJ_DEPTH=1"], "d3": ["GNN_PROJ_DEPTH=3"],
            "d4": ["GNN_PROJ_DEPTH=4"], "d2g1024": ["GNN_PROJ_GRID=1024"],
            "d3g1024": ["GNN_PROJ_DEPTH=3", "GNN_PROJ_GRID=1024"], "oldlds": ["GNN_TILE_OLD_LDS", "GNN_PROJ_BLOCK_SYNC=1"],
            "blocksync": ["GNN_PROJ_BLOCK_SYNC=1"], "oldlds_wave": ["GNN_TILE_OLD_LDS"], "blds": ["GNN_PROJ_B_LDS"], "nowh": ["GNN_PROJ_NO_WH"],
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
    res = {v: [] for v in names}
    ref = None
    import statistics
    for rnd in range(5):
        for v in names:
            _lib.use_variant(ROOT / "graphneuralnetwork_amd" / "lib" / "variants" /
                             f"libgnn_proj_{v}.so")
            for _ in range(3):
                out = gat_project(x, w, H, fh, s, d)
            torch.cuda.synchronize()
            if rnd == 0:
                if ref is None:
                    ref = [t.clone() for t in out]
                elif not all(torch.equal(a_, b_) for a_, b_ in zip(out, ref)):
                    print(f"variant {v}: output differs from {names[0]}")
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                gat_project(x, w, H, fh, s, d)
            b.record()
            torch.cuda.synchronize()
            res[v].append(a.elapsed_time(b) / 20)
    res = {v: round(statistics.median(t), 4) for v, t in res.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
