"""A/B of gnn_gat_project_rows_f32 builds (lib/variants) at the cfg3 shape (rows scattered
into a column order as bench.py's cfg3 step writes them).

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
            "g2": ["GNN_PROJ_G=2"], "g2_512": ["GNN_PROJ_G=2", "GNN_PROJ_GRID=512"],
            "old": None}  # "old": lib/variants/libgnn_proj_old.so, built from another tree


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--inorder", action="store_true",
                    help="gnn_gat_project_f32 (rows in place) instead of the column-order scatter")
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        from graphneuralnetwork_amd.build import build_variant
        for n in names:
            if VARIANTS[n] is not None:
                print(build_variant("proj_" + n, VARIANTS[n], only=["project.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    dev = torch.device("cuda:0")
    n, k, H, fh = 1_000_000, 64, 8, 8
    x = torch.randn(n, k, device=dev)
    w = torch.randn(k, H * fh, device=dev)
    s, d = torch.randn(H * fh, device=dev), torch.randn(H * fh, device=dev)
    # cfg3's column order: 262,144 "hub" ids (random here) first in random order, the rest
    # ascending (graph.degree_order(prefix=...)); inv = old -> new row
    g = torch.Generator(device=dev).manual_seed(3)
    hub = torch.randperm(n, device=dev, generator=g)[:262144]
    is_hub = torch.zeros(n, dtype=torch.bool, device=dev)
    is_hub[hub] = True
    perm = torch.cat([hub, torch.nonzero(~is_hub).view(-1)])
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(n, device=dev)
    w2 = torch.empty(k * 16, device=dev)  # the scratch older builds fold the logits into

    def gat_project(x, w, H, fh, s, d):
        lib = _lib.load()
        wh = torch.empty(n, H * fh, device=dev)
        el = torch.empty(n, H, device=dev)
        er = torch.empty(n, H, device=dev)
        if args.inorder:
            _lib.check(lib.gnn_gat_project_f32(
                x.data_ptr(), k, n, k, w.data_ptr(), H * fh, s.data_ptr(), d.data_ptr(), H, fh,
                wh.data_ptr(), H * fh, el.data_ptr(), er.data_ptr(), H, w2.data_ptr(),
                _lib.stream_handle(dev)), "gnn_gat_project_f32")
            return wh, el, er
        _lib.check(lib.gnn_gat_project_rows_f32(
            x.data_ptr(), k, n, k, w.data_ptr(), H * fh, s.data_ptr(), d.data_ptr(), H, fh,
            wh.data_ptr(), H * fh, el.data_ptr(), er.data_ptr(), H, inv.data_ptr(),
            w2.data_ptr(), _lib.stream_handle(dev)), "gnn_gat_project_rows_f32")
        return wh, el, er
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
