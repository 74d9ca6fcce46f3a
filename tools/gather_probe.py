"""Random 512-B row-gather bandwidth probe (what bounds the north-star SpMM).

Times gnn_gather_rows_f32 (read one fp32 row of F=128 per index, write it out) for
sequential vs uniform-random vs R-MAT-column indices over a 1M-row (512 MB, ~2x the
Infinity Cache) and a 10M-row (5.1 GB) table. Reports (read + write bytes) / time.

    python tools/gather_probe.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from graphneuralnetwork_amd.ops import gather_rows
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    F, n_idx = 128, 20_000_000
    res = {}
    for n_rows in (1_000_000, 10_000_000):
        table = torch.randn(n_rows, F, device=dev)
        out = torch.empty(n_idx, F, device=dev)
        _, d = rmat_edges(n_rows, n_idx, 1)
        pats = {"sequential": torch.arange(n_idx, device=dev) % n_rows,
                "uniform": torch.randint(0, n_rows, (n_idx,), device=dev),
                "rmat_cols": torch.from_numpy(d[:n_idx]).to(dev)}
        for name, idx in pats.items():
            for _ in range(2):
                gather_rows(table, idx, out=out, check=False)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                gather_rows(table, idx, out=out, check=False)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 5
            res[f"{n_rows // 1_000_000}M_{name}"] = {"ms": round(ms, 3),
                                                     "GBps": round(2 * n_idx * F * 4 / ms / 1e6)}
            print(f"table {n_rows} rows, {name}: {ms:.3f} ms, {2 * n_idx * F * 4 / ms / 1e6:.0f} GB/s",
                  flush=True)
        del table, out
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
