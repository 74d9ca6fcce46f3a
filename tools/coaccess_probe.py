"""CPU probe: could row-to-XCD affinity make pass 2's hub gathers XCD-local?

Pass 2 of the XCD-sliced SpMM runs every row of < 128 edges ("short rows") on whichever XCD its
task lands on, so its hub gathers read the whole 128 MiB hub table from every XCD (L2 hit rate
0.11 at the north star). If each short row instead ran on the XCD whose slice holds the most of
its hub edges (its plurality slice), that share of its hub gathers would read an XCD-local slice.
This probe measures, for the graph in the column-degree order the bench uses (hub rank r =
column r, K = 256 Ki hub ranks, slices of 4 consecutive ranks dealt to 8 XCDs):

  * baseline: the fraction of short-row hub gathers that land on the XCD a row is run on today
    (rows dealt to XCDs with no regard to their hubs: 1/8 in expectation);
  * plurality (today's slices): the fraction in each row's plurality slice, i.e. what row
    affinity alone would make XCD-local;
  * plurality after co-access clustering: hub ranks reassigned to slices (balanced by gather
    load, 2 % slack) by a few rounds of greedy label propagation toward the slices their rows
    already favour.

    python tools/coaccess_probe.py [--workload cfg2|ns] [--rounds 4]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

XCDS = 8
GROUP = 4
K_HUB = 256 * 1024
SHORT = 128


def plurality(rows: np.ndarray, slices: np.ndarray, n_rows: int):
    """(sum over rows of the largest per-slice count, per-(row, slice) counts)."""
    cnt = np.bincount(rows * XCDS + slices, minlength=n_rows * XCDS).reshape(n_rows, XCDS)
    return int(cnt.max(1).sum()), cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "ns"])
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, e = (1_000_000, 10_000_000) if a.workload == "cfg2" else (10_000_000, 100_000_000)
    t0 = time.time()
    s, d = rmat_edges(n, e, 0)
    g = gcn_normalized_csr(torch.from_numpy(s), torch.from_numpy(d), n)
    del s, d
    rowptr = g.rowptr.numpy()
    col = g.col.numpy().astype(np.int64)
    deg_in = np.bincount(col, minlength=n)
    # column-degree order (graph.degree_order: descending in-degree, ties by ascending id)
    order = np.lexsort((np.arange(n), -deg_in))
    rank = np.empty(n, np.int64)
    rank[order] = np.arange(n)
    rdeg = np.diff(rowptr)
    row_of = np.repeat(np.arange(n), rdeg)
    r_edge = rank[col]
    hub = r_edge < K_HUB
    short = rdeg[row_of] < SHORT
    sel = hub & short
    rows = row_of[sel]
    hr = r_edge[sel]
    n_g = int(sel.sum())
    print(f"[probe] {a.workload}: nnz {col.size}, short-row hub gathers {n_g} "
          f"({n_g / col.size:.1%} of all entries), built in {time.time() - t0:.0f}s", flush=True)
    out = {"workload": a.workload, "nnz": int(col.size), "short_row_hub_gathers": n_g,
           "hub_ranks": K_HUB, "slice_group": GROUP, "short_row_degree_below": SHORT}
    hs = np.bincount(rows, minlength=n)
    out["short_rows_with_hub_edges"] = int((hs > 0).sum())
    out["hub_edges_per_such_row_mean"] = float(n_g / max(1, (hs > 0).sum()))
    # today's slices; a row runs on an XCD unrelated to them (expected local share 1/8)
    sl = (hr // GROUP) % XCDS
    pl, _ = plurality(rows, sl, n)
    out["baseline_local_fraction"] = 1.0 / XCDS
    out["plurality_fraction_current_slices"] = pl / n_g
    print(f"[probe] plurality with today's slices: {pl / n_g:.3f} (baseline 0.125)", flush=True)
    # co-access clustering: greedy label propagation of hub ranks toward the slices their rows
    # favour, under a per-slice load cap
    slice_of = (np.arange(K_HUB) // GROUP) % XCDS
    load = np.bincount(hr, minlength=K_HUB).astype(np.float64)
    cap = load.sum() / XCDS * 1.02
    hist = []
    for it in range(a.rounds):
        t1 = time.time()
        sl = slice_of[hr]
        _, cnt = plurality(rows, sl, n)
        # affinity of hub h to slice s: its rows' counts in s (its own edge excluded)
        aff = np.zeros((K_HUB, XCDS))
        c_edge = cnt[rows]                               # [n_g, 8]
        c_edge[np.arange(n_g), sl] -= 1
        for s_ in range(XCDS):
            aff[:, s_] = np.bincount(hr, weights=c_edge[:, s_], minlength=K_HUB)
        del c_edge
        gain = aff - aff[np.arange(K_HUB), slice_of][:, None]
        best = gain.argmax(1)
        bgain = gain[np.arange(K_HUB), best]
        new = slice_of.copy()
        used = np.bincount(slice_of, weights=load, minlength=XCDS)
        for h in np.argsort(-bgain):
            if bgain[h] <= 0:
                break
            t = best[h]
            if used[t] + load[h] <= cap:
                used[t] += load[h]
                used[new[h]] -= load[h]
                new[h] = t
        moved = int((new != slice_of).sum())
        slice_of = new
        pl, _ = plurality(rows, slice_of[hr], n)
        hist.append({"round": it + 1, "moved_hubs": moved, "plurality_fraction": pl / n_g,
                     "max_slice_load_over_mean": float(
                         np.bincount(slice_of, weights=load, minlength=XCDS).max()
                         / (load.sum() / XCDS))})
        print(f"[probe] round {it + 1}: moved {moved}, plurality {pl / n_g:.3f} "
              f"({time.time() - t1:.0f}s)", flush=True)
    out["clustering"] = hist
    out["plurality_fraction_clustered"] = hist[-1]["plurality_fraction"] if hist else None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
