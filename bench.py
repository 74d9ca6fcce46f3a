"""Benchmark: GCN SpMM aggregation (the BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2|ns] [--feat F]

One "step" = one full GCN neighbour aggregation Y = A_hat . X + b over the
whole (per-rank) graph -- the op that replaces torch.spmm(adj, support) + bias
at GCN/GCN.py:43-45 -- with X and the CSR adjacency already resident in HBM.

Workloads (synthetic R-MAT, SURVEY.md section 8(d) recipe, reference GCN
normalisation):
  cfg2  BASELINE configs[1]: 1M nodes / 10M directed edges (nnz 20,073,500), F=128
  ns    north star: 10M nodes / 100M edges (nnz 206,948,698), F=128
With --gpus N > 1 (torchrun, one process per GPU, RCCL) the graph grows with N
(weak scaling: N x the per-GPU graph) and is edge-cut N ways by contiguous
nnz-balanced row blocks; each step exchanges halo feature rows with an RCCL
all-to-all-v and runs the interior SpMM concurrently on a second stream.

Rank 0 prints ONE JSON line (value = aggregated edges/s over all ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
import warnings
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "aggregated edges/sec + achieved HBM GB/s, GCN SpMM feat_dim=128 @1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
WORKLOADS = {
    "cfg2": dict(nodes=1_000_000, edges=10_000_000,
                 name="GCN SpMM, RMAT 1M nodes / 10M edges (BASELINE configs[1])"),
    "ns": dict(nodes=10_000_000, edges=100_000_000,
               name="GCN SpMM, RMAT 10M nodes / 100M edges (north star)"),
    # BASELINE configs[4]: the whole 10M / 100M graph at F=256 edge-cut over the N ranks
    # (strong scaling: the graph does not grow with N; at N=1 it is the single-GPU reference)
    "cfg5": dict(nodes=10_000_000, edges=100_000_000, feat=256, strong=True,
                 name="GCN SpMM, RMAT 10M nodes / 100M edges, F=256, edge-cut over N GPUs "
                      "(BASELINE configs[4])"),
    "cfg3": dict(nodes=1_000_000, edges=10_000_000,
                 name="GAT 8-head (64->8x8) edge-softmax + aggregate, RMAT 1M / 10M (BASELINE configs[2])"),
    "cfg4": dict(nodes=10_000_000, edges=100_000_000,
                 name="GraphSAGE 2-hop fanout [25,10] MEAN, F=H=128, 8192 seeds, RMAT 10M / 100M "
                      "(BASELINE configs[3])"),
}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


class Watchdog:
    """Per-rank phase deadlines for the N-rank bench: the first RCCL run
    happens on the driver's 8-GPU node, so a stall there must leave evidence. Each rank names
    its phase (``enter``); a daemon thread checks every few seconds, and a phase that outlives
    its limit makes the rank print which phase it stalled in (with every thread's Python stack)
    to stderr and leave with exit status 3 (os._exit: no exec, no cleanup that could block on
    the hung collective). On at N > 1, or with GNN_BENCH_WATCHDOG=1; GNN_BENCH_DEADLINE_SCALE
    scales every limit."""

    def __init__(self, rank: int, enabled: bool):
        import threading
        self.rank = rank
        self.enabled = enabled
        self.scale = float(os.environ.get("GNN_BENCH_DEADLINE_SCALE", "1"))
        self.phase, self.limit, self.t0 = "start", None, time.time()
        self.history = []
        self._lock = threading.Lock()
        if enabled:
            threading.Thread(target=self._run, name="bench-watchdog", daemon=True).start()

    def enter(self, phase: str, limit_s: float | None) -> None:
        with self._lock:
            now = time.time()
            self.history.append((self.phase, round(now - self.t0, 3)))
            self.phase, self.t0 = phase, now
            self.limit = None if limit_s is None else limit_s * self.scale

    def _run(self):
        import faulthandler
        while True:
            time.sleep(2.0)
            with self._lock:
                phase, limit, t0 = self.phase, self.limit, self.t0
            if limit is not None and time.time() - t0 > limit:
                print(f"[bench] WATCHDOG rank {self.rank}: phase '{phase}' made no progress for "
                      f"{time.time() - t0:.0f} s (limit {limit:.0f} s); earlier phases "
                      f"{self.history[-8:]}; exiting with status 3", file=sys.stderr, flush=True)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                os._exit(3)


WD = Watchdog(0, False)


def phase(name: str, limit_s: float | None) -> None:
    """Name the phase this rank is in (see Watchdog); None = no deadline."""
    WD.enter(name, limit_s)


def algorithmic_bytes(nnz: int, n_rows: int, feat: int) -> int:
    """SpMM gather-model bytes: per edge 4 col + 4 val + 4F gathered row;
    per output row 8 rowptr + 4F written row. Every gathered row is counted as an HBM read,
    so this is an upper bound on the traffic (hub rows are re-read from L2 / the Infinity
    Cache), not the minimum: reported as ``gather_model_*``."""
    return nnz * (8 + 4 * feat) + n_rows * (8 + 4 * feat)


def compulsory_bytes(nnz: int, n_rows: int, n_cols: int, feat: int) -> int:
    """SpMM compulsory bytes, the basis of ``roofline.achieved`` / ``frac``: every input read
    once and the output written once -- per edge 4 col + 4 val; per row 8 rowptr + 4F output;
    per column 4F of X (nnz*8 + N*(8 + 8F) for a square graph)."""
    return nnz * 8 + n_rows * (8 + 4 * feat) + n_cols * 4 * feat


def spmm_replay(ga, X, bias, Y, reps: int = 5, table_rows: int = 2048) -> dict | None:
    """The SpMM's ceiling measured on its own access stream (the model it
    replaces priced hub gathers at a rate the 16 MiB slices cannot reach): the product kernels
    over ``ga``'s real XCD hub plan, with only the gathered row ids rewritten in place --
      as_built            the step as benchmarked;
      hub_gathers_in_L2   every hub gather (rank < k, pass 1 and pass 2) to rank % T, a T-row
                          table that fits each XCD's 4 MiB L2 (the floor for hub locality);
      all_gathers_in_L2   every gather to rank % T: no HBM / Infinity-Cache gather at all, the
                          schedule's own cost (CSR, partial rows, output, gather issue);
    then the original ids restored. The rewritten steps compute wrong sums (never read).
    HIP events, median of ``reps``; None when ``ga`` has no XCD-direct hub plan."""
    from graphneuralnetwork_amd.graph import XcdHubPlan
    from graphneuralnetwork_amd.ops import spmm_forward
    xps = [p for p in ga._plans.values() if isinstance(p, XcdHubPlan) and p.prefix]
    if len(xps) != 1:
        return None
    items, rest = xps[0].direct()
    k, T = xps[0].k, table_rows
    i0, r0 = items.col.clone(), rest.col.clone()
    hub = (r0 >= 0) & (r0 < k)
    variants = {"as_built_ms": (i0, r0),
                "hub_gathers_in_L2_ms": (i0 % T, torch.where(hub, r0 % T, r0)),
                "all_gathers_in_L2_ms": (i0 % T, torch.where(r0 >= 0, r0 % T, r0))}
    times = {v: [] for v in variants}
    try:
        for _ in range(reps):
            for v, (ic, rc) in variants.items():
                items.col.copy_(ic)
                rest.col.copy_(rc)
                spmm_forward(ga, X, bias, out=Y)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                spmm_forward(ga, X, bias, out=Y)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1))
    finally:
        items.col.copy_(i0)
        rest.col.copy_(r0)
        torch.cuda.synchronize()
    out = {v: statistics.median(t) for v, t in times.items()}
    out["as_built_over_hub_floor"] = out["as_built_ms"] / out["hub_gathers_in_L2_ms"]
    out.update(hub_rows=k, table_rows=T, pass1_hub_gathers=int(i0.numel()),
               pass2_hub_gathers=int(hub.sum()), pass2_nonhub_gathers=int((r0 >= k).sum()),
               method="product kernels on the real plan, gathered ids rewritten (tools/spmm_replay.py)")
    return out


def gat_replay(ga, k: int, fn, reps: int = 5, table_rows: int = 2048) -> dict | None:
    """The GAT aggregation's ceiling measured the way ``spmm_replay`` measures the SpMM's
    (VERDICT r5 weak #4): the product kernels over ``ga``'s real hub plan (the column-ordered
    graph: hub columns renamed -1-c, their Wh / er rows read in place) with only the gathered ids
    rewritten -- hub gathers to rank % T (a T-row Wh table of T * 256 B fits each XCD's L2), then
    every gather -- and restored. ``fn`` runs the benchmarked aggregation. None without a hub
    plan."""
    hp = ga._plans.get(("_hub", k))
    if hp is None or getattr(hp, "col_hub", None) is None:
        return None
    col = hp.col_hub
    c0 = col.clone()
    T = table_rows
    hub = c0 < 0
    variants = {"as_built_ms": c0,
                "hub_gathers_in_L2_ms": torch.where(hub, -1 - ((-1 - c0) % T), c0),
                "all_gathers_in_L2_ms": torch.where(hub, -1 - ((-1 - c0) % T), c0 % T)}
    times = {v: [] for v in variants}
    try:
        for _ in range(reps):
            for v, cv in variants.items():
                col.copy_(cv)
                fn()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1))
    finally:
        col.copy_(c0)
        torch.cuda.synchronize()
    out = {v: statistics.median(t) for v, t in times.items()}
    out["as_built_over_hub_floor"] = out["as_built_ms"] / out["hub_gathers_in_L2_ms"]
    out.update(hub_rows=k, table_rows=T, hub_gathers=int(hub.sum()),
               nonhub_gathers=int((~hub).sum()),
               method="product kernels on the real plan, gathered ids rewritten")
    return out


BUILD_INFO = {}
HUB_INFO = {}


def build_graph(nodes: int, edges: int, dev, rank: int, world: int, edges_np=None):
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    phase("graph_edges", 600)
    t0 = time.time()
    if edges_np is not None:
        s = torch.from_numpy(edges_np[0]).to(dev)
        d = torch.from_numpy(edges_np[1]).to(dev)
    elif world > 1:
        # rank 0 draws the edge list (numpy recipe), every rank receives it (RCCL broadcast)
        bdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        if rank == 0:
            s, d = rmat_edges(nodes, edges, 0)
            buf = torch.from_numpy(np.stack([s, d])).to(bdev)
        else:
            buf = torch.empty((2, edges), dtype=torch.int64, device=bdev)
        dist.broadcast(buf, 0)
        buf = buf.to(dev)
        s, d = buf[0], buf[1]
    else:
        s, d = rmat_edges(nodes, edges, 0)
        s = torch.from_numpy(s).to(dev)
        d = torch.from_numpy(d).to(dev)
    log(f"[bench] rmat edges ready in {time.time() - t0:.1f}s")
    torch.cuda.synchronize(dev)
    phase("graph_build", 600)
    t0 = time.time()
    g = gcn_adjacency(s, d, nodes, device=dev)  # HIP graph builder (graph_build.hip)
    torch.cuda.synchronize(dev)
    BUILD_INFO["gcn_adjacency_build_s"] = time.time() - t0
    log(f"[bench] normalized CSR nnz={g.nnz} in {BUILD_INFO['gcn_adjacency_build_s']:.2f}s")
    return g


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants this job (cgroup v2 cpu.max), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        return None


def cpu_threads() -> int:
    """Host threads for the CPU lines: every CPU this process may use, capped by the box's
    per-GPU CPU share -- the cgroup quota (cpu.max: 16 CPUs of time on the GPU box, whose
    affinity mask lists all 256 host CPUs) and OMP_NUM_THREADS (16 there too).
    GNN_CPU_THREADS overrides. Round 4 also timed the sample on all 256 host CPUs: inside the
    16-CPU quota that oversubscribes, 0.600 s against 0.182 s at 16 threads
    (profiles/r04zd_bench_default.log), so the lines use the quota."""
    if os.environ.get("GNN_CPU_THREADS"):
        return int(os.environ["GNN_CPU_THREADS"])
    n = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    if quota:
        n = min(n, quota)
    share = os.environ.get("OMP_NUM_THREADS")
    return min(n, int(share)) if share and share.isdigit() and int(share) > 0 else n


def cpu_baseline(g, X, feat: int, threads: int | None = None):
    """Oracle C restatement of the reference SpMM timed on this host's cores (rank 0, N=1)."""
    from oracle import c_oracle
    threads = cpu_threads() if threads is None else threads
    c_oracle.set_threads(threads)
    rowptr = g.rowptr.cpu().numpy()
    col = g.col.cpu().numpy()
    val = g.val.cpu().numpy()
    Xn = X.cpu().numpy()
    # a bounded sample: the leading rows holding <= 25M entries (the whole graph at cfg2)
    r1 = max(1, min(g.n_rows, int(np.searchsorted(rowptr, 25_000_000, side="right")) - 1))
    e1 = int(rowptr[r1])
    c_oracle.spmm_csr(rowptr, col, val, Xn, None, 0, min(r1, 20000))  # warm-up
    times = []
    t_budget = time.perf_counter()
    for _ in range(5):
        t0 = time.perf_counter()
        c_oracle.spmm_csr(rowptr, col, val, Xn, None, 0, r1)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_budget > 15:
            break
    t = statistics.median(times)
    sample = "full graph" if r1 == g.n_rows else f"rows 0..{r1} of {g.n_rows}"
    return {"value": e1 / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"{sample} (nnz {e1}, F={feat}), oracle/spmm_oracle.c OpenMP "
                      f"double-accumulation SpMM, median of {len(times)} runs",
            "seconds_per_step": t, "host": host_cpu_info(threads)}


STAMP_SOURCES = ("graphneuralnetwork_amd/csrc", "graphneuralnetwork_amd/ops.py",
                 "graphneuralnetwork_amd/graph.py")


def source_stamp(root: Path = ROOT) -> str:
    """sha256 (16 hex) over the kernel sources and the schedule builders (csrc/, ops.py,
    graph.py): what a PMC traffic file or a kernel-stats summary was measured on. The profile
    summaries carry it (tools/summarize_profiles.py) and bench.py compares it with the tree it
    runs (roofline.traffic_stale)."""
    import hashlib
    h = hashlib.sha256()
    files = []
    for s in STAMP_SOURCES:
        p = root / s
        files += sorted(f for f in p.rglob("*") if f.is_file()) if p.is_dir() else [p]
    for f in files:
        if f.suffix not in (".hip", ".hpp", ".cpp", ".h", ".py", ".map"):
            continue
        h.update(str(f.relative_to(root)).encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


def library_stamps() -> dict:
    """The loaded library's embedded source stamp beside the tree's;
    _lib.load() already refused a mismatch, the line records both."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd import build as B
    lib_stamp, tree = _lib.build_stamp(), B.lib_source_stamp()
    return {"lib_stamp": lib_stamp, "lib_tree_stamp": tree, "lib_stamp_ok": lib_stamp == tree}


def traffic_record(path: Path):
    """(traffic bytes, source note, stamp, stale) of a profiles/traffic_*.json, or Nones."""
    try:
        t = json.loads(path.read_text())
        traffic = t["traffic_bytes"]
    except (OSError, ValueError, KeyError):
        return None, None, None, None
    stamp = t.get("source_stamp")
    src = (str(path.relative_to(ROOT)) if path.is_relative_to(ROOT) else str(path)) + \
        ": rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE of this command (round %s)" % t.get("round")
    return traffic, src, stamp, stamp != source_stamp()


def traffic_fields(path: Path) -> dict:
    """The roofline keys that say where ``traffic`` came from and whether it is current."""
    traffic, src, stamp, stale = traffic_record(path)
    return {"traffic": traffic, "traffic_source": src, "traffic_stamp": stamp,
            "tree_stamp": source_stamp(), "traffic_stale": stale}


def load_traffic(name: str):
    """PMC traffic summary profiles/traffic_<name>.json (tools/summarize_profiles.py) or None."""
    traffic, src, _, _ = traffic_record(ROOT / "profiles" / f"traffic_{name}.json")
    return traffic, src


def cpu_reference_ops(g, X, feat: int, budget_s: float = 25.0, max_nnz: int = 21_000_000):
    """SURVEY 8(d) CPU lines beside the port: the reference's own operator -- torch.spmm on
    the uncoalesced COO built as GCN/data_utils.py:63-70 (CSC -> COO order, int64 indices,
    GCN/GCN.py:43) -- and torch.sparse.mm on CSR, both with every allowed host thread."""
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        # bounded sample: the leading rows holding at most max_nnz edges (the whole graph at cfg2)
        rowptr = g.rowptr.cpu()
        r1 = min(g.n_rows, int(torch.searchsorted(rowptr, max_nnz, right=True)) - 1)
        r1 = max(r1, 1)
        e1 = int(rowptr[r1])
        rows = torch.repeat_interleave(torch.arange(r1, dtype=torch.int64),
                                       rowptr[1:r1 + 1] - rowptr[:r1])
        cols = g.col[:e1].cpu().to(torch.int64)
        vals = g.val[:e1].cpu()
        order = torch.argsort(cols, stable=True)          # scipy CSC -> COO order
        idx = torch.stack([rows[order], cols[order]])
        coo = torch.sparse_coo_tensor(idx, vals[order], (r1, g.n_cols))  # uncoalesced
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # "sparse CSR support is in beta"
            csr = torch.sparse_csr_tensor(rowptr[:r1 + 1], cols, vals, (r1, g.n_cols))
        # ATen's CPU sparse kernels index the dense operand with 32-bit offsets: at N*F >= 2^31
        # (cfg5: 10M x 256) torch.spmm segfaults, so the operand goes in column blocks there
        n_blk = -(-X.numel() // (2 ** 31 - 1))
        Xc = [c.contiguous() for c in X.cpu().chunk(n_blk, dim=1)]
        out = {}
        for name, fn in (("torch_spmm_coo", lambda: [torch.spmm(coo, c) for c in Xc]),
                         ("torch_sparse_mm_csr", lambda: [torch.sparse.mm(csr, c) for c in Xc])):
            t_all = time.perf_counter()
            fn()                                          # warm-up
            times = []
            while not times or (len(times) < 5 and time.perf_counter() - t_all < budget_s / 2):
                t0 = time.perf_counter()
                fn()
                times.append(time.perf_counter() - t0)
            t = statistics.median(times)
            out[name] = {"value": e1 / t, "unit": "edges/s", "threads": threads,
                         "seconds_per_step": t, "runs": len(times)}
        sample = "full graph" if r1 == g.n_rows else f"rows 0..{r1} ({e1} edges)"
        if n_blk > 1:
            sample += f", X in {n_blk} column blocks (N*F >= 2^31 crashes ATen's CPU spmm)"
        out["note"] = ("torch_spmm_coo is the reference's CPU operator on the reference's tensor "
                       "layout (effectively single-threaded in ATen); %s, F=%d" % (sample, feat))
        return out
    finally:
        torch.set_num_threads(prev)


def _cpu_time(fn, budget_s: float):
    """Median wall seconds of fn() (1 warm-up, up to 5 runs within the budget)."""
    t_all = time.perf_counter()
    fn()
    times = []
    while not times or (len(times) < 5 and time.perf_counter() - t_all < budget_s):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return statistics.median(times), len(times)


def cpu_spgat_ops(g, X, W, a_s, a_d, H: int, Fh: int, max_edges: int = 2_000_000,
                  budget_s: float = 20.0):
    """The reference's CPU operator sequence for one SpGAT layer (SpGraphAttentionLayer.forward,
    GAT/models/layers.py:94-131, one head after another as GAT.py:16 does): h = X W; the E x 2F
    edge matrix [h_i | h_j]; exp(-LeakyReLU(a . edge_h)); row sums and h' by COO matmuls
    (SpecialSpmm, layers.py:43-69); h' / rowsum.  Restated with torch CPU ops on the leading
    rows holding <= max_edges edges, every allowed host thread."""
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rowptr = g.rowptr.cpu()
        r1 = max(1, min(g.n_rows, int(torch.searchsorted(rowptr, max_edges, right=True)) - 1))
        e1 = int(rowptr[r1])
        src = torch.repeat_interleave(torch.arange(r1), rowptr[1:r1 + 1] - rowptr[:r1])
        dst = g.col[:e1].cpu().to(torch.int64)
        edge = torch.stack([src, dst])
        ones = torch.ones(g.n_cols, 1)
        Ws = W.view(-1, H, Fh)
        a = torch.cat([a_s.view(H, Fh), a_d.view(H, Fh)], 1)  # [H, 2 Fh]

        hs = [X @ Ws[:, hd, :] for hd in range(H)]  # the N x Fh transforms: outside the sample

        def layer():
            outs = []
            for hd in range(H):
                h = hs[hd]
                edge_h = torch.cat([h[src], h[dst]], 1)
                e = torch.exp(-torch.nn.functional.leaky_relu(edge_h @ a[hd], 0.2))
                A = torch.sparse_coo_tensor(edge, e, (r1, g.n_cols))
                outs.append(torch.sparse.mm(A, h) / torch.sparse.mm(A, ones))
            return torch.cat(outs, 1)

        t, runs = _cpu_time(layer, budget_s)
        return {"torch_spgat_layer": {"value": e1 / t, "unit": "edges/s", "threads": threads,
                                      "seconds_per_step": t, "runs": runs},
                "note": f"torch CPU restatement of SpGraphAttentionLayer x {H} heads on rows "
                        f"0..{r1} ({e1} edges), the X W transforms excluded (generous to the CPU); the dense "
                        f"GraphAttentionLayer is O(N^2) at this size"}
    finally:
        torch.set_num_threads(prev)


def cpu_sage_ops(table, batch, F: int, H: int, budget_s: float = 20.0):
    """The reference's CPU GraphSAGE forward for this batch (GraphSAGE/GraphSAGE.py:38-52 with
    graph_utils.Aggregator MEAN): the collate-side neighbour tensor [M, k1, F]
    (data_utils.py:141-147) is materialised once outside the timed region, then
    mean -> Linear(cat) -> ReLU, the torch.embedding re-gathers, mean -> Linear -> ReLU,
    classifier.  torch CPU ops, every allowed host thread, same shapes, random weights."""
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        T = torch.from_numpy(table)
        front = batch.frontier.cpu()
        nb1 = batch.frontier_nbrs.cpu()
        cmap, nmap = batch.center_map.cpu(), batch.neigh_map.cpu()
        self_feats = T[front]
        neigh_feats = T[nb1]                                   # [M, k1, F]
        gen = torch.Generator().manual_seed(0)
        W0 = torch.randn(H, 2 * F, generator=gen) * 0.05
        W1 = torch.randn(H, 2 * H, generator=gen) * 0.05
        Wc = torch.randn(3, H, generator=gen) * 0.05

        def forward():
            h1 = torch.relu(torch.cat([self_feats, neigh_feats.mean(1)], 1) @ W0.T)
            agg = torch.embedding(h1, nmap).mean(1)
            h2 = torch.relu(torch.cat([torch.embedding(h1, cmap), agg], 1) @ W1.T)
            return h2 @ Wc.T

        t, runs = _cpu_time(forward, budget_s)
        return {"torch_graphsage_forward": {"value": batch.sampled_edges / t, "unit": "edges/s",
                                            "threads": threads, "seconds_per_step": t,
                                            "runs": runs},
                "note": "torch CPU restatement of GraphSAGE.forward (MEAN, 2 layers) on the same "
                        "sampled batch, neighbour tensor pre-materialised as collate_fn does"}
    finally:
        torch.set_num_threads(prev)


def describe_path(g, feat: int):
    """The kernels one single-GPU step launched (read from the plans the warm-up built)."""
    xp = next((v for k, v in g._plans.items()
               if isinstance(k, tuple) and k[0] == "_xcd" and v is not None), None)
    if xp is not None and xp.prefix:
        from graphneuralnetwork_amd import ops
        if ops.XCD_DIRECT:
            return ("spmm_csr_kernel pass 1 (%d XCD-sliced hub items of rows with >= %d edges, "
                    "workgroup w on XCD w %% 8, reading the %d hub rows in place: the first "
                    "%.0f MiB of X in the column-degree order) + spmm_csr_kernel<HUB, tasks> pass "
                    "2 (remaining edges + partial refs, short rows as packed row tasks) + "
                    "spmm_fixup_kernel, per-step HIP events"
                    % (xp.n_items, xp.min_deg, xp.k, xp.k * 4 * feat / 2**20))
    if xp is not None:
        return ("gather_rows_kernel (hub staging: the %d highest-degree rows of X, %.0f MiB) + "
                "spmm_csr_kernel<HUB> pass 1 (%d XCD-sliced hub items of rows with >= %d edges, "
                "workgroup w on XCD w %% 8) + spmm_csr_kernel<HUB> pass 2 (remaining edges + "
                "partial refs) + spmm_fixup_kernel, per-step HIP events"
                % (xp.k, xp.k * 4 * feat / 2**20, xp.n_items, xp.min_deg))
    hub = next((v for k, v in g._plans.items() if isinstance(k, tuple) and k[0] == "_hub"), None)
    if hub is not None:
        return ("gather_rows_kernel (hub staging: the %d highest-degree rows of X, %.0f MiB) + "
                "spmm_csr_kernel<HUB> + spmm_fixup_kernel, per-step HIP events"
                % (hub.k, hub.k * 4 * feat / 2**20))
    return "spmm_csr_kernel (+ spmm_fixup_kernel), per-step HIP events"


def _all_gather_phase_values(v: list, world: int, dev):
    """[world, len(v)] float64 of every rank's phase times (an all-to-all-v of one row)."""
    from graphneuralnetwork_amd.distributed import _all_gather_floats
    return _all_gather_floats(v, world, dev)


def time_steps(step, steps: int, warmup: int, dev):
    """Per-step HIP-event times (ms) on the current stream + wall seconds for `steps` steps."""
    stream = torch.cuda.current_stream(dev)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize(dev)
    return [a.elapsed_time(b) for a, b in ev], time.perf_counter() - t0


def run_gat(args, dev, rank: int = 0, world: int = 1):
    """cfg3: one 8-head GAT layer (dense softmax semantics, ELU) over the 1M/10M RMAT graph."""
    from graphneuralnetwork_amd.ops import (GAT_DENSE, GAT_SPARSE, gat_aggregate, gat_logits,
                                            gat_project)
    if world != 1:
        return run_gat_edgecut(args, dev, rank, world)
    wl = WORKLOADS["cfg3"]
    g = build_graph(wl["nodes"], wl["edges"], dev, 0, 1)
    H, Fh, Fin = 8, 8, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(g.n_rows, Fin, device=dev, generator=gen)
    W = torch.randn(Fin, H * Fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    Wh = torch.mm(X, W)
    el, er = gat_logits(Wh, H, Fh, a_s, a_d)
    out = torch.empty_like(Wh)
    # as the drop-in attention layers run at inference (gat._AttentionBase._ordered): over the
    # column-degree-ordered graph A P^T, the projection writing Wh / er in its column order
    from graphneuralnetwork_amd.ops import gat_column_order
    t0 = time.perf_counter()
    order = gat_column_order(g, H, Fh)
    torch.cuda.synchronize(dev)
    order_s = time.perf_counter() - t0
    ga = g if order is None else order.graph
    inv = None if order is None else order.inv
    Wh_o, el_o, er_o = gat_project(X, W, H, Fh, a_s, a_d, col_rows=inv)

    def layer():  # GAT inference layer: fused MFMA transform + logits, then aggregation
        wh, e_l, e_r = gat_project(X, W, H, Fh, a_s, a_d, col_rows=inv)
        return gat_aggregate(ga, wh, e_l, e_r, H, Fh, 0.2, GAT_DENSE, "elu", out=out, a_dst=a_d)

    agg = {m: (lambda m=m: gat_aggregate(ga, Wh_o, el_o, er_o, H, Fh, 0.2, m, "elu", out=out,
                                         a_dst=a_d))
           for m in (GAT_DENSE, GAT_SPARSE)}
    layer_ms, wall = time_steps(layer, args.steps, args.warmup, dev)
    agg_ms = {m: time_steps(f, args.steps, args.warmup, dev)[0] for m, f in agg.items()}
    proj_ms = time_steps(lambda: gat_project(X, W, H, Fh, a_s, a_d, col_rows=inv), args.steps,
                         args.warmup, dev)[0]
    nnz, n = g.nnz, g.n_rows
    from graphneuralnetwork_amd.ops import hub_rows_for
    hub_k = hub_rows_for(g.n_cols, H * Fh + H)
    # SURVEY 8(d) gather model (every gathered Wh row / er entry from HBM) and the compulsory
    # bytes (each input read once, the output written once): col per edge; rowptr, el, the
    # Wh row, the er entry and the output row per node
    gm = nnz * (4 + 4 * H + 4 * H * Fh) + n * (8 + 4 * H + 4 * H * Fh)
    comp = nnz * 4 + n * (8 + 4 * H + 4 * H + 4 * H * Fh + 4 * H * Fh)
    k_ms = statistics.mean(agg_ms[GAT_DENSE])
    t = k_ms / 1e3
    achieved = comp / t / 1e9
    tf = traffic_fields(ROOT / "profiles" / "traffic_cfg3_F64.json")
    traffic = tf["traffic"]
    from graphneuralnetwork_amd.ops import transform_precision
    proj_arith = ("fp32 products from split-bf16 MFMAs (x and W in three bf16 pieces, six "
                  "v_mfma_f32_16x16x32_bf16 products accumulated in fp32)"
                  if transform_precision() == "split-bf16" else
                  "fp32 MFMA (v_mfma_f32_16x16x4_f32)")
    res = {"metric": "GAT 8-head aggregated edges/sec (all heads) + achieved HBM GB/s",
           "value": nnz * args.steps / wall, "unit": "edges/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
           "median_step_ms": statistics.median(layer_ms), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic R-MAT",
           "config": {"workload": wl["name"], "nodes": n, "nnz": nnz, "heads": H, "head_dim": Fh,
                      "in_dim": Fin,
                      "step": "gnn_gat_project_rows (X@W at K=64: %s; + the el / er logits; Wh / "
                              "er rows scattered into the column order) + gnn_gat_csr (dense, "
                              "ELU)" % proj_arith,
                      **({"column_order": "A P^T: columns relabelled by in-degree once per "
                                          "graph (%.2f s, outside the timed region); the "
                                          "projection writes Wh / er in that order (el in "
                                          "place); output rows in the original order"
                                          % order_s} if order is not None else {})},
           "layer_ms": statistics.median(layer_ms),
           "aggregate_ms": {"dense": statistics.median(agg_ms[GAT_DENSE]),
                            "sparse": statistics.median(agg_ms[GAT_SPARSE])},
           "project_ms": statistics.median(proj_ms), "project_arithmetic": proj_arith,
           "project_tflops": 2.0 * n * Fin * (H * Fh + 2 * H) / (statistics.median(proj_ms) / 1e3)
           / 1e12,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBPS, **tf,
                        "compulsory_bytes": comp,
                        "traffic_over_compulsory": traffic / comp if traffic else None,
                        "gather_model_bytes": gm, "gather_model_GBps": gm / t / 1e9,
                        "gather_model_frac": gm / t / 1e9 / HBM_PEAK_GBPS,
                        "traffic_GBps": traffic / t / 1e9 if traffic else None,
                        "traffic_frac": traffic / t / 1e9 / HBM_PEAK_GBPS if traffic else None,
                        "kernel": (("gat_eh_kernel<dense, er from the rows> (segments, mid "
                                    "and one-edge rows; the Wh rows of the %d highest-degree "
                                    "columns read in place, the first rows in the column-degree "
                                    "order) + " % hub_k) if order is not None
                                   else ("gather_rows_kernel x2 (hub staging: Wh / er rows of "
                                         "the %d highest-degree columns) + gat_eh_kernel<dense> + "
                                         % hub_k) if hub_k else "gat_eh_kernel<dense> + ")
                                  + "gat_short_kernel + gat_fixup_kernel",
                        "avg_launch_ms": k_ms,
                        "median_launch_ms": statistics.median(agg_ms[GAT_DENSE])}}
    if not args.no_replay and order is not None:
        rpf = gat_replay(ga, hub_k, agg[GAT_DENSE])
        if rpf is not None:
            rpf["frac_at_all_in_L2"] = comp / (rpf["all_gathers_in_L2_ms"] / 1e3) / 1e9 / \
                HBM_PEAK_GBPS
            res["roofline"]["replay_floor"] = rpf
    if not args.no_cpu_baseline:
        from oracle import c_oracle
        threads = cpu_threads()
        c_oracle.set_threads(threads)
        rp = g.rowptr.cpu().numpy()
        col = g.col.cpu().numpy()
        whn, eln, ern = Wh.cpu().numpy(), el.cpu().numpy(), er.cpu().numpy()
        c_oracle.gat_csr(rp, col, whn, eln, ern, H, Fh, 0.2, False, 0, 20000)  # warm-up
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            c_oracle.gat_csr(rp, col, whn, eln, ern, H, Fh, 0.2, False)
            times.append(time.perf_counter() - t0)
        tc = statistics.median(times)
        res["cpu_baseline"] = {"value": nnz / tc, "unit": "edges/s", "cores": threads,
                               "kind": "port", "seconds_per_step": tc,
                               "sample": f"full graph ({n} rows, nnz {nnz}), oracle/spmm_oracle.c "
                                         f"oracle_gat_csr (OpenMP, float64, dense softmax, "
                                         f"8 heads), median of {len(times)} runs",
                               "host": host_cpu_info(threads)}
        if not args.no_cpu_reference:
            try:
                res["cpu_reference_ops"] = cpu_spgat_ops(g, X.cpu(), W.cpu(), a_s.cpu(), a_d.cpu(),
                                                         H, Fh)
            except Exception as e:
                res["cpu_reference_ops"] = {"error": repr(e)}
    del Wh, out, Wh_o, el_o, er_o
    torch.cuda.empty_cache()
    if not args.no_train:
        res["train_step"] = gat_train_step(g, X, H, Fh, args, dev)
    del g, X
    torch.cuda.empty_cache()
    return res


def gat_train_step(g, X, H: int, Fh: int, args, dev) -> dict:
    """One training step of the drop-in 8-head GAT attention block at cfg3 (GAT.py:16's heads
    through GATBase._heads: one X W GEMM for all heads, the fused edge-softmax aggregation with
    ELU; GAT/train_eval.py:75-76's loss.backward()): forward + backward with W, a_src, a_dst
    requiring grad (X is the input features). The backward's HIP passes (csrc/gat_bwd.hip:
    the coalesced prep + the row pass, the recomputing node pass over A^T; replacing the
    autograd of GAT/models/layers.py:22-37 and SpecialSpmmFunction.backward :54-64) are also
    timed alone, each with a roofline on its compulsory bytes."""
    from graphneuralnetwork_amd.gat import GAT
    from graphneuralnetwork_amd.ops import (GAT_DENSE, gat_aggregate, gat_backward, gat_logits,
                                            gat_train_order)
    gen = torch.Generator(device=dev).manual_seed(3)
    net = GAT(X.shape[1], Fh, 3, dropout=0.0, alpha=0.2, nheads=H).to(dev).train()
    gy = torch.randn(g.n_rows, H * Fh, device=dev, generator=gen)
    steps = max(3, min(args.steps, 10))
    # the block runs over the graph GATBase.forward trains on: P A P^T (nodes in degree order,
    # gat_train_order; x permuted once per model forward, on entry) -- X, gy in that order
    t0 = time.perf_counter()
    order = gat_train_order(g, H, Fh)
    torch.cuda.synchronize(dev)
    order_s = time.perf_counter() - t0
    g_nat, X_nat, gy_nat = g, X, gy
    if order is not None:
        g, X, gy = order.graph, order.permute_rows(X), order.permute_rows(gy)

    def step():
        net.zero_grad(set_to_none=True)
        net._heads(X, g).backward(gy)

    step_ms = time_steps(step, steps, 2, dev)[0]
    fwd_ms = time_steps(lambda: net._heads(X, g), steps, 2, dev)[0]
    keep = {"y": net._heads(X, g)}
    bwd_ms = time_steps(lambda: keep["y"].backward(gy, retain_graph=True), steps, 2, dev)[0]
    del keep

    def step_nat():
        net.zero_grad(set_to_none=True)
        net._heads(X_nat, g_nat).backward(gy_nat)

    nat_ms = time_steps(step_nat, steps, 2, dev)[0] if order is not None else step_ms
    # the whole GAT model (8 heads, ELU, out_att 64 -> 3, ELU; GAT/train_eval.py:75-76 with a
    # NLL loss on log_softmax of the logits), x entering and the logits leaving in the
    # original order (GATBase.forward's two permutes inside the step)
    labels = torch.randint(0, 7, (g.n_rows,), device=dev, generator=gen)
    idx_train = torch.arange(0, g.n_rows, 10, device=dev)
    ce = torch.nn.CrossEntropyLoss()
    model = GAT(X.shape[1], Fh, 7, dropout=0.6, alpha=0.2, nheads=H).to(dev).train()

    def model_step():  # GAT/train_eval.py:72-76: CE on output[idx_train], backward
        model.zero_grad(set_to_none=True)
        ce(model(X_nat, g_nat)[idx_train], labels[idx_train]).backward()

    model_ms = time_steps(model_step, steps, 2, dev)[0]
    # the three backward passes alone (the tensors the autograd Function saves)
    W = torch.cat([m.W for m in net.attentions], 1).detach()
    a_s = torch.cat([m._a_parts()[0] for m in net.attentions]).detach()
    a_d = torch.cat([m._a_parts()[1] for m in net.attentions]).detach()
    Wh = torch.mm(X, W)
    el, er = gat_logits(Wh, H, Fh, a_s, a_d)
    stats = torch.empty((g.n_rows, H), device=dev)
    out = gat_aggregate(g, Wh, el, er, H, Fh, 0.2, GAT_DENSE, "elu", stats=stats)
    per = {}
    for i in range(steps + 2):
        tl = []
        gat_backward(g, Wh, el, er, stats, out, gy, a_s, a_d, H, Fh, 0.2, GAT_DENSE, True,
                     timings=tl)
        torch.cuda.synchronize(dev)
        if i >= 2:
            for name, a, b in tl:
                per.setdefault(name, []).append(a.elapsed_time(b))
    n, nnz, feat = g.n_rows, g.nnz, H * Fh
    two_pass = "rows" in per
    comp = {"prep": n * 4 * (3 * feat + H),
            "edges": nnz * (4 + 8 * H) + n * (8 + 16 * H + 4 * feat) + g.n_cols * (4 * H + 4 * feat),
            "rows": nnz * 4 + n * (8 + 12 * feat + 28 * H) + g.n_cols * (4 * H + 4 * feat),
            "nodes": (nnz * 4 + n * (8 + 12 * feat + 28 * H)) if two_pass else
                     (nnz * (12 + 8 * H) + n * (8 + 8 * feat + 8 * H))}
    what = {"prep": "gat_bwd_prep_kernel: dout = dy ELU'(out), D = dout . out",
            "edges": "gat_bwd_edge_kernel (+ del fix-up): SDDMM g = dout_i . Wh_j, edge weights "
                     "w_ij and softmax/LeakyReLU gradients ds_ij written per (edge, head)",
            "rows": "gat_bwd_prep_rec_kernel (dout, D_i and the per-(row, head) record {el, "
                    "lse, D}, coalesced) + gat_bwd_rows_kernel (+ del fix-up): SDDMM g = "
                    "dout_i . Wh_j and ds_ij summed into del_i",
            "nodes": ("gat_bwd_node_r_kernel (+ fix-up) over A^T (A itself when symmetric): "
                      "a_ij, g_ij, w_ij, ds_ij recomputed from the gathered dout_i and {el, lse, "
                      "D}_i; dWh_j = sum_i w_ij dout_i + der_j a_dst + del_j a_src") if two_pass
                     else ("gat_bwd_node_kernel (+ fix-up) over the transposed CSR: dWh_j = "
                           "sum_i w_ij dout_i + der_j a_dst + del_j a_src")}
    kernels = {}
    for name, ms in per.items():
        t = statistics.mean(ms) / 1e3
        kernels[name] = {"median_ms": statistics.median(ms), "kernel": what[name],
                         "roofline": {"bound": "hbm", "achieved": comp[name] / t / 1e9,
                                      "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                      "frac": comp[name] / t / 1e9 / HBM_PEAK_GBPS,
                                      "compulsory_bytes": comp[name], "avg_launch_ms": t * 1e3}}
    res = {"what": "GAT %d-head attention block (%d -> %dx%d, dense softmax, ELU) forward + "
                   "loss.backward() at cfg3; W, a_src, a_dst require grad" % (H, X.shape[1], H, Fh),
           "step_ms": statistics.median(step_ms), "forward_ms": statistics.median(fwd_ms),
           "backward_ms": statistics.median(bwd_ms),
           "edges_per_s": nnz / (statistics.median(step_ms) / 1e3),
           "node_order": ("P A P^T (gat_train_order: nodes relabelled by degree once per graph, "
                          "%.2f s outside the timed region; X, dy in that order as "
                          "GATBase.forward hands them to the block)" % order_s)
                         if order is not None else "natural",
           "natural_order_step_ms": statistics.median(nat_ms),
           "model_step_ms": statistics.median(model_ms),
           "model_step_what": "GAT(%d, %d, 7, dropout=0.6, nheads=%d).train() forward + "
                              "CrossEntropyLoss(output[idx_train]) backward, idx_train = every "
                              "10th node (GAT/train_eval.py:72-76; both attention layers, the "
                              "7-class out_att zero-padded to 8 features; x in and logits out "
                              "in the original order)" % (X.shape[1], Fh, H),
           "forward_path": "X W on the MFMA transform (_ProjectFn) + gat_logits + the edge-head "
                           "gat_aggregate (er from the gathered rows) with per-row log-sum-exp "
                           "stats",
           "backward_kernels": kernels,
           "compulsory_bytes_model": ({
               "rows": "4 nnz + N (8 + 12 H Fh + 28 H) + N (4 H + 4 H Fh): y, dy, el, lse, "
                       "rowptr, col read, dout, {el, lse, D, 0}, del written, er / Wh gathered "
                       "once",
               "nodes": "4 nnz + N (8 + 12 H Fh + 28 H): rowptr, sources, dout + record "
                        "gathered once, own Wh / er / del, dWh and der written"} if two_pass else {
               "prep": "4 N (3 H Fh + H)",
               "edges": "nnz (4 + 8 H) + N (8 + 16 H + 4 H Fh) + N (4 H + 4 H Fh)",
               "nodes": "nnz (12 + 8 H) + N (8 + 8 H Fh + 8 H)"})}
    if not args.no_cpu_baseline:
        try:
            res["cpu_reference_ops"] = cpu_gat_train_ops(g, X.cpu(), W.cpu(), a_s.cpu(),
                                                         a_d.cpu(), H, Fh)
        except Exception as e:
            res["cpu_reference_ops"] = {"error": repr(e)}
    del net, model, gy, Wh, out, stats, X_nat, gy_nat, g_nat
    torch.cuda.empty_cache()
    return res


def cpu_gat_train_ops(g, X, W, a_s, a_d, H: int, Fh: int, max_edges: int = 1_000_000,
                      budget_s: float = 10.0) -> dict:
    """The sparse attention layer's math (GAT/models/layers.py:94-131 per head, softmax-
    normalised and ELU as the dense layer) forward + backward by torch CPU autograd on an edge
    list (index_select / index_add: the reference's own backward materialises dense N x N
    gradients and cannot run at this size), on the leading rows holding <= max_edges edges,
    every allowed host thread."""
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rowptr = g.rowptr.cpu()
        r1 = max(1, min(g.n_rows, int(torch.searchsorted(rowptr, max_edges, right=True)) - 1))
        e1 = int(rowptr[r1])
        src = torch.repeat_interleave(torch.arange(r1), rowptr[1:r1 + 1] - rowptr[:r1])
        dst = g.col[:e1].cpu().to(torch.int64)
        Wp = W.clone().requires_grad_(True)
        asp = a_s.clone().requires_grad_(True)
        adp = a_d.clone().requires_grad_(True)
        gy = torch.randn(r1, H * Fh)

        def step():
            for t in (Wp, asp, adp):
                t.grad = None
            Wh = (X @ Wp).view(-1, H, Fh)
            el = (Wh[:r1] * asp.view(H, Fh)).sum(-1)
            er = (Wh * adp.view(H, Fh)).sum(-1)
            z = torch.nn.functional.leaky_relu(el[src] + er[dst], 0.2)
            m = torch.zeros(r1, H).index_reduce_(0, src, z.detach(), "amax", include_self=False)
            p = torch.exp(z - m[src])
            den = torch.zeros(r1, H).index_add_(0, src, p)
            num = torch.zeros(r1, H, Fh).index_add_(0, src, p.unsqueeze(-1) * Wh[dst])
            out = torch.nn.functional.elu(num / den.unsqueeze(-1))
            out.view(r1, -1).backward(gy)

        t, runs = _cpu_time(step, budget_s)
        return {"torch_cpu_train_step": {"value": e1 / t, "unit": "edges/s", "threads": threads,
                                         "seconds_per_step": t, "runs": runs},
                "note": f"torch CPU autograd of the edge-list attention layer, {H} heads, rows "
                        f"0..{r1} ({e1} edges; X W over all {X.shape[0]} rows)"}
    finally:
        torch.set_num_threads(prev)


def run_gat_edgecut(args, dev, rank: int, world: int):
    """cfg3 over N GPUs (weak scaling: N x the 1M / 10M R-MAT graph, edge-cut by nnz-balanced
    row blocks): one step = this rank's fused MFMA projection + logits (gat_project) and the
    EdgeCutGat layer -- the [Wh | er] halo rows exchanged by one RCCL all-to-all-v on a
    communication stream while the interior pass runs, then the halo pass with the interior
    result merged as a log-sum-exp pseudo-edge (distributed.EdgeCutGat). Value = all ranks'
    edges / the slowest rank's time."""
    from graphneuralnetwork_amd.distributed import EdgeCutGat, build_partition
    from graphneuralnetwork_amd.ops import GAT_DENSE, gat_project
    wl = WORKLOADS["cfg3"]
    nodes = int(wl["nodes"] * world * args.scale)
    edges = int(wl["edges"] * world * args.scale)
    g = build_graph(nodes, edges, dev, rank, world)
    H, Fh, Fin = 8, 8, 64
    phase("partition_build", 900)
    t0 = time.time()
    part = build_partition(g, rank, world)
    t_part = time.time() - t0
    r0, r1 = part.bounds[rank], part.bounds[rank + 1]
    nnz_local = int(g.rowptr[r1] - g.rowptr[r0])
    del g
    torch.cuda.empty_cache()
    gen = torch.Generator(device=dev).manual_seed(0)
    W = torch.randn(Fin, H * Fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    X = torch.randn(part.n_own, Fin, device=dev, generator=gen)
    layer = EdgeCutGat(part, H, Fh, dev)

    def step():
        wh, el, er = gat_project(X, W, H, Fh, a_s, a_d)
        return layer(wh, a_s, a_d, 0.2, GAT_DENSE, "elu", el=el, er=er)

    phase("first_step", 300)
    step()
    torch.cuda.synchronize(dev)
    phase("warmup", 300)
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize(dev)
    phase("timed_steps", 300)
    dist.barrier()
    step_ms, wall = time_steps(step, args.steps, 0, dev)
    dist.barrier()
    phase("reduce", 120)
    red = torch.tensor([wall, float(nnz_local), statistics.median(step_ms)], dtype=torch.float64,
                       device=dev if dist.get_backend() == "nccl" else "cpu")
    mx = red[0::2].clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    tot = red[1:2].clone()
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    T, nnz_all = float(mx[0]), float(tot[0])
    return {"metric": "GAT 8-head aggregated edges/sec (all heads), edge-cut over N GPUs",
            "value": nnz_all * args.steps / T, "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": T / args.steps * 1e3,
            "median_step_ms_max_over_ranks": float(mx[1]), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic R-MAT (N x 1M / 10M)",
            "config": {"workload": wl["name"] + f", edge-cut over {world} GPUs", "nodes": nodes,
                       "directed_edges": edges, "nnz": int(nnz_all), "heads": H, "head_dim": Fh,
                       "in_dim": Fin, "parallelism": f"edge-cut{world}",
                       "step": "gnn_gat_project + EdgeCutGat (RCCL all-to-all-v of [Wh | er] "
                               "halo rows overlapping the interior pass, then the halo pass "
                               "with the log-sum-exp pseudo-edge merge)"},
            "partition_build_s": t_part, "row_bounds": part.bounds,
            "exchange_rows_rank0": {"send": int(sum(part.send_counts)),
                                    "recv": int(sum(part.recv_counts))},
            "overlapped_two_pass": layer._halo_pass is not None}


def run_sage(args, dev, rank: int = 0, world: int = 1, edges_np=None):
    """cfg4: GraphSAGE 2-layer MEAN forward on a device-sampled [25, 10] batch of 8192 seeds.
    With N ranks (replicated table, no collective on the forward path) the global
    batch is 8192 x N seeds and rank r runs its shard (distributed.shard_seeds, its own
    sampler stream): weak scaling, value = all ranks' sampled edges / the slowest rank."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.ops import sage_gather_aggregate
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import degree_ordered, sample_batch, symmetric_adjacency
    wl = WORKLOADS["cfg4"]
    n = wl["nodes"]
    phase("sage_graph", 600)
    t0 = time.time()
    s, d = edges_np if edges_np is not None else rmat_edges(n, wl["edges"], 0)
    adj = symmetric_adjacency(s, d, n, device=dev)
    del s, d
    log(f"[bench] sage adjacency nnz={adj.nnz} in {time.time() - t0:.1f}s")
    # the dataset relabelled once by degree (sampler.degree_ordered: hub rows first in the
    # table); the table is synthetic, so it is drawn directly in the new ids
    t1 = time.perf_counter()
    adj, _, _ = degree_ordered(adj)
    torch.cuda.synchronize(dev)
    order_s = time.perf_counter() - t1
    F = H = args.feat or 128
    gen = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(n, F, device=dev, generator=gen)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    cand = torch.nonzero(deg > 0).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192 * world]]
    sample_seed = 0
    if world > 1:
        from graphneuralnetwork_amd.distributed import rank_sample_seed, shard_seeds
        seeds = shard_seeds(seeds, rank, world)
        sample_seed = rank_sample_seed(0, rank)
    phase("first_sample", 300)
    tb = time.perf_counter()
    batch = sample_batch(adj, seeds, (25, 10), seed=sample_seed)
    torch.cuda.synchronize(dev)
    t_sample = time.perf_counter() - tb
    net = GraphSAGE(2, F, H, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    fargs = batch.forward_args(table)
    with torch.no_grad():
        phase("timed_steps", 300)
        if world > 1:
            dist.barrier()
        fwd_ms, wall = time_steps(lambda: net(*fargs, None, None, None, None, None), args.steps,
                                  args.warmup, dev)
        edges_all = batch.sampled_edges
        if world > 1:
            dist.barrier()
            rdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
            red = torch.tensor([wall, float(batch.sampled_edges)], dtype=torch.float64,
                               device=rdev)
            mx = red[:1].clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(red[1:], op=dist.ReduceOp.SUM)
            wall, edges_all = float(mx.item()), int(red[1].item())
        phase("extras", None)
        agg_ms, _ = time_steps(lambda: sage_gather_aggregate(table, batch.frontier_nbrs, "MEAN",
                                                             check=False),
                               args.steps, args.warmup, dev)
        # the same launch replayed REP times from one HIP graph: the kernel's own duration
        # (a ~50 us launch is otherwise paced by the Python call that enqueues it)
        REP = 10
        agg_out = torch.empty(batch.frontier_nbrs.shape[0], F, device=dev)
        agg_graph_ms = None
        try:
            def agg_call():
                sage_gather_aggregate(table, batch.frontier_nbrs, "MEAN", check=False,
                                      out=agg_out)
            s_cap = torch.cuda.Stream(dev)
            s_cap.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s_cap):
                for _ in range(2):
                    agg_call()
            torch.cuda.current_stream(dev).wait_stream(s_cap)
            ag = torch.cuda.CUDAGraph()
            with torch.cuda.graph(ag):
                for _ in range(REP):
                    agg_call()
            agg_graph_ms = [t / REP for t in time_steps(ag.replay, args.steps, args.warmup,
                                                          dev)[0]]
        except Exception as e:
            log(f"[bench] graph capture of the aggregation failed: {e!r}")
        smp_ms, _ = time_steps(lambda: sample_batch(adj, seeds, (25, 10), seed=sample_seed),
                               args.steps, args.warmup, dev)
        # the same call with the sizes left on the device (the batch path below): its three
        # kernels and their enqueue, without the host read
        smp_pending = []
        smp_pending_ms, _ = time_steps(
            lambda: smp_pending.append(sample_batch(adj, seeds, (25, 10), seed=sample_seed,
                                                    sync=False)), args.steps, args.warmup, dev)
        for b in smp_pending:
            b.check()
        del smp_pending

        def batch_step_synced():  # sampling (sizes read back) + the forward
            b = sample_batch(adj, seeds, (25, 10), seed=sample_seed)
            return net(*b.forward_args(table), None, None, None, None, None)

        pending = []

        def batch_step():  # one whole mini-batch: device sampling + the forward, no host read
            b = sample_batch(adj, seeds, (25, 10), seed=sample_seed, sync=False)
            pending.append(b)  # its error bits are read after the timed steps
            return net(*b.forward_args(table), None, None, None, None, None)

        batch_synced_ms, _ = time_steps(batch_step_synced, args.steps, args.warmup, dev)
        batch_ms, _ = time_steps(batch_step, args.steps, args.warmup, dev)
        for b in pending:
            b.check()  # every timed batch's sampler error word (raises on an error)
        del pending
        # the same forward replayed from a HIP graph (fixed-shape serving): GPU time without
        # the Python launch overhead of the eager call
        graph_ms = None
        try:
            s_cap = torch.cuda.Stream(dev)
            s_cap.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s_cap):
                for _ in range(2):
                    net(*fargs, None, None, None, None, None)
            torch.cuda.current_stream(dev).wait_stream(s_cap)
            hg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(hg):
                net(*fargs, None, None, None, None, None)
            graph_ms, _ = time_steps(hg.replay, args.steps, args.warmup, dev)
            graph_ms = statistics.mean(graph_ms)
        except Exception as e:  # reported, never the headline
            log(f"[bench] graph capture of the forward failed: {e!r}")
    M, k1 = batch.frontier_nbrs.shape
    B, k0 = batch.neigh_map.shape
    edges = batch.sampled_edges
    # layer-0 gather-mean: the 8(d) gather model counts every gathered row; the compulsory
    # bytes count each distinct table row once (+ the index map and the output)
    bytes_l0 = M * k1 * (4 * F + 8) + M * 4 * F
    distinct = int(torch.unique(batch.frontier_nbrs).numel())
    comp_l0 = M * k1 * 8 + distinct * 4 * F + M * 4 * F
    k_ms = statistics.mean(agg_graph_ms) if agg_graph_ms else statistics.mean(agg_ms)
    t = k_ms / 1e3
    achieved = comp_l0 / t / 1e9
    tf = traffic_fields(ROOT / "profiles" / f"traffic_cfg4_F{F}.json")
    traffic = tf["traffic"]
    res = {"metric": "GraphSAGE sampled-neighbour aggregated edges/sec (2-layer forward)",
           "value": edges_all * args.steps / wall, "unit": "edges/s", "n_gpus": world,
           "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic R-MAT",
           "config": {"workload": wl["name"], "nodes": n, "adj_nnz": adj.nnz, "seeds": B,
                      "frontier": M, "fanout": [k0, k1], "sampled_edges": edges, "feat_dim": F,
                      "step": "GraphSAGE.forward (one [self | mean] gather launch + one K=2F "
                              "GEMM per SageLayer, classifier) on device-sampled index maps",
                      "sage_layer_gemm": transform_note(),
                      "node_order": "dataset relabelled once by degree (sampler.degree_ordered, "
                                    "%.2f s, outside the timed region); seeds drawn in the new "
                                    "ids" % order_s},
           "forward_ms": statistics.median(fwd_ms), "sample_ms": statistics.median(smp_ms),
           "batch_ms": statistics.median(batch_ms),
           "batch_ms_note": "sample_batch(sync=False) + forward: the layer sizes stay on the "
                            "device, every batch's error word is read after the timed steps",
           "batch_synced_ms": statistics.median(batch_synced_ms),
           "sample_pending_ms": statistics.median(smp_pending_ms),
           "median_step_ms": statistics.median(fwd_ms),
           "forward_hipgraph_ms": graph_ms,
           "first_sample_s": t_sample,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBPS, **tf,
                        "compulsory_bytes": comp_l0, "distinct_rows": distinct,
                        "traffic_over_compulsory": traffic / comp_l0 if traffic else None,
                        "gather_model_bytes": bytes_l0, "gather_model_GBps": bytes_l0 / t / 1e9,
                        "gather_model_frac": bytes_l0 / t / 1e9 / HBM_PEAK_GBPS,
                        "traffic_GBps": traffic / t / 1e9 if traffic else None,
                        "traffic_frac": traffic / t / 1e9 / HBM_PEAK_GBPS if traffic else None,
                        "kernel": "sage_aggregate_kernel<gather, mean> (layer 0: |S1| x 10 from the 10M table)"
                                  + (", %d launches per HIP-graph replay" % REP if agg_graph_ms else
                                     ", eager per-launch HIP events"),
                        "eager_launch_ms": statistics.median(agg_ms),
                        "avg_launch_ms": k_ms,
                        "median_launch_ms": statistics.median(agg_graph_ms or agg_ms)}}
    if world == 1 and not args.no_variants:
        res["aggregators"] = sage_aggregator_variants(args, dev, table, batch, fargs, F, H,
                                                      distinct)
    if world > 1:
        res["config"]["global_seeds"] = 8192 * world
        res["config"]["parallelism"] = f"seed-sharded{world} (replicated table, no collective)"
    if not args.no_cpu_baseline and world == 1:
        from oracle import c_oracle
        threads = cpu_threads()
        c_oracle.set_threads(threads)
        tn = table.cpu().numpy()
        idx = batch.frontier_nbrs.cpu().numpy()
        c_oracle.sage_gather(tn, idx[:1000], "MEAN")  # warm-up
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            c_oracle.sage_gather(tn, idx, "MEAN")
            times.append(time.perf_counter() - t0)
        tc = statistics.median(times)
        res["cpu_baseline"] = {"value": idx.size / tc, "unit": "edges/s", "cores": threads,
                               "kind": "port", "seconds_per_step": tc,
                               "sample": f"layer-0 gather-mean of the same batch ({M} frontier "
                                         f"rows x {k1}) by oracle/spmm_oracle.c oracle_sage_gather "
                                         f"(OpenMP, float64), median of {len(times)} runs",
                               "host": host_cpu_info(threads)}
        if not args.no_cpu_reference:
            try:
                res["cpu_reference_ops"] = cpu_sage_ops(tn, batch, F, H)
            except Exception as e:
                res["cpu_reference_ops"] = {"error": repr(e)}
    del table, adj, batch, fargs
    torch.cuda.empty_cache()
    return res


def sage_aggregator_variants(args, dev, table, batch, fargs, F: int, H: int,
                             distinct: int) -> dict:
    """cfg4 with the other aggregators the reference exposes: 'MAX'
    (graph_utils.py:7-8: torch.argmax over the neighbours, int64 indices, bit-exact) and the
    north star's value max-pool 'MAXPOOL' (torch.max(dim=1).values): the 2-layer forward on the
    same sampled batch and the layer-0 gather-reduce kernel alone, with its roofline
    (compulsory bytes: the index map, each distinct table row once, the output: 8 B per
    element for the argmax) and the C oracle's rate on the same gather (16 threads)."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.ops import sage_gather_aggregate
    from oracle import c_oracle
    M, k1 = batch.frontier_nbrs.shape
    steps = max(3, min(args.steps, 10))
    out = {}
    for agg in ("MAX", "MAXPOOL"):
        net = GraphSAGE(2, F, H, False, agg_func=agg, Unsupervised=False,
                        class_size=3).to(dev).eval()
        with torch.no_grad():
            fwd_ms = time_steps(lambda: net(*fargs, None, None, None, None, None), steps, 2,
                                dev)[0]
            k_ms = time_steps(lambda: sage_gather_aggregate(table, batch.frontier_nbrs, agg,
                                                            check=False), steps, 2, dev)[0]
        out_bytes = M * F * (8 if agg == "MAX" else 4)
        comp = M * k1 * 8 + distinct * 4 * F + out_bytes
        t = statistics.mean(k_ms) / 1e3
        r = {"forward_ms": statistics.median(fwd_ms),
             "value": batch.sampled_edges / (statistics.median(fwd_ms) / 1e3),
             "unit": "edges/s",
             "layer0_kernel_ms": statistics.median(k_ms),
             "roofline": {"bound": "hbm", "achieved": comp / t / 1e9, "peak": HBM_PEAK_GBPS,
                          "unit": "GB/s", "frac": comp / t / 1e9 / HBM_PEAK_GBPS,
                          "compulsory_bytes": comp, "avg_launch_ms": t * 1e3,
                          "kernel": "sage_aggregate_kernel<gather, %s> (layer 0: %d frontier "
                                    "rows x %d from the 10M table), eager per-launch HIP events"
                                    % (agg.lower(), M, k1)}}
        if not args.no_cpu_baseline:
            threads = cpu_threads()
            c_oracle.set_threads(threads)
            tn = table.cpu().numpy()
            idx = batch.frontier_nbrs.cpu().numpy()
            fn = ((lambda: c_oracle.sage_argmax(tn, idx)) if agg == "MAX" else
                  (lambda: c_oracle.sage_gather(tn, idx, "MAXPOOL")))
            tc, runs = _cpu_time(fn, 5.0)
            r["cpu_baseline"] = {"value": idx.size / tc, "unit": "edges/s", "cores": threads,
                                 "kind": "port", "seconds_per_step": tc,
                                 "sample": "layer-0 gather-%s of the same batch (%d x %d) by "
                                           "oracle/spmm_oracle.c %s, median of %d runs"
                                           % (agg.lower(), M, k1,
                                              "oracle_sage_argmax" if agg == "MAX"
                                              else "oracle_sage_gather", runs),
                                 "host": host_cpu_info(threads)}
        out[agg] = r
        del net
    return out


def transform_note() -> str:
    """The arithmetic of the MFMA feature transforms (the GEMM half of a layer, outside the
    aggregation the headline times)."""
    from graphneuralnetwork_amd.ops import transform_precision
    if transform_precision() == "split-bf16":
        return ("gnn_gcn_transform / gnn_linear_relu on v_mfma_f32_16x16x32_bf16 at K >= 128: fp32 "
                "inputs split into three bf16 pieces, the six products down to order 2^-16 "
                "accumulated in fp32 (error per product a few fp32 ulps, below the fp32-MFMA "
                "path's in tests/test_spmm_gpu.py::test_transform_split_bf16_accuracy); fp32 "
                "v_mfma_f32_16x16x4_f32 at K < 128")
    return "gnn_gcn_transform / gnn_linear_relu on v_mfma_f32_16x16x4_f32 (fp32 fmaf chain)"


def host_cpu_info(threads: int) -> dict:
    """What the CPU lines ran on: the threads used, the CPUs this process may run on and
    the machine's count. The GPU box allots 16 CPUs per GPU
    (OMP_NUM_THREADS=16 there) even though os.cpu_count() shows the whole machine."""
    info = {"threads": threads, "affinity_cpus": len(os.sched_getaffinity(0)),
            "os_cpu_count": os.cpu_count(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}
    try:  # a CPU quota (cgroup v2 "quota period"): the CPUs' worth of time this job may use
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        info["cgroup_cpu_max"] = f"{q} {per}"
        if q != "max":
            info["cgroup_cpu_quota_cpus"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    info["threads_rule"] = ("min(affinity CPUs, cgroup CPU quota, OMP_NUM_THREADS): the CPUs "
                            "of time this job is granted; more threads oversubscribe the quota")
    return info


def gcn_roofline(nnz: int, n_rows: int, n_cols: int, feat: int, step_ms: list, tf: dict,
                 kernel: str) -> dict:
    """The roofline object of one SpMM step (see compulsory_bytes / algorithmic_bytes); ``tf``
    = traffic_fields() of the workload's PMC file (all None without one)."""
    kern_ms = statistics.mean(step_ms)
    t = kern_ms / 1e3
    comp = compulsory_bytes(nnz, n_rows, n_cols, feat)
    gm = algorithmic_bytes(nnz, n_rows, feat)
    achieved = comp / t / 1e9
    traffic = tf.get("traffic")
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS, **tf,
            "compulsory_bytes": comp,
            "traffic_over_compulsory": traffic / comp if traffic else None,
            # the SURVEY 8(d) no-reuse gather model (every gathered row from HBM): an upper
            # bound on traffic, not a floor -- hub rows come from L2 / the Infinity Cache
            "gather_model_bytes": gm, "gather_model_GBps": gm / t / 1e9,
            "gather_model_frac": gm / t / 1e9 / HBM_PEAK_GBPS,
            # L2-miss bytes per second (Infinity Cache hits included): what the memory side
            # served, as a fraction of the 8 TB/s peak
            "traffic_GBps": traffic / t / 1e9 if traffic else None,
            "traffic_frac": traffic / t / 1e9 / HBM_PEAK_GBPS if traffic else None,
            "kernel": kernel,
            "avg_launch_ms": kern_ms, "median_launch_ms": statistics.median(step_ms),
            "min_launch_ms": min(step_ms)}


def tn_kernel_name(m: int, k: int, d_is_b: bool = False) -> str:
    """The gemm_tn kernel launch_tn picks for an (M, K) shape (csrc/gemm_tn.hip) in the
    transforms' arithmetic mode."""
    from graphneuralnetwork_amd.ops import transform_precision
    if not (m >= 64 and k >= 32):
        return "gemm_tn_partial_kernel"
    if transform_precision() == "split-bf16":
        return "gemm_tn_x6_kernel" + ("<DB: dsum from B's loads>" if d_is_b else "")
    return "gemm_tn_mfma_kernel"


def _ms_stats(ms: list) -> dict:
    return {"median_ms": statistics.median(ms), "mean_ms": statistics.mean(ms)}


def gcn_train_step(g, F: int, args, dev) -> dict:
    """One training step of the drop-in Graph_conv_layer(F, F) at cfg2 (GCN/GCN.py:41-47 under
    GCN/train_eval.py:43-48's loss.backward()), as a hidden layer (dX needed too), over P A P^T.
    F -> F trains as (A X) W^T + b (ops._GcnLayerFn, GCN_REASSOC): forward = SpMM Z = A X +
    MFMA transform with the bias epilogue; backward = the tall-skinny A^T B kernel (dW = dY^T Z
    with db = column sums of dY from the same loads; hipBLASLt's torch.mm timed beside it) +
    MFMA transform (dZ = dY W) + SpMM over A^T (A itself: the normalised adjacency is
    symmetric). The A (X W^T) form (GCN_REASSOC off) is timed beside it. Each backward
    component is also timed alone; the backward SpMM carries its own roofline (compulsory
    bytes, as the forward's)."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import GCN_Model, Graph_conv_layer
    from graphneuralnetwork_amd.ops import gcn_train_order, gcn_transform, gemm_tn, spmm_forward
    gen = torch.Generator(device=dev).manual_seed(1)
    layer = Graph_conv_layer(F, F).to(dev)
    X = torch.randn(g.n_cols, F, device=dev, generator=gen).requires_grad_(True)
    gy = torch.randn(g.n_rows, F, device=dev, generator=gen)
    steps = max(3, min(args.steps, 10))
    # a hidden layer of GCN_Model in training runs over P A P^T (gcn_train_order: nodes in
    # degree order, the model's input permuted once on entry): X, dY in that order
    t0 = time.perf_counter()
    order = gcn_train_order(g, F)
    torch.cuda.synchronize(dev)
    order_s = time.perf_counter() - t0
    g_nat, X_nat, gy_nat = g, X, gy
    if order is not None:
        g = order.graph
        X = order.permute_rows(X.detach()).requires_grad_(True)
        gy = order.permute_rows(gy)

    def step():
        X.grad = None
        layer.zero_grad(set_to_none=True)
        layer(X, g).backward(gy)

    step_ms = time_steps(step, steps, 2, dev)[0]

    def step_nat():
        X_nat.grad = None
        layer.zero_grad(set_to_none=True)
        layer(X_nat, g_nat).backward(gy_nat)

    nat_ms = time_steps(step_nat, steps, 2, dev)[0] if order is not None else step_ms
    reassoc = ops._reassociate(X, layer.dense.weight, g)
    prev_reassoc = ops.GCN_REASSOC
    ops.GCN_REASSOC = False
    try:
        plain_ms = time_steps(step, steps, 2, dev)[0] if reassoc else step_ms
    finally:
        ops.GCN_REASSOC = prev_reassoc
    # the two-layer model, input and logits in the original order (GCN_Model.forward's two
    # permutes inside the step), NLL loss (GCN/train_eval.py:43-48)
    model = GCN_Model(F, F, 7, 2, 0.5).to(dev).train()
    labels = torch.randint(0, 7, (g.n_rows,), device=dev, generator=gen)
    idx_train = torch.arange(0, g.n_rows, 10, device=dev)
    Xm = X_nat.detach()
    ce = torch.nn.CrossEntropyLoss()

    def model_step():  # GCN/train_eval.py:43-46: CE on output[idx_train], backward
        model.zero_grad(set_to_none=True)
        ce(model(Xm, g_nat)[idx_train], labels[idx_train]).backward()

    model_ms = time_steps(model_step, steps, 2, dev)[0]
    del model
    fwd_ms = time_steps(lambda: layer(X, g), steps, 2, dev)[0]
    keep = {"y": layer(X, g)}
    bwd_ms = time_steps(lambda: keep["y"].backward(gy, retain_graph=True), steps, 2, dev)[0]
    del keep
    gt = g.transpose()
    Wt = layer.dense.weight.detach().t().contiguous()
    Xd = X.detach()
    ds = torch.empty(g.n_rows, F, device=dev)
    if reassoc:  # (A X) W^T + b: dW = dY^T Z, db from dY's own loads; dZ = dY W; dX = A^T dZ
        Z = spmm_forward(g, Xd)
        dz = gcn_transform(gy, Wt)
        spmm_ms = time_steps(lambda: spmm_forward(gt, dz, out=ds), steps, 2, dev)[0]
        dx_ms = time_steps(lambda: gcn_transform(gy, Wt), steps, 2, dev)[0]
        tn_args = (Z, gy, gy)
    else:  # A (X W^T) + b: dS = A^T dY; dX = dS W; dW = dS^T X, db = colsum dY
        spmm_ms = time_steps(lambda: spmm_forward(gt, gy, out=ds), steps, 2, dev)[0]
        dx_ms = time_steps(lambda: gcn_transform(ds, Wt), steps, 2, dev)[0]
        tn_args = (Xd, ds, gy)
    ta, tb, td = tn_args
    tn = gemm_tn(ta, tb, td, trans=True) is not None
    dw_ms = (time_steps(lambda: gemm_tn(ta, tb, td, trans=True), steps, 2, dev)[0] if tn else
             time_steps(lambda: torch.mm(tb.t(), ta), steps, 2, dev)[0])
    mm_ms = time_steps(lambda: torch.mm(tb.t(), ta), steps, 2, dev)[0]
    db_ms = time_steps(lambda: gy.sum(0), steps, 2, dev)[0]
    comp = compulsory_bytes(g.nnz, g.n_rows, g.n_cols, F)
    t_sp = statistics.mean(spmm_ms) / 1e3
    nbytes_rows = g.n_rows * 4 * F
    # operands read: (Z, dY) with db from dY's own loads, or (X, dS) + dY for db
    dw_bytes = (2 if reassoc or not tn else 3) * nbytes_rows
    res = {
        "what": "Graph_conv_layer(%d, %d) forward + loss.backward() at cfg2, X requiring grad "
                "(a hidden layer: dX, dW, db)" % (F, F),
        "step_ms": statistics.median(step_ms), "forward_ms": statistics.median(fwd_ms),
        "backward_ms": statistics.median(bwd_ms),
        "edges_per_s": 2 * g.nnz / (statistics.median(step_ms) / 1e3),
        "edges_note": ("two SpMM passes per step (forward A X, backward A^T dZ)" if reassoc else
                       "two SpMM passes per step (forward A S, backward A^T dY)"),
        "layer_form": ("(A X) W^T + b (ops.GCN_REASSOC: in_features <= out_features)" if reassoc
                       else "A (X W^T) + b"),
        "a_xwt_form_step_ms": statistics.median(plain_ms),
        "node_order": ("P A P^T (gcn_train_order: nodes relabelled by degree once per graph, "
                       "%.2f s outside the timed region; X, dY in that order as GCN_Model's "
                       "hidden layers see them)" % order_s) if order is not None else "natural",
        "natural_order_step_ms": statistics.median(nat_ms),
        "model_step_ms": statistics.median(model_ms),
        "model_step_what": "GCN_Model(%d, %d, 7, num_layers=2, dropout=0.5).train() forward + "
                           "CrossEntropyLoss(output[idx_train]) backward, idx_train = every 10th "
                           "node (GCN/train_eval.py:43-46; x in and logits out in the original "
                           "order)" % (F, F),
        "backward_components_ms": {
            ("spmm_dX_AT_dZ" if reassoc else "spmm_dS_AT_dY"): statistics.median(spmm_ms),
            ("transform_dZ_dY_W" if reassoc else "transform_dX_dS_W"): statistics.median(dx_ms),
            ("gemm_tn_dW_db" if tn else "gemm_dW_hipblaslt"): statistics.median(dw_ms),
            "colsum_db" + ("_in_gemm_tn" if tn else ""): (0.0 if tn else statistics.median(db_ms))},
        "hipblaslt_mm_dW_for_comparison_ms": statistics.median(mm_ms),
        "backward_spmm_graph": "A itself (symmetric: no transposed copy)" if gt is g else
                               "transposed CSR",
        "roofline_backward_spmm": {
            "bound": "hbm", "achieved": comp / t_sp / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": comp / t_sp / 1e9 / HBM_PEAK_GBPS, "compulsory_bytes": comp,
            "avg_launch_ms": t_sp * 1e3,
            "kernel": ("spmm_csr_kernel pass 1 + pass 2 over P A P^T (XCD-direct: dY's hub rows "
                       "read in place) + fix-up") if order is not None else
                      ("spmm_csr_kernel pass 1 + pass 2 (XCD-sliced hub staging of the natural-"
                       "order graph: dY is not in the column order) + fix-up")},
        "roofline_backward_gemm_dW": {
            "bound": "hbm", "achieved": dw_bytes / (statistics.mean(dw_ms) / 1e3) / 1e9,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": dw_bytes / (statistics.mean(dw_ms) / 1e3) / 1e9 / HBM_PEAK_GBPS,
            "bytes": dw_bytes,
            "kernel": ("%s + gemm_tn_reduce_kernel (%s in one pass)"
                       % (tn_kernel_name(F, F, reassoc),
                          "dW = dY^T Z and db = colsum dY" if reassoc else
                          "dW^T = X^T dS and db = colsum dY")) if tn else "hipBLASLt (torch.mm)",
            "note": ("Z and dY read once, db from dY's loads" if reassoc and tn else
                     "X, dS and dY (the db operand) read once" if tn else
                     "two operands read once") + " (K = n_rows reduction, %.1f GFLOP)"
                    % (2 * g.n_rows * F * F / 1e9)},
        "roofline_backward_transform_dX": {
            "bound": "hbm", "achieved": 2 * nbytes_rows / (statistics.mean(dx_ms) / 1e3) / 1e9,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": 2 * nbytes_rows / (statistics.mean(dx_ms) / 1e3) / 1e9 / HBM_PEAK_GBPS,
            "bytes": 2 * nbytes_rows,
            "note": "dY read, dZ written" if reassoc else "dS read, dX written"},
    }
    if not args.no_cpu_baseline:
        try:
            res["cpu_reference_ops"] = cpu_gcn_train_ops(g, F)
        except Exception as e:  # reported, never the target
            res["cpu_reference_ops"] = {"error": repr(e)}
    del X, gy, ds, layer, X_nat, gy_nat, Xm, ta, tb, td, tn_args
    if reassoc:
        del Z, dz
    torch.cuda.empty_cache()
    return res


def cpu_gcn_train_ops(g, F: int, max_nnz: int = 2_000_000, budget_s: float = 10.0) -> dict:
    """The reference's CPU training step of one Graph_conv_layer (GCN/GCN.py:41-47: nn.Linear +
    torch.spmm on the uncoalesced COO + bias; loss.backward()) with torch CPU autograd, every
    allowed host thread, on the leading rows holding <= max_nnz edges (the COO is [rows, n]:
    X and dX stay full size)."""
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rowptr = g.rowptr.cpu()
        r1 = max(1, min(g.n_rows, int(torch.searchsorted(rowptr, max_nnz, right=True)) - 1))
        e1 = int(rowptr[r1])
        rows = torch.repeat_interleave(torch.arange(r1), rowptr[1:r1 + 1] - rowptr[:r1])
        cols = g.col[:e1].cpu().to(torch.int64)
        order = torch.argsort(cols, stable=True)
        coo = torch.sparse_coo_tensor(torch.stack([rows[order], cols[order]]),
                                      g.val[:e1].cpu()[order], (r1, g.n_cols))
        lin = torch.nn.Linear(F, F, bias=False)
        bias = torch.nn.Parameter(torch.zeros(F))
        X = torch.randn(g.n_cols, F, requires_grad=True)
        gy = torch.randn(r1, F)

        def step():
            X.grad = None
            lin.zero_grad(set_to_none=True)
            bias.grad = None
            (torch.spmm(coo, lin(X)) + bias).backward(gy)

        t, runs = _cpu_time(step, budget_s)
        return {"torch_cpu_train_step": {"value": 2 * e1 / t, "unit": "edges/s",
                                         "threads": threads, "seconds_per_step": t,
                                         "runs": runs},
                "note": f"torch CPU forward + backward of the reference layer on rows 0..{r1} "
                        f"({e1} edges; the X W^T transform and its backward over all "
                        f"{g.n_cols} rows), edges counted twice (forward + backward SpMM)"}
    finally:
        torch.set_num_threads(prev)


def gcn_model_forward(g, F: int, args, dev) -> dict:
    """The drop-in two-layer GCN_Model(F, F, F, 2) forward at the north star (GCN/GCN.py:21-27:
    Graph_conv_layer -> ReLU -> Dropout (eval: identity) -> Graph_conv_layer), each layer the
    MFMA transform into the column order + the XCD-sliced SpMM, the ReLU in the first SpMM's
    store epilogue."""
    from graphneuralnetwork_amd.gcn import GCN_Model
    gen = torch.Generator(device=dev).manual_seed(2)
    net = GCN_Model(F, F, F, 2, 0.5).to(dev).eval()
    X = torch.randn(g.n_cols, F, device=dev, generator=gen)
    with torch.no_grad():
        ms = time_steps(lambda: net(X, g), max(3, min(args.steps, 10)), 2, dev)[0]
    t = statistics.median(ms)
    res = {"what": "GCN_Model(%d, %d, %d, num_layers=2).eval() forward at the north star" % (F, F, F),
           "forward_ms": t, "value": 2 * g.nnz / (t / 1e3), "unit": "edges/s",
           "edges_note": "two aggregation layers per forward"}
    if not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_gcn_layer_rate(g, F)
        except Exception as e:
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    del X, net
    torch.cuda.empty_cache()
    return res


def cpu_gcn_layer_rate(g, F: int, max_nnz: int = 25_000_000) -> dict:
    """The CPU rate of the GCN layer math on a row block (rows 0..r1 holding <= max_nnz
    entries): the dense transform of those rows (torch CPU, row-separable) + the C oracle's
    SpMM of those rows; a 2-layer forward is two such passes, so edges/s is the same."""
    from oracle import c_oracle
    threads = cpu_threads()
    c_oracle.set_threads(threads)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rowptr = g.rowptr.cpu().numpy()
        r1 = max(1, min(g.n_rows, int(np.searchsorted(rowptr, max_nnz, side="right")) - 1))
        e1 = int(rowptr[r1])
        Xs = torch.randn(r1, F)
        W = torch.randn(F, F)
        S = torch.randn(g.n_cols, F).numpy()
        col, val = g.col.cpu().numpy(), g.val.cpu().numpy()
        t_mm, _ = _cpu_time(lambda: Xs @ W.t(), 5.0)
        c_oracle.spmm_csr(rowptr, col, val, S, None, 0, min(r1, 20000))
        t_sp, runs = _cpu_time(lambda: c_oracle.spmm_csr(rowptr, col, val, S, None, 0, r1), 10.0)
        return {"value": e1 / (t_mm + t_sp), "unit": "edges/s", "cores": threads, "kind": "port",
                "seconds_per_layer_sample": t_mm + t_sp,
                "sample": f"one layer on rows 0..{r1} ({e1} entries): torch CPU X W^T of those "
                          f"rows ({t_mm:.3f} s) + oracle/spmm_oracle.c SpMM of those rows "
                          f"({t_sp:.3f} s, median of {runs})",
                "host": host_cpu_info(threads)}
    finally:
        torch.set_num_threads(prev)


def run_gcn(args, dev, rank: int, world: int, workload: str, edges_np=None, extras=False):
    """GCN SpMM step (GCN/GCN.py:43-45) over the workload's graph: single GPU, or edge-cut over
    the N ranks (RCCL halo exchange). Returns rank 0's result dict (None elsewhere)."""
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    wl = WORKLOADS[workload]
    grow = 1 if wl.get("strong") else world
    nodes, edges = int(wl["nodes"] * grow * args.scale), int(wl["edges"] * grow * args.scale)
    F = args.feat if (args.feat is not None and not extras) else wl.get("feat", 128)
    g = build_graph(nodes, edges, dev, rank, world, edges_np=edges_np)
    gen = torch.Generator(device=dev).manual_seed(0)
    bias = torch.randn(F, device=dev, generator=gen)
    part = None
    HUB_INFO.clear()
    BUILD_INFO.pop("column_order_s", None)

    if world == 1:
        X = torch.randn(g.n_cols, F, device=dev, generator=gen)
        Y = torch.empty(g.n_rows, F, device=dev)
        # the aggregation as Graph_conv_layer runs it: over the column-degree-ordered graph
        # A P^T (built once per graph, like the CSR), whose transform writes the support rows
        # in that order -- X here stands for that support; Y rows are in the original order
        t0 = time.perf_counter()
        order = column_order(g, F)
        torch.cuda.synchronize(dev)
        ga = g if order is None else order.graph
        if order is not None:
            BUILD_INFO["column_order_s"] = time.perf_counter() - t0
        step = lambda: spmm_forward(ga, X, bias, out=Y)  # noqa: E731
        rows_local, nnz_local = g.n_rows, g.nnz
        halo_rows = 0
        HUB_INFO["graph"] = ga
    else:
        from graphneuralnetwork_amd.distributed import (EdgeCutSpmm,
                                                        build_cover_exchange_balanced,
                                                        build_partition, nnz_balanced_bounds)
        phase("partition_build", 900)
        t0 = time.time()
        if args.exchange == "cover":
            # row blocks re-cut for the work the cover moves (cost model, 2 refinements)
            part, hist = build_cover_exchange_balanced(
                g, rank, world, progress=lambda it, mx, mean, s: log(
                    f"[bench] cover partition, build {it}: max/mean cost {mx / mean:.3f} "
                    f"({s:.1f}s)"))
            BUILD_INFO["balance_max_mean_cost"] = hist
            work = (f"interior {part.interior.nnz}, partial {part.send_p.nnz}, halo "
                    f"{part.halo_x.nnz} + {part.halo_p.nnz}; "
                    f"recv {part.n_partial_recv} partial + {part.n_feature_recv} feature rows")
        else:
            part = build_partition(g, rank, world, bounds=nnz_balanced_bounds(g.rowptr, world))
            work = f"interior {part.interior.nnz}, halo {part.halo.nnz}"
        BUILD_INFO["partition_build_s"] = time.time() - t0
        X = torch.randn(part.n_own, F, device=dev, generator=gen)
        runner = EdgeCutSpmm(part, F, dev)
        step = lambda: runner(X, bias)  # noqa: E731
        r0, r1 = part.bounds[rank], part.bounds[rank + 1]
        rows_local = part.n_own
        nnz_local = int(g.rowptr[r1] - g.rowptr[r0])        # graph edges of the owned rows
        log(f"[bench] rank{rank} {args.exchange} exchange: rows {rows_local} edges {nnz_local} "
            f"({work}) recv rows {part.n_halo} send rows {sum(part.send_counts)}")
        halo_rows = part.n_halo
        del g
        g = None
        torch.cuda.empty_cache()

    stream = torch.cuda.current_stream(dev)
    # the first step also builds the per-graph plans (row classes, hub ranks, XCD-sliced
    # items): reported as first_step_s, never timed as a step
    torch.cuda.synchronize(dev)
    phase("first_step", 300)
    t_first = time.perf_counter()
    step()
    torch.cuda.synchronize(dev)
    BUILD_INFO["first_step_s"] = time.perf_counter() - t_first
    phase("warmup", 300)
    log(f"[bench] first step (builds the per-graph plans) {BUILD_INFO['first_step_s']:.2f}s")
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize(dev)
    if HUB_INFO.get("graph") is not None:
        HUB_INFO["kernel"] = describe_path(HUB_INFO.pop("graph"), F)
    phase("timed_steps", 300)
    if world > 1:
        dist.barrier()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    per_step = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for a, b in per_step:
        a.record(stream)
        step()
        b.record(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    step_ms = [a.elapsed_time(b) for a, b in per_step]
    phase("reduce", 120)
    elapsed = torch.tensor([max(wall, gpu_ms / 1e3)], dtype=torch.float64, device=dev)
    tot_nnz = torch.tensor([nnz_local], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot_nnz, op=dist.ReduceOp.SUM)
    T = float(elapsed.item())
    ms_per_step = T / args.steps * 1e3
    value = float(tot_nnz.item()) * args.steps / T

    cold = None
    if world == 1 and not args.no_cold:
        # the timed loop re-runs the same X, so the staged hub table and
        # part of X stay in the 256 MiB Infinity Cache between steps. Here every step is
        # preceded (outside its events) by a 1 GiB write that evicts it, as a fresh X from the
        # layer's GEMM would: the cache-cold step time, reported beside the headline.
        flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
        cold_ms = []
        for i in range(6):
            flush.fill_(float(i))
            a_ev, b_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a_ev.record(stream)
            step()
            b_ev.record(stream)
            torch.cuda.synchronize(dev)
            cold_ms.append(a_ev.elapsed_time(b_ev))
        cold = statistics.median(cold_ms[1:])
        del flush
        torch.cuda.empty_cache()
        log(f"[bench] {workload} cache-cold step (1 GiB written before each): {cold:.3f} ms")
    phases = None
    if world > 1 and dev.type == "cuda":
        # one more (untimed) step with events at every phase boundary: per-rank compute
        # phases, the compute stream's waits on the exchanges, and the all-to-all-v times
        phase("phase_profile", 180)
        prof = runner.profile(X, bias)
        names = sorted(prof)
        vals = _all_gather_phase_values([prof[k] for k in names], world, dev)
        phases = {"rank0": {k: round(v, 4) for k, v in prof.items()},
                  "max_over_ranks": {k: round(float(vals[:, i].max()), 4)
                                     for i, k in enumerate(names)},
                  "exchange_MB_rank0": {
                      "send": round(sum(part.send_counts) * 4 * F / 1e6, 1),
                      "recv": round(sum(part.recv_counts) * 4 * F / 1e6, 1)}}
    phase("extras", None)
    layer_ms = None
    log(f"[bench] {workload} aggregation timed: {statistics.mean(step_ms):.3f} ms/launch "
        f"(median {statistics.median(step_ms):.3f})")
    if world == 1 and not args.no_layer:
        # the whole drop-in Graph_conv_layer(F, F).forward (GCN/GCN.py:41-47): dense X W^T +
        # the SpMM with the bias epilogue -- reported beside the aggregation
        from graphneuralnetwork_amd.gcn import Graph_conv_layer
        layer = Graph_conv_layer(F, F).to(dev).eval()
        with torch.no_grad():
            layer_ms = statistics.median(time_steps(lambda: layer(X, g), min(args.steps, 10),
                                                    2, dev)[0])
        del layer
        log(f"[bench] Graph_conv_layer timed: {layer_ms:.3f} ms")
        torch.cuda.empty_cache()

    train = model_fwd = None
    if world == 1 and not args.no_train and workload == "cfg2":
        train = gcn_train_step(g, F, args, dev)
    if world == 1 and not args.no_layer and workload == "ns":
        model_fwd = gcn_model_forward(g, F, args, dev)

    tf = {}
    if world == 1:
        tpath = Path(args.traffic_json) if (args.traffic_json and not extras) else \
            ROOT / "profiles" / f"traffic_{workload}_F{F}.json"
        tf = traffic_fields(tpath)
    res = None
    if rank == 0:
        kernel = HUB_INFO["kernel"] if HUB_INFO.get("kernel") else (
            "EdgeCutSpmm step: send-side SpMM; the feature rows in %d chunked RCCL "
            "all-to-all-v's and the partial rows in one more (comm stream) overlapping the "
            "interior SpMM (hub-staged when its X is >= 192 MiB); the halo SpMM of each chunk as "
            "it lands, then the partial-row pass; per-step HIP events, max over ranks"
            % (runner.chunks if args.exchange == "cover" else 1) if world > 1 else
            "spmm_csr_kernel (+ spmm_fixup_kernel), per-step HIP events")
        roof = gcn_roofline(nnz_local, rows_local,
                            rows_local + halo_rows if world > 1 else g.n_cols, F, step_ms,
                            tf, kernel)
        if world == 1 and not args.no_replay and "column_order_s" in BUILD_INFO:
            phase("replay", 300)
            rp = spmm_replay(ga, X, bias, Y)
            if rp is not None:
                rp["frac_at_hub_floor"] = (roof["compulsory_bytes"] / (
                    rp["hub_gathers_in_L2_ms"] / 1e3) / 1e9 / HBM_PEAK_GBPS)
                rp["frac_at_all_in_L2"] = (roof["compulsory_bytes"] / (
                    rp["all_gathers_in_L2_ms"] / 1e3) / 1e9 / HBM_PEAK_GBPS)
                roof["replay_floor"] = rp
        res = {
            "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "median_step_ms": statistics.median(step_ms),
            **({"cache_cold_median_step_ms": cold,
                "cache_cold_note": "median of 5 steps, each after a 1 GiB device write "
                                   "(outside the step's events) that evicts the Infinity Cache"}
               if cold is not None else {}),
            "higher_is_better": True, "scaling": "strong" if wl.get("strong") else "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (R-MAT a=.57 b=.19 c=.19 d=.05, seed 0, reference GCN normalisation; "
                    "X ~ N(0,1))",
            "config": {"workload": wl["name"], "nodes": nodes, "directed_edges": edges,
                       "nnz": int(tot_nnz.item()), "feat_dim": F, "global_batch": nodes,
                       "parallelism": f"edge-cut{world}" if world > 1 else "single-gpu",
                       "nnz_rank0": nnz_local, "halo_rows_rank0": halo_rows,
                       **({"exchange": args.exchange} if world > 1 else {}),
                       **({"column_order": "A P^T: columns relabelled by in-degree once per "
                                           "graph (graph.degree_order(rows=False), %.2f s, "
                                           "outside the timed region); X = the support in "
                                           "that row order, as Graph_conv_layer's transform "
                                           "writes it; output rows in the original order"
                                           % BUILD_INFO["column_order_s"]}
                          if world == 1 and "column_order_s" in BUILD_INFO else {})},
            "achieved_GBps": roof["achieved"],
            "graph_build_s": BUILD_INFO.get("gcn_adjacency_build_s"),
            "first_step_s": BUILD_INFO.get("first_step_s"),
            **({"gcn_layer_ms": layer_ms, "gcn_layer_transform": transform_note()}
               if layer_ms is not None else {}),
            **({"train_step": train} if train is not None else {}),
            **({"gcn_model_forward": model_fwd} if model_fwd is not None else {}),
            **({"partition_build_s": BUILD_INFO.get("partition_build_s"),
                "row_bounds": part.bounds,
                "balance_max_mean_cost": BUILD_INFO.get("balance_max_mean_cost"),
                "phases_ms": phases}
               if world > 1 else {}),
            "roofline": roof,
        }
        if world == 1 and not args.no_cpu_baseline:
            log(f"[bench] {workload} cpu baseline (oracle port) ...")
            try:
                res["cpu_baseline"] = cpu_baseline(g, X, F)
            except Exception as e:  # the baseline is reported, never the target
                res["cpu_baseline"] = {"value": None, "error": repr(e)}
            if not args.no_cpu_reference and not extras:
                log("[bench] cpu reference operators ...")
                try:
                    res["cpu_reference_ops"] = cpu_reference_ops(g, X, F)
                except Exception as e:
                    res["cpu_reference_ops"] = {"error": repr(e)}
    del X, g
    if world == 1:
        del ga
    torch.cuda.empty_cache()
    return res


def _sub(res: dict) -> dict:
    """A workload's line as a sub-object of the headline (the keys that describe it)."""
    keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "median_step_ms",
            "cache_cold_median_step_ms", "dtype",
            "config", "roofline", "cpu_baseline", "cpu_reference_ops",
            "first_step_s", "graph_build_s", "gcn_layer_ms", "layer_ms", "aggregate_ms",
            "forward_ms", "forward_hipgraph_ms", "sample_ms", "sample_pending_ms", "batch_ms",
            "batch_ms_note", "batch_synced_ms", "project_ms",
            "project_tflops", "project_arithmetic", "train_step", "gcn_model_forward",
            "aggregators")
    return {k: res[k] for k in keep if k in res}


# The driver parses the ONE stdout line; a 20.9 KB line went unparsed in round 5 (VERDICT r5
# weak #1). The line keeps the contract's keys and one-level summaries, the full result goes
# to a sidecar JSON the line names.
LINE_MAX_BYTES = 8000
REQUIRED_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                 "roofline", "cpu_baseline")
ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_stale",
                 "compulsory_bytes", "traffic_over_compulsory", "avg_launch_ms")
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "seconds_per_step")
CONFIG_KEYS = ("workload", "nodes", "directed_edges", "nnz", "feat_dim", "global_batch",
               "parallelism", "exchange", "heads", "head_dim", "in_dim", "seeds", "fanout",
               "frontier", "sampled_edges")


def _rnd(v, sig: int = 5):
    """Floats to `sig` significant digits (the line's numbers are measurements, not ids)."""
    if isinstance(v, float):
        return float(f"{v:.{sig}g}")
    if isinstance(v, dict):
        return {k: _rnd(x, sig) for k, x in v.items()}
    if isinstance(v, list):
        return [_rnd(x, sig) for x in v]
    return v


def _short(text, n: int = 160):
    return text if not isinstance(text, str) or len(text) <= n else text[:n - 3] + "..."


def _pick(d, keys) -> dict:
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _roof(r) -> dict | None:
    if not isinstance(r, dict):
        return None
    out = _pick(r, ROOFLINE_KEYS)
    if r.get("kernel"):
        out["kernel"] = _short(r["kernel"], 120)
    if r.get("traffic_source"):
        out["traffic_source"] = r["traffic_source"].split(":")[0]
    rp = r.get("replay_floor")
    if isinstance(rp, dict):  # the measured ceiling (spmm_replay)
        out["replay_floor"] = _pick(rp, ("as_built_ms", "hub_gathers_in_L2_ms",
                                         "all_gathers_in_L2_ms", "as_built_over_hub_floor",
                                         "frac_at_all_in_L2"))
    return out


def _cpu(c) -> dict | None:
    if not isinstance(c, dict):
        return None
    out = _pick(c, CPU_KEYS)
    if "sample" in out:
        out["sample"] = _short(out["sample"], 200)
    if "error" in c:
        out["error"] = _short(c["error"], 120)
    return out


def _summary(sub: dict) -> dict:
    """A sub-workload (north star, cfg3, cfg4) as value / ms / frac and its few headline
    times; everything else stays in the sidecar."""
    roof = sub.get("roofline") or {}
    out = {"value": sub.get("value"), "unit": sub.get("unit"),
           "ms": sub.get("median_step_ms", sub.get("ms_per_step")),
           "frac": roof.get("frac"), "traffic": roof.get("traffic"),
           "avg_launch_ms": roof.get("avg_launch_ms"),
           "cpu_baseline_value": (sub.get("cpu_baseline") or {}).get("value")}
    for k in ("gcn_layer_ms", "layer_ms", "forward_ms", "sample_ms", "sample_pending_ms",
              "batch_ms", "batch_synced_ms", "project_ms"):
        if k in sub:
            out[k] = sub[k]
    if isinstance(sub.get("aggregate_ms"), dict):
        out["aggregate_ms"] = sub["aggregate_ms"]
    if isinstance(sub.get("config"), dict):
        out["workload"] = _short(sub["config"].get("workload"), 100)
    for k in ("train_step", "gcn_model_forward"):
        t = sub.get(k)
        if isinstance(t, dict):
            out[k + "_ms"] = t.get("step_ms", t.get("forward_ms"))
    if "target" in sub:
        out["target_met"] = bool(roof.get("frac") is not None and roof["frac"] >= 0.6)
    rp = roof.get("replay_floor")
    if isinstance(rp, dict):
        out["replay_floor"] = _pick(rp, ("hub_gathers_in_L2_ms", "all_gathers_in_L2_ms",
                                         "as_built_over_hub_floor", "frac_at_all_in_L2"))
    if isinstance(sub.get("aggregators"), dict):
        out["aggregators_forward_ms"] = {k: v.get("forward_ms") for k, v in
                                         sub["aggregators"].items() if isinstance(v, dict)}
    return {k: v for k, v in out.items() if v is not None}


def compact_line(res: dict, detail: str | None = None) -> dict:
    """The driver's line: the contract's keys, the headline roofline and CPU baseline, the
    library / tree stamps, one-level summaries of the other workloads and training steps, and
    the path of the sidecar holding the full result. Never longer than LINE_MAX_BYTES."""
    line = {k: res[k] for k in REQUIRED_KEYS[:12] if k in res}
    line["config"] = _pick(res.get("config", {}), CONFIG_KEYS)
    for k in ("median_step_ms", "cache_cold_median_step_ms", "gcn_layer_ms", "first_step_s",
              "graph_build_s", "partition_build_s", "lib_stamp", "lib_tree_stamp",
              "lib_stamp_ok", "bench_wall_s"):
        if k in res:
            line[k] = res[k]
    line["roofline"] = _roof(res.get("roofline"))
    line["cpu_baseline"] = _cpu(res.get("cpu_baseline"))
    if isinstance(res.get("train_step"), dict):
        t = res["train_step"]
        line["train_gcn_cfg2"] = {"step_ms": t.get("step_ms"), "forward_ms": t.get("forward_ms"),
                                  "backward_ms": t.get("backward_ms"),
                                  "edges_per_s": t.get("edges_per_s"),
                                  "natural_order_step_ms": t.get("natural_order_step_ms"),
                                  "model_step_ms": t.get("model_step_ms")}
    if isinstance(res.get("phases_ms"), dict):  # N > 1: the per-phase max over ranks
        line["phases_ms_max"] = res["phases_ms"].get("max_over_ranks")
        line["exchange_MB_rank0"] = res["phases_ms"].get("exchange_MB_rank0")
    for k in ("north_star", "cfg3", "cfg4"):
        if isinstance(res.get(k), dict):
            line[k] = _summary(res[k])
            if k == "cfg3" and isinstance(res[k].get("train_step"), dict):
                t = res[k]["train_step"]
                line["train_gat_cfg3"] = {"step_ms": t.get("step_ms"),
                                          "forward_ms": t.get("forward_ms"),
                                          "backward_ms": t.get("backward_ms"),
                                          "natural_order_step_ms":
                                              t.get("natural_order_step_ms"),
                                          "model_step_ms": t.get("model_step_ms")}
    if detail:
        line["detail"] = detail
    line = _rnd(line)
    for k in ("value", "ms_per_step"):  # the headline numbers at full precision
        if k in res:
            line[k] = res[k]
    # last resort (never expected): drop the summaries, then the optional extras
    for k in ("north_star", "cfg4", "cfg3", "train_gat_cfg3", "train_gcn_cfg2", "phases_ms_max",
              "exchange_MB_rank0"):
        if len(json.dumps(line)) <= LINE_MAX_BYTES:
            break
        line.pop(k, None)
    assert len(json.dumps(line)) <= LINE_MAX_BYTES
    return line


def write_detail(res: dict, world: int) -> str | None:
    """The full result beside the line: $GNN_BENCH_DETAIL or gpurun_out/bench_detail_n<N>.json
    (relative to the repo root); the line names it. A failed write leaves the line intact."""
    path = Path(os.environ.get("GNN_BENCH_DETAIL") or
                ROOT / "gpurun_out" / f"bench_detail_n{world}.json")
    try:
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_text(json.dumps(res, indent=1) + "\n")
    except OSError as e:
        log(f"[bench] detail file not written: {e!r}")
        return None
    return str(path.relative_to(ROOT)) if path.is_relative_to(ROOT) else str(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="one workload only (default: cfg2 as the headline, plus the north "
                         "star, cfg3 and cfg4 as sub-objects at N=1)")
    ap.add_argument("--feat", type=int, default=None,
                    help="feature width (default: the workload's, 128 except cfg5 = 256)")
    ap.add_argument("--no-extras", action="store_true",
                    help="headline only (no north_star / cfg3 / cfg4 sub-objects)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cold", action="store_true",
                    help="skip the cache-cold step timing (profiling runs: exactly warmup + steps)")
    ap.add_argument("--no-layer", action="store_true",
                    help="skip the Graph_conv_layer (GEMM + SpMM) timing beside the aggregation "
                         "(and the two-layer GCN_Model forward at the north star)")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the training-step (forward + backward) sub-objects (cfg2 GCN "
                         "layer, cfg3 GAT layer)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the cfg4 MAX / MAXPOOL aggregator sub-object (profiling runs: "
                         "only the headline kernels launch)")
    ap.add_argument("--no-replay", action="store_true",
                    help="skip the SpMM replay floor (roofline.replay_floor: the step with its hub "
                         "gathers / all gathers served from an L2-resident table)")
    ap.add_argument("--no-cpu-reference", action="store_true",
                    help="skip the torch CPU operator lines (torch.spmm COO / sparse.mm CSR)")
    ap.add_argument("--exchange", default="cover", choices=["cover", "gather"],
                    help="N>1 halo exchange: feature rows + remote partial sums (cover) or "
                         "feature rows only (gather)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = multi-rank rehearsal (host-staged exchange), never for numbers")
    ap.add_argument("--scale", type=float, default=1.0,
                    help="graph size factor (rehearsals of the N-rank path on one GPU only; the "
                         "JSON config reports the nodes / edges actually used)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic summary (tools/pmc_traffic.py); default profiles/traffic_<workload>_F<feat>.json")
    args = ap.parse_args()
    # stdout carries exactly ONE line, the JSON result: whatever the libraries print there
    # (RCCL's version banner at communicator init, gloo's peer messages) goes to stderr with
    # the bench's own log lines
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if os.environ.get("GNN_BENCH_STACKS"):  # rehearsals: every rank dumps its stack periodically
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GNN_BENCH_STACKS"]), repeat=True)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    global WD
    WD = Watchdog(rank, world > 1 or os.environ.get("GNN_BENCH_WATCHDOG") == "1")
    phase("set_device", 180)
    dev_index = int(os.environ.get("GNN_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    phase("init_process_group", 300)
    if world > 1:
        if args.backend == "nccl":
            if os.environ.get("LOCAL_WORLD_SIZE", str(world)) == str(world):
                os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # single node: loopback bootstrap
            dist.init_process_group("nccl", device_id=dev)
        else:
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # the box hostname may not resolve
            dist.init_process_group("gloo")

    phase("load_library", 180)
    from graphneuralnetwork_amd import _lib
    _lib.load()
    workload = args.workload or "cfg2"
    extras = (args.workload is None and world == 1 and not args.no_extras and args.scale == 1.0)
    t_all = time.perf_counter()
    if workload == "cfg3":
        res = run_gat(args, dev, rank, world)
    elif workload == "cfg4":
        res = run_sage(args, dev, rank, world)
    else:
        res = run_gcn(args, dev, rank, world, workload)
    if extras:
        # the other BASELINE configs that fit one GPU, timed in the same driver run: the north
        # star (10M / 100M, F=128), cfg3 (GAT) and cfg4 (GraphSAGE). The 10M / 100M R-MAT edge
        # list is drawn once for the north star and cfg4.
        from graphneuralnetwork_amd.rmat import rmat_edges
        t0 = time.time()
        e10 = rmat_edges(WORKLOADS["ns"]["nodes"], WORKLOADS["ns"]["edges"], 0)
        log(f"[bench] 10M / 100M rmat edges ready in {time.time() - t0:.1f}s")
        res["north_star"] = _sub(run_gcn(args, dev, 0, 1, "ns", edges_np=e10, extras=True))
        res["north_star"]["target"] = (
            "north_star: >= 60 % of the 8 TB/s HBM roofline on this SpMM, <= 2.5 ms on the "
            "compulsory bytes: NOT met. Measured ceiling (roofline.replay_floor): with every hub "
            "gather served from L2 the step takes ~10.1 ms, with every gather from L2 ~7.5 ms "
            "(frac 0.20): 207M gathered 512-B rows, not HBM bytes, set the time. SpMM work "
            "closed (DESIGN.md section 8)")
        res["cfg3"] = _sub(run_gat(args, dev, 0, 1))
        res["cfg4"] = _sub(run_sage(args, dev, 0, 1, edges_np=e10))
        del e10
    phase("report", 120)
    if rank == 0:
        res["bench_wall_s"] = time.perf_counter() - t_all
        res.update(library_stamps())
        line = compact_line(res, write_detail(res, world))
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()
    phase("done", None)


if __name__ == "__main__":
    main()
