"""Device-side GraphSAGE mini-batch sampling (reference: GraphSAGE/data_utils.py:82-162).

The reference's ``collate_fn`` samples on the host with Python sets and
``random``, needs one fanout for every layer (its maps are stacked with
``torch.tensor``) and materialises every neighbour feature row with
``torch.embedding``.  Here the frontier of a batch is built on the device:

    nb0  = sample(adj, seeds, fanouts[0])             # [B, k0]   (gnn_sample_neighbors)
    S1   = unique(seeds ++ nb0)                        # layer-0 centre nodes (sorted ids)
    nb1  = sample(adj, S1, fanouts[1])                 # [|S1|, k1] global ids
    maps = positions of seeds / nb0 inside S1          # the reference's -1-free index maps

and the batch is handed to ``GraphSAGE.forward`` as ``Gathered`` (table, index)
pairs, so no [M, k, F] neighbour tensor is ever written: the layer-0
aggregation gathers straight from the feature table (gnn_sage_gather_aggregate_f32).
Per-hop fanouts ([25, 10]) are supported.  The reference's set iteration order
and Mersenne-Twister draws are not reproduced (it is unseeded); the sampled
distribution is (tests/test_sampler_gpu.py).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib
from .graph import CsrGraph
from .graphsage import Gathered, trust_map


_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    """splitmix64 finaliser (the same mix the device RNG applies)."""
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def stream_seed(seed: int, layer: int) -> int:
    """The device RNG key of one (batch seed, layer) pair: hashed, so batch s's layer 1
    and batch s+1's layer 0 draw independently (seed + layer would collide)."""
    return _mix64(_mix64(int(seed) & _M64) ^ ((int(layer) * 0xD1B54A32D192ED03) & _M64))


def _sample_into(adj: CsrGraph, nodes: torch.Tensor, k: int, seed: int, layer: int,
                 err: torch.Tensor) -> torch.Tensor:
    """gnn_sample_neighbors without a host synchronisation (the error bits go to ``err``)."""
    if not adj.rowptr.is_cuda:
        raise RuntimeError("sampling runs on the ROCm device only (no CPU fallback)")
    nodes = nodes.to(device=adj.device, dtype=torch.int64).contiguous()
    out = torch.empty((nodes.numel(), k), dtype=torch.int64, device=adj.device)
    lib = _lib.load()
    _lib.check(lib.gnn_sample_neighbors(adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.n_rows,
                                        nodes.data_ptr(), nodes.numel(), k,
                                        stream_seed(seed, layer), out.data_ptr(),
                                        err.data_ptr(), _lib.stream_handle(adj.device)),
               "gnn_sample_neighbors")
    return out


def _raise_sample_error(e: int) -> None:
    if e & 2:
        raise IndexError("sample_neighbors: node id out of range")
    if e & 1:  # random.choices(list(set()), k) in the reference
        raise IndexError("Cannot choose from an empty sequence")


def sample_neighbors(adj: CsrGraph, nodes: torch.Tensor, k: int, seed: int = 0,
                     layer: int = 0) -> torch.Tensor:
    """[len(nodes), k] int64 sampled neighbour ids (random.sample / random.choices rule).

    Draws are keyed by (stream_seed(seed, layer), position in ``nodes``, draw): a node
    listed twice gets two independent neighbour lists, like the reference's sequential
    draws from one generator (GraphSAGE/data_utils.py:89-94)."""
    err = torch.zeros(1, dtype=torch.int32, device=adj.device)
    out = _sample_into(adj, nodes, k, seed, layer, err)
    _raise_sample_error(int(err.item()))
    return out


_FRONTIER_WS: dict = {}


def _frontier_ws(n_nodes: int, dev) -> torch.Tensor:
    key = (dev, n_nodes)
    ws = _FRONTIER_WS.get(key)
    if ws is None:
        ws = torch.empty(int(_lib.load().gnn_frontier_workspace_bytes(n_nodes)), dtype=torch.uint8,
                         device=dev)
        _FRONTIER_WS.clear()  # one graph at a time
        _FRONTIER_WS[key] = ws
    return ws


def build_frontier(ids_a: torch.Tensor, ids_b: torch.Tensor, n_nodes: int, err: torch.Tensor):
    """(sorted distinct ids of ids_a and ids_b, rank function) on the device: the
    reference's set union + index remap (GraphSAGE/data_utils.py:100-116), as
    torch.unique(cat[a, b]) + torch.searchsorted would give, with a node bitmap instead of
    a sort (gnn_frontier_*). One host synchronisation: the frontier size, read together
    with the pending sampler error bits ``err`` (raised first) and the marks' own."""
    dev = ids_a.device
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    ws = _frontier_ws(n_nodes, dev)
    a = ids_a.to(torch.int64).contiguous().view(-1)
    b = ids_b.to(torch.int64).contiguous().view(-1)
    stat = torch.zeros(3, dtype=torch.int64, device=dev)
    err_f = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(lib.gnn_frontier_build(a.data_ptr(), a.numel(), b.data_ptr(), b.numel(), n_nodes,
                                      ws.data_ptr(), ws.numel(), stat.data_ptr(), err_f.data_ptr(),
                                      stream), "gnn_frontier_build")
    stat[1:2].copy_(err.to(torch.int64))
    stat[2:3].copy_(err_f.to(torch.int64))
    count, e, ef = (int(v) for v in stat.cpu().tolist())
    _raise_sample_error(e)   # the sampler's own error first (its rows of -1 also trip ef)
    _raise_sample_error(ef)
    frontier = torch.empty(count, dtype=torch.int64, device=dev)
    _lib.check(lib.gnn_frontier_emit(n_nodes, ws.data_ptr(), frontier.data_ptr(), stream),
               "gnn_frontier_emit")

    def rank(ids: torch.Tensor) -> torch.Tensor:
        ids = ids.to(torch.int64).contiguous()
        pos = torch.empty_like(ids)
        _lib.check(lib.gnn_frontier_rank(ids.data_ptr(), ids.numel(), n_nodes, ws.data_ptr(),
                                         pos.data_ptr(), stream), "gnn_frontier_rank")
        return pos

    return frontier, rank


@dataclass
class SampledBatch:
    seeds: torch.Tensor        # [B] global ids
    frontier: torch.Tensor     # S1 [M] global ids (sorted), layer-0 centres
    frontier_nbrs: torch.Tensor  # [M, k1] global ids (index the feature table)
    center_map: torch.Tensor   # [B] positions of the seeds in S1
    neigh_map: torch.Tensor    # [B, k0] positions of the seeds' neighbours in S1

    @property
    def sampled_edges(self) -> int:
        return int(self.frontier_nbrs.numel() + self.neigh_map.numel())

    def forward_args(self, table: torch.Tensor):
        """The 4 leading arguments of GraphSAGE.forward (supervised branch)."""
        return (Gathered(table, self.frontier, True), [trust_map(self.center_map)],
                Gathered(table, self.frontier_nbrs, True), [trust_map(self.neigh_map)])


def sample_batch(adj: CsrGraph, seeds: torch.Tensor, fanouts=(25, 10), seed: int = 0,
                 gcn: bool = False) -> SampledBatch:
    """Two-layer frontier for ``seeds`` (fanouts[0] for the seeds, fanouts[1] for S1)."""
    if len(fanouts) != 2:
        raise NotImplementedError("two-layer sampling (the reference's num_layers=2 runs)")
    seeds = seeds.to(device=adj.device, dtype=torch.int64).contiguous()
    err = torch.zeros(1, dtype=torch.int32, device=adj.device)
    nb0 = _sample_into(adj, seeds, fanouts[0], seed, 0, err)
    if gcn:  # the reference appends the node itself (data_utils.py:95-96)
        nb0 = torch.cat([nb0, seeds[:, None]], dim=1)
    # S1 = sorted unique(seeds ++ nb0) and the maps into it (bitmap frontier, no sort); the
    # sampler's error bits are read with the frontier size (one host synchronisation)
    s1, rank = build_frontier(seeds, nb0, adj.n_rows, err)
    nb1 = _sample_into(adj, s1, fanouts[1], seed, 1, err)
    if gcn:
        nb1 = torch.cat([nb1, s1[:, None]], dim=1)
    batch = SampledBatch(seeds, s1, nb1, rank(seeds), rank(nb0))
    _raise_sample_error(int(err.item()))
    return batch


def symmetric_adjacency(src, dst, n: int, device=None) -> CsrGraph:
    """Undirected neighbour lists without self-loops (the reference's ``adj_lists`` of sets,
    GraphSAGE/data_utils.py:30-38) as a CSR with ascending neighbours."""
    s = torch.as_tensor(src, dtype=torch.int64, device=device)
    d = torch.as_tensor(dst, dtype=torch.int64, device=device)
    keep = s != d
    s, d = s[keep], d[keep]
    key = torch.unique(torch.cat([s * n + d, d * n + s]))
    r, c = key // n, key % n
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=s.device)
    torch.cumsum(torch.bincount(r, minlength=n), 0, out=rowptr[1:])
    return CsrGraph(rowptr, c.to(torch.int32), torch.ones(c.numel(), device=s.device), n, n)
