"""Device-side GraphSAGE mini-batch sampling (reference: GraphSAGE/data_utils.py:82-162).

The reference's ``collate_fn`` samples on the host with Python sets and
``random``, needs one fanout for every layer (its maps are stacked with
``torch.tensor``) and materialises every neighbour feature row with
``torch.embedding``.  Here the frontier of a batch is built on the device:

    nb_i    = sample(adj, S_i, fanouts[i])         # [|S_i|, k_i]  (gnn_sample_neighbors)
    S_{i+1} = unique(S_i ++ nb_i)                   # sorted ids, S_0 = the seeds
    maps_i  = positions of S_i / nb_i inside S_{i+1}  # the reference's -1-free index maps

and the batch is handed to ``GraphSAGE.forward`` as ``Gathered`` (table, index)
pairs, so no [M, k, F] neighbour tensor is ever written: the layer-0
aggregation gathers straight from the feature table (gnn_sage_gather_aggregate_f32).
Per-hop fanouts ([25, 10], or any number of layers) are supported.  The reference's set iteration order
and Mersenne-Twister draws are not reproduced (it is unseeded); the sampled
distribution is (tests/test_sampler_gpu.py).
"""
from __future__ import annotations

from dataclasses import dataclass

import ctypes

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
_FRONTIER_GEN = [0]  # bumped by every build_frontier: a rank() of an older build refuses to run


def _frontier_ws(n_nodes: int, dev) -> torch.Tensor:
    key = (dev, n_nodes)
    ws = _FRONTIER_WS.get(key)
    if ws is None:
        ws = torch.empty(int(_lib.load().gnn_frontier_workspace_bytes(n_nodes)), dtype=torch.uint8,
                         device=dev)
        _FRONTIER_WS.clear()  # one graph at a time
        _FRONTIER_WS[key] = ws
    return ws


_SAMPLE_WS = {}


def _sample_ws(n_nodes: int, dev, stream=None) -> torch.Tensor:
    """gnn_sample_layers' workspace for an n_nodes graph: zero-filled once here; every call
    leaves it zero-filled again (the frontier flags are cleared by the scan that reads them).
    One workspace per (device, graph size, stream), as the header requires: two streams
    sampling at once never share the flags / tile tags. Allocated on ``stream``
    (the sampler's), so the caching allocator reuses it only in that stream's order."""
    stream = stream if stream is not None else torch.cuda.current_stream(dev)
    key = (dev, n_nodes, stream.cuda_stream)
    ws = _SAMPLE_WS.get(key)
    if ws is None:
        for k in [k for k in _SAMPLE_WS if k[1] != n_nodes]:  # one graph size at a time
            del _SAMPLE_WS[k]
        with torch.cuda.stream(stream):
            ws = torch.zeros(int(_lib.load().gnn_sample_layers_workspace_bytes(n_nodes)),
                             dtype=torch.uint8, device=dev)
        _SAMPLE_WS[key] = ws
    return ws


def build_frontier(ids_a: torch.Tensor, ids_b: torch.Tensor, n_nodes: int, err: torch.Tensor):
    """(sorted distinct ids of ids_a and ids_b, rank function) on the device: the
    reference's set union + index remap (GraphSAGE/data_utils.py:100-116), as
    torch.unique(cat[a, b]) + torch.searchsorted would give, with a node bitmap instead of
    a sort (gnn_frontier_*). One host synchronisation: the frontier size, read together
    with the pending sampler error bits ``err`` (raised first) and the marks' own.

    The bitmap and prefix workspace is shared per (device, n_nodes): ``rank`` must run on
    the current stream before the next ``build_frontier`` (it raises once the workspace has
    been rebuilt)."""
    dev = ids_a.device
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    ws = _frontier_ws(n_nodes, dev)
    _FRONTIER_GEN[0] += 1
    gen = _FRONTIER_GEN[0]
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
        if _FRONTIER_GEN[0] != gen or _FRONTIER_WS.get((dev, n_nodes)) is not ws:
            raise RuntimeError("build_frontier: rank() called after the frontier workspace was "
                               "rebuilt by a later build_frontier / sample_batch")
        ids = ids.to(torch.int64).contiguous()
        pos = torch.empty_like(ids)
        _lib.check(lib.gnn_frontier_rank(ids.data_ptr(), ids.numel(), n_nodes, ws.data_ptr(),
                                         pos.data_ptr(), stream), "gnn_frontier_rank")
        return pos

    return frontier, rank


@dataclass
class SampledBatch:
    """The device form of collate_fn's output (GraphSAGE/data_utils.py:104-162) for L layers.

    Sampling layer i draws ``fanouts[i]`` neighbours for S_i (S_0 = the seeds) and
    S_{i+1} = sorted unique(S_i ++ those neighbours). The forward runs the other way round:
    its layer 0 aggregates S_{L-1}'s neighbours, so the maps are kept in forward order --
    ``center_maps[i]`` = positions of S_{L-2-i} in S_{L-1-i}, ``neigh_maps[i]`` = positions
    of S_{L-2-i}'s sampled neighbours in S_{L-1-i}, exactly the reference's
    nodes_map[1:] / neigh_nodes_map[1:] (without its -1 padding)."""
    seeds: torch.Tensor        # [B] global ids (S_0)
    frontier: torch.Tensor     # S_{L-1} global ids (sorted; the seeds when L = 1), layer-0 centres
    frontier_nbrs: torch.Tensor  # [|S_{L-1}|, k_{L-1}] global ids (index the feature table)
    center_maps: list          # L-1 tensors, forward order (see above)
    neigh_maps: list           # L-1 tensors [|S_{L-2-i}|, k_{L-2-i}], forward order
    layers: tuple = ()         # S_0 (the seeds), ..., S_{L-1} (= frontier)
    # sample_batch(..., sync=False): the tensors above are the buffers at their capacity,
    # live[i] = |S_i| as a device int64 scalar (None for the seeds), and _finish() reads the
    # sizes and error bits back and returns the batch at its real sizes
    live: tuple = ()
    _finish: object = None

    @property
    def pending(self) -> bool:
        """True for a sync=False batch whose sizes and error bits the host has not read."""
        return self._finish is not None

    def sync(self) -> "SampledBatch":
        """This batch at its real sizes (one host read for a pending batch; raises the
        sampler's errors exactly as sample_batch(..., sync=True) does)."""
        return self._finish() if self._finish is not None else self

    def check(self) -> None:
        """Raise the sampler's error, if any (a pending batch's one host read)."""
        self.sync()

    @property
    def layer_sizes(self) -> tuple:
        return tuple(int(t.numel()) for t in self.sync().layers)

    @property
    def center_map(self) -> torch.Tensor:
        """Positions of the seeds in S_1 (the last forward layer's centre map)."""
        return self.center_maps[-1]

    @property
    def neigh_map(self) -> torch.Tensor:
        """Positions of the seeds' sampled neighbours in S_1 ([B, k_0])."""
        return self.neigh_maps[-1]

    @property
    def sampled_edges(self) -> int:
        b = self.sync()
        return int(b.frontier_nbrs.numel() + sum(m.numel() for m in b.neigh_maps))

    def forward_args(self, table: torch.Tensor):
        """The 4 leading arguments of GraphSAGE.forward (supervised branch). A pending batch's
        arguments carry the device sizes (``Gathered.live``, the maps' ``_gnn_live``): the
        inference forward then runs without a host round trip."""
        lv = self.live[-1] if self.live else None
        return (Gathered(table, self.frontier, True, lv), [trust_map(m) for m in self.center_maps],
                Gathered(table, self.frontier_nbrs, True, lv),
                [trust_map(m) for m in self.neigh_maps])


_STAT_HOST = {}


def _stat_host(n: int) -> torch.Tensor:
    """A pinned host buffer of n int64 (cached) for sample_batch's one readback."""
    t = _STAT_HOST.get(n)
    if t is None:
        t = _STAT_HOST[n] = torch.empty(n, dtype=torch.int64, pin_memory=True)
    return t


def sample_batch(adj: CsrGraph, seeds: torch.Tensor, fanouts=(25, 10), seed: int = 0,
                 gcn: bool = False, sync: bool = True) -> SampledBatch:
    """L = len(fanouts) layer frontier for ``seeds`` (get_layer_adj_nodes,
    GraphSAGE/data_utils.py:82-103, with a fanout per layer like GraphSAGE_Pytorch's
    multihop_sampling): fanouts[i] neighbours for every node of S_i, chained per hop.

    One library call (gnn_sample_layers) issues every hop's kernels with the list lengths kept
    on the device -- for [25, 10] three launches: draw + frontier marks, the frontier scan,
    draw + the maps -- and ONE host read at the end fetches the layer sizes and the error bits:
    the same tensors as ``sample_batch_stepwise`` (which reads each frontier size back before
    the next hop), bit for bit.

    ``sync=False``: no host read at all -- the batch comes back pending (``SampledBatch.live``
    holds the layer sizes on the device, the tensors are the buffers at their capacity), so
    the inference forward is enqueued right behind the sampler; ``batch.check()`` /
    ``batch.sync()`` later read the sizes and error bits (the sampler's errors are raised
    there, after a forward that ran on the flawed lists -- its gathers are range-checked, so
    it reads nothing outside the tables)."""
    fanouts = tuple(int(k) for k in fanouts)
    if not fanouts or min(fanouts) < 1:
        raise ValueError("fanouts must hold at least one positive neighbour count")
    if not adj.rowptr.is_cuda:
        raise RuntimeError("sampling runs on the ROCm device only (no CPU fallback)")
    seeds = seeds.to(device=adj.device, dtype=torch.int64).contiguous()
    if seeds.numel() == 0 or max(fanouts) > 64 or adj.n_rows == 0:
        # fanouts above the lane sampler's 64 (and empty inputs) take the hop-by-hop path
        return sample_batch_stepwise(adj, seeds, fanouts, seed, gcn)
    dev = adj.device
    L = len(fanouts)
    plan = _batch_plan(adj.n_rows, seeds.numel(), fanouts, gcn)
    caps, offs, tot, fan_a, cap_a = plan
    # every output in ONE allocation at 256-B boundaries, its pieces addressed by offset and
    # viewed once, at their final sizes, after the readback: the call is host-bound at cfg4
    # size (three ~15 us kernels), so host work is what there is to cut
    buf = torch.empty(tot, dtype=torch.int64, device=dev)
    base = buf.data_ptr()
    ptr = [base + 8 * o for o in offs]  # layers 1.., nbrs 0.., cmaps, nmaps, stat
    stream = torch.cuda.current_stream(dev)  # the sampler's kernels and its readback
    ws = _sample_ws(adj.n_rows, dev, stream)
    P = ctypes.c_void_p
    seed_a = (ctypes.c_uint64 * L)(*[stream_seed(seed, i) for i in range(L)])
    lib = _lib.load()
    _lib.check(lib.gnn_sample_layers(adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.n_rows,
                                     seeds.data_ptr(), seeds.numel(), L, fan_a, seed_a,
                                     1 if gcn else 0, (P * L)(None, *ptr[:L - 1]), cap_a,
                                     (P * L)(*ptr[L - 1:2 * L - 1]),
                                     (P * max(1, L - 1))(*ptr[2 * L - 1:3 * L - 2]),
                                     (P * max(1, L - 1))(*ptr[3 * L - 2:4 * L - 3]), ptr[-1],
                                     ws.data_ptr(), ws.numel(), stream.cuda_stream),
               "gnn_sample_layers")
    widths = [k + (1 if gcn else 0) for k in fanouts]

    def view(o, rows, w=0):
        return buf.as_strided((rows, w) if w else (rows,), (w, 1) if w else (1,), o)

    def build(sizes, live=(), finish=None):
        layers = [seeds] + [view(offs[i - 1], sizes[i]) for i in range(1, L)]
        nbrs_last = view(offs[2 * L - 2], sizes[L - 1], widths[L - 1])
        cmaps = [view(offs[2 * L - 1 + i], sizes[i]) for i in range(L - 1)]
        nmaps = [view(offs[3 * L - 2 + i], sizes[i], widths[i]) for i in range(L - 1)]
        for i in range(1, L - 1) if live else ():  # rows of map i = |S_i| (i = 0: the seeds)
            cmaps[i]._gnn_live = live[i]
            nmaps[i]._gnn_live = live[i]
        return SampledBatch(seeds, layers[-1], nbrs_last, cmaps[::-1], nmaps[::-1],
                            tuple(layers), tuple(live), finish)

    def finish():
        # on the stream the sampler ran on, whatever stream is current when a pending batch is
        # synced: the copy waits for the scan kernels that wrote the sizes
        host = _stat_host(L + 1)
        with torch.cuda.stream(stream):
            host.copy_(buf[offs[-1]:offs[-1] + L + 1], non_blocking=True)  # pinned: no staging
        stream.synchronize()  # the one host synchronisation
        st = host.tolist()  # every layer size + the error bits
        sizes, e = st[:L], int(st[L]) & 0xFFFFFFFF
        _raise_sample_error(e & 3)  # the sampler's own errors first, as the step-by-step path
        if e & 8:
            raise IndexError("sample_batch: a sampled id outside the graph reached the frontier")
        if e & 4:
            raise RuntimeError("sample_batch: a frontier outgrew its buffer (internal bound "
                               "error)")
        if e & 16:
            raise RuntimeError("sample_batch: the frontier scan's look-back did not complete "
                               "(internal error)")
        return build(sizes)

    if sync:
        return finish()
    stat = offs[-1]
    live = [None] + [buf[stat + i:stat + i + 1] for i in range(1, L)]
    return build(caps, live, finish)


_BATCH_PLAN = {}


def _batch_plan(n_rows: int, n_seeds: int, fanouts: tuple, gcn: bool):
    """(caps, buffer offsets, total int64 count, fanout / cap ctypes arrays) of sample_batch's
    one output buffer, cached per (graph size, batch size, fanouts, gcn). Pieces, in order:
    layers 1..L-1 [cap_i], neighbour lists 0..L-1 [cap_i, w_i], centre maps 0..L-2 [cap_i],
    neighbour maps 0..L-2 [cap_i, w_i], the L + 1 status words."""
    key = (n_rows, n_seeds, fanouts, gcn)
    p = _BATCH_PLAN.get(key)
    if p is None:
        L = len(fanouts)
        widths = [k + (1 if gcn else 0) for k in fanouts]
        caps = [n_seeds]
        for i in range(L - 1):
            caps.append(min(n_rows, caps[i] * (1 + widths[i])))
        sizes = ([caps[i] for i in range(1, L)] + [caps[i] * widths[i] for i in range(L)] +
                 [caps[i] for i in range(L - 1)] + [caps[i] * widths[i] for i in range(L - 1)] +
                 [L + 1])
        offs, tot = [], 0
        for n in sizes:
            offs.append(tot)
            tot += -(-n // 32) * 32
        p = (caps, offs, tot, (ctypes.c_int64 * L)(*fanouts), (ctypes.c_int64 * L)(*caps))
        if len(_BATCH_PLAN) > 64:
            _BATCH_PLAN.clear()
        _BATCH_PLAN[key] = p
    return p


def sample_batch_stepwise(adj: CsrGraph, seeds: torch.Tensor, fanouts=(25, 10), seed: int = 0,
                          gcn: bool = False) -> SampledBatch:
    """``sample_batch`` hop by hop: gnn_sample_neighbors, then the frontier (gnn_frontier_*,
    whose size is read back before the next hop), per layer."""
    fanouts = tuple(int(k) for k in fanouts)
    if not fanouts or min(fanouts) < 1:
        raise ValueError("fanouts must hold at least one positive neighbour count")
    seeds = seeds.to(device=adj.device, dtype=torch.int64).contiguous()
    err = torch.zeros(1, dtype=torch.int32, device=adj.device)
    layers = [seeds]
    cmaps, nmaps = [], []
    nb = None
    for i, k in enumerate(fanouts):
        nb = _sample_into(adj, layers[i], k, seed, i, err)
        if gcn:  # the reference appends the node itself (data_utils.py:95-96)
            nb = torch.cat([nb, layers[i][:, None]], dim=1)
        if i == len(fanouts) - 1:
            break
        # S_{i+1} = sorted unique(S_i ++ nb) and the maps into it (bitmap frontier, no sort);
        # the sampler's error bits are read with the frontier size (one host synchronisation)
        nxt, rank = build_frontier(layers[i], nb, adj.n_rows, err)
        cmaps.append(rank(layers[i]))
        nmaps.append(rank(nb))
        layers.append(nxt)
    batch = SampledBatch(seeds, layers[-1], nb, cmaps[::-1], nmaps[::-1], tuple(layers))
    _raise_sample_error(int(err.item()))
    return batch


def degree_ordered(adj: CsrGraph, table: torch.Tensor | None = None):
    """The dataset relabelled once by degree (``graph.degree_order``, rows and columns): the
    highest-degree nodes get the smallest ids, so the rows the sampled batches gather most
    often sit together at the top of the feature table (fewer pages, more L2 / Infinity-Cache
    hits: cfg4 layer-0 gather 51.9 -> 45.5 us, forward 135 -> 128 us,
    profiles/r03j_sage_order_probe.log). Returns ``(adj', table', order)``: adj' keeps
    ascending neighbours per row (``symmetric_adjacency``'s layout), table' = table[perm];
    a seed v becomes ``order.inv[v]``, and every output row stays the row of its seed."""
    from .graph import degree_order
    o = degree_order(adj, rows=True)
    g = o.graph
    n = g.n_rows
    rows = torch.repeat_interleave(torch.arange(n, device=g.device, dtype=torch.int64),
                                   g.rowptr[1:] - g.rowptr[:-1])
    # each row's neighbours back in ascending order; the values follow their edges (a weighted
    # adjacency keeps every weight on its own edge)
    key, perm = torch.sort(rows * n + g.col.to(torch.int64), stable=True)
    del rows
    g2 = CsrGraph(g.rowptr, (key % n).to(torch.int32).contiguous(), g.val[perm].contiguous(),
                  n, n)
    return g2, (o.permute_rows(table) if table is not None else None), o


def symmetric_adjacency(src, dst, n: int, device=None) -> CsrGraph:
    """Undirected neighbour lists without self-loops (the reference's ``adj_lists`` of sets,
    GraphSAGE/data_utils.py:30-38) as a CSR with ascending neighbours."""
    s = torch.as_tensor(src, dtype=torch.int64, device=device)
    d = torch.as_tensor(dst, dtype=torch.int64, device=device)
    keep = s != d
    s, d = s[keep], d[keep]
    key = torch.unique(torch.cat([s * n + d, d * n + s]))
    r, c = key // n, key % n
    # r is sorted (torch.unique): row starts by binary search, not a histogram whose atomics
    # serialise on equal neighbours (torch.bincount took 33 ms at the cfg4 graph's 197M keys)
    rowptr = torch.searchsorted(r, torch.arange(n + 1, dtype=torch.int64, device=s.device))
    return CsrGraph(rowptr, c.to(torch.int32), torch.ones(c.numel(), device=s.device), n, n)
