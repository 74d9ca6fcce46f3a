"""Multi-GPU GCN aggregation: 1-D edge-cut with an RCCL halo exchange.

One process per GPU (torchrun), ``torch.distributed`` on the nccl (= RCCL)
backend; the same code runs on gloo/CPU for the tests.

Partition (built once per graph, ``build_partition``):
  * nodes are split into ``world`` contiguous row blocks balanced by nnz
    (``nnz_balanced_bounds``); rank p owns rows [b_p, b_{p+1}) of A and the
    same rows of the feature matrix X;
  * rank p's rows are split into an *interior* CSR (columns it owns, remapped
    to local ids) and a *halo* CSR (remote columns, remapped to slots of a
    compact halo buffer, sorted by global id so each peer's rows are one
    contiguous slice);
  * one count all-to-all + one id all-to-all-v tell every owner which of its
    rows each peer needs (the send lists).

Per aggregation (``EdgeCutSpmm.__call__``):
  1. pack the rows peers need (HIP row gather) on the compute stream;
  2. exchange them with ONE all-to-all-v (RCCL over xGMI: all 7 peer links at
     once) on a communication stream ...
  3. ... while the interior SpMM runs on the compute stream;
  4. halo SpMM accumulating into the same output (GNN_EPI_ACCUMULATE), bias
     applied once.
Y_p = A[p, own] X_own + A[p, halo] X_halo = (A X)[rows of p], bit-for-bit the
single-GPU reduction up to fp32 summation order.

``build_cover_exchange`` is the SpMM default: instead of shipping the feature
row of every remote column, each cut block is covered by feature rows AND
remotely computed partial row sums (a greedy vertex cover of the block's
bipartite edge set), which ships 2-3x fewer rows on an RMAT cut; the two kinds
travel in two all-to-all-v's that pipeline with the partial-sum, interior and
halo SpMMs. The feature rows go in ``HALO_CHUNKS`` chunked all-to-all-v's, so that the halo
SpMM of one chunk runs while the next is in flight (``EdgeCutSpmm(chunks=...)``).

GraphSAGE (``sage_forward_sharded``) needs no exchange on its forward path: seed batches
shard across ranks and the feature table is replicated (5.1 GB at 10M x 128 fits 288 GB).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .graph import CsrGraph, from_coo


def weighted_bounds(rowptr: torch.Tensor, world: int, weights=None, old_bounds=None) -> torch.Tensor:
    """Row boundaries [world+1] balancing  sum_i w_block(i) * (deg_i + 1)  per block, where
    ``weights[b]`` is a cost density for the rows of block b of ``old_bounds`` (all 1.0:
    plain edges + rows balance)."""
    n = rowptr.numel() - 1
    dev = rowptr.device
    c = (rowptr[1:] - rowptr[:-1]).to(torch.float64) + 1.0
    if weights is not None:
        ob = torch.as_tensor(old_bounds, dtype=torch.int64, device=dev)
        blk = torch.bucketize(torch.arange(n, device=dev), ob[1:-1], right=True)
        c = c * torch.as_tensor(weights, dtype=torch.float64, device=dev)[blk]
    cost = torch.zeros(n + 1, dtype=torch.float64, device=dev)
    torch.cumsum(c, 0, out=cost[1:])
    total = float(cost[-1])
    targets = torch.tensor([total * k / world for k in range(world + 1)], dtype=torch.float64,
                           device=dev)
    b = torch.searchsorted(cost, targets).clamp_(0, n)
    b[0] = 0
    b[-1] = n
    return torch.cummax(b, 0).values.to(torch.int64)


def nnz_balanced_bounds(rowptr: torch.Tensor, world: int) -> torch.Tensor:
    """Row boundaries [world+1] so each block holds ~nnz/world stored edges (+ rows as a tiebreak)."""
    n = rowptr.numel() - 1
    nnz = int(rowptr[-1])
    # balance edges + rows (output rows cost bytes too)
    cost = rowptr.to(torch.float64) + torch.arange(n + 1, dtype=torch.float64, device=rowptr.device)
    total = float(cost[-1])
    targets = torch.tensor([total * k / world for k in range(world + 1)], dtype=torch.float64,
                           device=rowptr.device)
    b = torch.searchsorted(cost, targets).clamp_(0, n)
    b[0] = 0
    b[-1] = n
    b = torch.cummax(b, 0).values
    del nnz
    return b.to(torch.int64)


@dataclass
class EdgeCutPartition:
    rank: int
    world: int
    bounds: list            # [world+1] row boundaries (python ints)
    interior: CsrGraph      # rows: owned rows; cols: owned rows (local ids)
    halo: CsrGraph          # rows: owned rows; cols: halo slots
    halo_ids: torch.Tensor  # int64 [n_halo] global ids of the halo slots (sorted)
    send_idx: torch.Tensor  # int64 [n_send] local row ids to send, grouped by peer
    send_counts: list
    recv_counts: list

    @property
    def n_own(self) -> int:
        return self.bounds[self.rank + 1] - self.bounds[self.rank]

    @property
    def n_halo(self) -> int:
        return int(self.halo_ids.numel())

    @property
    def nnz(self) -> int:
        return self.interior.nnz + self.halo.nnz


class LocalGroup:
    """``world`` ranks as threads of ONE process (one device): this module's collectives
    (all-to-all-v, the count all-reduce, the float all-gather) become copies between the
    ranks' tensors. It runs the whole N-rank path -- partition builders, handshakes and
    exchanges -- at full size on one GPU without N processes time-slicing it (tests,
    tools/rank_sim.py). Each thread calls ``bind(rank)`` first; every collective is entered
    by all ranks, in the same order, as with torch.distributed."""

    def __init__(self, world: int):
        import threading
        self.world = world
        self._bar = threading.Barrier(world)
        self._box: list = [None] * world
        self._tls = threading.local()

    def bind(self, rank: int) -> None:
        self._tls.rank = rank

    @property
    def rank(self) -> int:
        return self._tls.rank

    @staticmethod
    def _drain(t: torch.Tensor) -> None:
        if t.is_cuda:  # this rank's queued work on the tensor is done (the exchange stream's)
            torch.cuda.current_stream(t.device).synchronize()

    def all_to_all_v(self, out, inp, out_splits, in_splits) -> None:
        r = self.rank
        self._drain(inp)
        offs = [0]
        for v in in_splits:
            offs.append(offs[-1] + int(v))
        self._box[r] = [inp[offs[k]:offs[k + 1]] for k in range(self.world)]
        self._bar.wait()
        parts = [self._box[k][r] for k in range(self.world)]
        if sum(int(v) for v in out_splits) != sum(int(p.shape[0]) for p in parts):
            raise RuntimeError("LocalGroup.all_to_all_v: split sizes do not match the peers'")
        if out.numel():
            torch.cat([p.to(out.device) for p in parts], out=out)
        self._drain(out)  # the copies are done before any sender reuses its buffer
        self._bar.wait()

    def all_gather(self, v: list) -> list:
        r = self.rank
        self._box[r] = list(v)
        self._bar.wait()
        res = [list(self._box[k]) for k in range(self.world)]
        self._bar.wait()
        return res


def _all_to_all_v(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    """All-to-all-v (RCCL ncclAllToAllv under the nccl backend).

    Device tensors under a gloo group (multi-rank rehearsal on one GPU) are
    staged through host memory; the RCCL path never is."""
    if isinstance(group, LocalGroup):
        group.all_to_all_v(out, inp, out_splits, in_splits)
        return
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), output_split_sizes=list(out_splits),
                               input_split_sizes=list(in_splits), group=group)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp, output_split_sizes=list(out_splits),
                           input_split_sizes=list(in_splits), group=group)


def build_partition(g: CsrGraph, rank: int, world: int, group=None,
                    bounds: torch.Tensor | None = None) -> EdgeCutPartition:
    """Rank ``rank``'s edge-cut block of the (replicated) graph ``g`` + send/recv lists.

    Only this rank's rows of ``g`` are read; the send lists are negotiated with
    the peers (two all-to-alls), so the same code works when each rank only
    holds its own rows.
    """
    if bounds is None:
        bounds = nnz_balanced_bounds(g.rowptr, world)
    b = [int(v) for v in bounds.cpu().tolist()]
    r0, r1 = b[rank], b[rank + 1]
    n_own = r1 - r0
    dev = g.device
    e0, e1 = int(g.rowptr[r0]), int(g.rowptr[r1])
    rp = g.rowptr[r0:r1 + 1] - e0
    col = g.col[e0:e1].to(torch.int64)
    val = g.val[e0:e1]
    rows = torch.repeat_interleave(torch.arange(n_own, device=dev, dtype=torch.int64),
                                   rp[1:] - rp[:-1])
    own = (col >= r0) & (col < r1)
    interior = from_coo(rows[own], col[own] - r0, val[own], n_own, n_own)
    hcol = col[~own]
    halo_ids = torch.unique(hcol)                       # sorted global ids
    halo = from_coo(rows[~own], torch.searchsorted(halo_ids, hcol), val[~own], n_own,
                    int(halo_ids.numel()))
    bt = torch.tensor(b, dtype=torch.int64, device=dev)
    owner = torch.searchsorted(bt, halo_ids, right=True) - 1
    recv_counts_t = torch.bincount(owner, minlength=world).to(torch.int64)
    send_counts_t = torch.empty_like(recv_counts_t)
    _all_to_all_v(send_counts_t, recv_counts_t, [1] * world, [1] * world, group)
    recv_counts = [int(v) for v in recv_counts_t.cpu().tolist()]
    send_counts = [int(v) for v in send_counts_t.cpu().tolist()]
    req = torch.empty(sum(send_counts), dtype=torch.int64, device=dev)
    _all_to_all_v(req, halo_ids.contiguous(), send_counts, recv_counts, group)
    send_idx = req - r0
    return EdgeCutPartition(rank, world, b, interior, halo, halo_ids, send_idx, send_counts,
                            recv_counts)


@dataclass
class CoverExchange:
    """Edge-cut SpMM exchange that ships, per cut edge, EITHER the feature row
    of its column OR a partial sum of its row -- whichever covers more edges.

    For the cut block A[p, q] (rows owned by p, columns owned by q) every edge
    (i, j) is covered either by shipping X_j from q to p (column cover) or by q
    computing the partial row sum  s_qi = sum_{j in q} A_ij X_j  over its own
    rows of X and shipping s_qi to p (row cover).  Picking, per block, a small
    vertex cover of the bipartite edge set cuts the rows exchanged by an 8-way
    RMAT edge-cut ~2-3x (a hub row is covered once instead of once per
    neighbour), see DESIGN.md section 6.

    Per aggregation the two kinds travel in two all-to-all-v's so that the
    exchange pipelines with the compute:
      gather feature rows -> [exchange 1]  while the partial-sum SpMM (``send_p``)
      -> [exchange 2] while the interior SpMM, then the ``halo_x`` SpMM (A_ij over
      the received feature rows) -> ``halo_p`` (1.0 x each received partial row).
    """

    rank: int
    world: int
    bounds: list
    interior: CsrGraph      # rows: owned rows; cols: owned rows (local ids)
    send_x_idx: torch.Tensor  # int64: local rows whose features peers need, grouped by peer
    send_p: CsrGraph        # rows: partial-sum slots grouped by peer; cols: owned rows
    halo_x: CsrGraph        # rows: owned rows; cols: received feature-row slots
    halo_p: CsrGraph        # rows: owned rows; cols: received partial-row slots (values 1.0)
    send_x_counts: list
    send_p_counts: list
    recv_x_counts: list
    recv_p_counts: list
    any_x: bool             # some rank exchanges feature rows (collective is needed)
    any_p: bool             # some rank exchanges partial rows
    # feature rows rank p receives from rank q, for every (p, q): the same on every rank
    recv_x_matrix: list = field(default=None)

    @property
    def n_own(self) -> int:
        return self.bounds[self.rank + 1] - self.bounds[self.rank]

    @property
    def send_counts(self) -> list:
        return [a + b for a, b in zip(self.send_x_counts, self.send_p_counts)]

    @property
    def recv_counts(self) -> list:
        return [a + b for a, b in zip(self.recv_x_counts, self.recv_p_counts)]

    @property
    def n_halo(self) -> int:
        return int(sum(self.recv_counts))

    @property
    def n_partial_recv(self) -> int:
        return int(sum(self.recv_p_counts))

    @property
    def n_feature_recv(self) -> int:
        return int(sum(self.recv_x_counts))

    @property
    def nnz(self) -> int:
        """Stored entries this rank reduces per aggregation."""
        return self.interior.nnz + self.send_p.nnz + self.halo_x.nnz + self.halo_p.nnz


def _exclusive_cumsum(t: torch.Tensor) -> torch.Tensor:
    return torch.cumsum(t, 0) - t


def _global_sum(v: int, device, group=None) -> int:
    if isinstance(group, LocalGroup):
        return int(sum(x[0] for x in group.all_gather([int(v)])))
    on_dev = torch.device(device).type == "cuda" and dist.get_backend(group) != "gloo"
    t = torch.tensor([v], dtype=torch.int64, device=device if on_dev else "cpu")
    dist.all_reduce(t, group=group)
    return int(t.item())


# build the cover on the device through the C-ABI (csrc/cover_build.hip: gnn_cover_build /
# _fill / _send_partials, the arrays of the torch restatement below; up to 64 ranks)
NATIVE_COVER = True


def build_cover_exchange(g: CsrGraph, rank: int, world: int, group=None,
                         bounds: torch.Tensor | None = None) -> CoverExchange:
    """Rank ``rank``'s block of the cover exchange (see ``CoverExchange``).

    Only this rank's rows of ``g`` are read. The cover is chosen locally (the
    owner of a row block sees every edge of its blocks A[p, q]) with the greedy
    rule "cover (i, j) by its row when row i has more edges into q than column
    j has from p's rows", then tightened in two passes (an edge whose row is
    already shipped as a partial joins it; an edge whose column is already
    shipped drops its partial). The edges to be reduced remotely are handed to
    their column owners once, here. On the device the local choice and the
    partial-sum CSR are built by the C-ABI (``NATIVE_COVER``), the handshake is
    this module's collectives either way.
    """
    if bounds is None:
        bounds = nnz_balanced_bounds(g.rowptr, world)
    b = [int(v) for v in bounds.cpu().tolist()]
    r0, r1 = b[rank], b[rank + 1]
    n_own = r1 - r0
    dev = g.device
    i64 = torch.int64
    native = NATIVE_COVER and g.rowptr.is_cuda and world <= 64
    local = (_cover_local_native if native else _cover_local_torch)(g, rank, world, b)
    interior, xcols, nx, (pe_src_i, pe_src_j, pe_src_v), np_, npe, halo_x, halo_p = local

    # ---- one-time handshake -----------------------------------------------------------------
    mine = torch.stack([nx, np_, npe], 1).contiguous()        # [world, 3] what I ask of each peer
    theirs = torch.empty_like(mine)
    _all_to_all_v(theirs.view(-1), mine.view(-1), [3] * world, [3] * world, group)
    mine_l, theirs_l = mine.cpu().tolist(), theirs.cpu().tolist()
    req_x = torch.empty(sum(t[0] for t in theirs_l), dtype=i64, device=dev)
    _all_to_all_v(req_x, xcols.contiguous(), [t[0] for t in theirs_l], [m[0] for m in mine_l], group)
    spl_out, spl_in = [t[2] for t in theirs_l], [m[2] for m in mine_l]
    n_pe_in = sum(spl_out)
    pe_i = torch.empty(n_pe_in, dtype=i64, device=dev)
    pe_j = torch.empty(n_pe_in, dtype=i64, device=dev)
    pe_v = torch.empty(n_pe_in, dtype=g.val.dtype, device=dev)
    _all_to_all_v(pe_i, pe_src_i.contiguous(), spl_out, spl_in, group)
    _all_to_all_v(pe_j, pe_src_j.contiguous(), spl_out, spl_in, group)
    _all_to_all_v(pe_v, pe_src_v.contiguous(), spl_out, spl_in, group)

    # ---- what this rank computes / copies for its peers ------------------------------------
    n_p_send = sum(t[1] for t in theirs_l)
    if native:
        send_p = _cover_send_partials_native(pe_i, pe_j, pe_v, spl_out, world, r0, n_own, n_p_send)
    else:
        peer_e = torch.repeat_interleave(torch.arange(world, device=dev, dtype=i64),
                                         torch.tensor(spl_out, dtype=i64, device=dev))
        _, p_slot = torch.unique_consecutive(peer_e * b[-1] + pe_i, return_inverse=True)
        send_p = from_coo(p_slot.view(-1), pe_j - r0, pe_v, n_p_send, n_own)
    # every rank's feature-row requests ([world, world]: row p = rows p receives from each q),
    # so that a consumer of the exchange (EdgeCutSpmm's chunking) decides from data all ranks
    # hold, with no collective of its own
    x_matrix = [[int(v) for v in row] for row in
                _all_gather_floats([float(m[0]) for m in mine_l], world, dev, group).tolist()]
    any_x = sum(map(sum, x_matrix)) > 0
    any_p = _global_sum(int(halo_p.n_cols), dev, group) > 0
    return CoverExchange(rank, world, b, interior, (req_x - r0).contiguous(), send_p, halo_x,
                         halo_p, [t[0] for t in theirs_l], [t[1] for t in theirs_l],
                         [int(v) for v in nx.cpu().tolist()], [int(v) for v in np_.cpu().tolist()],
                         any_x, any_p, x_matrix)


def _cover_local_torch(g: CsrGraph, rank: int, world: int, b: list):
    """The local half of ``build_cover_exchange`` in torch ops: (interior, requested columns,
    feature rows asked of each peer, the partial edges (global row, global column, value) in
    (owner, row) order, partial rows / partial edges asked of each peer, halo_x, halo_p)."""
    r0, r1 = b[rank], b[rank + 1]
    n_own = r1 - r0
    dev = g.device
    i64 = torch.int64
    e0, e1 = int(g.rowptr[r0]), int(g.rowptr[r1])
    rp = g.rowptr[r0:r1 + 1] - e0
    col = g.col[e0:e1].to(i64)
    val = g.val[e0:e1]
    rows = torch.repeat_interleave(torch.arange(n_own, device=dev, dtype=i64), rp[1:] - rp[:-1])
    own = (col >= r0) & (col < r1)
    interior = from_coo(rows[own], col[own] - r0, val[own], n_own, n_own)

    # ---- choose the cover of the cut edges ------------------------------------------------
    cut = ~own
    rc, cc, vc = rows[cut], col[cut], val[cut]
    bt = torch.tensor(b, dtype=i64, device=dev)
    qc = torch.searchsorted(bt, cc, right=True) - 1           # column owner per cut edge
    _, inv_iq, cnt_iq = torch.unique(rc * world + qc, return_inverse=True, return_counts=True)
    _, inv_j, cnt_j = torch.unique(cc, return_inverse=True, return_counts=True)
    part = cnt_iq[inv_iq] > cnt_j[inv_j]
    hp = torch.zeros(cnt_iq.numel(), dtype=torch.bool, device=dev)
    hp[inv_iq[part]] = True
    part = hp[inv_iq]                                          # row already shipped: join it
    hx = torch.zeros(cnt_j.numel(), dtype=torch.bool, device=dev)
    hx[inv_j[~part]] = True
    part = part & ~hx[inv_j]                                   # column already shipped: use it

    # column cover: feature rows requested from each owner (sorted global ids)
    xr, xc, xv = rc[~part], cc[~part], vc[~part]
    xcols = torch.unique(xc)
    nx = torch.bincount(torch.searchsorted(bt, xcols, right=True) - 1, minlength=world).to(i64)
    # row cover: partial rows (q, i) and the edges the owner q reduces for them
    pr, pc, pv, pq = rc[part], cc[part], vc[part], qc[part]
    stride = max(n_own, 1)
    pkey = pq * stride + pr
    order = torch.sort(pkey, stable=True).indices              # by (peer, row), edge order kept
    pr, pc, pv, pq, pkey = pr[order], pc[order], pv[order], pq[order], pkey[order]
    pkeys = torch.unique_consecutive(pkey)
    np_ = torch.bincount(pkeys // stride, minlength=world).to(i64)
    npe = torch.bincount(pq, minlength=world).to(i64)

    # ---- how this rank folds in what it receives ------------------------------------------
    halo_x = from_coo(xr, torch.searchsorted(xcols, xc), xv, n_own, int(xcols.numel()))
    ki = pkeys - (pkeys // stride) * stride
    halo_p = from_coo(ki, torch.arange(pkeys.numel(), device=dev, dtype=i64),
                      torch.ones(pkeys.numel(), dtype=val.dtype, device=dev), n_own,
                      int(pkeys.numel()))
    return interior, xcols, nx, (pr + r0, pc, pv), np_, npe, halo_x, halo_p


def _cover_local_native(g: CsrGraph, rank: int, world: int, b: list):
    """``_cover_local_torch`` by gnn_cover_build / gnn_cover_fill (the same tensors)."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    dev = g.device
    r0, r1 = b[rank], b[rank + 1]
    n_own = r1 - r0
    e_loc = int(g.rowptr[r1]) - int(g.rowptr[r0])
    stream = _lib.stream_handle(dev)
    hb = (ctypes.c_int64 * (world + 1))(*b)
    ws = torch.empty(int(lib.gnn_cover_workspace_bytes(g.n_rows, e_loc, n_own, world)),
                     dtype=torch.uint8, device=dev)
    counts = (ctypes.c_int64 * (4 + 3 * world))()
    _lib.check(lib.gnn_cover_build(g.rowptr.data_ptr(), _lib.ptr(g.col), g.n_rows,
                                   ctypes.addressof(hb), rank, world, ctypes.addressof(counts),
                                   ws.data_ptr(), ws.numel(), stream), "gnn_cover_build")
    c = [int(v) for v in counts]
    n_int, n_x, n_hx, n_pk = c[:4]
    nx = torch.tensor(c[4:4 + world], dtype=torch.int64, device=dev)
    np_ = torch.tensor(c[4 + world:4 + 2 * world], dtype=torch.int64, device=dev)
    npe = torch.tensor(c[4 + 2 * world:4 + 3 * world], dtype=torch.int64, device=dev)
    n_pe = sum(c[4 + 2 * world:])
    i64, i32, f32 = (dict(dtype=t, device=dev) for t in (torch.int64, torch.int32, torch.float32))
    int_rp, int_col, int_val = (torch.empty(n_own + 1, **i64), torch.empty(n_int, **i32),
                                torch.empty(n_int, **f32))
    xcols = torch.empty(n_x, **i64)
    hx_rp, hx_col, hx_val = (torch.empty(n_own + 1, **i64), torch.empty(n_hx, **i32),
                             torch.empty(n_hx, **f32))
    pe_i, pe_j, pe_v = torch.empty(n_pe, **i64), torch.empty(n_pe, **i64), torch.empty(n_pe, **f32)
    hp_rp, hp_col, hp_val = (torch.empty(n_own + 1, **i64), torch.empty(n_pk, **i32),
                             torch.empty(n_pk, **f32))
    P = _lib.ptr
    _lib.check(lib.gnn_cover_fill(ws.data_ptr(), g.rowptr.data_ptr(), P(g.col), P(g.val), g.n_rows,
                                  ctypes.addressof(hb), rank, world, ctypes.addressof(counts),
                                  int_rp.data_ptr(), P(int_col), P(int_val), P(xcols),
                                  hx_rp.data_ptr(), P(hx_col), P(hx_val), P(pe_i), P(pe_j),
                                  P(pe_v), hp_rp.data_ptr(), P(hp_col), P(hp_val), stream),
               "gnn_cover_fill")
    interior = CsrGraph(int_rp, int_col, int_val, n_own, n_own)
    halo_x = CsrGraph(hx_rp, hx_col, hx_val, n_own, n_x)
    halo_p = CsrGraph(hp_rp, hp_col, hp_val, n_own, n_pk)
    return interior, xcols, nx, (pe_i, pe_j, pe_v), np_, npe, halo_x, halo_p


def _cover_send_partials_native(pe_i, pe_j, pe_v, recv_edges: list, world: int, r0: int,
                                n_own: int, n_p_send: int) -> CsrGraph:
    """The partial-sum CSR this rank computes for its peers (gnn_cover_send_partials)."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    dev = pe_i.device
    m = int(sum(recv_edges))
    ws = torch.empty(int(lib.gnn_cover_send_workspace_bytes(m)), dtype=torch.uint8, device=dev)
    he = (ctypes.c_int64 * world)(*[int(v) for v in recv_edges])
    rp = torch.empty(n_p_send + 1, dtype=torch.int64, device=dev)
    col = torch.empty(m, dtype=torch.int32, device=dev)
    val = torch.empty(m, dtype=torch.float32, device=dev)
    P = _lib.ptr
    _lib.check(lib.gnn_cover_send_partials(P(pe_i), P(pe_j), P(pe_v), ctypes.addressof(he), world,
                                           r0, n_own, n_p_send, rp.data_ptr(), P(col), P(val),
                                           ws.data_ptr(), ws.numel(), _lib.stream_handle(dev)),
               "gnn_cover_send_partials")
    return CsrGraph(rp, col, val, n_p_send, n_own)


def _all_gather_floats(v: list, world: int, device, group=None) -> torch.Tensor:
    """[world, len(v)] float64: every rank's ``v`` (an all-to-all-v of the same row)."""
    if isinstance(group, LocalGroup):
        return torch.tensor(group.all_gather([float(x) for x in v]), dtype=torch.float64)
    on_dev = torch.device(device).type == "cuda" and dist.get_backend(group) != "gloo"
    dev = device if on_dev else "cpu"
    inp = torch.tensor(v, dtype=torch.float64, device=dev).repeat(world)
    out = torch.empty(world * len(v), dtype=torch.float64, device=dev)
    _all_to_all_v(out, inp, [len(v)] * world, [len(v)] * world, group)
    return out.view(world, len(v)).cpu()


# cost of a row of 4F bytes moved over xGMI (RCCL all-to-all) relative to HBM (one
# gathered or written row): ~6 TB/s HBM vs ~0.4-0.5 TB/s of all-to-all per GPU, halved
# because the interior SpMM overlaps the exchange
XGMI_ROW_COST = 8.0


def cover_cost(part: CoverExchange, alpha: float = XGMI_ROW_COST) -> float:
    """Modelled per-aggregation cost of one rank, in units of one 4F-byte row through HBM:
    edges gathered + rows written (read-modify-written by the accumulate passes, only the
    rows with edges) + alpha x the rows this rank sends or receives, whichever is larger."""
    def touched(g: CsrGraph) -> int:
        return int(((g.rowptr[1:] - g.rowptr[:-1]) > 0).sum()) if g.n_rows else 0
    n_sx, n_sp = sum(part.send_x_counts), sum(part.send_p_counts)
    compute = (part.interior.nnz + part.n_own + part.send_p.nnz + n_sp + 2 * n_sx
               + part.halo_x.nnz + 2 * touched(part.halo_x)
               + part.halo_p.nnz + 2 * touched(part.halo_p))
    exchange = max(n_sx + n_sp, sum(part.recv_counts))
    return float(compute + alpha * exchange)


def build_cover_exchange_balanced(g: CsrGraph, rank: int, world: int, group=None,
                                  iters: int = 2, alpha: float = XGMI_ROW_COST, progress=None):
    """``build_cover_exchange`` with row blocks re-cut for the work the cover moves.

    The cover shifts work between ranks (partial sums are computed by the column
    owners; high-id R-MAT blocks hold millions of degree-1 rows), so edges + rows
    balanced blocks end up far apart in cost (8 ranks: 0.8 vs 2.4 ms of compute,
    173 vs 549 MB sent, tools/rank_sim.py). Each iteration gathers every rank's
    ``cover_cost``, turns it into a cost density per block (cost / (edges + rows)) and
    re-cuts with those densities; the partition with the lowest maximum cost is kept
    (the same choice on every rank: they all see the same costs). Returns
    (partition, per-iteration max/mean costs). ``progress(it, max_cost, mean_cost, seconds)``
    is called after each build.
    """
    import time
    bounds = nnz_balanced_bounds(g.rowptr, world)
    best, best_max, history = None, None, []
    deg1 = (g.rowptr[1:] - g.rowptr[:-1]).to(torch.float64) + 1.0
    for it in range(iters + 1):
        t0 = time.perf_counter()
        part = build_cover_exchange(g, rank, world, group, bounds=bounds)
        costs = _all_gather_floats([cover_cost(part, alpha)], world, g.device, group)[:, 0]
        mx, mean = float(costs.max()), float(costs.mean())
        history.append((mx, mean))
        if progress is not None:
            progress(it, mx, mean, time.perf_counter() - t0)
        if best_max is None or mx < best_max:
            best, best_max = part, mx
        else:
            del part
        if it == iters:
            break
        b = [int(v) for v in bounds.cpu().tolist()]
        cum = torch.zeros(deg1.numel() + 1, dtype=torch.float64, device=deg1.device)
        torch.cumsum(deg1, 0, out=cum[1:])
        units = torch.tensor([float(cum[b[k + 1]] - cum[b[k]]) for k in range(world)],
                             dtype=torch.float64)
        dens = (costs / units.clamp(min=1.0)).tolist()
        bounds = weighted_bounds(g.rowptr, world, dens, b)
    return best, history


def _overlaps(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Whether the byte ranges spanned by the views a and b intersect."""
    if a.device != b.device:
        return False

    def span(t):
        last = sum((n - 1) * st for n, st in zip(t.shape, t.stride()))
        return t.data_ptr(), t.data_ptr() + (last + 1) * t.element_size()

    a0, a1 = span(a)
    b0, b1 = span(b)
    return a0 < b1 and b0 < a1


def chunk_sizes(counts: list, chunks: int) -> list:
    """[chunks][world] row counts: peer q's block of counts[q] rows cut into ``chunks``
    contiguous pieces, piece k = rows [k n_q // C, (k+1) n_q // C). Sender and receiver derive
    the same pieces from the same count."""
    return [[(k + 1) * n // chunks - k * n // chunks for n in counts] for k in range(chunks)]


def chunk_major(counts: list, chunks: int, device) -> torch.Tensor:
    """int64 [sum(counts)]: for a buffer laid out peer-major (peer q's rows contiguous, in peer
    order), the source position of each row of the chunk-major layout (chunk k holds piece k
    of every peer, in peer order): new_buf = old_buf[chunk_major(...)]."""
    offs = [0]
    for n in counts:
        offs.append(offs[-1] + int(n))
    parts = []
    for k in range(chunks):
        for q, n in enumerate(counts):
            lo, hi = k * n // chunks, (k + 1) * n // chunks
            if hi > lo:
                parts.append(torch.arange(offs[q] + lo, offs[q] + hi, device=device,
                                          dtype=torch.int64))
    if not parts:
        return torch.zeros(0, dtype=torch.int64, device=device)
    return torch.cat(parts)


def split_halo_chunks(halo_x: CsrGraph, recv_counts: list, chunks: int) -> list:
    """``halo_x`` (columns = receive slots, peer-major) split into ``chunks`` CSRs by the
    chunk-major receive layout (``chunk_major``): graph k reads chunk k's slice of the receive
    buffer, its columns renumbered from 0. Each row keeps its edges' CSR order."""
    dev = halo_x.device
    src = chunk_major(recv_counts, chunks, dev)          # chunk-major position -> receive slot
    new_of_old = torch.empty_like(src)
    new_of_old[src] = torch.arange(src.numel(), device=dev, dtype=torch.int64)
    rows = torch.repeat_interleave(torch.arange(halo_x.n_rows, device=dev, dtype=torch.int64),
                                   halo_x.rowptr[1:] - halo_x.rowptr[:-1])
    newc = new_of_old[halo_x.col.to(torch.int64)] if halo_x.nnz else halo_x.col.to(torch.int64)
    out, lo = [], 0
    for piece in chunk_sizes(recv_counts, chunks):
        hi = lo + sum(piece)
        m = (newc >= lo) & (newc < hi)
        out.append(from_coo(rows[m], newc[m] - lo, halo_x.val[m], halo_x.n_rows, hi - lo,
                            check=False))
        lo = hi
    return out


# Feature-row exchange of the cover SpMM in this many chunked all-to-all-v's (each peer's rows
# cut into HALO_CHUNKS pieces): the halo_x SpMM of chunk k runs while chunk k+1 is in flight,
# instead of every halo gather waiting for the whole exchange. Each extra
# chunk costs one more RCCL launch and one more accumulate pass over the rows it touches.
HALO_CHUNKS = 2


class EdgeCutSpmm:
    """Y_own = (A X)[own rows] (+ bias) for one rank of the edge-cut, halo exchange overlapped.

    ``spmm`` / ``gather`` default to the HIP kernels; tests on gloo/CPU pass
    CPU checkers instead (they exercise the partition + exchange logic only).

    ``chunks`` (cover exchange; default HALO_CHUNKS): the feature rows travel in that many
    all-to-all-v's, laid out chunk-major in the send / receive buffers, and the halo_x SpMM is
    split by column chunk, so the halo gathers of chunk k start as soon as chunk k has landed.
    All ranks skip the same globally empty chunks, decided from the [world, world] count
    matrix ``build_cover_exchange`` gathered: the constructor itself runs no collective.
    """

    def __init__(self, part: EdgeCutPartition | CoverExchange, feat: int, device, group=None,
                 spmm=None, gather=None, chunks: int | None = None):
        self.part = part
        self.feat = feat
        self.group = group
        self.device = torch.device(device)
        if spmm is None or gather is None:
            from .ops import gather_rows, spmm_forward
            spmm = spmm or spmm_forward
            gather = gather or (lambda x, idx, out: gather_rows(x, idx, out=out, check=False))
        self._spmm = spmm
        self._gather = gather
        self.cover = isinstance(part, CoverExchange)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.chunks = max(1, int(HALO_CHUNKS if chunks is None else chunks))
        if self.cover:
            self._build_chunks()
            self.send_x = torch.empty((sum(part.send_x_counts), feat), **f32)
            self.send_p = torch.empty((sum(part.send_p_counts), feat), **f32)
            self.recv_x = torch.empty((sum(part.recv_x_counts), feat), **f32)
            self.recv_p = torch.empty((sum(part.recv_p_counts), feat), **f32)
        else:
            self.send_buf = torch.empty((sum(part.send_counts), feat), **f32)
            self.recv_buf = torch.empty((part.n_halo, feat), **f32)
        # two output buffers used in turn, so a result fed back as the next call's x
        # (stacked layers of one width) is never the buffer that call writes
        self._outs = [torch.empty((part.n_own, feat), **f32) for _ in range(2)]
        self._turn = 0
        self._last = None        # the tensor the most recent call wrote
        self._prof_out = None    # profile()'s own output (it must not use up a turn)
        self.cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._marks = None  # [(name, event)] while profile() runs

    def _build_chunks(self):
        """Chunk-major send / receive layouts of the feature rows and the halo_x SpMM split by
        column chunk (see ``chunks``)."""
        p = self.part
        C = self.chunks
        self.x_send_chunks = chunk_sizes(p.send_x_counts, C)
        self.x_recv_chunks = chunk_sizes(p.recv_x_counts, C)
        self.x_send_off = [0]
        self.x_recv_off = [0]
        for k in range(C):
            self.x_send_off.append(self.x_send_off[-1] + sum(self.x_send_chunks[k]))
            self.x_recv_off.append(self.x_recv_off[-1] + sum(self.x_recv_chunks[k]))
        # chunks that move no row on ANY rank are not issued at all (every rank sees the same
        # totals, so every rank skips the same collectives); a chunk empty on some ranks only
        # is an all-to-all-v with zero counts there, as any exchange can be
        self.x_chunk_live = [True] * C
        if C > 1 and p.any_x:
            if p.recv_x_matrix is not None:   # every rank holds the whole count matrix
                flat = [n for row in p.recv_x_matrix for n in row]
                self.x_chunk_live = [sum(piece) > 0 for piece in chunk_sizes(flat, C)]
            else:  # a CoverExchange built without it: one all-gather of the chunk sizes
                mine = [float(sum(self.x_send_chunks[k]) + sum(self.x_recv_chunks[k]))
                        for k in range(C)]
                tot = _all_gather_floats(mine, p.world, self.device, self.group).sum(0)
                self.x_chunk_live = [bool(v > 0) for v in tot.tolist()]
        if C == 1:
            self.send_x_idx = p.send_x_idx
            self.halo_x_chunks = [p.halo_x]
            return
        self.send_x_idx = p.send_x_idx[chunk_major(p.send_x_counts, C,
                                                   p.send_x_idx.device)].contiguous()
        self.halo_x_chunks = split_halo_chunks(p.halo_x, p.recv_x_counts, C)

    def _mark(self, name, stream):
        if self._marks is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            self._marks.append((name, ev))

    def _exchange(self, recv, send, recv_counts, send_counts, cur, tag="a2a"):
        """All-to-all-v on the communication stream after the work queued on ``cur``;
        returns an event marking its completion (None off-GPU: done on return)."""
        if not self.cuda:
            _all_to_all_v(recv, send, recv_counts, send_counts, self.group)
            return None
        self.comm_stream.wait_stream(cur)
        with torch.cuda.stream(self.comm_stream):
            self._mark(tag + ">", self.comm_stream)
            _all_to_all_v(recv, send, recv_counts, send_counts, self.group)
            self._mark(tag + "<", self.comm_stream)
            ev = torch.cuda.Event()
            ev.record(self.comm_stream)
        return ev

    def profile(self, x, bias=None, activation=None) -> dict:
        """One call with timing events at every phase boundary (GPU only): milliseconds of
        each compute-stream phase in issue order (a "wait_*" phase is the time the compute
        stream stalled on an exchange), of each all-to-all-v on the communication stream,
        and of the whole call. For the multi-GPU bench's per-rank breakdown."""
        if not self.cuda:
            raise RuntimeError("profile() needs the GPU path")
        self._marks = []
        cur = torch.cuda.current_stream(self.device)
        if self._prof_out is None:
            self._prof_out = torch.empty_like(self._outs[0])
        last = self._last
        try:
            self._mark("start", cur)
            self(x, bias, activation, out=self._prof_out)
            self._last = last
            self._mark("end", cur)
            torch.cuda.synchronize(self.device)
        finally:
            marks, self._marks = self._marks, None
        res, prev, opened = {}, None, {}
        t0 = marks[0][1]
        at = {}  # every mark's time since the start (ms)
        for name, ev in marks:
            at[name] = t0.elapsed_time(ev)
            if name.endswith(">"):
                opened[name[:-1]] = ev
            elif name.endswith("<"):
                res[name[:-1] + "_ms"] = opened.pop(name[:-1]).elapsed_time(ev)
            else:
                if prev is not None and name != "end":
                    res[name + "_ms"] = prev.elapsed_time(ev)
                prev = ev if name != "end" else prev
        res["total_ms"] = marks[0][1].elapsed_time(marks[-1][1])
        # the pipelined halo pass: when the first halo_x chunk starts (its wait ends) against
        # when the last feature-row chunk lands; > 0 = halo gathers ran before the last receive
        if self.cover and self.chunks > 1 and "wait_x0" in at:
            last = f"a2a_x{self.chunks - 1}<"
            res["halo_x0_start_at_ms"] = at["wait_x0"]
            if last in at:
                res["a2a_x_last_end_at_ms"] = at[last]
                res["halo_before_last_recv_ms"] = at[last] - at["wait_x0"]
        return res

    def _wait(self, ev, cur):
        if ev is not None:
            cur.wait_event(ev)

    @property
    def out(self) -> torch.Tensor | None:
        """The tensor the most recent call wrote (an internal buffer or the caller's ``out``;
        ``profile()`` calls are not counted)."""
        return self._last

    def __call__(self, x: torch.Tensor, bias: torch.Tensor | None = None,
                 activation: str | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
        """Returns ``out`` if given, else one of two internal buffers used in turn: an
        internal result stays valid until the call after next overwrites it."""
        p = self.part
        if x.shape != (p.n_own, self.feat):
            raise ValueError("x must be this rank's [n_own, feat] feature rows")
        if out is None:
            out = self._outs[self._turn]
            self._turn ^= 1
        elif out.shape != (p.n_own, self.feat) or out.dtype != torch.float32:
            raise ValueError("out must be float32 [n_own, feat]")
        if x.numel() and out.numel() and _overlaps(x, out):
            raise ValueError("x and the output buffer overlap: the interior SpMM would read "
                             "rows it is writing")
        self._last = out
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        if self.cover:
            C = self.chunks
            ev_x, ev_p = [None] * C, None
            if p.any_x:
                if self.send_x.shape[0]:
                    self._gather(x, self.send_x_idx, self.send_x)
                self._mark("gather_send_x", cur)
                so, ro = self.x_send_off, self.x_recv_off
                for k in range(C):  # every rank issues the same (globally non-empty) chunks
                    if not self.x_chunk_live[k]:
                        continue
                    ev_x[k] = self._exchange(self.recv_x[ro[k]:ro[k + 1]],
                                             self.send_x[so[k]:so[k + 1]], self.x_recv_chunks[k],
                                             self.x_send_chunks[k], cur,
                                             "a2a_x" if C == 1 else f"a2a_x{k}")
            if p.any_p:
                if self.send_p.shape[0]:
                    self._spmm(p.send_p, x, None, out=self.send_p)  # partial sums for peers
                self._mark("spmm_send_p", cur)
                ev_p = self._exchange(self.recv_p, self.send_p, p.recv_p_counts,
                                      p.send_p_counts, cur, "a2a_p")
            self._spmm(p.interior, x, bias, out=out)           # overlaps both exchanges
            self._mark("spmm_interior", cur)
            last = "p" if p.any_p else ("x" if p.any_x else None)
            if p.any_x:
                ro = self.x_recv_off
                for k in range(C):
                    sfx = "" if C == 1 else str(k)
                    self._wait(ev_x[k], cur)
                    self._mark("wait_x" + sfx, cur)
                    act = activation if (last == "x" and k == C - 1) else None
                    gk = self.halo_x_chunks[k]
                    if gk.nnz or act is not None:  # an activation pass touches every row
                        self._spmm(gk, self.recv_x[ro[k]:ro[k + 1]], None, out=out,
                                   accumulate=True, activation=act)
                    self._mark("spmm_halo_x" + sfx, cur)
            if p.any_p:
                self._wait(ev_p, cur)
                self._mark("wait_p", cur)
                self._spmm(p.halo_p, self.recv_p, None, out=out, accumulate=True,
                           activation=activation)
                self._mark("spmm_halo_p", cur)
            if last is None and activation is not None:
                self._spmm(p.halo_x, self.recv_x, None, out=out, accumulate=True,
                           activation=activation)
            return out
        if p.send_idx.numel():
            self._gather(x, p.send_idx, self.send_buf)
        self._mark("gather_send", cur)
        ev = self._exchange(self.recv_buf, self.send_buf, p.recv_counts, p.send_counts, cur)
        self._spmm(p.interior, x, bias, out=out)               # overlaps the exchange
        self._mark("spmm_interior", cur)
        self._wait(ev, cur)
        self._mark("wait", cur)
        self._spmm(p.halo, self.recv_buf, None, activation=activation, out=out,
                   accumulate=True)
        self._mark("spmm_halo", cur)
        return out


def extended_graph(part: EdgeCutPartition) -> CsrGraph:
    """Rank-local CSR over [own rows | halo slots]: rows = owned rows, columns
    0..n_own-1 = owned nodes, n_own + k = halo slot k (interior edges first in each row)."""
    g = getattr(part, "_ext", None)
    if g is None:
        dev = part.interior.device
        parts = []
        for csr, off in ((part.interior, 0), (part.halo, part.n_own)):
            rows = torch.repeat_interleave(torch.arange(part.n_own, device=dev, dtype=torch.int64),
                                           csr.rowptr[1:] - csr.rowptr[:-1])
            parts.append((rows, csr.col.to(torch.int64) + off, csr.val))
        g = from_coo(torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts]),
                     torch.cat([p[2] for p in parts]), part.n_own, part.n_own + part.n_halo)
        part._ext = g
    return g


class EdgeCutGat:
    """One GAT attention layer (all heads) on one rank of the edge-cut.

    The halo rows of Wh AND of the column logits er are packed into one buffer and
    exchanged with a single all-to-all-v (RCCL on a communication stream). The softmax of
    a row needs all its edges, so on the HIP path (``overlap``) the row is reduced in two
    passes whose partial softmaxes merge exactly:

      1. while the exchange is in flight, the interior pass aggregates each row over its
         OWNED columns (gat_aggregate with per-row log-sum-exp stats L_int, no activation);
      2. after it, the halo pass aggregates each row over its halo columns (read in place
         from the received [Wh | er] rows, halo slot s = staged row -1-s) plus ONE
         pseudo-edge: the row's interior result, whose logit is made to equal L_int
         (er_pseudo = LeakyReLU^-1(+-L_int) - el_i), so the online softmax weighs it by
         exp(L_int) = sum of the interior edges' weights -- the log-sum-exp merge that
         gat_fixup_kernel applies to segments -- and the activation is applied there.

    Otherwise (CPU checkers, rows with no edge at all) the fused aggregation runs once
    over the rank's extended graph [own | halo] after a blocking exchange.
    """

    def __init__(self, part: EdgeCutPartition, heads: int, fh: int, device, group=None,
                 logits=None, aggregate=None, gather=None, overlap: bool = True):
        self.part = part
        self.heads, self.fh = heads, fh
        self.group = group
        self.device = torch.device(device)
        hip_aggregate = aggregate is None
        if logits is None or aggregate is None or gather is None:
            from .ops import gat_aggregate, gat_logits, gather_rows
            logits = logits or gat_logits
            aggregate = aggregate or gat_aggregate
            gather = gather or (lambda x, idx, out: gather_rows(x, idx, out=out, check=False))
        self._logits, self._aggregate, self._gather = logits, aggregate, gather
        w = heads * fh + heads
        self.send_buf = torch.empty((part.send_idx.numel(), w), dtype=torch.float32,
                                    device=self.device)
        self.recv_buf = torch.empty((part.n_halo, w), dtype=torch.float32, device=self.device)
        self.ext = extended_graph(part)
        self.cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.cuda else None
        from .graph import CsrGraph
        # the HIP path reads the received [Wh | er] rows in place: halo slot s is column -1-s
        # of the staged tables (gat_aggregate_staged)
        self._staged = None
        self._halo_pass = None
        if hip_aggregate and self.cuda and part.n_halo and not self.ext.has_empty_rows():
            col = self.ext.col.to(torch.int64)
            col = torch.where(col < part.n_own, col, part.n_own - 1 - col).to(torch.int32)
            self._staged = CsrGraph(self.ext.rowptr, col.contiguous(), self.ext.val,
                                    part.n_own, part.n_own)
            if overlap:
                self._halo_pass = self._build_halo_pass()
        if self._halo_pass is not None:
            F = heads * fh
            f32 = dict(dtype=torch.float32, device=self.device)
            self.out_int = torch.empty((part.n_own, F), **f32)
            self.lse = torch.empty((part.n_own, heads), **f32)
            self.er_pseudo = torch.empty((part.n_own, heads), **f32)

    def _build_halo_pass(self):
        """Rows = owned rows; per row a pseudo-edge to column i (the row's interior result,
        only for rows with interior edges) followed by its halo edges as columns -1-slot."""
        p = self.part
        dev = self.device
        i64 = torch.int64
        deg_i = p.interior.rowptr[1:] - p.interior.rowptr[:-1]
        has_int = torch.nonzero(deg_i > 0).view(-1)
        hrows = torch.repeat_interleave(torch.arange(p.n_own, device=dev, dtype=i64),
                                        p.halo.rowptr[1:] - p.halo.rowptr[:-1])
        rows = torch.cat([has_int, hrows])
        cols = torch.cat([has_int, -1 - p.halo.col.to(i64)])
        vals = torch.ones(rows.numel(), dtype=torch.float32, device=dev)
        g = from_coo(rows, cols, vals, p.n_own, p.n_own, check=False)  # stable: pseudo first
        return None if g.has_empty_rows() else g

    def __call__(self, wh_own: torch.Tensor, a_src: torch.Tensor, a_dst: torch.Tensor,
                 negative_slope: float, mode: int, activation: str | None = None,
                 el: torch.Tensor | None = None, er: torch.Tensor | None = None):
        """``el`` / ``er``: this rank's logits when already computed (gat_project fuses them
        into the projection); otherwise they are computed here from ``wh_own``."""
        p = self.part
        F = self.heads * self.fh
        if el is None or er is None:
            el, er = self._logits(wh_own, self.heads, self.fh, a_src, a_dst)
        if p.send_idx.numel():  # [Wh | er] rows for the peers, gathered into their columns
            self._gather(wh_own, p.send_idx, self.send_buf[:, :F])
            self._gather(er.contiguous(), p.send_idx, self.send_buf[:, F:])
        if self._halo_pass is not None and wh_own.stride(1) == 1 and negative_slope > 0:
            from .ops import GAT_DENSE, gat_aggregate, gat_aggregate_staged
            cur = torch.cuda.current_stream(self.device)
            self.comm_stream.wait_stream(cur)
            with torch.cuda.stream(self.comm_stream):
                _all_to_all_v(self.recv_buf, self.send_buf, p.recv_counts, p.send_counts,
                              self.group)
                ev = torch.cuda.Event()
                ev.record(self.comm_stream)
            # interior pass over the owned columns, overlapping the exchange
            el_c, er_c = el.contiguous(), er.contiguous()
            gat_aggregate(p.interior, wh_own, el_c, er_c, self.heads, self.fh, negative_slope,
                          mode, None, out=self.out_int, stats=self.lse)
            y = self.lse if mode == GAT_DENSE else -self.lse
            torch.sub(torch.where(y >= 0, y, y / negative_slope), el_c, out=self.er_pseudo)
            cur.wait_event(ev)
            return gat_aggregate_staged(self._halo_pass, self.out_int, el_c, self.er_pseudo,
                                        self.recv_buf[:, :F], self.recv_buf[:, F:], self.heads,
                                        self.fh, negative_slope, mode, activation)
        _all_to_all_v(self.recv_buf, self.send_buf, p.recv_counts, p.send_counts, self.group)
        if self._staged is not None and wh_own.stride(1) == 1:
            from .ops import gat_aggregate_staged
            return gat_aggregate_staged(self._staged, wh_own, el, er, self.recv_buf[:, :F],
                                        self.recv_buf[:, F:], self.heads, self.fh,
                                        negative_slope, mode, activation)
        wh_ext = torch.cat([wh_own, self.recv_buf[:, :F]], dim=0)
        er_ext = torch.cat([er, self.recv_buf[:, F:]], dim=0)
        return self._aggregate(self.ext, wh_ext, el, er_ext, self.heads, self.fh,
                               negative_slope, mode, activation)


# ------------------------------------------------------------------------------ GraphSAGE
def shard_seeds(seeds: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Rank ``rank``'s contiguous block of a seed batch (sizes differ by at most one, order
    kept): GraphSAGE data parallelism -- each rank samples and runs its own
    seeds against a replicated feature table, with no collective on the forward path."""
    n = seeds.numel()
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return seeds[lo:hi]


def rank_sample_seed(seed: int, rank: int) -> int:
    """The sampler seed of one rank's shard: independent device RNG streams per rank (the
    reference draws every batch from one sequential generator)."""
    return (int(seed) * 0x9E3779B97F4A7C15 + int(rank) + 1) & 0xFFFFFFFFFFFFFFFF


def all_gather_rows(local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """Every rank's [n_r, ...] rows concatenated in rank order (an all-gather-v built from a
    count all-gather and one all-to-all-v of the rows each rank sends to every peer)."""
    dev = local.device
    counts = _all_gather_floats([float(local.shape[0])], world, dev, group)[:, 0]
    counts = [int(c) for c in counts.tolist()]
    width = 1
    for d in local.shape[1:]:
        width *= int(d)
    flat = local.reshape(local.shape[0], width).contiguous()
    out = torch.empty((sum(counts), width), dtype=local.dtype, device=dev)
    inp = flat.repeat(world, 1) if world > 1 else flat
    _all_to_all_v(out.view(-1), inp.view(-1), [c * width for c in counts],
                  [local.shape[0] * width] * world, group)
    return out.view(sum(counts), *local.shape[1:])


def sage_forward_sharded(net, adj, table: torch.Tensor, seeds: torch.Tensor, rank: int,
                         world: int, fanouts=(25, 10), seed: int = 0, group=None,
                         gather: bool = False):
    """Data-parallel GraphSAGE inference over one seed batch: rank ``rank`` samples its
    shard (``shard_seeds``; sampler stream ``rank_sample_seed(seed, rank)``) from the
    replicated adjacency and runs ``net`` (the drop-in GraphSAGE.forward, supervised
    branch) against the replicated table. Returns (embeddings, logits) of the shard, or of
    the whole batch in seed order with ``gather=True`` (``all_gather_rows``)."""
    from .sampler import sample_batch
    mine = shard_seeds(seeds, rank, world)
    if mine.numel():
        batch = sample_batch(adj, mine, fanouts, seed=rank_sample_seed(seed, rank))
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
    else:  # fewer seeds than ranks: an empty shard still joins the gather
        last = list(net.sage_blocks)[-1]
        emb = torch.empty((0, last.output_size), dtype=torch.float32, device=table.device)
        logits = (torch.empty((0, net.dense.out_features), dtype=torch.float32,
                              device=table.device) if not net.Unsupervised else None)
    if gather:
        emb = all_gather_rows(emb, world, group)
        logits = all_gather_rows(logits, world, group) if logits is not None else None
    return emb, logits
