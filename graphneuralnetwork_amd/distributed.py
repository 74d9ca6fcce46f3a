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
bipartite edge set), which ships ~1.8x fewer rows on an 8-way RMAT cut; step 1
becomes one SpMM over a "send" CSR and the exchange is still one all-to-all-v.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

from .graph import CsrGraph, from_coo


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


def _all_to_all_v(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    """All-to-all-v (RCCL ncclAllToAllv under the nccl backend).

    Device tensors under a gloo group (multi-rank rehearsal on one GPU) are
    staged through host memory; the RCCL path never is."""
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
    vertex cover of the bipartite edge set cuts the exchanged rows of an 8-way
    RMAT edge-cut ~1.8x (hub rows are covered once instead of once per
    neighbour), see DESIGN.md section 6.

    Per aggregation it is still ONE all-to-all-v: the send buffer is produced
    by one SpMM over ``send`` (rows = send slots grouped by peer,
    [partial rows | feature rows]; a feature row is a 1-entry row with value
    1.0, an exact copy), and the receive buffer is reduced by ``halo`` (rows =
    owned rows; a column entry carries A_ij, a partial entry 1.0).
    """

    rank: int
    world: int
    bounds: list
    interior: CsrGraph      # rows: owned rows; cols: owned rows (local ids)
    send: CsrGraph          # rows: send slots; cols: owned rows (local ids)
    halo: CsrGraph          # rows: owned rows; cols: receive slots
    send_counts: list       # rows sent to each peer
    recv_counts: list       # rows received from each peer
    n_partial_recv: int     # partial-sum rows among the received rows
    n_feature_recv: int     # feature rows among the received rows

    @property
    def n_own(self) -> int:
        return self.bounds[self.rank + 1] - self.bounds[self.rank]

    @property
    def n_halo(self) -> int:
        return int(sum(self.recv_counts))

    @property
    def nnz(self) -> int:
        """Stored edges this rank reduces per aggregation (interior + send + halo)."""
        return self.interior.nnz + self.send.nnz + self.halo.nnz


def _exclusive_cumsum(t: torch.Tensor) -> torch.Tensor:
    return torch.cumsum(t, 0) - t


def build_cover_exchange(g: CsrGraph, rank: int, world: int, group=None,
                         bounds: torch.Tensor | None = None) -> CoverExchange:
    """Rank ``rank``'s block of the cover exchange (see ``CoverExchange``).

    Only this rank's rows of ``g`` are read. The cover is chosen locally (the
    owner of a row block sees every edge of its blocks A[p, q]) with the greedy
    rule "cover (i, j) by its row when row i has more edges into q than column
    j has from p's rows", then tightened in two passes (an edge whose row is
    already shipped as a partial joins it; an edge whose column is already
    shipped drops its partial). The edges to be reduced remotely are handed to
    their column owners once, here.
    """
    if bounds is None:
        bounds = nnz_balanced_bounds(g.rowptr, world)
    b = [int(v) for v in bounds.cpu().tolist()]
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
    pkey = pq * max(n_own, 1) + pr
    order = torch.sort(pkey, stable=True).indices              # by (peer, row), edge order kept
    pr, pc, pv, pq, pkey = pr[order], pc[order], pv[order], pq[order], pkey[order]
    pkeys = torch.unique_consecutive(pkey)
    np_ = torch.bincount(pkeys // max(n_own, 1), minlength=world).to(i64)
    npe = torch.bincount(pq, minlength=world).to(i64)

    # ---- one-time handshake -----------------------------------------------------------------
    mine = torch.stack([nx, np_, npe], 1).contiguous()        # [world, 3] what I ask of each peer
    theirs = torch.empty_like(mine)
    _all_to_all_v(theirs.view(-1), mine.view(-1), [3] * world, [3] * world, group)
    mine_l, theirs_l = mine.cpu().tolist(), theirs.cpu().tolist()
    req_x = torch.empty(sum(t[0] for t in theirs_l), dtype=i64, device=dev)
    _all_to_all_v(req_x, xcols.contiguous(), [t[0] for t in theirs_l], [m[0] for m in mine_l], group)
    pe_send = torch.stack([pr + r0, pc], 0).contiguous()       # global (row, col) per edge
    n_pe_in = sum(t[2] for t in theirs_l)
    pe_ij = torch.empty((2, n_pe_in), dtype=i64, device=dev)
    spl_out, spl_in = [t[2] for t in theirs_l], [m[2] for m in mine_l]
    for k in range(2):
        buf = torch.empty(n_pe_in, dtype=i64, device=dev)
        _all_to_all_v(buf, pe_send[k].contiguous(), spl_out, spl_in, group)
        pe_ij[k] = buf
    pe_v = torch.empty(n_pe_in, dtype=val.dtype, device=dev)
    _all_to_all_v(pe_v, pv.contiguous(), spl_out, spl_in, group)

    # ---- send CSR (what this rank computes for its peers) ---------------------------------
    tx = torch.tensor([t[0] for t in theirs_l], dtype=i64, device=dev)
    tp = torch.tensor([t[1] for t in theirs_l], dtype=i64, device=dev)
    send_sizes = tx + tp
    send_off = _exclusive_cumsum(send_sizes)
    peer_e = torch.repeat_interleave(torch.arange(world, device=dev, dtype=i64),
                                     torch.tensor(spl_out, dtype=i64, device=dev))
    n_tot = b[-1]
    _, prow = torch.unique_consecutive(peer_e * n_tot + pe_ij[0], return_inverse=True)
    p_slot = send_off[peer_e] + (prow - _exclusive_cumsum(tp)[peer_e])
    peer_x = torch.repeat_interleave(torch.arange(world, device=dev, dtype=i64), tx)
    x_slot = send_off[peer_x] + tp[peer_x] + (torch.arange(req_x.numel(), device=dev, dtype=i64)
                                              - _exclusive_cumsum(tx)[peer_x])
    send = from_coo(torch.cat([p_slot, x_slot]), torch.cat([pe_ij[1] - r0, req_x - r0]),
                    torch.cat([pe_v, torch.ones(req_x.numel(), dtype=val.dtype, device=dev)]),
                    int(send_sizes.sum()), n_own)

    # ---- halo CSR (how this rank folds in what it receives) -------------------------------
    recv_off = _exclusive_cumsum(nx + np_)
    xq = torch.searchsorted(bt, xc, right=True) - 1
    xs = recv_off[xq] + np_[xq] + (torch.searchsorted(xcols, xc) - _exclusive_cumsum(nx)[xq])
    kq = pkeys // max(n_own, 1)
    ki = pkeys - kq * max(n_own, 1)
    ks = recv_off[kq] + (torch.arange(pkeys.numel(), device=dev, dtype=i64) - _exclusive_cumsum(np_)[kq])
    halo = from_coo(torch.cat([xr, ki]), torch.cat([xs, ks]),
                    torch.cat([xv, torch.ones(pkeys.numel(), dtype=val.dtype, device=dev)]),
                    n_own, int((nx + np_).sum()))
    return CoverExchange(rank, world, b, interior, send, halo,
                         [int(v) for v in send_sizes.cpu().tolist()],
                         [int(v) for v in (nx + np_).cpu().tolist()],
                         int(np_.sum()), int(nx.sum()))


class EdgeCutSpmm:
    """Y_own = (A X)[own rows] (+ bias) for one rank of the edge-cut, halo exchange overlapped.

    ``spmm`` / ``gather`` default to the HIP kernels; tests on gloo/CPU pass
    CPU checkers instead (they exercise the partition + exchange logic only).
    """

    def __init__(self, part: EdgeCutPartition | CoverExchange, feat: int, device, group=None,
                 spmm=None, gather=None):
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
        self.send_buf = torch.empty((sum(part.send_counts), feat), dtype=torch.float32,
                                    device=self.device)
        self.recv_buf = torch.empty((part.n_halo, feat), dtype=torch.float32, device=self.device)
        self.out = torch.empty((part.n_own, feat), dtype=torch.float32, device=self.device)
        self.cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.cuda else None

    def __call__(self, x: torch.Tensor, bias: torch.Tensor | None = None,
                 activation: str | None = None) -> torch.Tensor:
        p = self.part
        if x.shape != (p.n_own, self.feat):
            raise ValueError("x must be this rank's [n_own, feat] feature rows")
        if self.cover:
            if self.send_buf.shape[0]:
                self._spmm(p.send, x, None, out=self.send_buf)   # partial sums + feature rows
        elif p.send_idx.numel():
            self._gather(x, p.send_idx, self.send_buf)
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            self.comm_stream.wait_stream(cur)
            with torch.cuda.stream(self.comm_stream):
                _all_to_all_v(self.recv_buf, self.send_buf, p.recv_counts, p.send_counts,
                              self.group)
            # interior rows overlap the exchange on the compute stream
            self._spmm(p.interior, x, bias, out=self.out)
            cur.wait_stream(self.comm_stream)
        else:
            _all_to_all_v(self.recv_buf, self.send_buf, p.recv_counts, p.send_counts, self.group)
            self._spmm(p.interior, x, bias, out=self.out)
        self._spmm(p.halo, self.recv_buf, None, activation=activation, out=self.out,
                   accumulate=True)
        return self.out


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

    The halo rows of Wh AND of the column logits er are packed into one buffer
    and exchanged with a single all-to-all-v; the fused edge-softmax aggregation
    then runs over the rank's extended graph [own | halo] (the softmax of a row
    needs all its edges, so the interior and halo edges are reduced together).
    """

    def __init__(self, part: EdgeCutPartition, heads: int, fh: int, device, group=None,
                 logits=None, aggregate=None, gather=None):
        self.part = part
        self.heads, self.fh = heads, fh
        self.group = group
        self.device = torch.device(device)
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

    def __call__(self, wh_own: torch.Tensor, a_src: torch.Tensor, a_dst: torch.Tensor,
                 negative_slope: float, mode: int, activation: str | None = None):
        p = self.part
        F = self.heads * self.fh
        el, er = self._logits(wh_own, self.heads, self.fh, a_src, a_dst)
        packed = torch.cat([wh_own, er], dim=1)
        if p.send_idx.numel():
            self._gather(packed, p.send_idx, self.send_buf)
        _all_to_all_v(self.recv_buf, self.send_buf, p.recv_counts, p.send_counts, self.group)
        wh_ext = torch.cat([wh_own, self.recv_buf[:, :F]], dim=0)
        er_ext = torch.cat([er, self.recv_buf[:, F:]], dim=0)
        return self._aggregate(self.ext, wh_ext, el, er_ext, self.heads, self.fh,
                               negative_slope, mode, activation)
