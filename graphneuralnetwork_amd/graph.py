"""CSR graphs and row-split plans resident in HBM.

The reference hands its aggregation ops three adjacency forms:

* GCN: a torch sparse COO fp32 tensor, int64 indices, *uncoalesced*, built by
  ``sparse_mx_to_torch_sparse_tensor`` (GCN/data_utils.py:63-70);
* GAT (dense layer): a dense [N, N] tensor whose entries ``> 0`` are edges
  (GAT/models/layers.py:29, GAT/data_utils.py:85);
* GAT (sparse layer): the same dense tensor, edges = ``adj.nonzero()``
  (GAT/models/layers.py:98).

All of them become one ``CsrGraph`` (rowptr int64 [N+1], col int32 [nnz],
val fp32 [nnz]) on the device, built once and cached on the adjacency tensor
object (keyed by the tensor's version counter, so an in-place edit rebuilds
it).  Duplicate COO entries are kept as separate edges: the SpMM sums them,
exactly as ``torch.spmm`` does on an uncoalesced tensor.

Power-law rows (degree > ``seg_len``) get a ``RowSplitPlan`` built on the
device by the C-ABI (``gnn_spmm_plan_*``); it is cached per ``seg_len``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import torch

from . import _lib

# Long-row segment size: ~192 KiB of gathered feature rows per wavefront. A/B on
# MI355X with hub staging (tools/lib_ab.py): 384 edges at F=128 beats 192 by 2.6 %
# (1M-node graph) and 1 % (10M-node graph); 288-512 are within 1 % of each other, and at
# F=256 192 edges beat 96 by 1 %. (Before hub staging 192 was best at F=128.)
SEG_BYTES = 192 * 1024
# the GAT passes keep the 96 KiB segments they were tuned with (tools/gat_ab.py)
GAT_SEG_BYTES = 96 * 1024
MIN_SEG_LEN = 64


def seg_len_for(feat: int, seg_bytes: int = SEG_BYTES) -> int:
    return max(MIN_SEG_LEN, seg_bytes // max(1, 4 * feat))


@dataclass
class RowSplitPlan:
    """Row classes of a CSR graph (plan.hip): small (deg <= 1), mid, long (split)."""

    seg_len: int
    seg_row: torch.Tensor      # int32 [n_seg]
    seg_begin: torch.Tensor    # int64 [n_seg]
    long_row: torch.Tensor     # int32 [n_long]
    long_seg_ptr: torch.Tensor  # int32 [n_long + 1]
    small_row: torch.Tensor    # int32 [n_small]
    small_col: torch.Tensor    # int32 [n_small] (-1: no edge)
    small_val: torch.Tensor    # fp32  [n_small]
    mid_row: torch.Tensor      # int32 [n_mid]

    @property
    def n_seg(self) -> int:
        return int(self.seg_row.numel())

    @property
    def n_long(self) -> int:
        return int(self.long_row.numel())

    @property
    def n_small(self) -> int:
        return int(self.small_row.numel())

    @property
    def n_mid(self) -> int:
        return int(self.mid_row.numel())

    def row_list(self) -> torch.Tensor:
        """mid + small rows (every row that is not split into segments)."""
        if not hasattr(self, "_row_list"):
            self._row_list = torch.cat([self.mid_row, self.small_row]).contiguous()
        return self._row_list

    def gat_split(self, rowptr: torch.Tensor, max_deg: int):
        """(mid rows with deg > max_deg, short rows with deg <= max_deg), row order kept:
        the GAT launch's short-row class (lane-private softmax, several rows per wave).
        Cached per max_deg; no host round-trip beyond the two sizes."""
        cache = self.__dict__.setdefault("_gat_split", {})
        if max_deg not in cache:
            if max_deg < 2 or self.n_mid == 0:
                cache[max_deg] = (self.mid_row, self.mid_row[:0])
            else:
                r = self.mid_row.to(torch.int64)
                short = (rowptr[r + 1] - rowptr[r]) <= max_deg
                cache[max_deg] = (self.mid_row[~short].contiguous(),
                                  self.mid_row[short].contiguous())
        return cache[max_deg]

    def nonempty_small(self):
        """(small_row, small_col, small_val) without the edgeless rows (cached): an
        accumulate pass with no bias and no activation leaves those rows unchanged, so it
        need not read-modify-write them (the halo passes of the edge-cut SpMM, where most
        owned rows have no halo edge)."""
        if not hasattr(self, "_nonempty_small"):
            keep = self.small_col >= 0
            self._nonempty_small = (self.small_row[keep].contiguous(),
                                    self.small_col[keep].contiguous(),
                                    self.small_val[keep].contiguous())
        return self._nonempty_small

    def args(self, skip_empty: bool = False):
        """The plan arguments of gnn_spmm_csr_f32 / gnn_gat_csr_f32 (after seg_len);
        ``skip_empty`` drops the edgeless rows (see ``nonempty_small``)."""
        from ._lib import ptr
        small_row, small_col, small_val = (self.nonempty_small() if skip_empty else
                                           (self.small_row, self.small_col, self.small_val))
        return (ptr(self.seg_row), ptr(self.seg_begin), self.n_seg, ptr(self.long_row),
                self.long_seg_ptr.data_ptr(), self.n_long, ptr(small_row),
                ptr(small_col), ptr(small_val), int(small_row.numel()),
                # mid_row must be non-NULL whenever a plan is used (NULL = "no plan")
                self.mid_row.data_ptr() if self.n_mid else self.long_seg_ptr.data_ptr(),
                self.n_mid)


# Packed row tasks (gnn_spmm_csr_tasks_f32): runs of consecutive rows of degree <= TASK_MAX_DEG
# cut into tasks of at most TASK_ROWS rows and about TASK_COST (edges + rows) each; one
# wavefront streams a task's edges (its EPI edge slots take balanced sub-ranges of rows).
TASK_ROWS = 63  # spmm.hip kTaskRows: a task's rowptr values fit one VGPR


@dataclass
class TaskPlan:
    """Row classes for gnn_spmm_csr_tasks_f32: segments of long rows (as RowSplitPlan), mid
    rows (max_deg < degree <= seg_len, one wave each) and packed tasks (the other rows)."""

    seg_len: int
    base: RowSplitPlan         # seg_row / seg_begin / long_row / long_seg_ptr are used
    mid_row: torch.Tensor      # int32 [n_mid]
    task_row: torch.Tensor     # int32 [2 * n_task]: [begin, end) row ranges
    max_deg: int
    cost: int

    @property
    def n_task(self) -> int:
        return int(self.task_row.numel()) // 2

    @property
    def n_mid(self) -> int:
        return int(self.mid_row.numel())

    def args(self):
        """The plan arguments of gnn_spmm_csr_tasks_f32 after seg_len."""
        from ._lib import ptr
        b = self.base
        return (ptr(b.seg_row), ptr(b.seg_begin), b.n_seg, ptr(b.long_row),
                b.long_seg_ptr.data_ptr(), b.n_long,
                self.mid_row.data_ptr() if self.n_mid else b.long_seg_ptr.data_ptr(), self.n_mid,
                self.task_row.data_ptr() if self.n_task else None, self.n_task)


# The schedule builders run natively on the device (csrc/plan_build.hip: gnn_spmm_tasks_build,
# gnn_column_order, gnn_xcd_hub_plan_*), the same C-ABI a C caller uses; the torch versions
# below are the CPU path and the cross-check (tests/test_plan_build_gpu.py: equal arrays).
NATIVE_PLANS = True


def task_ranges(rowptr: torch.Tensor, max_deg: int, cost: int, rows: int = TASK_ROWS):
    """[2 * n_task] int32 [begin, end) row ranges: maximal runs of consecutive rows of degree
    <= max_deg, cut where the (edges + rows) prefix inside the run crosses a multiple of
    ``cost`` and every ``rows`` rows. On the device: gnn_spmm_tasks_build; else torch ops."""
    if NATIVE_PLANS and rowptr.is_cuda and rows == TASK_ROWS and cost >= 1:
        return task_ranges_native(rowptr, max_deg, cost)
    return task_ranges_torch(rowptr, max_deg, cost, rows)


def task_ranges_native(rowptr: torch.Tensor, max_deg: int, cost: int) -> torch.Tensor:
    """``task_ranges`` by gnn_spmm_tasks_build (one host sync for the count)."""
    n = rowptr.numel() - 1
    dev = rowptr.device
    if n <= 0:
        return torch.zeros(0, dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = torch.empty(int(lib.gnn_spmm_tasks_workspace_bytes(n)), dtype=torch.uint8, device=dev)
    out = torch.empty(2 * n, dtype=torch.int32, device=dev)
    nt = ctypes.c_int64(0)
    _lib.check(lib.gnn_spmm_tasks_build(rowptr.data_ptr(), n, int(max_deg), int(cost),
                                        out.data_ptr(), n, ctypes.addressof(nt), ws.data_ptr(),
                                        ws.numel(), _lib.stream_handle(dev)),
               "gnn_spmm_tasks_build")
    return out[:2 * nt.value].clone()


def task_ranges_torch(rowptr: torch.Tensor, max_deg: int, cost: int, rows: int = TASK_ROWS):
    """``task_ranges`` in torch ops (any device)."""
    dev = rowptr.device
    n = rowptr.numel() - 1
    if n == 0:
        return torch.zeros(0, dtype=torch.int32, device=dev)
    deg = rowptr[1:] - rowptr[:-1]
    pack = deg <= max_deg
    if not bool(pack.any()):
        return torch.zeros(0, dtype=torch.int32, device=dev)
    prev = torch.cat([torch.zeros(1, dtype=torch.bool, device=dev), pack[:-1]])
    run_start = pack & ~prev
    run_id = torch.cumsum(run_start.to(torch.int64), 0) - 1
    c = torch.where(pack, deg + 1, torch.zeros_like(deg))
    excl = torch.cumsum(c, 0) - c
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    first = idx[run_start]
    rid = run_id.clamp_(min=0)
    excl_in = excl - excl[first][rid]
    pos_in = idx - first[rid]
    bucket = excl_in // cost
    prev_bucket = torch.cat([bucket[:1] - 1, bucket[:-1]])
    start = pack & (run_start | (bucket != prev_bucket) | (pos_in % rows == 0))
    bounds = torch.nonzero(start | ~pack).view(-1)
    bounds = torch.cat([bounds, torch.full((1,), n, dtype=torch.int64, device=dev)])
    tb = torch.nonzero(start).view(-1)
    te = bounds[torch.searchsorted(bounds, tb, right=True)]
    return torch.stack([tb, te], 1).reshape(-1).to(torch.int32).contiguous()


def check_tasks(task_row: torch.Tensor, n_rows: int) -> None:
    """Raise if a task list breaks gnn_spmm_csr_tasks_f32's contract (1..63 rows inside
    [0, n_rows), ascending and disjoint): gnn_spmm_tasks_check on the device, one host read.
    The kernel skips such tasks, so a bad list would leave rows unwritten silently."""
    n_task = task_row.numel() // 2
    if n_task == 0 or not task_row.is_cuda:
        return
    err = torch.zeros(1, dtype=torch.int32, device=task_row.device)
    _lib.check(_lib.load().gnn_spmm_tasks_check(task_row.data_ptr(), n_task, n_rows,
                                                err.data_ptr(),
                                                _lib.stream_handle(task_row.device)),
               "gnn_spmm_tasks_check")
    e = int(err.item())
    if e:
        raise ValueError(f"packed row tasks break the kernel contract (gnn_spmm_tasks_check "
                         f"flags {e}: 1 = a task outside 1..{TASK_ROWS} rows in [0, {n_rows}), "
                         f"2 = overlapping / descending tasks)")


@dataclass
class HubPlan:
    """Hub staging of a graph's columns (gnn_spmm_csr_hub_f32): the k highest-degree
    columns, hottest first, and the column array with hub columns renamed -1-rank."""

    hub_ids: torch.Tensor   # int64 [k]
    col_hub: torch.Tensor   # int32 [nnz]
    err: torch.Tensor       # int32 [1] (gather index check flag)

    @property
    def k(self) -> int:
        return int(self.hub_ids.numel())

    @property
    def prefix(self) -> bool:
        """True when the hub rows are the first k rows in rank order (a graph relabelled by
        ``degree_order``): the staged table is then the operand itself, no copy needed."""
        v = self.__dict__.get("_prefix")
        if v is None:
            ids = self.hub_ids
            v = bool(torch.equal(ids, torch.arange(ids.numel(), device=ids.device,
                                                   dtype=ids.dtype)))
            self.__dict__["_prefix"] = v
        return v


# gfx950: 8 XCDs with one 4 MiB L2 each; the workgroups of a launch are dealt to them
# round-robin (workgroup w runs on XCD w % 8), and the SpMM kernel runs 4 waves per
# workgroup (spmm.hip kBlock = 256), one row per wave.
XCDS = 8
SPMM_WAVES_PER_WG = 4
# hub ranks per slice group of the XCD-sliced plan (xcd_hub_coo); plan_build.hip's
# GNN_XCD_SLICE_GROUP is the same constant for the device builder
XCD_SLICE_GROUP = 4


@dataclass
class XcdHubPlan:
    """XCD-sliced hub staging (built once per graph, hub count and row threshold).

    The staged hub ranks are dealt to the 8 XCDs ((rank // XCD_SLICE_GROUP) % 8). For every
    row of degree >= ``min_deg``, the hub edges that fall in one slice form an *item* (chunked
    to at most ``chunk`` edges). Pass 1 (``items``) reduces each item into one partial row;
    its rows are laid out so that workgroup w holds only items of slice w % 8, so each
    XCD's L2 serves 1/8 of the hub table. Pass 2 (``rest``) is every row's remaining
    edges followed by one edge of value 1.0 per partial row of that row.

    Both passes run the hub kernel (gnn_spmm_csr_hub_f32) over one staged buffer
    [hub table (k rows) | partial rows (n_pos rows)]: column c < 0 names its row -1-c.
    The row sums are regrouped (same terms, another order), so the result equals the
    unstaged kernel's to fp32 rounding, and is bitwise reproducible.
    """

    hub: HubPlan
    items: CsrGraph     # rows: item positions; cols: -1-rank (hub table rows)
    rest: CsrGraph      # rows: graph rows; cols: X rows, -1-rank, -1-(k + position)
    n_items: int        # real items (the other positions are 2-edge zero-valued pads)
    min_deg: int
    chunk: int
    item_row: torch.Tensor  # int64 [n_pos]: the graph row of each item position (pads: 0)

    @property
    def k(self) -> int:
        return self.hub.k

    @property
    def n_pos(self) -> int:
        return self.items.n_rows

    @property
    def prefix(self) -> bool:
        """True when the hub rows are X's first k rows in rank order (a graph relabelled by
        ``degree_order``): the staged table is then X itself and needs no copy."""
        return self.hub.prefix

    def direct(self) -> tuple["CsrGraph", "CsrGraph"]:
        """(items, rest) of a prefix plan with the hub references turned back into X row ids
        (-1-rank -> rank) and the partial refs renumbered -1-(k + pos) -> -1-pos: pass 1 reads
        X with the plain kernel, pass 2 reads X and a separate partial-row buffer (cached)."""
        d = self.__dict__.get("_direct")
        if d is None:
            k = self.k
            ic = (-1 - self.items.col.to(torch.int64)).to(torch.int32)
            items = CsrGraph(self.items.rowptr, ic.contiguous(), self.items.val,
                             self.items.n_rows, k)
            c = self.rest.col
            rc = torch.where(c >= 0, c, torch.where(c >= -k, -1 - c, c + k))
            rest = CsrGraph(self.rest.rowptr, rc.to(torch.int32).contiguous(), self.rest.val,
                            self.rest.n_rows, self.rest.n_cols)
            d = self.__dict__["_direct"] = (items, rest)
        return d

    def rest_plan(self, seg_len: int) -> RowSplitPlan:
        """The row-class plan of ``rest`` for the hub kernels (cached per seg_len).

        The packed small-row class reads its one pre-resolved column straight from X and
        treats a negative id as "no edge"; a one-edge row of ``rest`` whose edge is a hub
        or a partial row (negative id) therefore goes to the mid-row class instead, whose
        gather resolves negative ids through the staged buffer."""
        cache = self.__dict__.setdefault("_rest_plans", {})
        if seg_len not in cache:
            cache[seg_len] = staged_plan(self.rest, seg_len)
        return cache[seg_len]


def staged_plan(g: "CsrGraph", seg_len: int) -> RowSplitPlan:
    """The row-class plan of a graph whose negative column ids name rows of a staged table
    (the hub kernels' convention): one-edge rows whose edge is staged leave the packed
    small-row class (it reads its pre-resolved column from X and a negative id as "no
    edge") for the mid-row class, whose gather resolves negative ids."""
    p = g.plan(seg_len)
    rp = g.rowptr
    if p.n_small:
        r = p.small_row.to(torch.int64)
        staged = (p.small_col < 0) & ((rp[r + 1] - rp[r]) == 1)
        if bool(staged.any()):
            keep = ~staged
            p = RowSplitPlan(p.seg_len, p.seg_row, p.seg_begin, p.long_row,
                             p.long_seg_ptr, p.small_row[keep].contiguous(),
                             p.small_col[keep].contiguous(),
                             p.small_val[keep].contiguous(),
                             torch.cat([p.mid_row, p.small_row[staged]]).contiguous())
    return p


def xcd_hub_coo(rowptr: torch.Tensor, col_hub: torch.Tensor, val: torch.Tensor, k: int,
                min_deg: int, chunk: int, xcds: int = XCDS,
                waves_per_wg: int = SPMM_WAVES_PER_WG, phases: int = 1,
                item_k: int | None = None, small_item: int | None = None):
    """The two COO edge lists of ``XcdHubPlan`` (torch ops on any device; the CPU tests
    check them against the oracle SpMM).

    Returns ``None`` when no row has two hub edges in one slice, else
    ``((item_rows, item_cols, item_vals, n_pos, n_items), (rest_rows, rest_cols, rest_vals),
    pos_row)`` where ``pos_row[p]`` is the graph row of item position p (pads: 0).
    Item edges keep their CSR order; rest rows list their unmoved edges in CSR order,
    then their partial refs in (slice, chunk) order.

    Hub rank r belongs to slice (r // G) % S, S = xcds * phases, G = ``XCD_SLICE_GROUP``
    consecutive ranks (1 when fewer than S * G ranks may form items): G = 4 keeps 2 KiB of a
    slice's rows together in X at F = 128, 2.8 % faster at cfg2 than dealing single ranks
    (``profiles/r04sg_slice_group_ab.log``). ``phases`` > 1: the items of slice s run on XCD
    s % xcds in phase s // xcds, the phases one after another in the launch order, so each
    XCD's L2 holds 1 / (xcds * phases) of the table at a time.

    ``item_k`` < k limits the items to the item_k hottest hub rows (a smaller set per XCD
    slice); the edges to the other hub rows stay in ``rest`` and read the whole table.

    ``small_item`` (>= 2): rows below ``min_deg`` also get items, for the slices where they
    have at least ``small_item`` hub edges (a partial row pays off only when it replaces
    enough shared-table gathers)."""
    S = xcds * phases
    if chunk < 4 or k < S or phases < 1:  # balanced chunks of a >= 2-edge item hold >= 2 edges
        raise ValueError("xcd hub staging needs chunk >= 4 and k >= xcds * phases")
    dev = rowptr.device
    i64 = torch.int64
    n = rowptr.numel() - 1
    deg = rowptr[1:] - rowptr[:-1]
    rows_e = torch.repeat_interleave(torch.arange(n, device=dev, dtype=i64), deg)
    c = col_hub.to(i64)
    ik = k if item_k is None else min(int(item_k), k)
    if ik < S:
        raise ValueError("xcd hub staging needs item_k >= xcds * phases")
    if small_item is not None and small_item < 2:
        raise ValueError("small_item must be >= 2")
    if small_item is None:
        eid = torch.nonzero((c < 0) & (c >= -ik) & (deg[rows_e] >= min_deg)).view(-1)
    else:
        eid = torch.nonzero((c < 0) & (c >= -ik) & (deg[rows_e] >= 2)).view(-1)
    G = XCD_SLICE_GROUP if XCD_SLICE_GROUP > 1 and ik >= S * XCD_SLICE_GROUP else 1
    s_e = ((-1 - c[eid]) // G) % S
    key = rows_e[eid] * S + s_e
    order = torch.argsort(key, stable=True)                  # by (row, slice), CSR order kept
    eid, key, s_e = eid[order], key[order], s_e[order]
    _, inv, m = torch.unique_consecutive(key, return_inverse=True, return_counts=True)
    moved = m >= 2                                           # a 1-edge item saves nothing
    if small_item is not None:
        first = torch.cumsum(m, 0) - m                       # first edge of each group
        moved &= (deg[rows_e[eid[first]]] >= min_deg) | (m >= small_item)
    if not bool(moved.any()):
        return None
    em = moved[inv]
    eid, s_e, inv = eid[em], s_e[em], inv[em]
    grp = (torch.cumsum(moved.to(i64), 0) - 1)[inv]          # item group of each moved edge
    mg = m[moved]
    nch = (mg + chunk - 1) // chunk                          # balanced chunks of <= chunk edges
    pos_in = torch.arange(eid.numel(), device=dev, dtype=i64) - (torch.cumsum(mg, 0) - mg)[grp]
    item = (torch.cumsum(nch, 0) - nch)[grp] + pos_in * nch[grp] // mg[grp]
    n_items = int(nch.sum())
    it_slice = torch.empty(n_items, dtype=i64, device=dev)
    it_slice[item] = s_e
    it_row = torch.empty(n_items, dtype=i64, device=dev)
    it_row[item] = rows_e[eid]
    # position of an item: the j-th item of slice s (phase p = s // xcds) goes to workgroup
    # base[p] + (j // W) * xcds + s % xcds
    by_slice = torch.argsort(it_slice, stable=True)
    cnt = torch.bincount(it_slice, minlength=S)
    j = torch.empty(n_items, dtype=i64, device=dev)
    j[by_slice] = torch.arange(n_items, device=dev, dtype=i64) - (torch.cumsum(cnt, 0) - cnt)[
        it_slice[by_slice]]
    W = waves_per_wg
    per = [-(-int(v) // W) * W for v in cnt.view(phases, xcds).max(1).values.tolist()]
    base_l = [0]
    for v in per:
        base_l.append(base_l[-1] + v * xcds)                 # positions before each phase
    base = torch.tensor(base_l, dtype=i64, device=dev)
    pos = base[it_slice // xcds] + ((j // W) * xcds + it_slice % xcds) * W + j % W
    n_pos = base_l[-1]
    filled = torch.zeros(n_pos, dtype=torch.bool, device=dev)
    filled[pos] = True
    pad = torch.nonzero(~filled).view(-1)                    # 2 zero-valued edges of its slice
    pad_phase = torch.searchsorted(base, pad, right=True) - 1
    pad_col = -1 - (pad_phase * xcds + ((pad - base[pad_phase]) // W) % xcds) * G
    items = (torch.cat([pos[item], pad, pad]), torch.cat([c[eid], pad_col, pad_col]),
             torch.cat([val[eid], torch.zeros(2 * pad.numel(), dtype=val.dtype, device=dev)]),
             n_pos, n_items)
    keep = torch.ones(c.numel(), dtype=torch.bool, device=dev)
    keep[eid] = False
    kid = torch.nonzero(keep).view(-1)
    rest = (torch.cat([rows_e[kid], it_row]), torch.cat([c[kid], -1 - (k + pos)]),
            torch.cat([val[kid], torch.ones(n_items, dtype=val.dtype, device=dev)]))
    pos_row = torch.zeros(n_pos, dtype=i64, device=dev)
    pos_row[pos] = it_row
    return items, rest, pos_row


@dataclass
class CsrGraph:
    """Adjacency in CSR: row = output node, col = gathered node (torch.spmm orientation)."""

    rowptr: torch.Tensor  # int64 [n_rows + 1]
    col: torch.Tensor     # int32 [nnz]
    val: torch.Tensor     # fp32 [nnz]
    n_rows: int
    n_cols: int
    _plans: dict = field(default_factory=dict, repr=False)
    _transpose: "CsrGraph | None" = field(default=None, repr=False)
    # A == A^T (structure, and values to fp32 rounding): the SpMM backward's dX = A^T dY then
    # runs over A itself, with A's cached plans and no transposed copy. Set by the GCN
    # adjacency builders (D^-1/2 (A_sym + I) D^-1/2 is symmetric), or found by ``transpose``.
    symmetric: bool = False

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def has_empty_rows(self) -> bool:
        """Whether some row has no edge (one device reduction, cached)."""
        v = self._plans.get("_has_empty")
        if v is None:
            v = bool(((self.rowptr[1:] - self.rowptr[:-1]) == 0).any())
            self._plans["_has_empty"] = v
        return v

    def validate(self) -> None:
        assert self.rowptr.dtype == torch.int64 and self.rowptr.numel() == self.n_rows + 1
        assert self.col.dtype == torch.int32 and self.val.dtype == torch.float32
        assert self.col.numel() == self.val.numel()
        assert self.rowptr.is_contiguous() and self.col.is_contiguous() and self.val.is_contiguous()

    # ------------------------------------------------------------------ plans
    def plan(self, seg_len: int) -> RowSplitPlan:
        """Row-split plan for this graph (device-built once per seg_len, then cached)."""
        p = self._plans.get(seg_len)
        if p is None:
            p = _build_plan(self, seg_len)
            self._plans[seg_len] = p
        return p

    def task_plan(self, seg_len: int, max_deg: int, cost: int) -> TaskPlan:
        """Packed-task plan (built once per (seg_len, max_deg, cost), cached)."""
        key = ("_tasks", seg_len, max_deg, cost)
        p = self._plans.get(key)
        if p is None:
            base = self.plan(seg_len)
            deg = self.rowptr[1:] - self.rowptr[:-1]
            mid = torch.nonzero((deg > max_deg) & (deg <= base.seg_len)).view(-1)
            tasks = task_ranges(self.rowptr, min(max_deg, base.seg_len), cost)
            check_tasks(tasks, self.n_rows)
            p = TaskPlan(base.seg_len, base, mid.to(torch.int32).contiguous(), tasks, max_deg,
                         cost)
            self._plans[key] = p
        return p

    def hub_plan(self, k: int) -> HubPlan:
        """Hub staging plan for the k highest-degree columns (built once per k, cached)."""
        key = ("_hub", k)
        p = self._plans.get(key)
        if p is None:
            p = _build_hub_plan(self, k)
            self._plans[key] = p
        return p

    def xcd_hub_plan(self, k: int, min_deg: int, chunk: int, phases: int = 1,
                     item_k: int | None = None,
                     small_item: int | None = None) -> "XcdHubPlan | None":
        """XCD-sliced hub staging plan (built once per (k, min_deg, chunk, phases, item_k,
        small_item), cached); None when no row has two hub edges in one slice."""
        key = ("_xcd", k, min_deg, chunk, phases, item_k, small_item)
        if key not in self._plans:
            self._plans[key] = _build_xcd_hub_plan(self, k, min_deg, chunk, phases, item_k,
                                                   small_item)
        return self._plans[key]

    def transpose(self) -> "CsrGraph":
        """CSR of A^T (used by the SpMM backward: dX = A^T dY). A symmetric graph is its own
        transpose (no copy, its plans reused); a graph not marked symmetric whose transpose
        turns out equal to it (same structure, values within one fp32 rounding: the
        reference's scipy normalisation rounds v_ij and v_ji separately) is marked so and the
        copy dropped."""
        if self.symmetric:
            return self
        if self._transpose is None:
            rows = torch.repeat_interleave(
                torch.arange(self.n_rows, device=self.device, dtype=torch.int64),
                self.rowptr[1:] - self.rowptr[:-1])
            t = from_coo(self.col.to(torch.int64), rows, self.val, self.n_cols, self.n_rows)
            if (self.n_rows == self.n_cols and torch.equal(t.rowptr, self.rowptr)
                    and torch.equal(t.col, self.col)
                    and torch.allclose(t.val, self.val, rtol=2.0 ** -23, atol=0.0)):
                self.symmetric = True
                return self
            self._transpose = t
        return self._transpose

    def transpose_eid(self):
        """(rowptr_t, src_t int32, eid_t int64, plan-able CsrGraph of A^T) -- the GAT
        backward's column view: for node j, the CSR edges (i, j) and their ids."""
        t = self._plans.get("_transpose_eid")
        if t is None:
            rows = torch.repeat_interleave(
                torch.arange(self.n_rows, device=self.device, dtype=torch.int64),
                self.rowptr[1:] - self.rowptr[:-1])
            eid = torch.argsort(self.col.to(torch.int64), stable=True)
            rowptr_t = torch.zeros(self.n_cols + 1, dtype=torch.int64, device=self.device)
            torch.cumsum(torch.bincount(self.col.to(torch.int64), minlength=self.n_cols), 0,
                         out=rowptr_t[1:])
            src_t = rows[eid].to(torch.int32).contiguous()
            gt = CsrGraph(rowptr_t, src_t, torch.ones(src_t.numel(), device=self.device),
                          self.n_cols, self.n_rows)
            t = (rowptr_t, src_t, eid.contiguous(), gt)
            self._plans["_transpose_eid"] = t
        return t

    def to(self, device) -> "CsrGraph":
        return CsrGraph(self.rowptr.to(device), self.col.to(device), self.val.to(device),
                        self.n_rows, self.n_cols, symmetric=self.symmetric)


def _build_plan(g: CsrGraph, seg_len: int) -> RowSplitPlan:
    lib = _lib.load()
    dev = g.device
    stream = _lib.stream_handle(dev)
    nbytes = int(lib.gnn_spmm_plan_scratch_bytes(g.n_rows))
    scratch = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=dev)
    counts = torch.zeros(4, dtype=torch.int64, device=dev)
    _lib.check(lib.gnn_spmm_plan_count(g.rowptr.data_ptr(), g.n_rows, seg_len, counts.data_ptr(),
                                       scratch.data_ptr(), stream), "gnn_spmm_plan_count")
    # one host round-trip per graph
    n_long, n_seg, n_small, n_mid = (int(v) for v in counts.cpu().tolist())
    i32 = dict(dtype=torch.int32, device=dev)
    seg_row = torch.empty(n_seg, **i32)
    seg_begin = torch.empty(n_seg, dtype=torch.int64, device=dev)
    long_row = torch.empty(n_long, **i32)
    long_seg_ptr = torch.empty(n_long + 1, **i32)
    small_row = torch.empty(n_small, **i32)
    small_col = torch.empty(n_small, **i32)
    small_val = torch.empty(n_small, dtype=torch.float32, device=dev)
    mid_row = torch.empty(n_mid, **i32)
    col = g.col if g.nnz else torch.zeros(1, **i32)
    val = g.val if g.nnz else torch.zeros(1, dtype=torch.float32, device=dev)
    _lib.check(lib.gnn_spmm_plan_fill(g.rowptr.data_ptr(), col.data_ptr(), val.data_ptr(),
                                      g.n_rows, seg_len, _lib.ptr(seg_row), _lib.ptr(seg_begin),
                                      _lib.ptr(long_row), long_seg_ptr.data_ptr(),
                                      _lib.ptr(small_row), _lib.ptr(small_col),
                                      _lib.ptr(small_val), _lib.ptr(mid_row), scratch.data_ptr(),
                                      stream), "gnn_spmm_plan_fill")
    return RowSplitPlan(seg_len, seg_row, seg_begin, long_row, long_seg_ptr, small_row,
                        small_col, small_val, mid_row)


def _build_hub_plan(g: CsrGraph, k: int) -> HubPlan:
    """The k hottest columns (in-degree descending, ties by ascending id) and the renamed
    column array, built on the device by gnn_hub_plan_build (hub.hip)."""
    lib = _lib.load()
    dev = g.device
    k = max(1, min(int(k), g.n_cols))
    hub_ids = torch.empty(k, dtype=torch.int64, device=dev)
    col_hub = torch.empty_like(g.col)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(int(lib.gnn_hub_plan_workspace_bytes(g.n_cols)), dtype=torch.uint8,
                     device=dev)
    _lib.check(lib.gnn_hub_plan_build(_lib.ptr(g.col), g.nnz, g.n_cols, k, hub_ids.data_ptr(),
                                      _lib.ptr(col_hub), err.data_ptr(), ws.data_ptr(),
                                      ws.numel(), _lib.stream_handle(dev)), "gnn_hub_plan_build")
    return HubPlan(hub_ids, col_hub, err)


def _build_xcd_hub_plan(g: CsrGraph, k: int, min_deg: int, chunk: int, phases: int = 1,
                        item_k: int | None = None,
                        small_item: int | None = None) -> "XcdHubPlan | None":
    hub = g.hub_plan(k)
    if hub.k < XCDS * phases or g.nnz == 0:
        return None
    if item_k is not None and min(int(item_k), hub.k) < XCDS * phases:
        return None
    # the device builder's slice group is a compile-time constant: it runs only when it is the
    # one asked for here (a monkeypatched / edited XCD_SLICE_GROUP takes the torch builder,
    # which reads it at run time)
    if NATIVE_PLANS and g.rowptr.is_cuda and \
            int(_lib.load().gnn_xcd_slice_group()) == XCD_SLICE_GROUP:
        return _build_xcd_hub_plan_native(g, hub, min_deg, chunk, phases, item_k, small_item)
    coo = xcd_hub_coo(g.rowptr, hub.col_hub, g.val, hub.k, min_deg, chunk, phases=phases,
                      item_k=item_k, small_item=small_item)
    if coo is None:
        return None
    (ir, ic, iv, n_pos, n_items), (rr, rc, rv), pos_row = coo
    if hub.k + n_pos > 0x7fffffff:
        return None  # partial refs must fit int32 column ids
    items = from_coo(ir, ic, iv, n_pos, hub.k, check=False)
    rest = from_coo(rr, rc, rv, g.n_rows, g.n_cols, check=False)
    return XcdHubPlan(hub, items, rest, n_items, min_deg, chunk, pos_row)


def _build_xcd_hub_plan_native(g: CsrGraph, hub: HubPlan, min_deg: int, chunk: int,
                               phases: int, item_k: int | None,
                               small_item: int | None) -> "XcdHubPlan | None":
    """``_build_xcd_hub_plan`` by gnn_xcd_hub_plan_build / _fill (the same CSR arrays)."""
    if chunk < 4:
        raise ValueError("xcd hub staging needs chunk >= 4 and k >= xcds * phases")
    if small_item is not None and small_item < 2:
        raise ValueError("small_item must be >= 2")
    lib = _lib.load()
    dev = g.device
    stream = _lib.stream_handle(dev)
    ws = torch.empty(int(lib.gnn_xcd_hub_plan_workspace_bytes(g.n_rows, g.nnz)),
                     dtype=torch.uint8, device=dev)
    counts = (ctypes.c_int64 * 4)()
    _lib.check(lib.gnn_xcd_hub_plan_build(g.rowptr.data_ptr(), hub.col_hub.data_ptr(), g.n_rows,
                                          g.nnz, hub.k, int(min_deg), int(chunk), int(phases),
                                          0 if item_k is None else int(item_k),
                                          0 if small_item is None else int(small_item),
                                          ctypes.addressof(counts), ws.data_ptr(), ws.numel(),
                                          stream), "gnn_xcd_hub_plan_build")
    n_items, n_pos, nnz_items, nnz_rest = (int(v) for v in counts)
    if n_items == 0 or hub.k + n_pos > 0x7fffffff:
        return None
    i64, i32, f32 = (dict(dtype=t, device=dev) for t in (torch.int64, torch.int32, torch.float32))
    irp = torch.empty(n_pos + 1, **i64)
    icol = torch.empty(nnz_items, **i32)
    ival = torch.empty(nnz_items, **f32)
    pos_row = torch.empty(n_pos, **i64)
    rrp = torch.empty(g.n_rows + 1, **i64)
    rcol = torch.empty(nnz_rest, **i32)
    rval = torch.empty(nnz_rest, **f32)
    _lib.check(lib.gnn_xcd_hub_plan_fill(ws.data_ptr(), g.rowptr.data_ptr(),
                                         hub.col_hub.data_ptr(), g.val.data_ptr(), g.n_rows, g.nnz,
                                         hub.k, int(phases), ctypes.addressof(counts),
                                         irp.data_ptr(), icol.data_ptr(), ival.data_ptr(),
                                         pos_row.data_ptr(), rrp.data_ptr(), rcol.data_ptr(),
                                         rval.data_ptr(), stream), "gnn_xcd_hub_plan_fill")
    items = CsrGraph(irp, icol, ival, n_pos, hub.k)
    rest = CsrGraph(rrp, rcol, rval, g.n_rows, g.n_cols)
    return XcdHubPlan(hub, items, rest, n_items, min_deg, chunk, pos_row)


@dataclass
class DegreeOrder:
    """A relabelling of a square graph's nodes by in-degree (descending, ties by ascending
    id): new id i is old node ``perm[i]``; ``inv[old]`` is its new id. Under it the hub rows
    that the staging would copy (the same ranking as hub.hip) are the first rows of X, so
    the SpMM reads them in place (``XcdHubPlan.direct``)."""

    perm: torch.Tensor  # int64 [n]: new -> old
    inv: torch.Tensor   # int64 [n]: old -> new
    graph: "CsrGraph"   # P A P^T, or A P^T (degree_order(rows=False))

    def permute_rows(self, x: torch.Tensor) -> torch.Tensor:
        """X' = P X (rows in the new order)."""
        return x.index_select(0, self.perm)

    def unpermute_rows(self, y: torch.Tensor) -> torch.Tensor:
        """Y = P^T Y' (rows back in the original order)."""
        return y.index_select(0, self.inv)


def in_degree(g: "CsrGraph") -> torch.Tensor:
    """int64 [n_cols] column in-degrees. On the device: gnn_in_degree_u32 (LDS-privatised
    counts for the hot ids; torch.bincount serialises on the hub columns: 26 ms at the north
    star, profiles/r04d_sample_kernel_stats.csv); on the CPU: torch.bincount."""
    n = g.n_cols
    if not g.col.is_cuda or g.nnz == 0 or n == 0:
        return torch.bincount(g.col.to(torch.int64), minlength=n)
    deg = torch.empty(n, dtype=torch.int32, device=g.device)
    err = torch.zeros(1, dtype=torch.int32, device=g.device)
    _lib.check(_lib.load().gnn_in_degree_u32(g.col.data_ptr(), g.nnz, n, deg.data_ptr(),
                                             err.data_ptr(), _lib.stream_handle(g.device)),
               "gnn_in_degree_u32")
    # a column id outside [0, n_cols) is not counted by the kernel; torch.bincount would raise
    # (negative) or return a longer vector, so it is an error here too
    if int(err.item()) != 0:
        raise ValueError(f"column ids outside [0, {n}) in the graph (in_degree)")
    # uint32 counts < 2^31 here (nnz < 2^31 per column): the int32 view is exact
    return deg.to(torch.int64)


def degree_order(g: "CsrGraph", rows: bool = True, prefix: int | None = None,
                 tail: str | None = None) -> DegreeOrder:
    """Relabel a CSR graph by column in-degree (gnn_column_order on the device, torch ops on
    the CPU; tail "first_use" in torch ops everywhere). The edges of each
    row keep their CSR order (renamed), so every row sum runs in the same order: the result
    is bit-identical to the original graph's, permuted.

    ``rows=True`` (square graphs): both sides, A' = P A P^T, for Y' = A' X' = P Y.
    ``rows=False``: the columns only, A' = A P^T, for Y = A' (P X) -- the output rows stay
    in the original order.
    ``prefix``: only the ``prefix`` highest-degree ids are ranked (first, by degree); the rest
    follow in their original id order, so a producer that writes its rows in the new order
    (a transform or projection with scattered output rows) stores all but the prefix rows in
    ascending address order. The hub ranking of any K <= prefix is the full order's.
    ``tail`` (with ``prefix``): the order of the ids after the prefix -- "degree" (the full
    degree order), "id" (ascending ids, the default when only ``prefix`` is given) or
    "first_use" (by the CSR position of their first edge: the rows a row-ordered SpMM touches
    for the first time lie together in memory; columns without edges last)."""
    n = g.n_cols
    dev = g.device
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    if tail not in (None, "id", "degree", "first_use"):
        raise ValueError(f"unknown tail order {tail!r}")
    col_new = None
    if NATIVE_PLANS and g.col.is_cuda and n > 0 and tail != "first_use":
        ranked = prefix if (prefix is not None and prefix < n and tail != "degree") else -1
        perm, inv, col_new = column_order_native(g, ranked)
    else:
        perm, inv = _degree_perm_torch(g, prefix, tail)
    if not rows:
        col = col_new if col_new is not None else inv[g.col.to(torch.int64)].to(torch.int32)
        return DegreeOrder(perm, inv, CsrGraph(g.rowptr, col.contiguous(), g.val, g.n_rows, n))
    if g.n_rows != g.n_cols:
        raise ValueError("degree_order(rows=True) needs a square adjacency")
    deg = g.rowptr[1:] - g.rowptr[:-1]
    new_deg = deg[perm]
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(new_deg, 0, out=rowptr[1:])
    # edge e of new row i is edge (rowptr_old[perm[i]] + j) of the old graph
    rows_new = torch.repeat_interleave(idx, new_deg)
    src = g.rowptr[perm][rows_new] + (torch.arange(rows_new.numel(), device=dev,
                                                   dtype=torch.int64) - rowptr[rows_new])
    if col_new is not None:
        col = col_new[src].contiguous()
    else:
        col = inv[g.col.to(torch.int64)[src]].to(torch.int32).contiguous()
    val = g.val[src].contiguous()
    return DegreeOrder(perm, inv, CsrGraph(rowptr, col, val, n, n))


def column_order_native(g: "CsrGraph", prefix: int = -1):
    """(perm, inv, renamed int32 columns) of ``degree_order`` by gnn_column_order
    (``prefix`` < 0: every id ranked)."""
    n = g.n_cols
    dev = g.device
    lib = _lib.load()
    ws = torch.empty(int(lib.gnn_column_order_workspace_bytes(n)), dtype=torch.uint8, device=dev)
    perm = torch.empty(n, dtype=torch.int64, device=dev)
    inv = torch.empty(n, dtype=torch.int64, device=dev)
    col = torch.empty_like(g.col)
    _lib.check(lib.gnn_column_order(_lib.ptr(g.col), g.nnz, n, int(prefix), perm.data_ptr(),
                                    inv.data_ptr(), _lib.ptr(col), ws.data_ptr(), ws.numel(),
                                    _lib.stream_handle(dev)), "gnn_column_order")
    return perm, inv, col


def _degree_perm_torch(g: "CsrGraph", prefix: int | None, tail: str | None):
    """(perm, inv) of ``degree_order`` in torch ops (any device)."""
    n = g.n_cols
    dev = g.device
    indeg = in_degree(g)
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    # descending in-degree, ascending id on ties: one stable sort of -indeg
    perm = torch.sort(-indeg, stable=True).indices
    if prefix is not None and prefix < n:
        rest = perm[prefix:]
        if tail == "first_use":
            nnz = g.col.numel()
            first = torch.full((n,), nnz, dtype=torch.int64, device=dev)
            first.scatter_reduce_(0, g.col.to(torch.int64),
                                  torch.arange(nnz, device=dev, dtype=torch.int64), "amin")
            rest = rest[torch.sort(first[rest], stable=True).indices]
        elif tail in (None, "id"):
            rest = torch.sort(rest).values
        elif tail != "degree":
            raise ValueError(f"unknown tail order {tail!r}")
        perm = torch.cat([perm[:prefix], rest])
    inv = torch.empty_like(perm)
    inv[perm] = idx
    return perm, inv


# ---------------------------------------------------------------- builders
def from_coo(row: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n_rows: int,
             n_cols: int, check: bool = True) -> CsrGraph:
    """CSR from COO triplets (any order, duplicates kept), rows stably sorted.

    ``check=False`` skips the (host-syncing) index range check for indices the
    caller has already validated."""
    row = row.to(torch.int64)
    if check and row.numel() and (int(row.min()) < 0 or int(row.max()) >= n_rows
                        or int(col.min()) < 0 or int(col.max()) >= n_cols):
        raise IndexError("COO index out of range for the adjacency shape")
    order = torch.argsort(row, stable=True)
    counts = torch.bincount(row, minlength=n_rows)
    rowptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=row.device)
    torch.cumsum(counts, 0, out=rowptr[1:])
    g = CsrGraph(rowptr, col[order].to(torch.int32).contiguous(),
                 val[order].to(torch.float32).contiguous(), n_rows, n_cols)
    return g


def from_dense(adj: torch.Tensor, predicate: str) -> CsrGraph:
    """CSR of a dense [N, M] adjacency; edges where ``adj > 0`` ('positive') or ``adj != 0`` ('nonzero')."""
    if predicate == "positive":
        mask = adj > 0
    elif predicate == "nonzero":
        mask = adj != 0
    else:
        raise ValueError(predicate)
    idx = mask.nonzero()  # row-major order
    return from_coo(idx[:, 0], idx[:, 1], adj[mask], adj.shape[0], adj.shape[1])


def _edge_mask(val: torch.Tensor, predicate: str):
    if predicate == "all":
        return None
    if predicate == "positive":
        return val > 0
    if predicate == "nonzero":
        return val != 0
    raise ValueError(predicate)


def from_torch_sparse(adj: torch.Tensor, predicate: str = "all") -> CsrGraph:
    """CSR of a torch sparse COO/CSR tensor; ``predicate`` filters stored entries
    ('all' keeps every stored entry, as torch.spmm uses them)."""
    if adj.layout == torch.sparse_coo:
        if predicate != "all":  # edge-set semantics (GAT): one edge per (i, j)
            adj = adj.coalesce()
        idx = adj._indices()
        row, col, val = idx[0], idx[1], adj._values()
    elif adj.layout == torch.sparse_csr:
        crow = adj.crow_indices().to(torch.int64)
        val = adj.values()
        mask = _edge_mask(val, predicate)
        if mask is None:
            return CsrGraph(crow.contiguous(), adj.col_indices().to(torch.int32).contiguous(),
                            val.to(torch.float32).contiguous(), adj.shape[0], adj.shape[1])
        row = torch.repeat_interleave(torch.arange(adj.shape[0], device=crow.device),
                                      crow[1:] - crow[:-1])
        col = adj.col_indices()
    else:
        raise TypeError(f"unsupported sparse layout {adj.layout}")
    mask = _edge_mask(val, predicate)
    if mask is not None:
        row, col, val = row[mask], col[mask], val[mask]
    return from_coo(row, col, val, adj.shape[0], adj.shape[1])


def as_csr(adj, predicate: str = "all") -> CsrGraph:
    """The CsrGraph of a reference adjacency (cached on the tensor object).

    predicate: which entries are edges -- 'all' (every stored entry of a sparse
    tensor / every nonzero of a dense one: torch.spmm semantics), 'positive'
    (adj > 0: dense GAT layer), 'nonzero' (adj != 0: sparse GAT layer).
    """
    if isinstance(adj, CsrGraph):
        return adj
    if not isinstance(adj, torch.Tensor) or adj.dim() != 2:
        raise TypeError("adj must be a 2-D torch tensor (dense, sparse COO or sparse CSR) or a CsrGraph")
    key = (predicate, adj._version, adj.device)
    cache = getattr(adj, "_gnn_csr_cache", None)
    if cache is not None and key in cache:
        return cache[key]
    if adj.layout == torch.strided:
        g = from_dense(adj, "nonzero" if predicate == "all" else predicate)
    else:
        g = from_torch_sparse(adj, predicate)
    if cache is None:
        cache = {}
        try:
            adj._gnn_csr_cache = cache
        except (AttributeError, RuntimeError):
            return g
    cache[key] = g
    return g
