"""Vertex-range sharded MaxK aggregation over torch.distributed.

One process per GPU (RCCL over xGMI on MI355X; gloo in the CPU tests).  The
graph is cut into contiguous row ranges balanced by nnz; rank p owns rows
[bounds[p], bounds[p+1]) of A, their CSR slice, and the CBSR (top-k) rows of
those vertices.  There is no reference counterpart (the reference is
single-GPU); the oracle for this path is "identical to the
1-GPU result".

Two exchange modes, the same result ("auto" picks halo when every shard's halo is at most
HALO_SHARE of the vertices, else gather):
  "gather" (default)  forward: one all-gather of every vertex's CBSR row (k f32 +
            k u8); backward: the local push into a CBSR-shaped gradient for ALL
            vertices, then a reduce-scatter that sums the partials on the owners.
            Vertex ids are remapped once to a padded space (owner * vmax + local
            row), so both collectives are plain equal-size calls.
  "halo"    only the rows a shard's edges touch travel: once per graph each rank
            sends every owner the sorted list of the owner's vertices it needs
            (all-to-allv), which becomes the owner's send plan.  Forward: one
            all-to-allv of the needed CBSR rows into a compact column space (the
            shard's halo, in global-id order); backward: the local push into that
            compact space, one all-to-allv back to the owners, and each owner adds
            what it receives into its rows (index_add).  Bytes per step and rank:
            halo rows x k x 5 each way instead of (world-1)/world x V x k x 5
            (exchange_bytes()).  On graphs without locality (the randomly
            labelled synthetic ones) a shard's halo is nearly every vertex.

`kernels` is the compute backend: by default the HIP library through
maxk_cuda_kernels; the CPU tests inject an object with the same two methods
backed by the oracle.
"""
from __future__ import annotations

from typing import List, Optional

import os

import torch
import torch.distributed as dist
from torch.autograd import Function


def _staged(group) -> bool:
    """gloo has no device collectives for these calls: stage through host memory (the CPU
    tests, and rehearsing N ranks on a one-GPU box).  RCCL ("nccl") runs them on device."""
    return dist.get_backend(group) == "gloo"


def all_gather_rows(out: torch.Tensor, inp: torch.Tensor, group=None, async_op=False):
    """out[p * n:(p + 1) * n] = inp of rank p (equal n on every rank).  async_op (RCCL): the
    call is queued on the communicator's stream and its work handle returned; wait() on it
    makes the current stream wait (the host does not block).  Staged (gloo) calls complete
    before returning (None)."""
    if _staged(group) and inp.is_cuda:
        tmp = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(tmp, inp.cpu(), group=group)
        out.copy_(tmp)
        return None
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def reduce_scatter_rows(out: torch.Tensor, inp: torch.Tensor, group=None, async_op=False):
    """out = sum over ranks of inp[rank * n:(rank + 1) * n]; async_op as all_gather_rows."""
    if _staged(group) and inp.is_cuda:
        tmp = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(tmp, inp.cpu(), group=group)
        out.copy_(tmp)
        return None
    return dist.reduce_scatter_tensor(out, inp, group=group, async_op=async_op)


def _wait(work) -> None:
    if work is not None:
        work.wait()


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    """all_to_all_single along dim 0 (None splits: equal); gloo is staged through host."""
    if _staged(group) and inp.is_cuda:
        tmp = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(tmp, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(tmp)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _all_reduce_max(t: torch.Tensor, group=None) -> None:
    if _staged(group) and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)


def balanced_bounds(row_ptr: torch.Tensor, world: int) -> List[int]:
    """Row boundaries [0 = b0 <= b1 <= ... <= b_world = V] with ~E/world edges per shard."""
    rp = row_ptr.detach().to("cpu", torch.int64)
    V = rp.numel() - 1
    E = int(rp[-1])
    targets = torch.arange(world + 1, dtype=torch.int64) * E // world
    b = torch.searchsorted(rp, targets).tolist()
    b[0], b[-1] = 0, V
    for i in range(1, world + 1):  # monotone, inside [0, V]
        b[i] = min(max(b[i], b[i - 1]), V)
    return b


class _HipKernels:
    def __init__(self, bwd_mode=None):
        import maxk_cuda_kernels as mk
        self.mk = mk
        self.bwd_mode = bwd_mode  # None: "auto" per shard (or pipeline part)

    def spgemm_forward(self, indptr, indices, values, cbsr_val, cbsr_idx, D, row_div=None,
                       out=None, accumulate=False, edge_sel_out=None):
        return self.mk.spgemm_forward(indptr, indices, values, cbsr_val, cbsr_idx, D,
                                      row_div=row_div, out=out, accumulate=accumulate,
                                      edge_sel_out=edge_sel_out)

    def sspmm_backward(self, indptr, indices, values, grad, cbsr_idx, row_div=None, plan=None,
                       edge_sel=None):
        return self.mk.sspmm_backward(indptr, indices, values, grad, cbsr_idx, row_div=row_div,
                                      plan=plan, mode=self.bwd_mode, edge_sel=edge_sel)

    # the transport-record forward (ShardedMaxK._records / _aggregate_records)
    def records_ok(self, num_rows, num_cols, num_e, dim, k):
        return self.mk.records_ok(num_rows, num_cols, num_e, dim, k)

    def cbsr_records(self, cbsr_val, cbsr_idx, dim):
        return self.mk.cbsr_records(cbsr_val, cbsr_idx, dim)

    def spgemm_forward_records(self, indptr, indices, values, rec, k, D, row_div=None, out=None,
                               accumulate=False):
        return self.mk.spgemm_forward_records(indptr, indices, values, rec, k, D,
                                              row_div=row_div, out=out, accumulate=accumulate)

    def stream_mode(self, indptr, indices, k, num_cols, num_rows=None, dim=None):
        """Whether a (part's) forward should write the edge-selector stream for its backward:
        the backward this graph resolves to reads one ("csc" / "bsort") and
        edge_selectors_wanted(k); maxk_cuda_kernels.edge_selector_mode with this backend's
        mode."""
        if indices.numel() == 0 or not self.mk.edge_selectors_wanted(k):
            return False
        mode = self.mk._bwd_mode(self.bwd_mode, k, indices.numel(), num_cols, num_rows, dim,
                                 (indptr, indices))
        return mode in ("csc", "bsort")

    def backward_plan(self, indptr, indices, values, num_cols, k, num_rows=None, dim=None):
        return self.mk.backward_plan(indices, num_cols, k, mode=self.bwd_mode, num_rows=num_rows,
                                     indptr=indptr, values=values, dim=dim)


class ShardedMaxK:
    """Rank-local view of a vertex-partitioned graph for the MaxK aggregation.

    k (optional): the CBSR width the shard will carry; with it, "gather" mode pipelines only
    an exchange of at least PIPELINE_MIN_BYTES per rank and step (without it: PIPELINE parts
    at world > 1, as before).

    mode "gather": column space = padded [world * vmax] (all vertices);
    mode "halo":   column space = this shard's halo (the distinct columns of its edges, in
                   global-id order).  n_cols is its size either way."""

    MODES = ("gather", "halo", "auto")
    # "gather" mode, world > 1: the exchange runs in PIPELINE column parts (each owner's rows
    # cut into PIPELINE equal ranges, one sub-CSR per range): the forward adds part j's
    # product while part j+1's all-gather is in flight, and the backward's reduce-scatter of
    # part j runs beside part j+1's backward
    PIPELINE = 2
    # mode "auto": halo when every shard's halo is at most this share of the vertices (an
    # ordered graph's shards need a fraction of the others' rows: the exchange shrinks and
    # the per-column work -- record pack, selector ordering, tile reduce, phase-2 walk --
    # covers the halo only); gather otherwise (a randomly labelled graph's halo is nearly
    # every vertex, and one all-gather / reduce-scatter beats all-to-allv of the same bytes)
    HALO_SHARE = 0.6
    # the pipeline pays only where the exchange is large enough to hide: each part adds two
    # all-gathers and a reduce-scatter, and a collective costs tens of microseconds however
    # small.  With the width k known at construction, a shard whose whole-step exchange (CBSR
    # rows received, k f32 + k u8 each) is below this stays in one part -- Reddit-sized at
    # N = 8 moves ~16 MB per rank and step (one all-gather and one reduce-scatter instead of
    # six collectives), ogbn-products-sized ~390 MB (pipelined)
    PIPELINE_MIN_BYTES = 64 << 20

    def __init__(self, row_ptr: torch.Tensor, col_idx: torch.Tensor, values: torch.Tensor,
                 rank: int, world: int, group=None, device=None, kernels=None,
                 bounds: Optional[List[int]] = None, mode: str = "gather",
                 pipeline: Optional[int] = None, k: Optional[int] = None):
        if mode not in self.MODES:
            raise ValueError(f"mode must be one of {self.MODES}, got {mode!r}")
        self.rank, self.world, self.group = rank, world, group
        self.device = torch.device(device) if device is not None else row_ptr.device
        self.kernels = kernels if kernels is not None else _HipKernels()
        self.bounds = bounds if bounds is not None else balanced_bounds(row_ptr, world)
        b = self.bounds
        self.V = b[-1]
        self.v0, self.v1 = b[rank], b[rank + 1]
        self.n_local = self.v1 - self.v0
        self.vmax = max(max(b[i + 1] - b[i] for i in range(world)), 1)
        rp = row_ptr.to(self.device, torch.int64)
        e0, e1 = int(rp[self.v0]), int(rp[self.v1])
        self.row_ptr = (rp[self.v0:self.v1 + 1] - e0).to(torch.int32).contiguous()
        cols = col_idx[e0:e1].to(self.device, torch.int64)
        starts = torch.tensor(b, dtype=torch.int64, device=self.device)
        if mode == "auto":  # every rank must pick the same collectives: decide on the max
            share = torch.tensor([torch.unique(cols).numel() / max(1, self.V)],
                                 dtype=torch.float64, device=self.device)
            _all_reduce_max(share, group)
            self.halo_share = float(share.item())
            mode = "halo" if self.halo_share <= self.HALO_SHARE else "gather"
        self.mode = mode
        if mode == "gather":
            owner = torch.searchsorted(starts[1:], cols, right=True)
            loc = cols - starts[owner]
            self.col_idx = (owner * self.vmax + loc).to(torch.int32).contiguous()
            self.n_cols = world * self.vmax
        else:
            self._halo_plan(cols, starts)
        self.values = values[e0:e1].to(self.device, torch.float32).contiguous()
        self._plans = {}
        # default: pipelined at world > 1; an explicit part count also applies at world 1 (the
        # one-GPU RCCL test runs the async collectives and part kernels that way)
        P = self.PIPELINE if pipeline is None else int(pipeline)
        if pipeline is None and k is not None and \
                (world - 1) * self.vmax * 5 * int(k) < self.PIPELINE_MIN_BYTES:
            P = 1  # latency-bound exchange: one part
        on = mode == "gather" and (world > 1 or pipeline is not None)
        self.pipeline = max(1, min(P, self.vmax)) if on else 1
        if self.pipeline > 1:
            self._split_parts(owner, loc)

    # ---- pipelined gather mode: column parts (once per graph)
    def _split_parts(self, owner: torch.Tensor, loc: torch.Tensor) -> None:
        """Part j = the columns whose row inside their owner lies in [j * vh, (j + 1) * vh);
        its sub-CSR keeps the shard's rows (CSR order inside each row) and numbers its columns
        owner * vh + (loc - j * vh), the padded space of that part's all-gather."""
        P = self.pipeline
        vh = -(-self.vmax // P)
        self.vh = vh
        part = loc // vh
        counts = torch.diff(self.row_ptr.to(torch.int64))
        rows_e = torch.repeat_interleave(torch.arange(self.n_local, device=self.device), counts)
        self.parts = []
        for j in range(P):
            m = part == j
            cnt = torch.bincount(rows_e[m], minlength=self.n_local)
            rp = torch.zeros(self.n_local + 1, dtype=torch.int64, device=self.device)
            rp[1:] = torch.cumsum(cnt, 0)
            col = (owner[m] * vh + (loc[m] - j * vh)).to(torch.int32).contiguous()
            self.parts.append((rp.to(torch.int32).contiguous(), col,
                               self.values[m].contiguous()))
        self.n_cols_part = self.world * vh

    # ---- halo send plan (once per graph)
    def _halo_plan(self, cols: torch.Tensor, starts: torch.Tensor) -> None:
        halo = torch.unique(cols)  # sorted global ids: grouped by owner, owners ascending
        self.halo = halo
        self.n_cols = int(halo.numel())
        self.col_idx = torch.searchsorted(halo, cols).to(torch.int32).contiguous()
        owner = torch.searchsorted(starts[1:], halo, right=True)
        need = torch.bincount(owner, minlength=self.world)  # rows I receive from each owner
        give = torch.empty_like(need)                       # rows each requester wants of mine
        _all_to_all(give, need, None, None, self.group)
        self.recv_counts = [int(x) for x in need.tolist()]
        self.send_counts = [int(x) for x in give.tolist()]
        req = torch.empty(sum(self.send_counts), dtype=torch.int64, device=self.device)
        _all_to_all(req, halo, self.send_counts, self.recv_counts, self.group)
        self.send_rows = (req - self.v0).contiguous()  # my local rows, per requester in order

    def exchange_bytes(self, k: int) -> dict:
        """Bytes this rank sends / receives per step (forward CBSR + backward gradient)."""
        row_f, row_b = k * 5, k * 4  # k f32 + k u8 forward, k f32 backward
        if self.mode == "gather":
            rows = self.vh * self.pipeline if self.pipeline > 1 else self.vmax  # padded chunk
            others = (self.world - 1) * rows
            return {"fwd_recv": others * row_f, "fwd_send": others * row_f,
                    "bwd_send": others * row_b, "bwd_recv": others * row_b}
        own = self.recv_counts[self.rank]
        recv_rows = self.n_cols - own
        send_rows = sum(self.send_counts) - self.send_counts[self.rank]
        return {"fwd_recv": recv_rows * row_f, "fwd_send": send_rows * row_f,
                "bwd_send": recv_rows * row_b, "bwd_recv": send_rows * row_b}

    # ---- helpers
    def gather_cbsr(self, val_local: torch.Tensor, idx_local: torch.Tensor):
        """The CBSR rows of the shard's column space: [n_cols, k] values and selectors.

        One collective per call: each row travels as one byte record [k values | k selectors],
        so values and selectors move together; "gather" all-gathers every rank's vmax rows
        (padding rows zero), "halo" sends each owner's requested rows only."""
        k = val_local.shape[1]
        dev = val_local.device
        vb = k * val_local.element_size()
        rb = vb + k * idx_local.element_size()
        if self.mode == "gather":
            send = torch.zeros(self.vmax, rb, dtype=torch.uint8, device=dev)
            send[:self.n_local, :vb] = val_local.contiguous().view(torch.uint8).view(-1, vb)
            send[:self.n_local, vb:] = idx_local.contiguous().view(torch.uint8).view(-1, rb - vb)
            recv = torch.empty(self.world * self.vmax, rb, dtype=torch.uint8, device=dev)
            all_gather_rows(recv.view(-1), send.view(-1), self.group)
        else:
            rows = self.send_rows.to(dev)
            send = torch.empty(rows.numel(), rb, dtype=torch.uint8, device=dev)
            send[:, :vb] = val_local.contiguous().view(torch.uint8).view(-1, vb)[rows]
            send[:, vb:] = idx_local.contiguous().view(torch.uint8).view(-1, rb - vb)[rows]
            recv = torch.empty(self.n_cols, rb, dtype=torch.uint8, device=dev)
            _all_to_all(recv, send, self.recv_counts, self.send_counts, self.group)
        val_all = recv[:, :vb].contiguous().view(val_local.dtype).view(self.n_cols, k)
        idx_all = recv[:, vb:].contiguous().view(idx_local.dtype).view(self.n_cols, k)
        return val_all, idx_all

    def scatter_grad(self, partial: torch.Tensor) -> torch.Tensor:
        """Sum the per-rank partial gradients [n_cols, k] onto the owners: [n_local, k]."""
        k = partial.shape[1]
        if self.mode == "gather":
            out = torch.empty(self.vmax, k, dtype=partial.dtype, device=partial.device)
            reduce_scatter_rows(out, partial.contiguous(), self.group)
            return out[:self.n_local]
        recv = torch.empty(sum(self.send_counts), k, dtype=partial.dtype, device=partial.device)
        _all_to_all(recv, partial.contiguous(), self.send_counts, self.recv_counts, self.group)
        out = torch.zeros(self.n_local, k, dtype=partial.dtype, device=partial.device)
        # one index_add per requester, in rank order: a requester's rows are distinct, so no
        # add races another and the sum order is fixed (run to run bitwise)
        rows = self.send_rows.to(partial.device)
        o = 0
        for n in self.send_counts:
            if n:
                out.index_add_(0, rows[o:o + n], recv[o:o + n])
            o += n
        return out

    def plan(self, k: int, D: Optional[int] = None, part: Optional[int] = None):
        """The backward's per-graph plan at width k and feature width D (built once per
        (k, D) and pipeline part; None for a kernel backend without plans, e.g. the CPU oracle
        in the tests, or a part without edges)."""
        key = (k, D, part)
        if key not in self._plans:
            bp = getattr(self.kernels, "backward_plan", None)
            rp, col, val, nc = ((self.row_ptr, self.col_idx, self.values, self.n_cols)
                                if part is None else self.parts[part] + (self.n_cols_part,))
            self._plans[key] = (bp(rp, col, val, nc, k, num_rows=self.n_local, dim=D)
                                if bp is not None and col.numel() > 0 else None)
        return self._plans[key]

    # ---- one aggregation step (gather + forward; backward + scatter), pipelined or not
    def aggregate(self, val_local: torch.Tensor, idx_local: torch.Tensor, D: int,
                  row_div_local=None, out: Optional[torch.Tensor] = None):
        """(Y_local [n_local, D], saved) -- saved is what grad() needs: the gathered
        selectors (one tensor, or one per pipeline part)."""
        if self.pipeline == 1:
            val_all, idx_all = self.gather_cbsr(val_local, idx_local)
            y = self.kernels.spgemm_forward(self.row_ptr, self.col_idx, self.values, val_all,
                                            idx_all, D, row_div=row_div_local,
                                            **({} if out is None else {"out": out}))
            return y, idx_all
        k = val_local.shape[1]
        dev = val_local.device
        P, vh = self.pipeline, self.vh
        sv = torch.zeros(P * vh, k, dtype=val_local.dtype, device=dev)
        si = torch.zeros(P * vh, k, dtype=idx_local.dtype, device=dev)
        sv[:self.n_local] = val_local
        si[:self.n_local] = idx_local
        # every part's two all-gathers (values, selectors: each lands as the contiguous
        # [world * vh, k] array the kernels take, no unpacking copy) queued at once, in part order
        recvs, works = [], []
        if self._records(k, D):
            return self._aggregate_records(sv, si, k, D, row_div_local, out)
        for j in range(P):
            rv = torch.empty(self.world * vh, k, dtype=sv.dtype, device=dev)
            ri = torch.empty(self.world * vh, k, dtype=si.dtype, device=dev)
            wv = all_gather_rows(rv.view(-1), sv[j * vh:(j + 1) * vh].reshape(-1), self.group,
                                 async_op=True)
            wi = all_gather_rows(ri.view(-1), si[j * vh:(j + 1) * vh].reshape(-1), self.group,
                                 async_op=True)
            recvs.append((rv, ri))
            works.append((wv, wi))
        y, saved = out, []
        for j in range(P):
            _wait(works[j][0])
            _wait(works[j][1])
            val_j, idx_j = recvs[j]
            rp, col, val = self.parts[j]
            # the part's edge-selector stream when its backward reads one (csc / bsort)
            es = (torch.empty(col.numel(), k, dtype=torch.uint8, device=dev)
                  if self._stream(k, D, j) else None)
            kw = {} if es is None else {"edge_sel_out": es}
            saved.append((idx_j, es))
            if j == 0:  # writes every row (zeros where part 0 has no edges)
                if y is not None:
                    kw["out"] = y
                y = self.kernels.spgemm_forward(rp, col, val, val_j, idx_j, D,
                                                row_div=row_div_local, **kw)
            elif col.numel() > 0:
                self.kernels.spgemm_forward(rp, col, val, val_j, idx_j, D, row_div=row_div_local,
                                            out=y, accumulate=True, **kw)
        return y, saved

    def _records(self, k: int, D: int) -> bool:
        """Whether the pipelined gather exchanges transport records (decided once per (k, D)):
        the kernels offer them (cbsr_records / spgemm_forward_records), no part writes an
        edge-selector stream, and every part with edges takes the records forward
        (records_ok: a sparse part graph, k % 4 == 0 in [24, 32]).  MAXK_DIST_RECORDS=0: never."""
        key = ("records", k, D)
        if key not in self._plans:
            kn = self.kernels
            ok = (os.environ.get("MAXK_DIST_RECORDS", "1") != "0" and self.mode == "gather" and
                  all(hasattr(kn, f) for f in ("cbsr_records", "spgemm_forward_records",
                                                "records_ok")))
            for j in range(self.pipeline):
                rp, col, _ = self.parts[j]
                if not ok:
                    break
                if col.numel() > 0:
                    ok = (not self._stream(k, D, j) and
                          kn.records_ok(self.n_local, self.n_cols_part, col.numel(), D, k))
            self._plans[key] = bool(ok)
        return self._plans[key]

    def _aggregate_records(self, sv, si, k: int, D: int, row_div_local, out):
        """The pipelined gather over transport records: each owner builds its part-j rows'
        records ([k f32 | k u8], the bytes the two CBSR all-gathers carry), one all-gather per
        part lands them as the [world * vh, 5k] buffer the records forward walks (no pack over
        the gathered vertices); the part's selectors for the backward are its columns 4k..5k."""
        P, vh = self.pipeline, self.vh
        dev = sv.device
        # every part's send buffer stays referenced until its all-gather has been waited on (the
        # caching allocator also holds a block used on the communicator's stream, but the
        # lifetime does not rest on that)
        recvs, works, sends = [], [], []
        for j in range(P):
            send = self.kernels.cbsr_records(sv[j * vh:(j + 1) * vh], si[j * vh:(j + 1) * vh], D)
            rr = torch.empty(self.world * vh, 5 * k, dtype=torch.uint8, device=dev)
            works.append(all_gather_rows(rr.view(-1), send.view(-1), self.group, async_op=True))
            recvs.append(rr)
            sends.append(send)
        y, saved = out, []
        for j in range(P):
            _wait(works[j])
            sends[j] = None
            rr = recvs[j]
            rp, col, val = self.parts[j]
            saved.append((rr[:, 4 * k:].contiguous(), None))
            if j == 0:  # writes every row (zeros where part 0 has no edges)
                y = self.kernels.spgemm_forward_records(rp, col, val, rr, k, D,
                                                        row_div=row_div_local, out=y)
            elif col.numel() > 0:
                self.kernels.spgemm_forward_records(rp, col, val, rr, k, D,
                                                    row_div=row_div_local, out=y,
                                                    accumulate=True)
        return y, saved

    def _stream(self, k: int, D: int, part: int) -> bool:
        """Whether pipeline part `part` carries an edge-selector stream at (k, D) (decided once,
        as its plan is)."""
        key = ("stream", k, D, part)
        if key not in self._plans:
            sm = getattr(self.kernels, "stream_mode", None)
            rp, col, _ = self.parts[part]
            self._plans[key] = bool(sm is not None and col.numel() > 0 and
                                    sm(rp, col, k, self.n_cols_part, self.n_local, D))
        return self._plans[key]

    def grad(self, grad_local: torch.Tensor, saved, row_div_local=None) -> torch.Tensor:
        """CBSR gradient of the owned vertices [n_local, k] from aggregate()'s saved state."""
        if self.pipeline == 1:
            return self.backward(grad_local, saved, row_div_local)
        g = grad_local.contiguous()
        parts = [s if isinstance(s, tuple) else (s, None) for s in saved]
        k = parts[0][0].shape[1]
        outs, works, keep = [], [], []
        for j in range(self.pipeline):  # part j's reduce-scatter beside part j+1's backward
            rp, col, val = self.parts[j]
            idx_j, es = parts[j]
            if col.numel() > 0:
                partial = self.kernels.sspmm_backward(rp, col, val, g, idx_j,
                                                      row_div=row_div_local,
                                                      plan=self.plan(k, g.shape[1], j),
                                                      **({} if es is None else {"edge_sel": es}))
            else:
                partial = torch.zeros(self.n_cols_part, k, dtype=g.dtype, device=g.device)
            o = torch.empty(self.vh, k, dtype=g.dtype, device=g.device)
            works.append(reduce_scatter_rows(o, partial.contiguous(), self.group, async_op=True))
            outs.append(o)
            keep.append(partial)
        for w in works:
            _wait(w)
        return torch.cat(outs)[:self.n_local]

    # ---- the two aggregation passes
    def forward(self, val_all, idx_all, D: int, row_div_local=None) -> torch.Tensor:
        """Y_local [n_local, D] from the gathered CBSR."""
        return self.kernels.spgemm_forward(self.row_ptr, self.col_idx, self.values, val_all,
                                           idx_all, D, row_div=row_div_local)

    def backward(self, grad_local: torch.Tensor, idx_all: torch.Tensor,
                 row_div_local=None) -> torch.Tensor:
        """CBSR gradient of the owned vertices [n_local, k] (partials summed on the owners)."""
        partial = self.kernels.sspmm_backward(self.row_ptr, self.col_idx, self.values,
                                              grad_local.contiguous(), idx_all,
                                              row_div=row_div_local,
                                              plan=self.plan(idx_all.shape[1],
                                                             grad_local.shape[1]))
        return self.scatter_grad(partial)


class ShardedMaxKFunction(Function):
    """Autograd over one sharded aggregation: Y_local = (A . scatter(CBSR))[owned rows] / deg.
    Gradient flows to the local top-k values (the v4 surface, spgemmfunction_v4:76-101)."""

    @staticmethod
    def forward(ctx, shard: ShardedMaxK, topk_values, topk_indices, dim_origin: int,
                degrees_local=None):
        idx = topk_indices if topk_indices.dtype == torch.uint8 else topk_indices.to(torch.uint8)
        y, saved = shard.aggregate(topk_values.float().contiguous(), idx.contiguous(),
                                   dim_origin, degrees_local)
        # pipelined: one (selectors, edge-selector stream or None) pair per part, flattened
        flat = ([t if t is not None else torch.empty(0) for pair in saved for t in pair]
                if isinstance(saved, list) else [saved])
        ctx.shard = shard
        ctx.save_for_backward(*flat, degrees_local if degrees_local is not None
                              else torch.empty(0))
        ctx.has_div = degrees_local is not None
        return y

    @staticmethod
    def backward(ctx, grad_output):
        *flat, deg = ctx.saved_tensors
        st = ([(flat[i], flat[i + 1] if flat[i + 1].numel() else None)
               for i in range(0, len(flat), 2)] if ctx.shard.pipeline > 1 else flat[0])
        g = ctx.shard.grad(grad_output.float(), st, deg if ctx.has_div else None)
        return None, g, None, None, None


def sharded_maxk_spgemm(shard: ShardedMaxK, topk_values, topk_indices, dim_origin: int = 256,
                        degrees_local=None):
    return ShardedMaxKFunction.apply(shard, topk_values, topk_indices, dim_origin, degrees_local)
