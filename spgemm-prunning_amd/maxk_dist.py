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

import torch
import torch.distributed as dist
from torch.autograd import Function


def _staged(group) -> bool:
    """gloo has no device collectives for these calls: stage through host memory (the CPU
    tests, and rehearsing N ranks on a one-GPU box).  RCCL ("nccl") runs them on device."""
    return dist.get_backend(group) == "gloo"


def all_gather_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out[p * n:(p + 1) * n] = inp of rank p (equal n on every rank)."""
    if _staged(group) and inp.is_cuda:
        tmp = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(tmp, inp.cpu(), group=group)
        out.copy_(tmp)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def reduce_scatter_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = sum over ranks of inp[rank * n:(rank + 1) * n]."""
    if _staged(group) and inp.is_cuda:
        tmp = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(tmp, inp.cpu(), group=group)
        out.copy_(tmp)
    else:
        dist.reduce_scatter_tensor(out, inp, group=group)


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
    def __init__(self):
        import maxk_cuda_kernels as mk
        self.mk = mk

    def spgemm_forward(self, indptr, indices, values, cbsr_val, cbsr_idx, D, row_div=None):
        return self.mk.spgemm_forward(indptr, indices, values, cbsr_val, cbsr_idx, D,
                                      row_div=row_div)

    def sspmm_backward(self, indptr, indices, values, grad, cbsr_idx, row_div=None, plan=None):
        return self.mk.sspmm_backward(indptr, indices, values, grad, cbsr_idx, row_div=row_div,
                                      plan=plan)

    def backward_plan(self, indptr, indices, values, num_cols, k, num_rows=None, dim=None):
        return self.mk.backward_plan(indices, num_cols, k, num_rows=num_rows, indptr=indptr,
                                     values=values, dim=dim)


class ShardedMaxK:
    """Rank-local view of a vertex-partitioned graph for the MaxK aggregation.

    mode "gather": column space = padded [world * vmax] (all vertices);
    mode "halo":   column space = this shard's halo (the distinct columns of its edges, in
                   global-id order).  n_cols is its size either way."""

    MODES = ("gather", "halo", "auto")
    # mode "auto": halo when every shard's halo is at most this share of the vertices (an
    # ordered graph's shards need a fraction of the others' rows: the exchange shrinks and
    # the per-column work -- record pack, selector ordering, tile reduce, phase-2 walk --
    # covers the halo only); gather otherwise (a randomly labelled graph's halo is nearly
    # every vertex, and one all-gather / reduce-scatter beats all-to-allv of the same bytes)
    HALO_SHARE = 0.6

    def __init__(self, row_ptr: torch.Tensor, col_idx: torch.Tensor, values: torch.Tensor,
                 rank: int, world: int, group=None, device=None, kernels=None,
                 bounds: Optional[List[int]] = None, mode: str = "gather"):
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
            self.col_idx = (owner * self.vmax + (cols - starts[owner])).to(torch.int32).contiguous()
            self.n_cols = world * self.vmax
        else:
            self._halo_plan(cols, starts)
        self.values = values[e0:e1].to(self.device, torch.float32).contiguous()
        self._plans = {}

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
            others = self.n_cols - self.vmax
            return {"fwd_recv": others * row_f, "fwd_send": (self.world - 1) * self.vmax * row_f,
                    "bwd_send": others * row_b, "bwd_recv": (self.world - 1) * self.vmax * row_b}
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

    def plan(self, k: int, D: Optional[int] = None):
        """The backward's per-graph plan at width k and feature width D (built once per
        (k, D); None for a kernel backend without plans, e.g. the CPU oracle in the tests)."""
        if (k, D) not in self._plans:
            bp = getattr(self.kernels, "backward_plan", None)
            self._plans[(k, D)] = (bp(self.row_ptr, self.col_idx, self.values, self.n_cols, k,
                                      num_rows=self.n_local, dim=D)
                                   if bp is not None else None)
        return self._plans[(k, D)]

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
        val_all, idx_all = shard.gather_cbsr(topk_values.float().contiguous(), idx.contiguous())
        ctx.shard = shard
        ctx.save_for_backward(idx_all, degrees_local if degrees_local is not None
                              else torch.empty(0))
        ctx.has_div = degrees_local is not None
        return shard.forward(val_all, idx_all, dim_origin, degrees_local)

    @staticmethod
    def backward(ctx, grad_output):
        idx_all, deg = ctx.saved_tensors
        g = ctx.shard.backward(grad_output.float(), idx_all, deg if ctx.has_div else None)
        return None, g, None, None, None


def sharded_maxk_spgemm(shard: ShardedMaxK, topk_values, topk_indices, dim_origin: int = 256,
                        degrees_local=None):
    return ShardedMaxKFunction.apply(shard, topk_values, topk_indices, dim_origin, degrees_local)
