"""MaxK-GNN layers on the drop-in aggregation, without DGL.

The reference's integrated models (model_integrated_v3.py: OPTMaxK :28-43,
MaxKSAGEConv :62-192, MaxKGraphConv :194-398, MaxKGINConv :400-520, MaxKSAGE
:522-588) wrap DGL graphs; here a layer takes a `CSRGraph` (row r = destination,
its columns = source vertices) and every aggregation goes through
`maxk_spgemm_function.maxk_spgemm` (v4 shape) -> the HIP kernels.  The MaxK
nonlinearity runs on the HIP top-k.

Caller defects of the reference fixed here, each documented
where it applies:
  * OPTMaxK.backward drops the gradient of topk_values (:39-43) -> MaxK below
    returns grad = scatter(gather(g_dense) + g_topk);
  * GCN "both"/"left" normalisation scales feat_src, but the kernel is then fed
    the unnormalised topk_values AND divides by degree (:301-310, 341-345,
    380-389) -> here the symmetric normalisation is folded into the edge values
    once per graph and the kernel divides by nothing;
  * lin_before_mp paths apply the Linear to the [V, k] top-k values (:166, 330)
    -> here aggregation always runs on the CBSR and the Linear after it (equal by
    linearity, and the aggregation keeps its k-sparse input);
  * GIN "sum" passes the degrees, i.e. computes a mean (:493) -> here a sum;
  * the models' feat_drop masks x_sparse but the aggregation is fed the undropped
    topk_values (:153-181, :661-664, :743-746) -> here the aggregated values are the
    dropped ones.

`reference_compat=True` (on `maxk`, the convolutions and the models) reproduces every one of
these behaviours instead, so a model trained with the reference computes the same function
here (tests/test_layers_gpu.py checks each against a dense restatement of the reference's
lines).  The reference's lin_before_mp branches (in_feats > out_feats) multiply the [V, k]
top-k values by an [in_feats, out] matrix, which raises and sends the reference to its DGL
fallback, i.e. the normalised aggregation; compat mode computes that fallback there.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
from torch.autograd import Function

import maxk_cuda_kernels as mk
from maxk_spgemm_function import maxk_spgemm


def _clamped(graph, name: str) -> torch.Tensor:
    """graph.<name> clamped to >= 1: CSRGraph's cached tensor, or computed for a graph-like
    object without the cache."""
    f = getattr(graph, "clamped", None)
    return f(name) if f is not None else getattr(graph, name).clamp(min=1.0)


class CSRGraph:
    """Adjacency in CSR with rows = destinations: out[r] aggregates x[indices[e]], e in row r."""

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor,
                 values: Optional[torch.Tensor] = None):
        self.indptr = indptr.int().contiguous()
        self.indices = indices.int().contiguous()
        self.num_nodes = self.indptr.numel() - 1
        self.values = (torch.ones(self.indices.numel(), device=self.indices.device)
                       if values is None else values.float().contiguous())
        # in-degree of a destination row, out-degree of a source (column counts)
        self.in_degrees = torch.diff(self.indptr).float()
        self.out_degrees = torch.bincount(self.indices.long(),
                                          minlength=self.num_nodes).float()
        self._rows = None
        self._clamped = {}

    def clamped(self, name: str) -> torch.Tensor:
        """in_degrees / out_degrees clamped to >= 1, built once: the same divisor tensor
        every call, so per-(plan, divisor) work in the backward (maxk_cuda_kernels'
        pre-scaled pull entries) is done once per graph."""
        if name not in self._clamped:
            self._clamped[name] = getattr(self, name).clamp(min=1.0)
        return self._clamped[name]

    def edge_rows(self) -> torch.Tensor:
        if self._rows is None:
            self._rows = torch.repeat_interleave(
                torch.arange(self.num_nodes, device=self.indptr.device),
                torch.diff(self.indptr).long())
        return self._rows

    def aggregate(self, topk_values, topk_indices, dim: int, values=None, row_div=None):
        """(A . scatter(CBSR))[r] / row_div[r] through the drop-in v4 surface."""
        return maxk_spgemm(self.indices, self.values if values is None else values,
                           topk_values, topk_indices, None, 0, self.indptr, row_div,
                           dim_origin=dim)


class MaxK(Function):
    """MaxK nonlinearity (model_integrated_v3.py:28-60): keeps the k largest entries of each
    row.  Returns (dense masked output, topk_values, topk_indices u8); gradients from the
    dense output and from topk_values both reach the input (the reference drops the latter).

    Both directions are single fused HIP passes: the forward writes the
    CBSR and the masked dense row from one top-k kernel (maxk_topk_cbsr_dense); the backward
    gathers the dense gradient at the selected columns, adds the topk_values gradient and
    writes the whole dense row in one kernel (maxk_topk_backward)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, k: int, drop_topk_grad: bool = False):
        dense, vals, idx = mk.topk_cbsr_dense(x.float(), int(k))
        ctx.save_for_backward(idx)
        ctx.D = x.shape[1]
        ctx.drop = bool(drop_topk_grad)
        ctx.mark_non_differentiable(idx)
        return dense, vals, idx

    @staticmethod
    def backward(ctx, g_dense, g_vals, g_idx):
        idx, = ctx.saved_tensors
        # drop_topk_grad: OPTMaxK.backward (model_integrated_v3.py:39-43) returns
        # grad_output * mask and ignores the topk_values gradient
        gv = None if g_vals is None or ctx.drop else g_vals.float().contiguous()
        gd = None if g_dense is None else g_dense.float().contiguous()
        if gv is None and gd is None:
            return None, None, None
        return mk.topk_backward(gv, gd, idx, ctx.D), None, None


def maxk(x: torch.Tensor, k: int, reference_compat: bool = False):
    """(masked dense x, topk_values, topk_indices u8).  reference_compat: the topk_values
    gradient is dropped, as the reference's OPTMaxK does."""
    return MaxK.apply(x, k, reference_compat)


def _dropped_values(x_sparse: torch.Tensor, topk_values: torch.Tensor,
                    topk_indices: torch.Tensor, drop: nn.Module) -> tuple:
    """(dropout(x_sparse), its values at the selected columns): the CBSR of the dropped
    features, so the aggregation sees what the layer's dense input sees.  Without an
    active dropout both are returned unchanged."""
    if not drop.training or getattr(drop, "p", 0.0) == 0.0:
        return x_sparse, topk_values
    xd = drop(x_sparse)
    return xd, xd.gather(1, topk_indices.long())


# ---- dense parts of a full-graph layer (N = all vertices) ---------------------------------
# rocBLAS / hipBLASLt pick a weight-gradient kernel for G^T X with K = N = 2.45M rows that
# runs at ~60 TFLOP/s (5.1 ms for 256x256 on ogbn-products); as a batched GEMM over 256
# row chunks plus a sum it takes 2.2 ms.  PyTorch's bias gradient g.sum(0) over [2.45M, 47]
# takes 19 ms; as a chunked sum 0.11 ms (tools/dense_probe.py).  Same sums, regrouped.

_CHUNKS = 256


def _wgrad(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """g^T @ x ([O, I]) for tall g [N, O], x [N, I]."""
    n = g.shape[0]
    if n < _CHUNKS * 1024:
        return g.t() @ x
    m = n // _CHUNKS * _CHUNKS
    out = torch.bmm(g[:m].view(_CHUNKS, m // _CHUNKS, g.shape[1]).transpose(1, 2),
                    x[:m].view(_CHUNKS, m // _CHUNKS, x.shape[1])).sum(0)
    if m < n:
        out.addmm_(g[m:].t(), x[m:])
    return out


def _bgrad(g: torch.Tensor) -> torch.Tensor:
    """g.sum(0) for tall g [N, O]."""
    n = g.shape[0]
    if n < _CHUNKS * 1024:
        return g.sum(0)
    m = n // _CHUNKS * _CHUNKS
    out = g[:m].view(_CHUNKS, m // _CHUNKS, g.shape[1]).sum(1).sum(0)
    return out + g[m:].sum(0) if m < n else out


class _Linear(Function):
    """out = x1 W1^T (+ x2 W2^T) (+ b): nn.Linear (or two summed, SAGE's fc_self + fc_neigh,
    accumulated by a second addmm in place) with the tall-matrix weight/bias gradients above."""

    @staticmethod
    def forward(ctx, x1, w1, b, x2, w2):
        out = torch.addmm(b, x1, w1.t()) if b is not None else x1 @ w1.t()
        if x2 is not None:
            out.addmm_(x2, w2.t())
        ctx.save_for_backward(x1, w1, x2, w2)
        ctx.has_b = b is not None
        return out

    @staticmethod
    def backward(ctx, g):
        x1, w1, x2, w2 = ctx.saved_tensors
        g = g.contiguous()
        n = ctx.needs_input_grad
        gx1 = g @ w1 if n[0] else None
        gw1 = _wgrad(g, x1) if n[1] else None
        gb = _bgrad(g) if ctx.has_b and n[2] else None
        gx2 = g @ w2 if x2 is not None and n[3] else None
        gw2 = _wgrad(g, x2) if x2 is not None and n[4] else None
        return gx1, gw1, gb, gx2, gw2


def linear(x: torch.Tensor, layer: nn.Linear, x2: Optional[torch.Tensor] = None,
           layer2: Optional[nn.Linear] = None) -> torch.Tensor:
    """layer(x) (+ layer2(x2)) through _Linear; layer2's bias (if any) is added separately."""
    out = _Linear.apply(x, layer.weight, layer.bias, x2,
                        None if layer2 is None else layer2.weight)
    if layer2 is not None and layer2.bias is not None:
        out = out + layer2.bias
    return out


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """F.cross_entropy(logits, target) (mean over rows) as log_softmax + gather + mean:
    PyTorch's nll_loss reduction kernel takes 5 ms forward + 4 ms backward on 2.45M rows,
    this form 1.3 ms for both (tools/dense_probe.py)."""
    return -torch.log_softmax(logits, 1).gather(1, target[:, None]).mean()


class MaxKSAGEConv(nn.Module):
    """GraphSAGE-mean on MaxK features (model_integrated_v3.py:62-192):
    rst = fc_self(x_sparse) + fc_neigh(mean_{u in N(v)} x_sparse[u])."""

    def __init__(self, in_feats: int, out_feats: int, bias: bool = True, feat_drop: float = 0.,
                 activation=None, norm: Optional[nn.Module] = None,
                 reference_compat: bool = False):
        super().__init__()
        self.in_feats, self.out_feats = in_feats, out_feats
        self.reference_compat = reference_compat
        self.fc_neigh = nn.Linear(in_feats, out_feats, bias=False)
        self.fc_self = nn.Linear(in_feats, out_feats, bias=bias)
        self.feat_drop = nn.Dropout(feat_drop)
        self.activation, self.norm = activation, norm
        gain = nn.init.calculate_gain("relu")
        nn.init.xavier_uniform_(self.fc_self.weight, gain=gain)
        nn.init.xavier_uniform_(self.fc_neigh.weight, gain=gain)

    def forward(self, graph: CSRGraph, x_sparse, topk_values, topk_indices):
        deg = _clamped(graph, "in_degrees")
        if self.reference_compat:  # :153-181: only h_self sees the dropout
            h_self = self.feat_drop(x_sparse)
        else:
            h_self, topk_values = _dropped_values(x_sparse, topk_values, topk_indices,
                                                  self.feat_drop)
        agg = graph.aggregate(topk_values, topk_indices, self.in_feats, row_div=deg)
        # fc_self(x) + fc_neigh(agg) as one accumulated pair of GEMMs
        rst = linear(h_self, self.fc_self, agg, self.fc_neigh)
        if self.activation is not None:
            rst = self.activation(rst)
        if self.norm is not None:
            rst = self.norm(rst)
        return rst


class MaxKGraphConv(nn.Module):
    """GCN on MaxK features (model_integrated_v3.py:194-398): rst = (N A N') x_sparse W + b,
    norm "both" = D_in^-1/2 A D_out^-1/2, "right" = D_in^-1 A, "left" = A D_out^-1."""

    def __init__(self, in_feats: int, out_feats: int, norm: str = "both", weight: bool = True,
                 bias: bool = True, activation=None, reference_compat: bool = False):
        super().__init__()
        if norm not in ("none", "both", "right", "left"):
            raise ValueError(f'Invalid norm value. Must be either "none", "both", "right" or '
                             f'"left". But got "{norm}".')
        self.in_feats, self.out_feats, self._norm = in_feats, out_feats, norm
        self.reference_compat = reference_compat
        self.weight = nn.Parameter(torch.empty(in_feats, out_feats)) if weight else None
        self.bias = nn.Parameter(torch.zeros(out_feats)) if bias else None
        self.activation = activation
        if self.weight is not None:
            nn.init.xavier_uniform_(self.weight)
        self._graph_key = None
        self._edge_values = None

    def _norm_values(self, graph: CSRGraph) -> torch.Tensor:
        if self._graph_key is not graph:  # once per graph, like the reference's set_graph_data
            v = graph.values
            if self._norm in ("left", "both"):
                src = _clamped(graph, "out_degrees")
                src = src.pow(-0.5) if self._norm == "both" else 1.0 / src
                v = v * src[graph.indices.long()]
            if self._norm in ("right", "both"):
                dst = _clamped(graph, "in_degrees")
                dst = dst.pow(-0.5) if self._norm == "both" else 1.0 / dst
                v = v * dst[graph.edge_rows()]
            self._edge_values, self._graph_key = v.contiguous(), graph
        return self._edge_values

    def forward(self, graph: CSRGraph, x_sparse, topk_values, topk_indices):
        if self.reference_compat and self.in_feats <= self.out_feats:
            # :302-310 normalise feat_src, which the kernel never reads; :341-345 feed it the
            # raw topk_values with the in-degrees as divisor; :381-389 then apply the right
            # normalisation on top
            deg = _clamped(graph, "in_degrees")
            rst = graph.aggregate(topk_values, topk_indices, self.in_feats, row_div=deg)
            if self.weight is not None:
                rst = rst @ self.weight
            if self._norm in ("right", "both"):
                rst = rst * (deg.pow(-0.5) if self._norm == "both" else 1.0 / deg)[:, None]
        else:
            rst = graph.aggregate(topk_values, topk_indices, self.in_feats,
                                  values=self._norm_values(graph))
            if self.weight is not None:
                rst = rst @ self.weight
        if self.bias is not None:
            rst = rst + self.bias
        if self.activation is not None:
            rst = self.activation(rst)
        return rst


class MaxKGINConv(nn.Module):
    """GIN-sum on MaxK features (model_integrated_v3.py:400-520):
    rst = apply_func((1 + eps) x + sum_{u in N(v)} x_sparse[u])."""

    def __init__(self, apply_func: Optional[nn.Module] = None, init_eps: float = 0.,
                 learn_eps: bool = False, activation=None, reference_compat: bool = False):
        super().__init__()
        self.apply_func, self.activation = apply_func, activation
        self.reference_compat = reference_compat
        if learn_eps:
            self.eps = nn.Parameter(torch.tensor([float(init_eps)]))
        else:
            self.register_buffer("eps", torch.tensor([float(init_eps)]))

    def forward(self, graph: CSRGraph, x, topk_values, topk_indices):
        # reference_compat: the "sum" kernel call passes the in-degrees (:491-495), a mean
        row_div = _clamped(graph, "in_degrees") if self.reference_compat else None
        neigh = graph.aggregate(topk_values, topk_indices, x.shape[1], row_div=row_div)
        rst = (1 + self.eps) * x + neigh
        if self.apply_func is not None:
            rst = self.apply_func(rst)
        if self.activation is not None:
            rst = self.activation(rst)
        return rst


class MaxKSAGE(nn.Module):
    """lin_in -> [MaxK -> MaxKSAGEConv] x L -> lin_out (model_integrated_v3.py:522-588; same
    constructor arguments; graph_name is accepted and unused: no schedule files are needed)."""

    def __init__(self, in_size: int, hid_size: int, num_hid_layers: int, out_size: int,
                 maxk: int = 32, feat_drop: float = 0.5, norm: bool = False,
                 nonlinear: str = "maxk", graph_name: str = "", reference_compat: bool = False):
        super().__init__()
        if nonlinear != "maxk":
            raise ValueError(f"Only 'maxk' supported, got {nonlinear}")
        self.k, self.num_layers, self.graph_name = maxk, num_hid_layers, graph_name
        self.reference_compat = reference_compat
        self.lin_in = nn.Linear(in_size, hid_size)
        self.layers = nn.ModuleList([
            MaxKSAGEConv(hid_size, hid_size, feat_drop=feat_drop,
                         norm=nn.LayerNorm(hid_size) if norm else None,
                         reference_compat=reference_compat)
            for _ in range(num_hid_layers)])
        self.lin_out = nn.Linear(hid_size, out_size)
        nn.init.xavier_uniform_(self.lin_in.weight)
        nn.init.xavier_uniform_(self.lin_out.weight)

    def forward(self, graph: CSRGraph, x):
        x = linear(x, self.lin_in)
        for layer in self.layers:
            x_sparse, vals, idx = maxk(x, self.k, self.reference_compat)
            x = layer(graph, x_sparse, vals, idx)
        return linear(x, self.lin_out)


class _MaxKStack(nn.Module):
    """Shared body of MaxKGCN / MaxKGIN (model_integrated_v3.py:590-752): lin_in + relu, then
    per layer Linear -> MaxK -> dropout -> conv (-> LayerNorm), then lin_out."""

    def __init__(self, in_size, hid_size, num_hid_layers, out_size, maxk, feat_drop, norm,
                 nonlinear, graph_name, reference_compat, make_conv):
        super().__init__()
        if nonlinear != "maxk":
            raise ValueError(f"Only 'maxk' supported, got {nonlinear}")
        self.k, self.num_layers, self.graph_name = maxk, num_hid_layers, graph_name
        self.reference_compat = reference_compat
        self.dropoutlayers = nn.ModuleList([nn.Dropout(feat_drop) for _ in range(num_hid_layers)])
        self.convs = nn.ModuleList([make_conv() for _ in range(num_hid_layers)])
        self.normlayers = nn.ModuleList([nn.LayerNorm(hid_size) for _ in range(num_hid_layers)]
                                        if norm else [])
        self.linlayers = nn.ModuleList([nn.Linear(hid_size, hid_size)
                                        for _ in range(num_hid_layers)])
        for lin in self.linlayers:
            nn.init.xavier_uniform_(lin.weight)
        self.lin_in = nn.Linear(in_size, hid_size)
        self.lin_out = nn.Linear(hid_size, out_size)
        nn.init.xavier_uniform_(self.lin_in.weight)
        nn.init.xavier_uniform_(self.lin_out.weight)

    def forward(self, graph: CSRGraph, x):
        x = linear(x, self.lin_in).relu()
        for i in range(self.num_layers):
            x = linear(x, self.linlayers[i])
            x_sparse, vals, idx = maxk(x, self.k, self.reference_compat)
            if self.reference_compat:  # :661, :743: the kernel gets the undropped values
                x_sparse = self.dropoutlayers[i](x_sparse)
            else:
                x_sparse, vals = _dropped_values(x_sparse, vals, idx, self.dropoutlayers[i])
            x = self.convs[i](graph, x_sparse, vals, idx)
            if self.normlayers:
                x = self.normlayers[i](x)
        return linear(x, self.lin_out)


class MaxKGCN(_MaxKStack):
    """GCN model (model_integrated_v3.py:590-670): MaxKGraphConv(norm="both", no weight, no
    bias) after a per-layer Linear."""

    def __init__(self, in_size: int, hid_size: int, num_hid_layers: int, out_size: int,
                 maxk: int = 32, feat_drop: float = 0.5, norm: bool = False,
                 nonlinear: str = "maxk", graph_name: str = "", reference_compat: bool = False):
        super().__init__(in_size, hid_size, num_hid_layers, out_size, maxk, feat_drop, norm,
                         nonlinear, graph_name, reference_compat,
                         lambda: MaxKGraphConv(hid_size, hid_size, norm="both", weight=False,
                                               bias=False, reference_compat=reference_compat))

    @property
    def gcnlayers(self):
        return self.convs


class MaxKGIN(_MaxKStack):
    """GIN model (model_integrated_v3.py:672-752): MaxKGINConv(sum, learnable eps from 0)
    after a per-layer Linear."""

    def __init__(self, in_size: int, hid_size: int, num_hid_layers: int, out_size: int,
                 maxk: int = 32, feat_drop: float = 0.5, norm: bool = False,
                 nonlinear: str = "maxk", graph_name: str = "", reference_compat: bool = False):
        super().__init__(in_size, hid_size, num_hid_layers, out_size, maxk, feat_drop, norm,
                         nonlinear, graph_name, reference_compat,
                         lambda: MaxKGINConv(None, init_eps=0.0, learn_eps=True,
                                             reference_compat=reference_compat))

    @property
    def ginlayers(self):
        return self.convs
