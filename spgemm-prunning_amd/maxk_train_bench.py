#!/usr/bin/env python3
"""End-to-end MaxK-GraphSAGE training epoch on one MI355X (BASELINE.json configs[2]).

The reference reports full-graph training speed-ups of its MaxK kernels over the same
model aggregating with cuSPARSE (README.md:178, images/speedup_acc.png: ogbn-products SAGE
k=32 1.53x).  This driver times one full-graph epoch of `maxk_layers.MaxKSAGE`
(lin_in -> 3 x [MaxK -> SAGEConv] -> lin_out; forward, cross-entropy, backward, Adam step):

  maxk     aggregation through the drop-in maxk_spgemm (HIP SpGEMM / SSpMM kernels);
  library  the same model and weights, aggregation = rocSPARSE SpMM of the CSR with the
           dense MaxK output (backward on the transposed CSR) -- the vendor-SpMM
           denominator, as DGL drives cuSPARSE.

Both start from identical weights; the first epoch's losses must agree to 1e-4 (checked), and
the last epoch's, which follow Adam steps on each side's own gradients, to 1e-3 (the
backward through both aggregations; `last_loss_match`).
Graph: <graph>.indptr|.indices when found (maxk_graph.find_graph), else the synthetic
stand-in; features / labels are synthetic (randn, uniform classes).

  python maxk_train_bench.py [products] [--hidden 256] [--k 32] [--layers 3] [--epochs 5]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402
import maxk_layers  # noqa: E402

# (input feature dim, classes) of the published datasets (ogbn-products: 100 / 47)
DATASET_SHAPES = {"products": (100, 47), "products_comm": (100, 47), "reddit": (602, 41),
                  "proteins": (8, 112),
                  "flickr": (500, 7)}


class _LibrarySpMM(torch.autograd.Function):
    """Y = A @ X by rocSPARSE SpMM (int32 CSR, the reference's cusparseSpMM call,
    kernels/spmm_cusparse.cu:6-62), dX = A^T @ dY on the transposed graph built once --
    how DGL drives cuSPARSE for a SpMM aggregation.  One plan per direction, rebound to
    each call's dense buffers."""

    @staticmethod
    def forward(ctx, lib, x):
        ctx.lib = lib
        return lib.run(lib.fwd, x.contiguous())

    @staticmethod
    def backward(ctx, g):
        return None, ctx.lib.run(ctx.lib.bwd, g.contiguous())


class _LibraryPlans:
    def __init__(self, indptr, indices, values, V, dim):
        dev = indices.device
        self.A = (indptr, indices, values)
        rows = torch.repeat_interleave(torch.arange(V, device=dev), torch.diff(indptr).long())
        order = torch.argsort(indices.long(), stable=True)  # CSR of A^T
        t_ptr = torch.zeros(V + 1, dtype=torch.int64, device=dev)
        t_ptr[1:] = torch.cumsum(torch.bincount(indices.long(), minlength=V), 0)
        self.AT = (t_ptr.int(), rows[order].int().contiguous(), values[order].contiguous())
        dummy = torch.zeros(V, dim, device=dev)
        self.fwd = mk.DenseSpMMPlan(*self.A, dummy)
        self.bwd = mk.DenseSpMMPlan(*self.AT, dummy)

    @staticmethod
    def run(plan, x):
        return plan.run(x, torch.empty_like(x))


class LibraryGraph(maxk_layers.CSRGraph):
    """Same graph, aggregation by the vendor sparse library (rocSPARSE SpMM) on the dense MaxK
    output: the reference's cuSPARSE denominator."""

    def __init__(self, g: maxk_layers.CSRGraph):
        self.__dict__.update(g.__dict__)
        self._plans = {}

    def aggregate(self, topk_values, topk_indices, dim, values=None, row_div=None):
        x = torch.zeros(topk_values.shape[0], dim, device=topk_values.device).scatter(
            1, topk_indices.long(), topk_values)
        v = self.values if values is None else values
        key = (id(v), dim)
        if key not in self._plans:
            self._plans[key] = _LibraryPlans(self.indptr, self.indices, v, self.num_nodes, dim)
        y = _LibrarySpMM.apply(self._plans[key], x)
        return y if row_div is None else y / row_div[:, None]


def epoch(model, g, x, y, opt):
    opt.zero_grad(set_to_none=True)
    loss = maxk_layers.cross_entropy(model(g, x), y)  # = F.cross_entropy, parallel kernels
    loss.backward()
    opt.step()
    return loss


def time_epochs(model, g, x, y, epochs, warmup):
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    first = None
    for i in range(warmup + epochs):
        if i == warmup:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        loss = epoch(model, g, x, y, opt)
        if first is None:
            first = loss.item()
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / epochs, first, loss.item()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("graph", nargs="?", default="products")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--graph-dir", default=None)
    ap.add_argument("--no-library", action="store_true")
    ap.add_argument("--reorder", action="store_true",
                    help="relabel the graph by maxk_graph.locality_order first (untimed, once "
                         "per graph; features and labels are synthetic, so none to permute)")
    args = ap.parse_args(argv)
    if not torch.cuda.is_available():
        raise SystemExit("maxk_train_bench needs an MI355X (HIP device)")
    dev = torch.device("cuda")
    gdir = maxk_graph.find_graph(args.graph, [args.graph_dir] if args.graph_dir else [])
    if gdir:
        d = maxk_graph.GraphDataLoader(gdir).load_graph(args.graph)
        indptr, indices = torch.from_numpy(d["indptr"]).to(dev), torch.from_numpy(d["indices"]).to(dev)
        source = f"{gdir}/{args.graph}.indptr|.indices"
    else:
        indptr, indices = maxk_graph.synthetic_graph(args.graph, device=dev)
        source = "synthetic"
    t_reorder = None
    if args.reorder:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        indptr, indices, _ = maxk_graph.permute_graph(
            indptr, indices, maxk_graph.locality_order(indptr, indices))
        torch.cuda.synchronize()
        t_reorder = round(time.perf_counter() - t0, 3)
    g = maxk_layers.CSRGraph(indptr, indices)  # SAGE: unit edge weights, mean by in-degree
    V = g.num_nodes
    f_in, n_cls = DATASET_SHAPES.get(args.graph, (128, 16))
    gen = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(V, f_in, generator=gen, device=dev)
    y = torch.randint(0, n_cls, (V,), generator=gen, device=dev)
    torch.manual_seed(0)
    model = maxk_layers.MaxKSAGE(f_in, args.hidden, args.layers, n_cls, maxk=args.k,
                                 feat_drop=0.0).to(dev)
    ref = copy.deepcopy(model)
    ms, loss0, loss_n = time_epochs(model, g, x, y, args.epochs, args.warmup)
    out = {"graph": args.graph, "source": source, "V": V, "E": indices.numel(),
           "hidden": args.hidden, "k": args.k, "layers": args.layers, "epochs": args.epochs,
           "maxk_epoch_ms": round(ms, 3), "first_loss": loss0, "last_loss": loss_n}
    if args.reorder:
        out["reorder_s"] = t_reorder
    if not args.no_library:
        ms_lib, loss_lib, loss_lib_n = time_epochs(ref, LibraryGraph(g), x, y, args.epochs,
                                                   args.warmup)
        out.update({"library_epoch_ms": round(ms_lib, 3), "speedup": round(ms_lib / ms, 3),
                    "first_loss_library": loss_lib, "last_loss_library": loss_lib_n,
                    "loss_match": abs(loss0 - loss_lib) <= 1e-4 * max(1.0, abs(loss_lib)),
                    "last_loss_match": abs(loss_n - loss_lib_n) <= 1e-3 * max(1.0, abs(loss_lib_n))})
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
