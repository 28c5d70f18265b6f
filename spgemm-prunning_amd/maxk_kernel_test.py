#!/usr/bin/env python3
"""maxk_kernel_test -- the reference's kernel benchmark, on MI355X.

Restates `./maxk_kernel_test <graph>` (kernels/main.cu:50-221): for each k of
{16, 32, 64} (main.cu:111-117) every row gets k distinct columns of D sampled uniformly,
in ascending order, with U(0,1) values (main.cu:122-133); the dense copy of that input is
multiplied by the sparse library SpMM (rocSPARSE here, cuSPARSE there, main.cu:163-166)
once, then the MaxK forward SpGEMM and backward SSpMM are timed (spmm_base.h:34-61).
Output keeps the reference's lines:

    num graph dim_origin dim_k kernel time(ms)
    1/1 reddit 256 16 cusparse 20.1
    1/1 reddit 256 16 maxk 1.70
    1/1 reddit 256 16 maxk_backward 4.70

Graph: <dir>/<graph>.indptr|.indices when present (maxk_graph.find_graph: MAXK_GRAPH_DIR,
kernels/graphs, processed_graphs, graphs), else the synthetic stand-in of the same size.
Timing: HIP events on the current stream, median of --runs after --warmup (the reference
used 4 + 4 wall-clock runs).  Adds one validation line per k: MaxK forward vs the library
SpMM, max |diff| / max(1, |ref|) (the reference's check: direct_kernel_interface.py:221-372).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402


def sample_cbsr(V: int, D: int, k: int, gen: torch.Generator, device):
    """main.cu:122-133: k distinct columns per row (ascending) with U(0,1) values."""
    keys = torch.rand(V, D, generator=gen, device=device)
    sel = torch.topk(keys, k, dim=1).indices.sort(dim=1).values.to(torch.uint8).contiguous()
    vals = torch.rand(V, k, generator=gen, device=device)
    return vals, sel


def time_ms(fn, warmup: int, runs: int) -> float:
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(runs):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


# rocSPARSE CSR SpMM algorithms (dense_spmm_rocsparse.cpp kAlgs order); "default" is the
# cusparseSpMM(CUSPARSE_SPMM_ALG_DEFAULT) equivalent of spmm_cusparse.cu:30-46
LIBRARY_ALGS = ("default", "csr", "csr_row_split", "csr_merge_path", "csr_nnz_split")


def library_spmm_times(row_ptr, col, val, dense, warmup: int, runs: int):
    """Median ms of the library SpMM A . dense for every rocSPARSE CSR algorithm, the first
    plan's output (ALG_DEFAULT) and the errors of the others against it.  Returns
    ({alg: ms or None if the library refuses it}, y_default)."""
    times, y0 = {}, None
    for a, name in enumerate(LIBRARY_ALGS):
        try:
            lib = mk.DenseSpMMPlan(row_ptr, col, val, dense, alg=a)
        except RuntimeError:
            times[name] = None
            continue
        try:
            times[name] = time_ms(lib.run, warmup, runs)
            if y0 is None:
                y0 = lib.y.clone()
            elif float((lib.y - y0).abs().max()) > 1e-3 * max(1.0, float(y0.abs().max())):
                times[name] = None  # a wrong result does not count as the library's best
        finally:
            lib.close()
    return times, y0


def best_library(times):
    """(name, ms) of the fastest accepted algorithm; (None, None) if the library refused or
    mis-computed every one."""
    ok = {n: t for n, t in times.items() if t is not None}
    if not ok:
        return None, None
    n = min(ok, key=ok.get)
    return n, ok[n]


def _ratio(a, b):
    return None if a is None or b is None or b <= 0 else a / b


def _fmt(t):
    return "refused" if t is None else f"{t:.4f}"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("graph", nargs="?", default="reddit")
    ap.add_argument("--k", type=int, nargs="+", default=[16, 32, 64])
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--graph-dir", default=None)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--bwd-mode", default="auto", choices=["auto", "pull", "bsort", "csc", "atomic", "dense"])
    ap.add_argument("--json", action="store_true", help="also print one JSON summary line")
    args = ap.parse_args(argv)
    if not torch.cuda.is_available():
        raise SystemExit("maxk_kernel_test needs an MI355X (HIP device)")
    dev = torch.device("cuda")
    gdir = maxk_graph.find_graph(args.graph, [args.graph_dir] if args.graph_dir else [])
    if gdir:
        g = maxk_graph.GraphDataLoader(gdir).load_graph(args.graph)
        row_ptr = torch.from_numpy(g["indptr"]).to(dev)
        col = torch.from_numpy(g["indices"]).to(dev)
        source = f"{gdir}/{args.graph}.indptr|.indices"
    elif args.graph in maxk_graph.PRESETS:
        row_ptr, col = maxk_graph.synthetic_graph(args.graph, device=dev)
        source = "synthetic"
    else:
        raise SystemExit(f"no {args.graph}.indptr/.indices found and no synthetic preset "
                         f"(presets: {sorted(maxk_graph.PRESETS)})")
    V, E, D = row_ptr.numel() - 1, col.numel(), args.dim
    gen = torch.Generator(device=dev).manual_seed(123)  # main.cu:74-77
    val = torch.rand(E, generator=gen, device=dev)
    print(f"# graph {args.graph} ({source}): V={V} E={E}", file=sys.stderr)
    print("num graph dim_origin dim_k kernel time(ms)")
    results = []
    t_lib = None
    for n, k in enumerate(args.k):
        tag = f"1/1 {args.graph} {D} {k}"
        vals, sel = sample_cbsr(V, D, k, gen, dev)
        dense = mk.cbsr_scatter_dense(vals, sel, D)
        y = torch.empty(V, D, device=dev)
        gs = torch.empty(V, k, device=dev)
        mk.spgemm_forward(row_ptr, col, val, vals, sel, D, out=y, validate=True)
        if n == 0:  # main.cu:163-166: the library SpMM once, on the first k's dense input;
            # ALG_DEFAULT keeps the reference's line, the fastest CSR algorithm is reported too
            t_algs, y_lib = library_spmm_times(row_ptr, col, val, dense, args.warmup, args.runs)
            t_lib = t_algs["default"]
            best_name, t_best = best_library(t_algs)
            print(f"{tag} cusparse {_fmt(t_lib)}")
            print(f"{tag} cusparse_best {_fmt(t_best)}")
            print("# library SpMM per algorithm (ms): " + ", ".join(
                f"{a} {'refused' if t is None else f'{t:.4f}'}" for a, t in t_algs.items()),
                file=sys.stderr)
        else:
            try:
                lib = mk.DenseSpMMPlan(row_ptr, col, val, dense)
                y_lib = lib.run().clone()
                lib.close()
            except RuntimeError:
                y_lib = None
        torch.cuda.synchronize()
        err = (None if y_lib is None else
               float(((y - y_lib).abs().max() / y_lib.abs().max().clamp(min=1))))
        t_f = time_ms(lambda: mk.spgemm_forward(row_ptr, col, val, vals, sel, D, out=y,
                                                validate=False), args.warmup, args.runs)
        print(f"{tag} maxk {t_f:.4f}")
        t_b = time_ms(lambda: mk.sspmm_backward(row_ptr, col, val, dense, sel, out=gs,
                                                validate=False, mode=args.bwd_mode),
                      args.warmup, args.runs)
        print(f"{tag} maxk_backward {t_b:.4f}")
        if err is None:
            print(f"# {tag} check maxk vs library SpMM: skipped (library refused)",
                  file=sys.stderr)
        else:
            print(f"# {tag} check maxk vs library SpMM: max rel err {err:.3e} "
                  f"({'PASS' if err < 1e-3 else 'FAIL'})", file=sys.stderr)
        results.append({"k": k, "bwd_mode": mk._bwd_mode(args.bwd_mode, k, E, V, V, D,
                                                         (row_ptr, col)),
                        "maxk_ms": t_f, "maxk_backward_ms": t_b, "max_rel_err": err,
                        "speedup_fwd": _ratio(t_lib, t_f), "speedup_bwd": _ratio(t_lib, t_b),
                        "speedup_fwd_vs_best": _ratio(t_best, t_f),
                        "speedup_bwd_vs_best": _ratio(t_best, t_b),
                        "gteps_fwd": E / t_f / 1e6, "gteps_bwd": E / t_b / 1e6})
        del dense, y, gs, y_lib
    if args.json:
        print(json.dumps({"graph": args.graph, "source": source, "V": V, "E": E, "dim": D,
                          "library_spmm_ms": t_lib, "library_spmm_ms_best": t_best,
                          "library_best_alg": best_name, "library_spmm_ms_by_alg": t_algs,
                          "bwd_mode": args.bwd_mode,
                          "results": results}))
    return results


if __name__ == "__main__":
    main()
