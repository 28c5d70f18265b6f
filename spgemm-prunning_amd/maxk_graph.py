"""On-disk graph format and preprocessing for the MaxK aggregation.

Format (the reference's, kernels/main.cu `cuda_read_array`, graph_loader.py:19-85,
dataset_gen.py:104-115): `<dir>/<name>.indptr` and `<dir>/<name>.indices`, raw
little-endian int32 arrays of the CSR (V+1 and E entries), no header.

`GraphDataLoader` keeps the reference loader's API (graph_loader.py:13-107): same
method names, same returned keys, same synthetic edge weights (numpy seed 123,
U(0,1) float32).  `build_csr` restates dataset_gen.py:59-104 (make undirected ->
add a self loop on every vertex -> drop multi-edges -> CSR) as device-side
sorts instead of a Python set loop, so the real Reddit / ogbn-products /
ogbn-proteins graphs can be prepared on the GPU box in seconds; its output has
sorted column indices, which the reference's DGL `adj_tensors('csr')` does not
promise (the kernels accept either).

`synthetic_graph` / `PRESETS`: the stand-ins used when the real files are absent
(symmetric Chung-Lu power law with self loops at the published V and E).  They are randomly
labelled, so they have no locality at all; `community_graph` adds planted communities (the
structure real graphs such as ogbn-products have), and `locality_order` / `permute_graph`
find and apply a vertex order that makes such structure contiguous (once per graph, like the
reference's offline .warp4 files).
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Dict, Optional

import numpy as np
import torch


def read_binary_array(filepath: str, dtype=np.int32) -> np.ndarray:
    """graph_loader.py:19-38: the whole file as one array."""
    if not os.path.exists(filepath):
        raise FileNotFoundError(f"Graph file not found: {filepath}")
    if dtype not in (np.int32, np.float32):
        raise ValueError(f"Unsupported dtype: {dtype}")
    if os.path.getsize(filepath) % 4:
        raise ValueError(f"{filepath}: size is not a multiple of 4 bytes")
    return np.fromfile(filepath, dtype=dtype)


def edge_values(e_num: int, seed: int = 123) -> np.ndarray:
    """graph_loader.py:69-71: np.random.seed(123); U(0,1) float32 per edge."""
    np.random.seed(seed)
    return np.random.uniform(0, 1, e_num).astype(np.float32)


def validate_csr(indptr: np.ndarray, indices: np.ndarray) -> None:
    """Structural checks the reference skips: monotone indptr from 0 to E, columns in range."""
    if indptr.ndim != 1 or indptr.size < 1:
        raise ValueError("indptr must be a non-empty 1-D array")
    if int(indptr[0]) != 0 or int(indptr[-1]) != indices.size:
        raise ValueError(f"indptr must run from 0 to E={indices.size}")
    if indptr.size > 1 and (np.diff(indptr) < 0).any():
        raise ValueError("indptr must be non-decreasing")
    V = indptr.size - 1
    if indices.size and (int(indices.min()) < 0 or int(indices.max()) >= V):
        raise ValueError(f"indices out of range [0, {V})")


class GraphDataLoader:
    """Reference-compatible loader (graph_loader.py:13): base_dir/<stem>.indptr|.indices."""

    def __init__(self, base_dir: str = "kernels/graphs/"):
        self.base_dir = base_dir

    def read_binary_array(self, filepath, dtype=np.int32):
        return read_binary_array(filepath, dtype)

    def load_graph(self, graph_name: str, validate: bool = True) -> Dict:
        stem = Path(graph_name).stem
        indptr = read_binary_array(os.path.join(self.base_dir, f"{stem}.indptr"))
        indices = read_binary_array(os.path.join(self.base_dir, f"{stem}.indices"))
        if validate:
            validate_csr(indptr, indices)
        v_num, e_num = indptr.size - 1, indices.size
        return {"graph_name": stem, "indptr": indptr, "indices": indices,
                "values": edge_values(e_num), "v_num": v_num, "e_num": e_num}

    def to_cuda_tensors(self, graph_data: Dict, device="cuda") -> Dict:
        """graph_loader.py:87-100."""
        out = {}
        for key, value in graph_data.items():
            out[key] = torch.from_numpy(np.ascontiguousarray(value)).to(device) \
                if isinstance(value, np.ndarray) else value
        return out


def build_csr(src: torch.Tensor, dst: torch.Tensor, num_nodes: int, symmetrize: bool = True,
              self_loops: bool = True, dedupe: bool = True):
    """dataset_gen.py:59-104 on the tensors' device: edges (src -> dst) -> CSR rows = src.

    Returns (indptr int32 [V+1], indices int32 [E]) with columns sorted within each row."""
    src = src.to(torch.int64).flatten()
    dst = dst.to(torch.int64).flatten()
    if src.numel() != dst.numel():
        raise ValueError("src and dst must have the same length")
    V = int(num_nodes)
    if src.numel() and (int(torch.minimum(src.min(), dst.min())) < 0 or
                        int(torch.maximum(src.max(), dst.max())) >= V):
        raise ValueError(f"edge endpoints out of range [0, {V})")
    if symmetrize:                      # :61-66 add reverse edges
        src, dst = torch.cat([src, dst]), torch.cat([dst, src])
    if self_loops:                      # :75-76 dgl.add_self_loop: one more per vertex
        loops = torch.arange(V, device=src.device)
        src, dst = torch.cat([src, loops]), torch.cat([dst, loops])
    key = src * V + dst
    key = torch.unique(key) if dedupe else torch.sort(key).values  # :82-101 multi-edges
    src, dst = key // V, key % V
    indptr = torch.zeros(V + 1, dtype=torch.int64, device=key.device)
    indptr[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0)
    return indptr.to(torch.int32), dst.to(torch.int32)


def save_graph(indptr, indices, out_dir: str, name: str) -> None:
    """dataset_gen.py:106-115: raw int32 files <out_dir>/<name>.indptr / .indices."""
    os.makedirs(out_dir, exist_ok=True)
    ip = indptr.cpu().numpy() if torch.is_tensor(indptr) else np.asarray(indptr)
    ix = indices.cpu().numpy() if torch.is_tensor(indices) else np.asarray(indices)
    ip.astype(np.int32).tofile(os.path.join(out_dir, f"{name}.indptr"))
    ix.astype(np.int32).tofile(os.path.join(out_dir, f"{name}.indices"))


def find_graph(name: str, dirs=None) -> Optional[str]:
    """First directory holding <name>.indptr and <name>.indices (the reference keeps them under
    kernels/graphs/ or ./processed_graphs/; MAXK_GRAPH_DIR adds one)."""
    dirs = list(dirs or [])
    if os.environ.get("MAXK_GRAPH_DIR"):
        dirs.insert(0, os.environ["MAXK_GRAPH_DIR"])
    dirs += ["kernels/graphs", "processed_graphs", "graphs"]
    for d in dirs:
        if os.path.exists(os.path.join(d, f"{name}.indptr")) and \
                os.path.exists(os.path.join(d, f"{name}.indices")):
            return d
    return None


# ---------------------------------------------------------------------------- synthetic graphs
# name: V, E (published sizes), power-law (alpha, offset) fitted so
# the max/avg degree ratio resembles the real graph
PRESETS = {
    "reddit": dict(V=232_965, E=114_615_891, alpha=0.7, i0=200, D=256, k=16),
    "products": dict(V=2_449_029, E=123_718_280, alpha=0.75, i0=3000, D=256, k=32),
    # ogbn-products' size and degree skew with planted communities (~1,200 vertices each,
    # 90 % of the edges inside one), randomly labelled: the locality a real graph has, hidden
    "products_comm": dict(V=2_449_029, E=123_718_280, alpha=0.75, i0=3000, D=256, k=32,
                          communities=2_000, p_in=0.9),
    # the same with half of the edges inside a community: a weaker locality, to place the
    # hybrid backward's switch-over (maxk_cuda_kernels._bwd_mode)
    "products_comm_p50": dict(V=2_449_029, E=123_718_280, alpha=0.75, i0=3000, D=256, k=32,
                              communities=2_000, p_in=0.5),
    "proteins": dict(V=132_534, E=79_122_504, alpha=0.45, i0=2000, D=256, k=64),
    "flickr": dict(V=89_250, E=989_006, alpha=0.9, i0=30, D=64, k=16),
}


def make_graph(V, E, alpha, i0, seed, device, trace=None):
    """Symmetric Chung-Lu power-law graph with self loops, deduplicated, CSR with sorted
    columns (the shape dataset_gen.py:44-115 produces), exactly E edges when E-V is even.
    `trace` (a list) collects (stage, seconds) pairs, each stage synchronised."""
    import time
    t_last = [time.perf_counter()]

    def mark(name):
        if trace is not None:
            if torch.device(device).type == "cuda":
                torch.cuda.synchronize(device)
            t = time.perf_counter()
            trace.append((name, round(t - t_last[0], 3)))
            t_last[0] = t
    g = torch.Generator(device=device).manual_seed(seed)
    pairs_target = (E - V) // 2
    w = (torch.arange(V, device=device, dtype=torch.float64) + i0) ** (-alpha)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    keys = torch.empty(0, dtype=torch.int64, device=device)
    need = pairs_target
    while keys.numel() < pairs_target:
        m = int(need * 1.25) + 4096
        a = torch.searchsorted(cdf, torch.rand(m, generator=g, device=device, dtype=torch.float64))
        b = torch.searchsorted(cdf, torch.rand(m, generator=g, device=device, dtype=torch.float64))
        a.clamp_(max=V - 1)
        b.clamp_(max=V - 1)
        lo, hi = torch.minimum(a, b), torch.maximum(a, b)
        k = (lo * V + hi)[lo != hi]
        mark("sample")
        keys = torch.unique(torch.cat([keys, k]))
        need = pairs_target - keys.numel()
        mark("unique")
        del a, b, lo, hi, k
    keys = keys[torch.randperm(keys.numel(), generator=g, device=device)[:pairs_target]]
    relabel = torch.randperm(V, generator=g, device=device)
    lo, hi = relabel[keys // V], relabel[keys % V]
    del keys
    loops = torch.arange(V, device=device)
    src = torch.cat([lo, hi, loops])
    dst = torch.cat([hi, lo, loops])
    del lo, hi
    mark("permute")
    key = torch.sort(src * V + dst).values
    del src, dst
    mark("sort")
    src, dst = key // V, key % V
    row_ptr = torch.zeros(V + 1, dtype=torch.int64, device=device)
    row_ptr[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0)
    return row_ptr.to(torch.int32), dst.to(torch.int32)


def synthetic_graph(name: str, seed: int = 1, device="cuda"):
    """(row_ptr int32, col int32) of the synthetic stand-in for a published graph: its exact V,
    E (E - V made even) and a degree skew like the real one; presets with
    `communities` plant them (community_graph)."""
    P = PRESETS[name]
    V = P["V"]
    E = P["E"] - ((P["E"] - V) % 2)
    if "communities" in P:
        return community_graph(V, E, P["alpha"], P["i0"], P["communities"], P["p_in"], seed,
                               torch.device(device))
    return make_graph(V, E, P["alpha"], P["i0"], seed, torch.device(device))


def _csr_from_pairs(lo: torch.Tensor, hi: torch.Tensor, V: int):
    """Symmetric CSR (sorted columns) of the undirected pairs lo < hi plus a self loop on
    every vertex."""
    loops = torch.arange(V, device=lo.device)
    src = torch.cat([lo, hi, loops])
    dst = torch.cat([hi, lo, loops])
    key = torch.sort(src * V + dst).values
    del src, dst
    src, dst = key // V, key % V
    row_ptr = torch.zeros(V + 1, dtype=torch.int64, device=lo.device)
    row_ptr[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0)
    return row_ptr.to(torch.int32), dst.to(torch.int32)


def community_graph(V, E, alpha, i0, communities, p_in, seed, device):
    """Symmetric graph with planted communities, self loops, exactly E edges (E - V even).

    Vertex weights follow make_graph's power law, assigned to vertices in random order;
    communities are `communities` equal blocks of that order.  Each undirected pair takes
    one endpoint by weight and the other, with probability p_in, uniformly from the first
    one's community, else by weight from the whole graph.  A final random relabelling
    hides the blocks, as a dataset's arbitrary vertex ids would."""
    g = torch.Generator(device=device).manual_seed(seed)
    pairs_target = (E - V) // 2
    w = (torch.arange(V, device=device, dtype=torch.float64) + i0) ** (-alpha)
    w = w[torch.randperm(V, generator=g, device=device)]  # hubs spread over the communities
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    size = -(-V // communities)
    keys = torch.empty(0, dtype=torch.int64, device=device)
    need = pairs_target
    while keys.numel() < pairs_target:
        m = int(need * 1.25) + 4096
        a = torch.searchsorted(cdf, torch.rand(m, generator=g, device=device,
                                               dtype=torch.float64)).clamp_(max=V - 1)
        b = torch.searchsorted(cdf, torch.rand(m, generator=g, device=device,
                                               dtype=torch.float64)).clamp_(max=V - 1)
        inside = torch.rand(m, generator=g, device=device) < p_in
        c0 = a // size * size
        span = torch.clamp(V - c0, max=size)
        bc = c0 + (torch.rand(m, generator=g, device=device, dtype=torch.float64) * span).long()
        b = torch.where(inside, bc.clamp_(max=V - 1), b)
        lo, hi = torch.minimum(a, b), torch.maximum(a, b)
        k = (lo * V + hi)[lo != hi]
        keys = torch.unique(torch.cat([keys, k]))
        need = pairs_target - keys.numel()
        del a, b, inside, c0, span, bc, lo, hi, k
    keys = keys[torch.randperm(keys.numel(), generator=g, device=device)[:pairs_target]]
    relabel = torch.randperm(V, generator=g, device=device)
    lo, hi = relabel[keys // V], relabel[keys % V]
    del keys
    return _csr_from_pairs(lo, hi, V)


def locality_order(indptr: torch.Tensor, indices: torch.Tensor, iters: int = 20,
                   seed: int = 0) -> torch.Tensor:
    """A vertex order that makes a graph's communities contiguous: `perm[new] = old`.

    Label propagation on the device (each round a random half of the vertices takes the most
    frequent label among its neighbours, its own counted through the self loop; ties go to
    a per-round random hash of the label, so no label floods by id, and updating half the
    vertices per round keeps neighbours from swapping labels back and forth), then vertices
    sorted by (label, old id).  Once per graph; apply with permute_graph.  On a randomly
    labelled graph without structure it returns an arbitrary order and costs nothing later."""
    V = indptr.numel() - 1
    dev = indices.device
    rows = torch.repeat_interleave(torch.arange(V, device=dev), torch.diff(indptr.long()))
    cols = indices.long()
    lab = torch.arange(V, device=dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    for _ in range(iters):
        h = torch.randint(0, 1 << 20, (V,), generator=g, device=dev)  # tie-break hash per label
        uniq, cnt = torch.unique(rows * V + lab[cols], return_counts=True)
        r, lb = uniq // V, uniq % V
        score = (cnt << 20) | h[lb]
        del uniq, cnt
        best = torch.full((V,), -1, dtype=torch.int64, device=dev).scatter_reduce_(
            0, r, score, "amax", include_self=True)
        cand = torch.where(score == best[r], lb, torch.full_like(lb, V))
        new = torch.full((V,), V, dtype=torch.int64, device=dev).scatter_reduce_(
            0, r, cand, "amin", include_self=True)
        move = (torch.rand(V, generator=g, device=dev) < 0.5) & (new < V)
        new = torch.where(move, new, lab)
        del r, lb, score, cand, best, move
        lab = new
    return torch.argsort(lab * V + torch.arange(V, device=dev))


def degree_order(indptr: torch.Tensor) -> torch.Tensor:
    """Vertices by decreasing degree (ties by id): `perm[new] = old`.  A probe of how much
    the pull backward gains when heavy destinations share buckets."""
    deg = torch.diff(indptr.long())
    return torch.sort(-deg, stable=True).indices


def permute_graph(indptr: torch.Tensor, indices: torch.Tensor, perm: torch.Tensor):
    """The CSR of the graph relabelled by `perm` (perm[new] = old): row and column i of the
    result are vertex perm[i].  Returns (indptr int32, indices int32, edge_perm int64) with
    sorted columns; edge_perm[e'] is the old edge id of new edge e' (values_new =
    values[edge_perm]).  Features follow with x[perm], outputs go back with y[inv]."""
    V = indptr.numel() - 1
    dev = indices.device
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(V, device=dev)
    rows = torch.repeat_interleave(torch.arange(V, device=dev), torch.diff(indptr.long()))
    key = inv[rows] * V + inv[indices.long()]
    key, eperm = torch.sort(key)
    src, dst = key // V, key % V
    ip = torch.zeros(V + 1, dtype=torch.int64, device=dev)
    ip[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0)
    return ip.to(torch.int32), dst.to(torch.int32), eperm
