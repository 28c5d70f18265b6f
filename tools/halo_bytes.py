"""Model, not product: CBSR exchange bytes per rank and step of maxk_dist's two modes on the
synthetic graphs (CPU), N = 2/4/8 vertex-range shards balanced by nnz (balanced_bounds).

  gather: forward all-gather of every vertex's CBSR row (k x 5 B), backward reduce-scatter of
          a [world * vmax, k] fp32 partial: each rank receives (world-1) * vmax rows forward
          and sends as many k x 4 B rows backward.
  halo:   only the rows a shard's edges touch (its distinct remote columns) travel, each way.
    python tools/halo_bytes.py [--graph products] [--k 32] [--reorder]
--reorder relabels the graph by maxk_graph.locality_order first (a planted-community graph,
--graph products_comm, then keeps most edges inside a shard)."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_dist  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="products")
ap.add_argument("--k", type=int, default=None)
ap.add_argument("--reorder", action="store_true")
ap.add_argument("--device", default="cpu")
a = ap.parse_args()
k = a.k or maxk_graph.PRESETS[a.graph]["k"]
rp, col = maxk_graph.synthetic_graph(a.graph, device=a.device)
if a.reorder:
    rp, col, _ = maxk_graph.permute_graph(rp, col, maxk_graph.locality_order(rp, col))
rp, col = rp.cpu(), col.cpu()
V, E = rp.numel() - 1, col.numel()
print(f"{a.graph} (synthetic{', locality order' if a.reorder else ''}) V={V} E={E} k={k}: "
      f"MB per rank and step (max over ranks), "
      f"forward receive + backward send")
for world in (2, 4, 8):
    b = maxk_dist.balanced_bounds(rp, world)
    vmax = max(b[i + 1] - b[i] for i in range(world))
    halo_rows = []
    for p in range(world):
        e0, e1 = int(rp[b[p]]), int(rp[b[p + 1]])
        c = torch.unique(col[e0:e1].long())
        remote = int(((c < b[p]) | (c >= b[p + 1])).sum())
        halo_rows.append(remote)
    g_fwd = (world - 1) * vmax * k * 5
    g_bwd = (world - 1) * vmax * k * 4
    h = max(halo_rows)
    print(f"  N={world}: gather {(g_fwd + g_bwd) / 1e6:8.1f} MB (fwd {g_fwd / 1e6:.1f} + bwd "
          f"{g_bwd / 1e6:.1f});  halo {h * k * 9 / 1e6:8.1f} MB ({h} remote rows = "
          f"{h / (V - vmax):.1%} of the other ranks' rows)")
