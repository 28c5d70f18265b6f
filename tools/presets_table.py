"""Markdown table of a round's preset bench lines (profiles/rNN/presets/*.json), for DESIGN.md 6.
    python tools/presets_table.py profiles/r02/presets"""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02/presets"
ORDER = ["reddit", "reddit_bucket", "reddit_csc", "reddit_atomic", "reddit_k8", "reddit_k32",
         "reddit_k64", "products_k4", "products_k8", "products_k16", "products", "products_k32",
         "products_k64", "proteins", "flickr", "products_comm_ordered"]
rows = {}
for p in glob.glob(os.path.join(d, "*.json")):
    name = os.path.basename(p)[:-5]
    if name.startswith("train_"):
        continue
    with open(p) as f:
        rows[name] = json.load(f)
print("| graph | V | E | D | k | GTEPS | fwd ms | bwd ms (mode) | bwd roofline frac | "
      "top-k ms | rocSPARSE SpMM ms (default / best) | fwd / bwd speed-up vs best | "
      "CPU reference path GTEPS (cores) |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
for name in ORDER + sorted(set(rows) - set(ORDER)):
    if name not in rows:
        continue
    r = rows[name]
    c, e = r["config"], r["extra"]
    lib = ""
    if e.get("rocsparse_spmm_ms"):
        lib = f"{e['rocsparse_spmm_ms']:.2f} / {e['rocsparse_spmm_ms_best']:.2f}"
    topk = f"{e['topk_ms']:.2f}" if e.get("topk_ms") else ""
    sp = ""
    if e.get("speedup_fwd_vs_rocsparse_best"):
        sp = f"{e['speedup_fwd_vs_rocsparse_best']:.1f}× / {e['speedup_bwd_vs_rocsparse_best']:.1f}×"
    cpu = ""
    if r.get("cpu_baseline"):
        cpu = f"{r['cpu_baseline']['value']:.4f} ({r['cpu_baseline']['cores']})"
    graph = c["graph"] + (" (ordered)" if "ordered" in name else "")
    print(f"| {graph} | {c['V']:,} | {c['E'] / 1e6:.1f}M | {c['D']} | {c['k']} | "
          f"{r['value']:.1f} | {e['fwd_ms']:.2f} | {e['bwd_ms']:.2f} ({e['bwd_mode']}) | "
          f"{e.get('bwd_alg_GBs', r['roofline']['frac'] * 8000) / 8000:.2f} | {topk} | {lib} | "
          f"{sp} | {cpu} |")
