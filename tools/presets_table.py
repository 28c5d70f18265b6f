"""Markdown table of a round's preset bench lines (profiles/rNN/presets/*.json), for DESIGN.md 6.
    python tools/presets_table.py profiles/r05/presets

Roofline columns: each op against the ceiling that binds it
(bench.binding_roofline: the largest of its compulsory bytes at the HBM peak, its measured
fabric bytes at the Infinity Cache's random-line rate and its measured tag accesses at the
texture path's rate), from the newest counters for the line's traffic_key; the fraction is
floor / measured time and cannot pass 1.  The algorithmic-bytes rate is shown
in TB/s: it counts per-edge gathers the caches serve, so it can pass the HBM peak."""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r05/presets"
ORDER = ["reddit", "reddit_bucket", "reddit_csc", "reddit_atomic", "reddit_k8", "reddit_k32",
         "reddit_k64", "products_k4", "products_k8", "products_k16", "products", "products_k32",
         "products_k64", "proteins", "flickr", "products_comm_ordered"]
SHORT = {"hbm_compulsory": "hbm", "fabric_lines": "lines", "tag_rate": "tags"}
rows = {}
for p in glob.glob(os.path.join(d, "*.json")):
    name = os.path.basename(p)[:-5]
    if name.startswith("train_"):
        continue
    with open(p) as f:
        rows[name] = json.loads(f.read().strip().splitlines()[-1])


def binding(r, op, t_ms, which):
    c = r["config"]
    C_f, C_b = bench.compulsory_bytes(c["V"], c["E"], c["D"], c["k"])
    rec, _ = bench.load_traffic_record(r["roofline"]["traffic_key"], op)
    b = bench.binding_roofline(t_ms, C_f if which == "f" else C_b, rec)
    return f"{b['frac']:.2f} ({SHORT[b['bound']]})"


print("| graph | V | E | D | k | GTEPS | fwd ms | bwd ms (mode) | fwd / bwd vs binding ceiling | "
      "fwd / bwd alg. TB/s | top-k ms | rocSPARSE SpMM ms (default / best) | "
      "fwd / bwd speed-up vs best | CPU reference path GTEPS (cores) |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
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
    bop = f"sspmm_backward_{e['bwd_mode']}"
    bind = (f"{binding(r, 'spgemm_forward', e['fwd_ms'], 'f')} / "
            f"{binding(r, bop, e['bwd_ms'], 'b')}")
    alg = f"{e['fwd_alg_GBs'] / 1000:.2f} / {e['bwd_alg_GBs'] / 1000:.2f}"
    print(f"| {graph} | {c['V']:,} | {c['E'] / 1e6:.1f}M | {c['D']} | {c['k']} | "
          f"{r['value']:.1f} | {e['fwd_ms']:.2f} | {e['bwd_ms']:.2f} ({e['bwd_mode']}) | "
          f"{bind} | {alg} | {topk} | {lib} | {sp} | {cpu} |")
