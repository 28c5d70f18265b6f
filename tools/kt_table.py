"""Markdown table of the kernel-test speed-ups over the library SpMM (maxk_kernel_test.py --json
output under profiles/rNN/kernel_test/), beside the reference's A100-vs-cuSPARSE ratios read off
its chart, for DESIGN.md 6.
    python tools/kt_table.py profiles/r02/kernel_test"""
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02/kernel_test"
REF = {  # (graph, op) -> {k: ratio}, SURVEY.md 6
    ("reddit", "forward"): {8: "≈6.2×", 16: "≈5.5×", 32: "≈2.9×", 64: "≈1.5×"},
    ("reddit", "backward"): {8: "≈9.8×", 16: "≈8.0×", 32: "≈2.9×", 64: "≈1.5×"},
    ("products", "forward"): {16: "≈3.9×", 32: "≈2.8×"},
    ("products", "backward"): {16: "≈3.8×", 32: "≈2.5×"},
    ("proteins", "forward"): {16: "≈3.8×", 64: "≈1.2×"},
    ("proteins", "backward"): {16: "≈4.9×", 64: "≈1.4×"},
    ("flickr", "forward"): {16: "≈2.7×"},
    ("flickr", "backward"): {16: "≈4.2×"},
}
KS = (8, 16, 32, 64)
# the reference's headline (README.md:136; averaged as main_runner_direct.py:138-213 does: the
# mean over graphs with average degree > 50 of the library SpMM time over the MaxK kernel time)
REF_AVG = {8: 6.93, 16: 5.39, 32: 2.55, 64: 1.46}
avg = {}  # (op, "default"|"best") -> {k: [ratios]}
dense_graphs = []
print("| graph, op | k=8 | k=16 | k=32 | k=64 |")
print("|---|---|---|---|---|")
for g in ("reddit", "products", "proteins", "flickr"):
    p = os.path.join(d, f"{g}.txt")
    if not os.path.exists(p):
        continue
    js = [json.loads(line) for line in open(p) if line.startswith("{")]
    if not js:
        continue
    res = {r["k"]: r for r in js[-1]["results"]}
    lib, best = js[-1]["library_spmm_ms"], js[-1]["library_spmm_ms_best"]
    if js[-1]["E"] / js[-1]["V"] > 50:
        dense_graphs.append(g)
        for op, key in (("forward", "speedup_fwd"), ("backward", "speedup_bwd")):
            for lb, suf in (("default", ""), ("best", "_vs_best")):
                for k in KS:
                    if k in res and res[k].get(key + suf):
                        avg.setdefault((op, lb), {}).setdefault(k, []).append(res[k][key + suf])
    for op, key in (("forward", "speedup_fwd"), ("backward", "speedup_bwd")):
        ours = [f"{res[k][key]:.1f}× ({res[k][key + '_vs_best']:.1f}×)" if k in res else ""
                for k in (8, 16, 32, 64)]
        print(f"| {g} {op}, ours (vs default ({best / lib:.2f}·default best)) | " +
              " | ".join(ours) + " |" if False else
              f"| {g} {op}, ours: vs ALG_DEFAULT (vs best alg) | " + " | ".join(ours) + " |")
        ref = REF.get((g, op), {})
        print(f"| {g} {op}, reference (A100 vs cuSPARSE) | " +
              " | ".join(ref.get(k, "") for k in (8, 16, 32, 64)) + " |")
    print(f"<!-- {g}: library SpMM {lib:.2f} ms (ALG_DEFAULT), {best:.2f} ms (best: "
          f"{js[-1]['library_best_alg']}) -->")

if avg:
    print()
    print("| average over graphs with average degree > 50 | k=8 | k=16 | k=32 | k=64 |")
    print("|---|---|---|---|---|")
    for op in ("forward", "backward"):
        for lb in ("default", "best"):
            a = avg.get((op, lb), {})
            print(f"| ours, {op} vs rocSPARSE {'ALG_DEFAULT' if lb == 'default' else 'best algorithm'}"
                  f" ({', '.join(dense_graphs)}) | " +
                  " | ".join(f"{sum(a[k]) / len(a[k]):.2f}× (n={len(a[k])})" if k in a else ""
                             for k in KS) + " |")
    print("| reference, A100 vs cuSPARSE (README.md:136) | " +
          " | ".join(f"{REF_AVG[k]:.2f}×" for k in KS) + " |")
