"""Model, not product: texture-path cycles of the pull backward's G' gathers for lane layouts,
on the synthetic Reddit graph's real tile streams (CPU).

Cost model (tools/ta_probe.hip on MI355X, L2-resident data): a dword gather wave instruction
costs, per 16-lane quarter, max(4, distinct 128-B lines the quarter touches) cycles; a
dwordx2/x4 instruction costs, per 4-lane group, max(1, distinct lines) cycles (16 groups).
Selectors: a uniform random k-subset per destination (what top-k of random features gives),
sorted.  Tiles: rows cut into S slices, destinations into 2^shift buckets, entries of a tile
in CSR order (row, column).
    python tools/pull_model.py [--graph reddit] [--k 16] [--tiles 24]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="reddit")
ap.add_argument("--k", type=int, default=16)
ap.add_argument("--slices", type=int, default=66)
ap.add_argument("--shift", type=int, default=10)
ap.add_argument("--tiles", type=int, default=24)
ap.add_argument("--cache", default="/tmp/pull_model_graph.npz")
ap.add_argument("--seg", type=int, default=64, help="bytes per tag access unit")
a = ap.parse_args()
SEGS = 1024 // a.seg

if os.path.exists(a.cache):
    z = np.load(a.cache)
    rp, col = z["rp"], z["col"]
else:
    r, c = maxk_graph.synthetic_graph(a.graph, device="cpu")
    rp, col = r.numpy().astype(np.int64), c.numpy()
    np.savez(a.cache, rp=rp, col=col)
V, E, k = len(rp) - 1, len(col), a.k
rng = np.random.default_rng(5)
sel = np.sort(np.argsort(rng.random((V, 256)), axis=1)[:, :k], axis=1).astype(np.int32)
rps = -(-V // a.slices)
nb = -(-V // (1 << a.shift))
rows = np.repeat(np.arange(V), np.diff(rp))


def tile(t):
    s, j = divmod(t, nb)
    lo, hi = rp[s * rps], rp[min(V, (s + 1) * rps)]
    r, c = rows[lo:hi], col[lo:hi]
    m = (c >> a.shift) == j
    return r[m], c[m]


L2_LINES = [0]


def quarter_cost(lines, group):  # lines: [n_instr, 64] line ids (-1 = idle lane)
    n = lines.shape[0]
    x = np.sort(lines, axis=1)  # lines each instruction requests from L2 (no L1 reuse)
    L2_LINES[0] += ((np.diff(x, axis=1) != 0).sum(1) + 1 - (x[:, 0] < 0)).sum()
    q = lines.reshape(n, 64 // group, group)
    cost = 0
    for g in range(q.shape[1]):
        x = np.sort(q[:, g, :], axis=1)
        d = (np.diff(x, axis=1) != 0).sum(1) + 1 - (x[:, 0] < 0)
        cost += np.maximum(d, 1 if group == 4 else 4).sum()
    return cost


def layout_A(r, c, LR):
    """LR lanes per entry, k/LR values per lane; instruction i gathers sorted positions
    i*LR + q (the i-th of k/LR quantile bands) of 64/LR consecutive entries."""
    n = len(r)
    epi = 64 // LR
    pad = (-n) % epi
    rr = np.concatenate([r, np.full(pad, -1)])
    cc = np.concatenate([c, np.zeros(pad, np.int64)])
    ni = len(rr) // epi
    S = sel[cc]  # [n, k]
    cost = 0
    for i in range(k // LR):
        pos = i * LR + np.arange(LR)
        ln = rr[:, None] * SEGS + S[:, pos] // (256 // SEGS)  # [n, LR]
        ln[rr < 0] = -1
        cost += quarter_cost(ln.reshape(ni, 64), 16)
    return cost


def layout_rowalign(r, c, LR):
    """As A, but a quarter (16/LR entries) never mixes rows: each row's run is padded to a
    multiple of the entries per quarter."""
    epq = 16 // LR
    _, start, cnt = np.unique(r, return_index=True, return_counts=True)
    pr, pc = [], []
    for s0, n0 in zip(start, cnt):
        p = (-n0) % epq
        pr.append(np.concatenate([r[s0:s0 + n0], np.full(p, -1)]))
        pc.append(np.concatenate([c[s0:s0 + n0], np.zeros(p, np.int64)]))
    return layout_A(np.concatenate(pr), np.concatenate(pc), LR)


tot = {}
n_ent = 0
ts = rng.choice(a.slices * nb, size=a.tiles, replace=False)
for t in ts:
    r, c = tile(int(t))
    n_ent += len(r)
    for LR in (1, 2, 4, 8, 16):
        if LR > k:
            continue
        for nm, f in (("A", layout_A), ("rowalign", layout_rowalign)):
            if nm == "rowalign" and LR < 2:
                continue
            L2_LINES[0] = 0
            cyc = f(r, c, LR)
            key = f"{nm} LR={LR}"
            o = tot.get(key, (0, 0))
            tot[key] = (o[0] + cyc, o[1] + L2_LINES[0])
print(f"{a.graph} V={V} E={E} k={k} S={a.slices} shift={a.shift}: {a.tiles} tiles, "
      f"{n_ent} entries ({n_ent / a.tiles:.0f} per tile)")
for name, (cyc, l2) in tot.items():
    per = cyc / n_ent
    ms = per * E / 256 / 2.4e6
    l2e = l2 / n_ent
    l2ms = l2e * 128 * E / 34.5e9
    print(f"  {name:16s} {per:6.2f} TA cycles per entry -> {ms:5.2f} ms at 2.4 GHz;  "
          f"{l2e:5.2f} L2 lines per entry -> {l2ms:5.2f} ms at 34.5 TB/s")

# floor: every (row, tile) run fetches each line its entries touch exactly once
lines_min = 0
for t in ts:
    r, c = tile(int(t))
    ln = r[:, None] * 8 + sel[c] // 32
    lines_min += len(np.unique(ln))
print(f"  floor: {lines_min / n_ent:5.2f} distinct lines per entry (each (row, tile) line once)")
for H in (2, 4):
    if k % H or k // H < 4:
        continue
    kp = k // H
    lm = 0
    for t in ts:
        r, c = tile(int(t))
        for h in range(H):
            ln = r[:, None] * 8 + sel[c][:, h * kp:(h + 1) * kp] // 32
            lm += len(np.unique(ln))
    print(f"  floor with {H} parts (sorted positions split by rank): {lm / n_ent:5.2f} lines per entry")


def layout_parts(r, c, LR, H):
    """H rank parts (part h: sorted positions [h*kp, (h+1)*kp)), each a pass over the tile's
    entries with LR lanes per entry; instruction i of part h gathers positions h*kp + i*LR + q."""
    kp = k // H
    n = len(r)
    epi = 64 // LR
    pad = (-n) % epi
    rr = np.concatenate([r, np.full(pad, -1)])
    cc = np.concatenate([c, np.zeros(pad, np.int64)])
    ni = len(rr) // epi
    S = sel[cc]
    cost = 0
    for h in range(H):
        for i in range(kp // LR):
            pos = h * kp + i * LR + np.arange(LR)
            ln = rr[:, None] * SEGS + S[:, pos] // (256 // SEGS)
            ln[rr < 0] = -1
            cost += quarter_cost(ln.reshape(ni, 64), 16)
    return cost


if os.environ.get("PARTS"):
    print("parts (rank split): TA cycles and L2 lines (no L1 reuse) per entry")
    for H in (1, 2, 4):
        for LR in (2, 4, 8, 16):
            if k % H or LR > k // H:
                continue
            cyc = l2 = 0
            for t in ts:
                r, c = tile(int(t))
                L2_LINES[0] = 0
                cyc += layout_parts(r, c, LR, H)
                l2 += L2_LINES[0]
            print(f"  H={H} LR={LR:2d} VPL={k // H // LR:2d}: {cyc / n_ent:6.2f} TA cyc  "
                  f"{l2 / n_ent:5.2f} L2 lines per entry")


def order_hybrid(r, c, epq, T):
    """Entries of a tile reordered: rows whose run is >= T first, each run padded to a
    multiple of epq (dummy entries -1), then the shorter runs packed in CSR order."""
    u, start, cnt = np.unique(r, return_index=True, return_counts=True)
    lr, lc, sr, sc = [], [], [], []
    for s0, n0 in zip(start, cnt):
        if n0 >= T:
            p = (-n0) % epq
            lr.append(np.concatenate([r[s0:s0 + n0], np.full(p, -1)]))
            lc.append(np.concatenate([c[s0:s0 + n0], np.zeros(p, np.int64)]))
        else:
            sr.append(r[s0:s0 + n0])
            sc.append(c[s0:s0 + n0])
    rr = np.concatenate(lr + sr) if lr or sr else r
    cc = np.concatenate(lc + sc) if lc or sc else c
    return rr, cc


if os.environ.get("HYBRID"):
    H = int(os.environ.get("H", "2"))
    LR = k // H // 4
    epq = 16 // LR
    print(f"hybrid order, H={H} parts, LR={LR} (tag model: max(4, lines) per quarter)")
    for T in (0, 4, 8, 16, 32):
        cyc = l2 = pads = 0
        for t in ts:
            r, c = tile(int(t))
            rr, cc = (r, c) if T == 0 else order_hybrid(r, c, epq, T)
            pads += (rr < 0).sum()
            L2_LINES[0] = 0
            cyc += layout_parts(rr, np.where(rr < 0, 0, cc), LR, H)
            l2 += L2_LINES[0]
        print(f"  T={T:2d}: {cyc / n_ent:6.2f} TA cyc/entry  {l2 / n_ent:5.2f} L2 lines/entry (no L1)  "
              f"padding {pads / n_ent:.1%}")

if os.environ.get("DEGSORT"):
    # relabel vertices by descending degree (rows and columns alike) and redo the floor
    deg = np.diff(rp)
    order = np.argsort(-deg, kind="stable")
    newid = np.empty(V, np.int64)
    newid[order] = np.arange(V)
    r2 = newid[rows]
    c2 = newid[col]
    o = np.lexsort((c2, r2))
    rows, col = r2[o], c2[o].astype(np.int32)
    rp = np.zeros(V + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=V), out=rp[1:])
    sel = sel[order]  # selectors follow their vertex
    lm = 0
    n2 = 0
    cyc = 0
    for t in ts:
        r, c = tile(int(t))
        n2 += len(r)
        if len(r):
            lm += len(np.unique(r[:, None] * 8 + sel[c] // 32))
            cyc += layout_A(r, c, 4)
    print(f"degree-sorted labels: {n2} entries in the same tiles; floor {lm / max(n2,1):5.2f} lines/entry, "
          f"TA model LR=4 {cyc / max(n2,1):5.2f} cyc/entry")
    # all tiles weighted: sample more tiles uniformly over entries
    tot_l = tot_e = 0
    for t in rng.choice(a.slices * nb, size=64, replace=False):
        r, c = tile(int(t))
        if len(r):
            tot_l += len(np.unique(r[:, None] * 8 + sel[c] // 32))
            tot_e += len(r)
    print(f"  64 random tiles: floor {tot_l / tot_e:5.2f} lines/entry over {tot_e} entries")

if os.environ.get("ROWSTAGE"):
    # rows whose run in a tile is >= T entries: one coalesced 1-KB load of the row per
    # (row, tile, part) = 4 quarters x max(4, 2 lines) = 16 cycles, the values then picked
    # from registers; shorter runs as now (layout_parts, CSR order)
    H = int(os.environ.get("H", "2"))
    LR = k // H // 4
    print(f"row-staged hybrid, H={H} parts, LR={LR}: TA cycles per entry")
    for T in (0, 4, 8, 16, 32, 64):
        cyc = ent_long = 0
        for t in ts:
            r, c = tile(int(t))
            u, start, cnt = np.unique(r, return_index=True, return_counts=True)
            longm = np.repeat(cnt >= T if T else np.zeros_like(cnt, bool), cnt)
            order = np.argsort(r, kind="stable")  # r already sorted (CSR order)
            ent_long += longm.sum()
            lg = cnt[cnt >= T] if T else cnt[:0]
            # per part: the row (16) and its entries, one b64 per lane per 64 (16 each)
            cyc += H * int((16 + 16 * -(-lg // 64)).sum())
            rs, cs = r[~longm], c[~longm]
            if len(rs):
                cyc += layout_parts(rs, cs, LR, H)
        print(f"  T={T:3d}: {cyc / n_ent:6.2f} TA cyc/entry (all parts)  long-run entries {ent_long / n_ent:.1%}")
