"""CPU: the C-ABI library loads, exports every symbol include/maxk_hip.h declares,
validates arguments on the host, and the Python surfaces refuse to compute
without a GPU (no fallback).  No kernel is launched here."""
import ctypes
import os
import re

import pytest
import torch

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "maxk_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(maxk_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_path():
    syms = declared_symbols()
    for s in ("maxk_spgemm_forward", "maxk_sspmm_backward", "maxk_topk_cbsr",
              "maxk_warp4_build", "maxk_warp4_to_row_ptr", "maxk_cbsr_scatter_dense",
              "maxk_dense_spmm_run", "maxk_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libmaxk_hip.so"))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_every_symbol():
    from maxk_cuda_kernels import _capi
    assert set(_capi.SIGNATURES) == set(declared_symbols())


def test_version_and_device_probe():
    import maxk_cuda_kernels as mk
    assert mk.version() == 100
    assert mk.device_count() >= 0  # 0 here (no GPU); never raises


def source_digest():
    """The Makefile's DIGEST: SHA-256 of csrc/*.hip|*.cpp|*.h and include/maxk_hip.h,
    concatenated in C-locale order of their paths relative to spgemm-prunning_amd/."""
    import glob
    import hashlib
    paths = [os.path.relpath(p, PKG) for pat in ("*.hip", "*.cpp", "*.h")
             for p in glob.glob(os.path.join(PKG, "csrc", pat))]
    paths.append(os.path.join("..", "include", "maxk_hip.h"))
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(os.path.join(PKG, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


@pytest.mark.skipif("MAXK_HIP_LIB" in os.environ, reason="a tuning variant is under test")
def test_library_built_from_tree():
    """The loaded libmaxk_hip.so was compiled from exactly the sources in this tree (the GPU
    tests run whatever library is present, so a stale binary would otherwise go unnoticed)."""
    from maxk_cuda_kernels import _capi
    assert _capi.load().maxk_source_digest().decode() == source_digest()


@pytest.mark.skipif("MAXK_HIP_LIB" in os.environ, reason="a tuning variant is under test")
def test_library_build_config_is_default():
    """The product library carries no MAXK_* tuning or ablation macro (EXTRA_HIPFLAGS)."""
    from maxk_cuda_kernels import _capi
    assert _capi.load().maxk_build_config().decode() == ""


def test_flagged_build_fails_provenance():
    """A library built with a tuning macro (tools/ builds) gets a digest that
    differs from the tree's, so test_library_built_from_tree rejects it (make -n: the digest
    the Makefile would bake in, nothing compiled)."""
    import subprocess
    cmd = ["make", "-n", "-B", "-C", PKG, "OBJDIR=/tmp/maxk_prov_obj", "OUTDIR=/tmp/maxk_prov_lib"]
    out_plain = subprocess.run(cmd, capture_output=True, text=True, check=True).stdout
    out_abl = subprocess.run(cmd + ["EXTRA_HIPFLAGS=-DMAXK_PULL_QU=4"], capture_output=True,
                             text=True, check=True).stdout
    dig = lambda out: re.search(r"MAXK_SRC_DIGEST='\"([0-9a-f]+)\"'", out).group(1)  # noqa: E731
    flags = lambda out: re.search(r"MAXK_BUILD_FLAGS='\"([^\"]*)\"'", out).group(1)  # noqa: E731
    assert dig(out_plain) == source_digest()
    assert dig(out_abl) != source_digest()
    assert flags(out_plain) == "" and flags(out_abl) == "-DMAXK_PULL_QU=4"


def test_host_side_argument_validation():
    from maxk_cuda_kernels import _capi
    L = _capi.load()
    # k > D, D > 256, negative sizes: rejected before any HIP call
    assert L.maxk_spgemm_forward(None, None, None, None, None, None, None, 10, 10, 0, 64, 65, 0,
                                 None, 0, None) == -1
    assert b"dim_k" in L.maxk_last_error()
    assert L.maxk_spgemm_forward(None, None, None, None, None, None, None, 10, 10, 0, 257, 16, 0,
                                 None, 0, None) == -1
    assert L.maxk_sspmm_backward(None, None, None, None, None, None, None, -1, 10, 0, 64, 16, 0,
                                 None, 0, None) == -1
    assert L.maxk_topk_cbsr(None, 64, None, None, None, 10, 64, 0, None) == -1
    assert L.maxk_topk_cbsr(None, 32, None, None, None, 10, 64, 8, None) == -1  # ld_x < D
    # forward needs a workspace when rows exist
    assert L.maxk_spgemm_forward(ctypes.c_void_p(16), None, None, None, None, None,
                                 ctypes.c_void_p(16), 10, 10, 0, 64, 16, 0, None, 0, None) == -1
    assert b"workspace" in L.maxk_last_error()
    # the reference-convention uint8 top-k: rows of 256 bytes, 1 <= k <= 256
    assert L.maxk_topk_u8_reference(None, None, None, 10, 128, 16, None) == -1
    assert b"256" in L.maxk_last_error()
    assert L.maxk_topk_u8_reference(None, None, None, 10, 256, 0, None) == -1
    assert L.maxk_topk_u8_reference(None, None, None, 10, 256, 16, None) == -1  # NULL buffers
    assert L.maxk_topk_u8_reference(None, None, None, 0, 256, 16, None) == 0
    # empty problems are valid no-ops
    assert L.maxk_spgemm_forward(None, None, None, None, None, None, None, 0, 0, 0, 64, 16, 0,
                                 None, 0, None) == 0
    assert L.maxk_last_error() == b""


def test_workspace_sizes():
    from maxk_cuda_kernels import _capi
    L = _capi.load()
    # slabs: one D-row per work item + a row id per item
    n = L.maxk_spgemm_forward_workspace_size(1000, 1000, 100000, 256, 16, 512)
    items = -(-101000 // 512)
    assert n >= items * (256 * 4 + 4) + 1000 * 128  # slabs + row ids + packed CBSR records
    assert L.maxk_spgemm_forward_workspace_size(0, 0, 0, 256, 16, 0) > 0  # one item minimum
    assert L.maxk_warp4_build_workspace_size(1000) >= 2 * 4000


def test_binding_refuses_cpu_tensors():
    import maxk_cuda_kernels as mk
    x = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match="CUDA"):
        mk.topk_cbsr(x, 2)
    ip = torch.zeros(5, dtype=torch.int32)
    with pytest.raises(RuntimeError, match="CUDA"):
        mk.spgemm_forward(ip, torch.zeros(0, dtype=torch.int32), torch.zeros(0),
                          torch.zeros(4, 2), torch.zeros(4, 2, dtype=torch.uint8), 8)


def test_autograd_surface_no_cpu_fallback():
    import maxk_spgemm_function as F
    assert F.MAXK_KERNELS_AVAILABLE is True
    ip = torch.tensor([0, 1, 2], dtype=torch.int32)
    idx = torch.tensor([1, 0], dtype=torch.int32)
    val = torch.ones(2)
    x = torch.randn(2, 8, requires_grad=True)
    with pytest.raises(RuntimeError):
        F.maxk_spgemm(idx, val, x, 2, graph_indptr=ip)
    w = F.MaxKSpmmWrapper("does_not_exist")
    assert w.load_metadata() is False  # reference contract: report and return False


def test_backward_mode_resolution():
    """mode "auto": pull for k % 4 == 0 or k <= 64, dim % 4 == 0 and >= 1/2 edge per (source
    row, bucket) or a small G, else csc; "bsort" refuses k % 4 != 0, "pull" k % 4 != 0 above
    64 and dim % 4 != 0; unknown modes are rejected (no silent fallback), "bucket" (removed in
    r06) among them; a dense graph past the pull's 256 x 65536 rows goes to csc."""
    import maxk_cuda_kernels as mk
    reddit = dict(num_e=114_615_891, num_cols=232_965, num_rows=232_965)
    products = dict(num_e=123_718_280, num_cols=2_449_029, num_rows=2_449_029)
    assert mk._bwd_mode("auto", 16, **reddit) == "pull"
    assert mk._bwd_mode("auto", 16, **reddit, dim=256) == "pull"
    assert mk._bwd_mode("auto", 16, **reddit, dim=9) == "csc"
    assert mk._bwd_mode("auto", 8, **reddit) == "pull"
    assert mk._bwd_mode("auto", 32, **reddit) == "pull"
    assert mk._bwd_mode("auto", 64, **reddit) == "pull"
    proteins = dict(num_e=79_122_504, num_cols=132_534, num_rows=132_534)
    assert mk._bwd_mode("auto", 64, **proteins) == "pull"
    assert mk._bwd_mode("auto", 32, **products) == "csc"
    assert mk._bwd_mode("auto", 16, **products, dim=256) == "csc"
    # a sparse graph whose vertex order groups its neighbours (pull_locality >= 1.5): "hybrid"
    # (the C ABI's rule on the locality; tests/test_hybrid_gpu.py reads it off real CSRs)
    from maxk_cuda_kernels import _capi
    L = _capi.load()
    P = (products["num_rows"], products["num_cols"], products["num_e"])
    assert L.maxk_backward_mode_auto(*P, 256, 32, 2.0) == 3    # MAXK_BWD_HYBRID
    assert L.maxk_backward_mode_auto(*P, 256, 32, 1.5) == 3
    assert L.maxk_backward_mode_auto(*P, 256, 32, 1.02) == 1   # MAXK_BWD_CSC
    assert L.maxk_backward_mode_auto(*P, 256, 32, -1.0) == 1   # locality unknown
    assert L.maxk_backward_mode_auto(*P, 256, 30, 9.0) == 1    # k % 4 != 0
    assert L.maxk_backward_mode_auto(*P, 9, 32, 9.0) == 1      # dim % 4 != 0
    R = (reddit["num_rows"], reddit["num_cols"], reddit["num_e"])
    assert L.maxk_backward_mode_auto(*R, 256, 16, 1.0) == 0    # MAXK_BWD_PULL
    assert L.maxk_backward_mode_auto(*R, -1, 16, -1.0) == 0    # dim unknown
    # a small gradient (Flickr, 23 MB) stays cache-resident: pull however sparse the graph
    flickr = dict(num_e=989_006, num_cols=89_250, num_rows=89_250)
    assert mk._bwd_mode("auto", 16, **flickr) == "csc"
    assert mk._bwd_mode("auto", 16, **flickr, dim=128) == "pull"
    assert mk._bwd_mode("auto", 10, **flickr, dim=64) == "pull"
    assert mk._bwd_mode("auto", 16, **flickr, dim=9) == "csc"
    assert mk._bwd_mode("auto", 12, **reddit) == "pull"
    assert mk._bwd_mode("auto", 10, **reddit) == "pull"  # one l per lane below k % 4
    assert mk._bwd_mode("auto", 66, **reddit) == "csc"
    assert mk._bwd_mode("auto", 16, **products) == "csc"
    # k <= 8 on the sparse graph: window-sorted contribution rows (a window of
    # maxk_bsort_window(k) edges holds >= 2 rows per destination bucket on average)
    assert mk._bwd_mode("auto", 8, **products) == "bsort"
    assert mk._bwd_mode("auto", 4, **products, dim=256) == "bsort"
    assert mk._bwd_mode("auto", 12, **products) == "csc"
    assert L.maxk_backward_mode_auto(*P, 256, 8, 1.02) == 5   # MAXK_BWD_BSORT
    assert L.maxk_backward_mode_auto(*P, 256, 8, 2.0) == 3    # locality still asks for hybrid
    W8, S8 = L.maxk_bsort_window(8), L.maxk_bucket_shift(8)
    big = W8 * (1 << S8) // 2  # the most columns whose windows keep 2 rows per bucket
    assert L.maxk_backward_mode_auto(big, big, 50 * big, 256, 8, -1.0) == 5
    assert L.maxk_backward_mode_auto(big + 1, big + 1, 50 * big, 256, 8, -1.0) == 1
    assert mk._bwd_mode("bsort", 8, **reddit) == "bsort"
    with pytest.raises(RuntimeError):
        mk._bwd_mode("bsort", 6, **reddit)
    # a shard of 1/8 of the rows keeps Reddit's per-row degree: still the pull form
    assert mk._bwd_mode("auto", 16, num_e=14_326_986, num_cols=232_968, num_rows=29_121) == "pull"
    with pytest.raises(RuntimeError, match="backward mode must be one of"):
        mk._bwd_mode("bucket", 16, **reddit)
    huge = 256 * 65536 + 1  # Reddit's density past the pull's row limit: csc
    assert L.maxk_backward_mode_auto(huge, huge, 492 * huge, 256, 16, -1.0) == 1
    assert mk._bwd_mode("csc", 16, **reddit) == "csc"
    assert mk._bwd_mode("atomic", 3, **reddit) == "atomic"
    with pytest.raises(RuntimeError):
        mk._bwd_mode("pull", 66, **reddit)
    with pytest.raises(RuntimeError):
        mk._bwd_mode("pull", 16, **reddit, dim=9)
    with pytest.raises(RuntimeError):
        mk._bwd_mode("nope", 16, **reddit)
    # k >= D / 2 at D <= 128 (r05): the dense route, both directions
    assert mk._bwd_mode("dense", 16, **reddit) == "dense"
    with pytest.raises(RuntimeError):
        mk._bwd_mode("dense", 6, **reddit)
    with pytest.raises(RuntimeError):
        mk._bwd_mode("dense", 16, **reddit, dim=9)
    assert mk._bwd_mode("auto", 32, **flickr, dim=64) == "dense"
    assert mk._bwd_mode("auto", 64, **flickr, dim=64) == "dense"
    # small narrow graphs at D / 4 <= k < D / 2: the dense backward's pick form (r05)
    assert mk._bwd_mode("auto", 28, **flickr, dim=64) == "dense"
    assert mk._bwd_mode("auto", 16, **flickr, dim=64) == "dense"
    assert mk._bwd_mode("auto", 8, **flickr, dim=64) == "pull"
    assert mk._bwd_mode("auto", 16, **flickr, dim=128) == "pull"
    assert mk._bwd_mode("auto", 16, **reddit, dim=64) == "pull"  # a dense graph keeps the pull
    assert mk._bwd_mode("auto", 64, **reddit, dim=128) == "dense"
    assert mk._bwd_mode("auto", 128, **reddit, dim=256) != "dense"  # past MAXK_DENSE_DMAX
    F = (flickr["num_rows"], flickr["num_cols"], flickr["num_e"])
    assert L.maxk_backward_mode_auto(*F, 64, 32, -1.0) == 6   # MAXK_BWD_DENSE
    assert L.maxk_backward_mode_auto(*F, -1, 32, -1.0) != 6   # dim unknown: no dense route
    assert [L.maxk_dense_route(64, k) for k in (16, 30, 32, 64)] == [0, 0, 1, 1]
    assert [L.maxk_dense_route(D, 64) for D in (100, 128, 132, 256)] == [1, 1, 0, 0]


def test_bucket_shift_rule():
    """2^shift destinations of k + 1 doubles fill the 144 KiB fp64 LDS accumulator."""
    from maxk_cuda_kernels import _capi
    L = _capi.load()
    for k in (1, 4, 8, 12, 16, 32, 64, 100, 256):
        sh = L.maxk_bucket_shift(k)
        assert ((k + 1) << sh) <= 18432 < ((k + 1) << (sh + 1)), k
    assert L.maxk_bucket_shift(0) == -1
    assert L.maxk_bucket_count(232965, 10) == 228
    assert L.maxk_bucket_count(0, 10) == 0


def test_pull_slice_rule():
    """~3.5 MiB of G rows per slice and rank part (at most 3 parts' worth), clamped to
    [1, 256]; the pull workspace is G / row_div plus one fp32 partial [num_cols padded to
    buckets, k] per slice."""
    from maxk_cuda_kernels import _capi
    L = _capi.load()
    assert L.maxk_pull_slices(232965, 0, 256, 16) == 28  # Reddit: 238.6 MB of G rows, 2 parts
    assert L.maxk_pull_slices(232965, 0, 256, 8) == 44   # 1 part
    assert L.maxk_pull_slices(232965, 0, 256, 32) == 33  # 2 parts
    assert L.maxk_pull_slices(232965, 0, 256, 64) == 22  # 4 parts, factor capped at 3
    assert L.maxk_pull_slices(29121, 0, 256, 16) == 4    # one of 8 row shards
    assert L.maxk_pull_slices(1, 0, 256, 16) == 1 and L.maxk_pull_slices(0, 0, 256, 16) == 1
    assert L.maxk_pull_slices(100_000_000, 0, 256, 16) == 256
    assert L.maxk_pull_slices(2_449_029, 0, 256, 64) == 228
    assert L.maxk_pull_slices(4_000_000, 0, 16, 64) == 62  # rows in a slice stay <= 65536
    # Flickr-sized (89k rows, D = 64): 132 / 352 / 264 tiles at k = 16 / 32 / 64 would leave
    # a nearly empty last round of workgroups; the slices drop to 2 (k = 8 keeps 5: 220, one round)
    assert [L.maxk_pull_slices(89250, 0, 64, k) for k in (8, 16, 32, 64)] == [5, 2, 2, 2]
    assert [L.maxk_pull_slices(89250, 89250, 64, k) for k in (8, 16, 32, 64)] == [5, 2, 2, 2]
    # a rectangular shard (a quarter of the rows, every column): rounds counted over the
    # columns' buckets, not the rows'
    assert L.maxk_pull_slices(44625, 0, 256, 8) == 9
    assert L.maxk_pull_slices(44625, 89250, 256, 8) == 5
    gp = (232965 * 256 * 4 + 255) // 256 * 256
    selq = 2 * ((232965 * 16 + 255) // 256 * 256)  # slot-ordered selectors + their l map
    assert L.maxk_sspmm_backward_pull_workspace_size(232965, 232965, 256, 16, 65) == \
        gp + 65 * 228 * (16 << 10) * 4 + selq
    assert L.maxk_sspmm_backward_pull_workspace_size(10, 10, 0, 16, 1) == 0


def test_edge_selector_rule(monkeypatch):
    """The forward writes the per-edge selector stream for a csc / bsort backward where it
    measured a net gain (k % 4 == 0, k <= 16); MAXK_EDGE_SEL=0 / 1 force it off / on."""
    import maxk_cuda_kernels as mk
    monkeypatch.delenv("MAXK_EDGE_SEL", raising=False)
    assert [mk.edge_selectors_wanted(k) for k in (4, 8, 12, 16, 32, 64, 10)] == \
        [True, True, True, True, False, False, False]
    monkeypatch.setenv("MAXK_EDGE_SEL", "1")
    assert mk.edge_selectors_wanted(64) and not mk.edge_selectors_wanted(10)
    monkeypatch.setenv("MAXK_EDGE_SEL", "0")
    assert not mk.edge_selectors_wanted(8)


def test_edge_selector_grid_capped():
    """maxk_edge_selectors walks its words grid-stride over a capped grid, so
    num_e * k one-byte words past 2^32 (products-sized graphs at k = 64 with unaligned
    streams) still fit one grid dimension."""
    from maxk_cuda_kernels import _capi
    lib = _capi.load()
    assert lib.maxk_edge_selectors_blocks(0) == 0
    assert lib.maxk_edge_selectors_blocks(1) == 1
    assert lib.maxk_edge_selectors_blocks(256 * 1000) == 1000
    for n_words in (1 << 32, 123_718_280 * 64, 1 << 40):
        b = lib.maxk_edge_selectors_blocks(n_words)
        assert 0 < b and b * 256 < (1 << 32) and b <= 256 * 64


def test_bench_launches_its_own_ranks(monkeypatch):
    """`python bench.py --gpus N` with no WORLD_SIZE (the driver's BENCH command shape at
    N > 1) starts the N ranks as a child torch.distributed.run on 127.0.0.1 and exits with its
    status; nothing here touches a GPU (the child command is captured, not run)."""
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("MAXK_DIST_BACKEND", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3", "--warmup", "1"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]
    assert cmd[-7].endswith("bench.py")
    # no GPU here: fewer visible devices than ranks -> gloo-staged collectives
    assert seen["env"]["MAXK_DIST_BACKEND"] == "gloo"


def test_bench_binding_roofline_and_traffic_order():
    """roofline.binding: the launch's floor is the largest of the HBM,
    Infinity-Cache-line and tag-rate terms, its fraction at most 1 for a launch no faster
    than the floor; counters are read from the newest round, its final build first."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    files = [os.path.relpath(p, ROOT) for p in bench.traffic_files()]
    rounds = [int(p.split(os.sep)[1][1:]) for p in files]
    assert rounds == sorted(rounds, reverse=True)
    for i, p in enumerate(files[:-1]):
        nxt = files[i + 1]
        if p.split(os.sep)[1] == nxt.split(os.sep)[1]:  # same round: final/ first
            assert p.endswith(os.path.join("final", "traffic.json"))
    rec = {"bytes": 13.0e9, "tag_accesses": 1.13e9}
    b = bench.binding_roofline(2.1248, 1.175e9, rec)
    assert b["bound"] == "tag_rate" and 0 < b["frac"] <= 1
    assert b["terms_ms"]["fabric_lines"] == round(13.0e9 / 8.6e12 * 1e3, 4)
    b = bench.binding_roofline(1.59, 1.2e9, {"bytes": 11.9e9})
    assert b["bound"] == "fabric_lines" and b["frac"] <= 1
    b = bench.binding_roofline(1.0, 1e9, None)
    assert b["bound"] == "hbm_compulsory" and b["frac"] == 0.125

