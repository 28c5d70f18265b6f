"""The compiled C++ consumer of include/maxk_hip.h (spgemm-prunning_amd/harness/
maxk_kernel_test.cpp): the reference's kernel benchmark (kernels/main.cu:50-221, timing
spmm_base.h:34-61) built against the C ABI alone.  CPU: it builds and starts; GPU: on a golden
fixture graph it reproduces the fixture's forward and backward outputs (--inputs / --dump,
every backward mode), and its benchmark run prints the reference's lines and passes the
reference's own forward check (check_err, main.cu:19-48)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, golden_cases, load_golden

BIN = os.path.join(PKG, "bin", "maxk_kernel_test")


def run(*args, timeout=300):
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=timeout)


def test_harness_builds_and_starts():
    assert os.access(BIN, os.X_OK), "make -C spgemm-prunning_amd builds bin/maxk_kernel_test"
    r = run("--help")
    assert r.returncode == 0 and "usage:" in r.stdout
    r = run("--bwd", "nope", "g")
    assert r.returncode == 1 and "--bwd" in r.stderr


def test_harness_no_device(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    r = run("g")
    assert r.returncode == 4 and "no HIP device" in r.stderr


def _write_graph(d, z):
    z["row_ptr"].astype(np.int32).tofile(os.path.join(d, "g.indptr"))
    z["col_idx"].astype(np.int32).tofile(os.path.join(d, "g.indices"))


@pytest.mark.gpu
@pytest.mark.parametrize("bwd", ["auto", "pull", "csc", "hybrid", "bsort", "atomic"])
@pytest.mark.parametrize("path", golden_cases()[:4], ids=lambda p: os.path.basename(p)[:-4])
def test_harness_reproduces_golden(cuda, tmp_path, path, bwd):
    z = load_golden(path)
    k, D = int(z["k"]), int(z["D"])
    if bwd in ("bsort", "hybrid") and k % 4:
        pytest.skip("needs k % 4 == 0")
    if bwd in ("pull", "hybrid") and D % 4:
        pytest.skip("needs D % 4 == 0")
    _write_graph(tmp_path, z)
    inp = tmp_path / "in"
    out = tmp_path / "out"
    inp.mkdir()
    out.mkdir()
    z["val"].astype(np.float32).tofile(inp / "val.f32")
    z["topk_val"].astype(np.float32).tofile(inp / "cbsr_val.f32")
    z["topk_idx"].astype(np.uint8).tofile(inp / "cbsr_idx.u8")
    z["g"].astype(np.float32).tofile(inp / "grad.f32")
    z["deg"].astype(np.float32).tofile(inp / "row_div.f32")
    r = run("g", "--dir", str(tmp_path), "--k", str(k), "--dim", str(D), "--bwd", bwd,
            "--inputs", str(inp), "--dump", str(out), "--runs", "1", "--lib-runs", "1")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "num graph dim_origin dim_k kernel time(ms)"
    assert [ln.split()[4] for ln in lines[1:]] == ["cusparse", "maxk", "maxk_backward"]
    V = z["row_ptr"].size - 1
    y = np.fromfile(out / "y.f32", np.float32).reshape(V, D)
    gs = np.fromfile(out / "gs.f32", np.float32).reshape(V, k)
    for got, ref in ((y, z["y_ref"]), (gs, z["grad_cbsr_ref"])):
        err = np.abs(got.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= 1e-4, err.max()


@pytest.mark.gpu
def test_harness_benchmark_run(cuda, tmp_path):
    """The reference's own run: random inputs from default_random_engine(123), k = 16, 32, 64,
    the library once, then MaxK forward and backward; --check passes the reference's
    check_err against the library SpMM for every k."""
    z = load_golden(next(c for c in golden_cases() if "sym_d256_k16" in c))
    _write_graph(tmp_path, z)
    r = run("g", "--dir", str(tmp_path), "--check")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "num graph dim_origin dim_k kernel time(ms)"
    kernels = [(ln.split()[3], ln.split()[4]) for ln in lines if ln.startswith("1/1 g 256")]
    assert kernels == [("16", "cusparse"), ("16", "maxk"), ("16", "maxk_backward"),
                       ("32", "maxk"), ("32", "maxk_backward"), ("64", "maxk"),
                       ("64", "maxk_backward")]
    assert r.stdout.count("validation pass!") == 3
