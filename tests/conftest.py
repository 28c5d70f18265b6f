import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spgemm-prunning_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("MAXK_VALIDATE", "1")  # tests validate CSR/selector ranges before launch


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def _ensure_lib():
    """Incremental make every session: a library older than any source is rebuilt, and
    test_library_built_from_tree checks the loaded library's source digest against the tree
    (MAXK_HIP_LIB, a variant under test, is left alone)."""
    lib = os.path.join(PKG, "lib", "libmaxk_hip.so")
    if "MAXK_HIP_LIB" not in os.environ:
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG])
    return lib


_ensure_lib()


def golden_cases():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_golden(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
