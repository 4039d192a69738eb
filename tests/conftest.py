import importlib
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    return {
        "inputs": dict(np.load(os.path.join(GOLDEN, "inputs_h.npz"))),
        "ref": dict(np.load(os.path.join(GOLDEN, "ref_vectors.npz"))),
        "matlab": dict(np.load(os.path.join(GOLDEN, "matlab_pins.npz"))),
    }


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.load()
    return oracle_py


def _ensure_libwce():
    """Build libwce.so unless it exists AND was linked from exactly the
    current sources (content hash written by the Makefile beside it): a
    pushed, older library is rebuilt, never tested silently."""
    pkg = os.path.join(REPO, "80211parallelestimation_amd")
    lib = os.path.join(pkg, "libwce.so")
    sys.path.insert(0, pkg)
    import srchash
    stamp = lib + ".srchash"
    fresh = os.path.exists(lib) and os.path.exists(stamp) and open(stamp).read().strip() == srchash.source_hash()
    if not fresh:
        subprocess.check_call(["make", "-C", os.path.join(pkg, "csrc"), "-B", "-j8"], stdout=subprocess.DEVNULL)
    return lib


@pytest.fixture(scope="session")
def wce():
    _ensure_libwce()
    mod = importlib.import_module("80211parallelestimation_amd")
    mod.load()
    return mod


@pytest.fixture(scope="session")
def gpu_wce(wce):
    # GPU tests must run on the HIP path: fail (not skip) if the device is absent.
    n = wce.device_count()
    assert n > 0, "gpu test without a HIP device"
    return wce
