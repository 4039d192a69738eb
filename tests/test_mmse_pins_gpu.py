"""The MMSE kernels against WiFi_channel_estimation_PS_MMSE.m's formula as the
reference's OWN routines compute it: multiply() and the cofactor inverse() of
utils.c composed in its long double complex (oracle/ref_harness.cpp:
refh_mmse_formula, fixtures from tests/golden/make_mmse_pins.py).

This is the reference pin the TEXTBOOK headline kernel (mmse_solve_fc_kernel:
exact first pivot step, Cholesky row panels, bordered read-out) and both
WCE_MMSE_COV forms (low-rank Gram path for the 6-tap profile, dense solve +
MFMA apply for the 53-tap one) had lacked: the reference holds no MMSE
output, but it does hold the arithmetic the formula needs.  Its cofactor
inverse is accurate only up to cond(Ryy) ~4e4 (4e-9 off at the frames' own
noise power), so the pins run at ow2 = 1e-3, 1e-4, 1e-5; accuracy at the
frames' own cond ~4e6 is covered by tests/test_accuracy_gpu.py and
tests/test_cov_lowrank_gpu.py against the long double oracle."""
import os

import numpy as np
import pytest

from oracle_py import N, NBLK, from_split, normrel

pytestmark = pytest.mark.gpu
PINS = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "mmse_formula_pins.npz")))


@pytest.mark.parametrize("kind", ["textbook", "pdp6", "pdp53"])
def test_mmse_vs_reference_routines(gpu_wce, golden, kind):
    wce = gpu_wce
    inp = golden["inputs"]
    tx = np.zeros((PINS["frames_tx"].shape[0], NBLK, N), np.complex128)
    rx = np.zeros_like(tx)
    tx[:, 0], rx[:, 0] = PINS["frames_tx"], PINS["frames_rx"]
    worst = 0.0
    for wi, ow2 in enumerate(PINS["ow2"]):
        if kind == "textbook":
            ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], float(ow2), wce.MMSE_TEXTBOOK)
        else:
            ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], float(ow2), Rhh=PINS["rhh_" + kind])
            assert ctx.cov_info()[1] == (kind == "pdp6")       # rank 6: low-rank path; 53 taps: dense
        H = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"]
        for f in range(tx.shape[0]):
            worst = max(worst, float(normrel(H[f], from_split(PINS["H_" + kind][wi, f]))))
    print(f"\n{kind}: max norm-relative error vs the reference's routines {worst:.2e}")
    assert worst < 1e-10, worst
