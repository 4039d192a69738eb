"""WCE_MMSE_COV on the GPU against an INDEPENDENT literal evaluation of
WiFi_channel_estimation_PS_MMSE.m:26-32 with a model covariance Rhh, in
mpmath at 50 digits (tests/golden/make_cov_mp.py), at the operating noise
power ow2 = 9.6172e-8.  One profile per solve form the library selects:
4 / 8 taps (one frame per lane), 12 / 16 (16 lanes per frame), 24 (two Gram
rows per lane), 53 taps (the tap-domain wave kernel) and the full-rank
exp(-0.12 t) profile (the dense solve + MFMA C W).  Frames: inputs.h, two of
the bench batch, one QPSK frame.  North-star tolerance 1e-10; measured
~1e-13 (the CPU test in tests/test_oracle.py pins the long double oracle to
the same fixtures)."""
import os

import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu
PINS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cov_mp_pins.npz")
KERNELS = {4: "mmse_lr_lane_staged_kernel<4, 1, true>", 8: "mmse_lr_lane_staged_kernel<8, 1, true>",
           12: "mmse_lr_quad_kernel<12, true>", 16: "mmse_lr_quad_kernel<16, true>", 24: "mmse_lr_quad2_kernel<24>",
           53: "mmse_lr_kernel<0, true>"}


@pytest.fixture(scope="module")
def pins():
    return dict(np.load(PINS))


@pytest.mark.parametrize("pi", range(7))
def test_cov_vs_mp_literal(gpu_wce, golden, pins, pi):
    inp = golden["inputs"]
    L, dec = int(pins["taps"][pi]), float(pins["decay"][pi])
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=np.diag(pins["pdp"][pi]).astype(np.complex128))
    r, lowrank, _, _ = ctx.cov_info()
    kern = ctx.lr_kernel(1 << 16) if lowrank else "mmse_solve_kernel<false> + apply_kernel"
    if dec == 0.5:
        assert lowrank and kern == KERNELS[L], (L, kern)
    else:
        assert not lowrank                      # the full-rank wide profile: the dense solve
    tx = np.repeat(pins["tx"][:, None, :], NBLK, 1)
    rx = np.repeat(pins["rx"][:, None, :], NBLK, 1)
    H = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    Hm = pins["H_hi"][pi].astype(np.clongdouble) + pins["H_lo"][pi]
    errs = np.array([normrel(H[f], Hm[f]) for f in range(len(H))])
    print(f"\nL={L} decay={dec} ({kern}): max {errs.max():.2e}")
    assert errs.max() < 1e-10, errs
    assert errs.max() < 1e-12, errs
