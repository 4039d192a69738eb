"""The headline mode (TEXTBOOK, WiFi_channel_estimation_PS_MMSE.m:26-32) on the
GPU against an INDEPENDENT evaluation of the .m formula at its operating
noise power (ow2 = 9.6172e-8, cond(Ryy) ~ 4e6): tests/golden/make_textbook_mp.py
forms F, Rhh = ifft(H_EST) ifft(H_EST)', Ryy and pinv(Ryy) literally in
mpmath at 50 digits (no closed form, nothing from the oracle).  Frames: the
inputs.h frame, 8 frames of the bench's own seed-0x80211 batch, 4 frames with
unrelated channels (one QPSK).  North-star tolerance 1e-10 norm-relative."""
import os

import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu

TOL = 1e-10
PINS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "textbook_mp_pins.npz")


@pytest.fixture(scope="module")
def pins():
    d = dict(np.load(PINS))
    d["H"] = d["H_hi"].astype(np.clongdouble) + d["H_lo"]
    return d


@pytest.fixture(scope="module")
def ctx(gpu_wce, golden):
    inp = golden["inputs"]
    return gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)


def test_textbook_vs_mp_literal_on_fixture_inputs(gpu_wce, ctx, pins):
    """The fixture's own fp64 inputs through the C ABI (block 0 estimated;
    the other 14 blocks are copies and do not enter C semantics)."""
    B = len(pins["tx"])
    tx = np.repeat(pins["tx"][:, None, :], NBLK, 1)
    rx = np.repeat(pins["rx"][:, None, :], NBLK, 1)
    H = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    errs = np.array([normrel(H[f], pins["H"][f]) for f in range(B)])
    print("\nGPU vs mp literal .m: max %.2e median %.2e (%d frames)" % (errs.max(), np.median(errs), B))
    assert errs.max() < TOL, errs


def test_bench_batch_frames_are_the_fixture_frames(gpu_wce, ctx, pins):
    """The bench's 65,536-frame batch generated on the device exactly as
    bench.py main() does: the picked frames' block 0 equals the fixture's
    inputs (tx exactly; rx to <= 2 ulp -- the device may fuse h*t + noise into
    one fma), and the in-HBM estimate of those frames is within 1e-10 of the
    mp literal formula."""
    B = 65536
    hs = gpu_wce.DeviceArray.from_numpy(np.ascontiguousarray(pins["h_shared"]))
    assert np.array_equal(pins["h_shared"], ctx.shared()[0])          # bench.py: hs = ctx.shared()[0]
    tx, rx = gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, NBLK, N))
    ctx.synth(tx, rx, None, B, first_frame=0, seed=int(pins["seed"]), h_shared=hs, amplitude=float(pins["amp"]))
    H = gpu_wce.DeviceArray((B, N), zero=True)
    ctx.estimate(ctx.frames(tx, rx, B), gpu_wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                 gpu_wce.PS_MMSE)
    gpu_wce.synchronize()
    sel = np.nonzero(pins["kind"] == "bench")[0]
    assert len(sel) == 8
    errs = []
    for i in sel:
        f = int(pins["bench_frame"][i])
        t0, r0 = tx.rows(f)[0, 0], rx.rows(f)[0, 0]
        assert np.array_equal(t0, pins["tx"][i]), f
        d = np.abs(r0 - pins["rx"][i])
        assert (d <= 2 * np.spacing(np.abs(pins["rx"][i]))).all(), (f, d.max())
        errs.append(float(normrel(H.rows(f)[0], pins["H"][i])))
    print("\nbench batch vs mp literal .m: max %.2e" % max(errs))
    assert max(errs) < TOL, errs
