"""The HBM kernels' variants (wce_debug_set_variant) are interchangeable:
bit-identical outputs on ragged batch sizes, across launch splits
(wce_debug_set_flat_chunk), for fp64 and fp32 outputs.  LS configs[1]: one
element per thread (ls_elem_kernel, default, 2) against the per-frame LIGHT
kernel (3); REF: 512-element chunks on a capped grid (default, 0) against an
uncapped grid (2).  (Round 4 retired ls_flat_kernel and the 64-frame REF
tiles from the library.)"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, NBLK = 53, 15


@pytest.fixture()
def lib(gpu_wce):
    lib = gpu_wce.load()
    yield lib
    assert lib.wce_debug_set_variant(0, 0) == 0
    assert lib.wce_debug_set_variant(1, 2) == 0
    assert lib.wce_debug_set_variant(4, 0) == 0
    assert lib.wce_debug_set_flat_chunk(ctypes.c_longlong(0)) == 0


@pytest.mark.parametrize("chunk", [0, 4096])
def test_ls_variants_identical(gpu_wce, golden, lib, chunk):
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_REF)
    B = 40003
    tx, rx, pre = gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=0x1A)
    assert lib.wce_debug_set_flat_chunk(ctypes.c_longlong(chunk)) == 0
    for f32, dt in ((0, np.complex128), (gpu_wce.OUT_LS_F32, np.complex64)):
        got = []
        for v in (2, 3):
            assert lib.wce_debug_set_variant(1, v) == 0
            lt, lin = gpu_wce.DeviceArray((B, N), dt, zero=True), gpu_wce.DeviceArray((B, N), dt, zero=True)
            ctx.estimate(ctx.frames(tx, rx, B, rx_pre=pre),
                         gpu_wce.Outputs(lt.addr, lin.addr, None, None, None, None, N, 0, 0, 0, f32),
                         gpu_wce.LT_LS | gpu_wce.PS_LINEAR)
            gpu_wce.synchronize()
            got.append((lt.numpy(), lin.numpy()))
        assert np.array_equal(got[1][0], got[0][0]) and np.array_equal(got[1][1], got[0][1]), f32


@pytest.mark.parametrize("frame_cov", [False, True])
def test_ref_variants_identical(gpu_wce, golden, lib, frame_cov):
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_REF)
    B = 33331
    tx, rx, pre = gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=0x2B)
    ctx.reserve(B)
    mask = gpu_wce.PS_MMSE | (gpu_wce.FRAME_COV if frame_cov else 0)
    # per-frame factors reach the REF read-out through the four-launch
    # FRAME_COV path (which 4 = 1); the default fuses it into ref_fc_kernel
    assert lib.wce_debug_set_variant(4, 1 if frame_cov else 0) == 0
    got = []
    for v in (0, 1, 2, 3):
        assert lib.wce_debug_set_variant(0, v) == 0
        H = gpu_wce.DeviceArray((B, N), zero=True)
        ctx.estimate(ctx.frames(tx, rx, B, rx_pre=pre if frame_cov else None),
                     gpu_wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0), mask)
        gpu_wce.synchronize()
        got.append(H.numpy())
    assert np.isfinite(got[0]).all()
    for g in got[1:]:
        assert np.array_equal(g, got[0])


def test_ref_frame_cov_ls_variant_full_w_rows(gpu_wce, golden, lib):
    """REF + FRAME_COV + the LS family on the wave-per-frame REF_LS variant
    (1) reads all 53 rows of w: the factor launch must write them, not only
    the 4 pilot rows.  The workspace is first filled with NaN
    by a call on NaN preambles; the next call must be finite and agree with
    the default one-element-per-thread form (0)."""
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_REF)
    B = 4099
    tx, rx, pre = gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=0x3C)
    ctx.reserve(B)
    nanpre = gpu_wce.DeviceArray.from_numpy(np.full((B, N), np.nan + 1j * np.nan))
    mask = gpu_wce.ALL | gpu_wce.FRAME_COV
    got = []
    try:
        for v in (0, 1):
            assert lib.wce_debug_set_variant(2, v) == 0
            outs = [gpu_wce.DeviceArray((B, N), zero=True) for _ in range(5)]
            eq = gpu_wce.DeviceArray((B, NBLK, N), zero=True)
            o = gpu_wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, 0)
            ctx.estimate(ctx.frames(tx, rx, B, rx_pre=nanpre), o, mask)      # poisons the workspace
            ctx.estimate(ctx.frames(tx, rx, B, rx_pre=pre), o, mask)
            gpu_wce.synchronize()
            got.append([x.numpy() for x in outs] + [eq.numpy()])
    finally:
        assert lib.wce_debug_set_variant(2, 0) == 0
    for a, b in zip(got[0], got[1]):
        assert np.isfinite(b).all()
        scale = np.abs(a).max(axis=-1, keepdims=True)
        assert (np.abs(a - b) <= 1e-12 * scale).all()
