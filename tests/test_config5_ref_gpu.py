"""BASELINE configs[4] in main.c semantics: REF PS_MMSE plus the LS family and
equalization in one call (main.c:66-212, WiFi_Equalization.m:1-9).

Since round 3 that request runs ref_ls_elem_kernel -- one HBM pass, one
(frame, subcarrier) element per thread -- instead of riding in the
wave-per-frame solve kernel.  Its outputs must equal the separate passes
(launch_ls + mmse_ref_flat_kernel) bit for bit, every mask and output
precision, shared or per-frame factors, across launch chunks; and sampled
frames must match the bit-exact oracle of main.c."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu
NAMES = ("lt_ls", "ps_linear", "ps_cubic", "ps_sinc", "ps_mmse")


@pytest.fixture(scope="module")
def frames(gpu_wce, golden):
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_REF)
    B = 3001
    tx, rx, pre = (gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, NBLK, N)),
                   gpu_wce.DeviceArray((B, N)))
    ctx.synth(tx, rx, pre, B, seed=0xC5)
    gpu_wce.synchronize()
    t, r, p = tx.numpy(), rx.numpy(), pre.numpy()
    t[0], r[0] = inp["tx_symb"], inp["rx_symb"]
    p[0] = inp["rx_pre"]
    return ctx, t, r, p


def _run(ctx, wce, t, r, p, mask, f32, variant=0, fuse=True):
    lib = wce.load()
    assert lib.wce_debug_set_variant(2, variant) == 0
    ctx.set_fusion(fuse)
    try:
        return ctx.estimate_host(t, r, rx_pre=p, mask=mask, ls_f32=f32)
    finally:
        ctx.set_fusion(True)
        assert lib.wce_debug_set_variant(2, 0) == 0


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("mask_name", ["ALL", "MMSE_LIN", "MMSE_CUB_SINC_EQ", "ALL_FC", "ALL_SHARED_PRE"])
def test_flat_equals_separate_passes(gpu_wce, frames, mask_name, f32):
    wce = gpu_wce
    ctx, t, r, p = frames
    mask = {"ALL": wce.ALL, "MMSE_LIN": wce.PS_MMSE | wce.PS_LINEAR,
            "MMSE_CUB_SINC_EQ": wce.PS_MMSE | wce.PS_CUBIC | wce.PS_SINC | wce.EQUALIZE,
            "ALL_FC": wce.ALL | wce.FRAME_COV, "ALL_SHARED_PRE": wce.ALL}[mask_name]
    pre = None if mask_name == "ALL_SHARED_PRE" else p
    flat = _run(ctx, wce, t, r, pre, mask, f32)
    sep = _run(ctx, wce, t, r, pre, mask, f32, fuse=False)
    old = _run(ctx, wce, t, r, pre, mask, f32, variant=1)
    for name in list(NAMES) + ["eq"]:
        if name not in flat:
            continue
        assert np.array_equal(flat[name], sep[name]), name
        # the wave-per-frame kernel reduces s over 64 lanes in another order
        tol = 1e-14 if name == "ps_mmse" else 0.0
        assert normrel(flat[name].reshape(len(t), -1), old[name].reshape(len(t), -1)).max() <= tol, name


def test_flat_across_launch_chunks(gpu_wce, frames):
    """53 * frames < 2^32 per launch: a 1,024-frame chunk makes the 3,001-frame
    batch take four launches (f_begin > 0), bit-identical to one."""
    wce = gpu_wce
    ctx, t, r, p = frames
    whole = _run(ctx, wce, t, r, p, wce.ALL, False)
    lib = wce.load()
    assert lib.wce_debug_set_flat_chunk(1024) == 0
    try:
        chunked = _run(ctx, wce, t, r, p, wce.ALL, False)
    finally:
        assert lib.wce_debug_set_flat_chunk(0) == 0
    for name in list(NAMES) + ["eq"]:
        assert np.array_equal(whole[name], chunked[name]), name


def test_flat_vs_oracle(gpu_wce, golden, oracle, frames):
    """Sampled frames (frame 0 = inputs.h) against main.c's own functions
    restated bit-exactly: LS family 1e-13, REF PS_MMSE 1e-10, eq 1e-12."""
    wce = gpu_wce
    ctx, t, r, p = frames
    inp, ref = golden["inputs"], golden["ref"]
    F, invF = oracle.from_split(ref["F"]), oracle.from_split(ref["invF"])
    hls_shared = oracle.lt_ls(inp["tx_pre"], inp["rx_pre"])
    out = _run(ctx, wce, t, r, p, wce.ALL, False)
    for f in [0, 1, 1500, len(t) - 1]:
        t0, r0 = t[f, 0], r[f, 0]
        hlt = oracle.lt_ls(inp["tx_pre"], p[f])
        assert normrel(out["lt_ls"][f], hlt) < 1e-13
        assert normrel(out["ps_linear"][f], oracle.ps_linear(t0, r0)) < 1e-13
        assert normrel(out["ps_cubic"][f], oracle.ps_cubic(t0, r0)) < 1e-13
        assert normrel(out["ps_sinc"][f], oracle.ps_sinc(t0, r0)) < 1e-13
        # shared-preamble C_ref (the ctx's), as main.c builds it from H_EST_LS
        mm = oracle.mmse_ref_repaired(t0, r0, F, inp["ow2"], hls_shared, invF)
        assert normrel(out["ps_mmse"][f], mm) < 1e-10
        eq = oracle.equalize(r[f], hlt, oracle.ps_linear(t0, r0))
        assert normrel(out["eq"][f].reshape(-1), eq.reshape(-1)) < 1e-12
