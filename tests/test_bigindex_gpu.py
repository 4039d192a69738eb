"""Element indices past 2^31: frames laid out with a 64 MB frame stride, so
that frame 599 starts at complex element 2.5e9 (40 GB into each buffer).
Every estimator path must index in 64 bits; the outputs must equal those of
the same frames packed densely, bit for bit (the reference's frames are
independent, main.c:41-53, so the layout may not change a single bit)."""
import numpy as np
import pytest

from oracle_py import N, NBLK

pytestmark = pytest.mark.gpu

B = 600
S = 1 << 22                     # frame stride in complex elements (64 MB)


@pytest.fixture(scope="module")
def layouts(gpu_wce, golden):
    wce = gpu_wce
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    tx, rx, pre = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=99)
    wce.synchronize()
    assert (B - 1) * S + NBLK * N > 2**31
    big = [wce.DeviceArray((B * S,)) for _ in range(3)]
    lib = wce.load()
    for f in range(B):
        for dst, src, cnt in ((big[0], tx, NBLK * N), (big[1], rx, NBLK * N), (big[2], pre, N)):
            assert lib.wce_memcpy_dtod(dst.addr + f * S * 16, src.addr + f * cnt * 16, cnt * 16, None) == 0
    wce.synchronize()
    yield wce, inp, (tx, rx, pre), big
    del big


def _run(wce, ctx, fr, mask, f32=False):
    outs = [wce.DeviceArray((B, N), np.complex64 if (f32 and i < 4) else np.complex128, zero=True) for i in range(5)]
    eq = wce.DeviceArray((B, NBLK, N), np.complex64 if f32 else np.complex128, zero=True)
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32 if f32 else 0)
    ctx.estimate(fr, o, mask)
    wce.synchronize()
    return [x.numpy() for x in outs] + [eq.numpy()]


@pytest.mark.parametrize("mode,mask,f32,sem", [
    ("TEXTBOOK", "PS_MMSE", False, "C"),             # mmse_solve_fc_kernel
    ("REF", "PS_MMSE", False, "C"),                  # mmse_ref_flat_kernel
    ("TEXTBOOK", "LT_LS|PS_LINEAR", False, "C"),     # ls_elem_kernel
    ("TEXTBOOK", "ALL", True, "C"),                  # fused solve + LS family + equalization, fp32 outputs
    ("COV", "PS_MMSE", False, "C"),                  # dense solve + MFMA apply
    ("COV8", "PS_MMSE", False, "C"),                 # 8-tap PDP: one frame per lane, mmse_lr_lane_staged_kernel<8, 1, true>
    ("COV8", "PS_MMSE", False, "MATLAB"),            # the same, split per-block solves + block mean
    ("COV12", "PS_MMSE", False, "C"),                # 12 taps: 16 lanes per frame, mmse_lr_quad_kernel<12, true>
    ("COV24", "PS_MMSE", False, "C"),                # 24 taps: 16 lanes, two rows each, mmse_lr_quad2_kernel<24>
    ("COV24", "PS_MMSE", False, "MATLAB"),           # the same, split per-block solves
    ("REF", "ALL", True, "C"),                       # ref_ls_elem_kernel, fp32 LS / eq
    ("TEXTBOOK", "PS_MMSE|FRAME_COV", False, "C"),   # per-frame covariance: factor matvecs + solve
    ("REF", "PS_MMSE|FRAME_COV", False, "C"),        # ref_fc_kernel: LT_LS, factors and H = u s in one launch
    ("REF", "ALL|FRAME_COV", True, "C"),             # ref_fc_kernel factors, then ref_ls_elem_kernel
    ("TEXTBOOK", "LS_ALL", False, "MATLAB"),         # ls_kernel, MATLAB semantics (4-block averages)
    ("TEXTBOOK", "PS_MMSE|FRAME_COV", False, "MATLAB"),   # split per-block solves + fc_finish
])
def test_64bit_frame_indexing(layouts, mode, mask, f32, sem):
    wce, inp, (tx, rx, pre), big = layouts
    if mode == "COV":
        p = np.exp(-0.12 * np.arange(N))
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=np.diag(p / p.sum()).astype(np.complex128) * 1.1e-4)
    elif mode.startswith("COV"):
        L = int(mode[3:])
        p = np.zeros(N)
        p[:L] = np.exp(-0.5 * np.arange(L))
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=np.diag(p / p.sum()).astype(np.complex128) * 1.1e-4)
        assert ctx.cov_info()[:2] == (L, True)
        units = B * (4 if sem == "MATLAB" else 1)
        assert ctx.lr_kernel(units) == {8: "mmse_lr_lane_staged_kernel<8, 1, true>", 12: "mmse_lr_quad_kernel<12, true>",
                                        24: "mmse_lr_quad2_kernel<24>"}[L]
    else:
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], getattr(wce, "MMSE_" + mode))
    m = 0
    ctx.reserve(B)
    for name in mask.split("|"):
        m |= getattr(wce, name)
    se = getattr(wce, "SEM_" + sem)
    dense = ctx.frames(tx, rx, B, rx_pre=pre, semantics=se)
    strided = ctx.frames(big[0], big[1], B, frame_stride=S, rx_pre=big[2], pre_stride=S, semantics=se)
    want = _run(wce, ctx, dense, m, f32)
    got = _run(wce, ctx, strided, m, f32)
    for i, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, w), (mode, mask, i)
    assert any(np.any(w) for w in want)
