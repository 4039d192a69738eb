"""GPU parity for per-frame-covariance MMSE (WCE_MMSE_FRAME_COV):
Rhh_f from each frame's own preamble, i.e. main.c's PS_MMSE called per frame
with H_EST_LS = that frame's LT_LS (REF), or WiFi_channel_estimation_PS_MMSE.m
with the frame's H_EST_LT_LS (TEXTBOOK).  Oracles: the bit-exact REF-repaired
restatement (pinned to the compiled reference) and the long double unified
solve with the frame's own C_f."""
import numpy as np
import pytest

from oracle_py import N, NBLK, from_split, normrel

pytestmark = pytest.mark.gpu

TOL = 1e-10


def _frames(tx0, rx0):
    B = tx0.shape[0]
    tx = np.zeros((B, NBLK, N), np.complex128)
    rx = np.zeros((B, NBLK, N), np.complex128)
    tx[:, 0], rx[:, 0] = tx0, rx0
    return tx, rx


def test_ref_per_frame_preamble_golden(gpu_wce, golden, oracle):
    """REF: frames alternate between the two golden preambles; expected =
    main.c's PS_MMSE with that frame's own LT_LS (oracle bit-exact to the
    reference); frames on preamble 0 equal the reference's golden output."""
    r = golden["ref"]
    ctx = gpu_wce.Context(r["pre_tx"][0], r["pre_rx"][0], r["ow2"], gpu_wce.MMSE_REF)
    tx, rx = _frames(r["frames_tx"], r["frames_rx"])
    B = tx.shape[0]
    pre = np.stack([r["pre_rx"][f % 2] for f in range(B)])
    out = ctx.estimate_host(tx, rx, rx_pre=pre, mask=gpu_wce.PS_MMSE | gpu_wce.FRAME_COV)["ps_mmse"]
    F, invF = from_split(r["F"]), from_split(r["invF"])
    for f in range(B):
        hls = oracle.lt_ls(r["pre_tx"][0], pre[f])
        exp = oracle.mmse_ref_repaired(tx[f, 0], rx[f, 0], F, r["ow2"], hls, invF)
        assert normrel(out[f], exp) < TOL, f
        if f % 2 == 0:
            assert normrel(out[f], from_split(r["ps_mmse_ref"][0][f])) < TOL, f


@pytest.mark.parametrize("mode", ["ref", "textbook"])
def test_frame_cov_with_shared_preamble_equals_shared_mode(gpu_wce, golden, mode):
    """Every frame carrying the context's own preamble: the per-frame path
    (rank-1 factors, no apply GEMM) reproduces the shared-C path."""
    inp = golden["inputs"]
    m = gpu_wce.MMSE_REF if mode == "ref" else gpu_wce.MMSE_TEXTBOOK
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m)
    hlt, _, _, _ = ctx.shared()
    B = 300
    tx = gpu_wce.DeviceArray((B, NBLK, N))
    rx = gpu_wce.DeviceArray((B, NBLK, N))
    ctx.synth(tx, rx, None, B, seed=21, h_shared=gpu_wce.DeviceArray.from_numpy(hlt))
    gpu_wce.synchronize()
    txh, rxh = tx.numpy(), rx.numpy()
    pre = np.repeat(inp["rx_pre"][None], B, axis=0)
    for sem in (gpu_wce.SEM_C, gpu_wce.SEM_MATLAB):
        a = ctx.estimate_host(txh, rxh, mask=gpu_wce.PS_MMSE, semantics=sem)["ps_mmse"]
        b = ctx.estimate_host(txh, rxh, rx_pre=pre, mask=gpu_wce.PS_MMSE | gpu_wce.FRAME_COV,
                              semantics=sem)["ps_mmse"]
        assert normrel(b, a).max() < 1e-11, (mode, sem)


def test_textbook_per_frame_vs_oracle(gpu_wce, golden, oracle):
    """TEXTBOOK with per-frame channels and preambles (device-generated):
    sampled frames against the long double solve with the frame's own C_f
    and against the closed form beta_f c_f."""
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 2000
    tx = gpu_wce.DeviceArray((B, NBLK, N))
    rx = gpu_wce.DeviceArray((B, NBLK, N))
    pre = gpu_wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=99)
    gpu_wce.synchronize()
    txh, rxh, preh = tx.numpy(), rx.numpy(), pre.numpy()
    ctx.reserve(B)
    outs = ctx.estimate_host(txh, rxh, rx_pre=preh, mask=gpu_wce.PS_MMSE | gpu_wce.FRAME_COV | gpu_wce.LT_LS)
    F = oracle.fmatrix()
    ones = np.ones(N, np.uint8)
    rng = np.random.default_rng(4)
    for f in np.concatenate([[0, B - 1], rng.choice(B, 10, replace=False)]):
        hls = oracle.lt_ls(inp["tx_pre"], preh[f])
        assert normrel(outs["lt_ls"][f], hls) < 1e-13
        C = oracle.mmse_textbook_cmatrix(F, hls)
        exp = oracle.mmse_unified(C, ones, 1, inp["ow2"], txh[f, 0], rxh[f, 0])
        assert normrel(outs["ps_mmse"][f], exp) < TOL, f
        cvec = F @ (F.conj() @ hls / N)
        closed = oracle.mmse_textbook_closed(cvec, txh[f, 0], rxh[f, 0], inp["ow2"])
        assert normrel(outs["ps_mmse"][f], closed) < TOL, f


def test_matlab_per_frame_preamble(gpu_wce, golden, oracle):
    """MATLAB semantics: each frame's LT_LS (proper conj) feeds its own
    PS_MMSE.m covariance; 4-block average vs the oracle."""
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 64
    tx = gpu_wce.DeviceArray((B, NBLK, N))
    rx = gpu_wce.DeviceArray((B, NBLK, N))
    pre = gpu_wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=123)
    gpu_wce.synchronize()
    txh, rxh, preh = tx.numpy(), rx.numpy(), pre.numpy()
    out = ctx.estimate_host(txh, rxh, rx_pre=preh, mask=gpu_wce.PS_MMSE | gpu_wce.FRAME_COV,
                            semantics=gpu_wce.SEM_MATLAB)["ps_mmse"]
    F = oracle.fmatrix()
    ones = np.ones(N, np.uint8)
    for f in (0, 17, B - 1):
        hls = oracle.matlab_lt_ls(inp["tx_pre"], preh[f])
        C = oracle.mmse_textbook_cmatrix(F, hls)
        per = [oracle.mmse_unified(C, ones, 1, inp["ow2"], txh[f, b], rxh[f, b]) for b in range(4)]
        assert normrel(out[f], np.mean(np.stack(per), axis=0)) < TOL, f


def test_frame_cov_errors(gpu_wce, golden):
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_REF)
    tx = gpu_wce.DeviceArray((2, NBLK, N), zero=True)
    rx = gpu_wce.DeviceArray((2, NBLK, N), zero=True)
    h = gpu_wce.DeviceArray((2, N), zero=True)
    o = gpu_wce.Outputs(None, None, None, None, h.addr, None, N, 0, 0, 0, 0)
    with pytest.raises(gpu_wce.WceError):   # modifier without PS_MMSE
        ctx.estimate(ctx.frames(tx, rx, 2), o, gpu_wce.FRAME_COV)
    with pytest.raises(gpu_wce.WceError):   # needs per-frame preambles
        ctx.estimate(ctx.frames(tx, rx, 2), o, gpu_wce.PS_MMSE | gpu_wce.FRAME_COV)
    with pytest.raises(gpu_wce.WceError):
        ctx.reserve(-1)


@pytest.mark.parametrize("mask_name", ["MMSE", "ALL", "MMSE_LIN"])
@pytest.mark.parametrize("f32", [False, True])
def test_ref_fused_factor_kernel_equals_four_launches(gpu_wce, golden, oracle, mask_name, f32):
    """REF + FRAME_COV in C semantics runs ref_fc_kernel (round 5 form): LT_LS
    of the frame's preamble, u = Mu h (Mu = F invF_ref) on MFMA, w at the 4
    pilot rows from the folded 80-bit real map State::Wp (g = invF h is never
    formed), s and H = u s -- H is always written by this launch; when the
    call also asks for LS outputs they come from a second launch,
    ref_ls_elem_kernel with mmse_done = 1.  The four-launch variant path
    (WCE_VARIANT_REF_FC = 1: LT_LS pass, matvec launches, ref_w_kernel from the
    same Wp, REF read-out) rounds alike, so H and every LS output are
    bit-identical between the two, on a ragged batch (not a multiple of 16
    frames), block 2 of the frame, a caller tx_pre, and a non-dense output
    stride.  Against main.c's PS_MMSE with the frame's own LT_LS (the oracle,
    main.c:37-53, 148-205) parity is held by tolerance, not bitwise: the Wp
    fold rounds once where main.c rounds g, q(g) and w separately."""
    wce = gpu_wce
    lib = wce.load()
    r = golden["ref"]
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
    B = 1037
    tx, rx, pre = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=0xFC)
    wce.synchronize()
    t, x, p = tx.numpy(), rx.numpy(), pre.numpy()
    p[1] = r["pre_rx"][1]                                   # a golden preamble of its own
    tpre = inp["tx_pre"] * (1.0 + 0.0j)
    mask = {"MMSE": wce.PS_MMSE, "ALL": wce.ALL, "MMSE_LIN": wce.PS_MMSE | wce.PS_LINEAR}[mask_name] | wce.FRAME_COV
    got = {}
    try:
        for v in (0, 1):
            assert lib.wce_debug_set_variant(4, v) == 0
            got[v] = ctx.estimate_host(t, x, rx_pre=p, mask=mask, block=2, tx_pre=tpre, ls_f32=f32)
    finally:
        assert lib.wce_debug_set_variant(4, 0) == 0
    for k in got[0]:
        assert np.array_equal(got[0][k], got[1][k]), k
    H = got[0]["ps_mmse"]
    assert np.isfinite(H).all()
    F, invF = from_split(r["F"]), from_split(r["invF"])
    for f in (0, 1, 2, 511, B - 1):
        hls = oracle.lt_ls(tpre, p[f])
        exp = oracle.mmse_ref_repaired(t[f, 2], x[f, 2], F, inp["ow2"], hls, invF)
        assert normrel(H[f], exp) < TOL, f


@pytest.mark.parametrize("B", [1, 15, 16, 17, 33])
def test_ref_fc_kernel_small_ragged_batches(gpu_wce, golden, oracle, B):
    """ref_fc_kernel (persistent, 16-frame tiles) on batches of 1..33 frames:
    the last tile partially live, waves without a tile leaving at once; each
    frame against main.c's PS_MMSE with its own LT_LS (the bit-exact oracle),
    and the four-launch variant bit for bit."""
    wce = gpu_wce
    lib = wce.load()
    r = golden["ref"]
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
    tx, rx, pre = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=0x1F0 + B)
    wce.synchronize()
    t, x, p = tx.numpy(), rx.numpy(), pre.numpy()
    got = {}
    try:
        for v in (0, 1):
            assert lib.wce_debug_set_variant(4, v) == 0
            got[v] = ctx.estimate_host(t, x, rx_pre=p, mask=wce.PS_MMSE | wce.FRAME_COV)["ps_mmse"]
    finally:
        assert lib.wce_debug_set_variant(4, 0) == 0
    assert np.array_equal(got[0], got[1])
    F, invF = from_split(r["F"]), from_split(r["invF"])
    for f in range(B):
        exp = oracle.mmse_ref_repaired(t[f, 0], x[f, 0], F, inp["ow2"], oracle.lt_ls(inp["tx_pre"], p[f]), invF)
        assert normrel(got[0][f], exp) < TOL, f


@pytest.mark.parametrize("B,mask_name", [(1037, "MMSE"), (1037, "MMSE_LIN_EQ"), (1, "MMSE"), (17, "MMSE"), (33, "MMSE_LIN_EQ")])
def test_textbook_fused_factor_kernel_equals_general_path(gpu_wce, golden, oracle, B, mask_name):
    """TEXTBOOK + FRAME_COV in C semantics without an LT_LS output: LT_LS of
    each preamble and u = Mu h (Mu = F conj(F) / 53) in one launch
    (ref_fc_kernel<UOUT>, round 5) where the general path (variant
    WCE_VARIANT_REF_FC = 1) runs the LT_LS pass and matvec_kernel.  Same
    arithmetic, so H and every output are bit-identical: ragged batches (1,
    17, 33, 1,037 frames), block 2, a caller tx_pre, a non-dense output
    stride; sampled frames against the long double solve with the frame's
    own C_f (WiFi_channel_estimation_PS_MMSE.m:26-33 on its own H_LT)."""
    wce = gpu_wce
    lib = wce.load()
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    tx, rx, pre = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, seed=0x7B + B)
    wce.synchronize()
    t, x, p = tx.numpy(), rx.numpy(), pre.numpy()
    tpre = inp["tx_pre"] * (1.0 + 0.0j)
    mask = {"MMSE": wce.PS_MMSE, "MMSE_LIN_EQ": wce.PS_MMSE | wce.PS_LINEAR | wce.EQUALIZE}[mask_name] | wce.FRAME_COV
    got = {}
    try:
        for v in (0, 1):
            assert lib.wce_debug_set_variant(4, v) == 0
            got[v] = ctx.estimate_host(t, x, rx_pre=p, mask=mask, block=2, tx_pre=tpre)
    finally:
        assert lib.wce_debug_set_variant(4, 0) == 0
    for k in got[0]:
        assert np.array_equal(got[0][k], got[1][k]), k
    H = got[0]["ps_mmse"]
    assert np.isfinite(H).all()
    F = oracle.fmatrix()
    ones = np.ones(N, np.uint8)
    for f in sorted({0, B // 2, B - 1}):
        hls = oracle.lt_ls(tpre, p[f])
        C = oracle.mmse_textbook_cmatrix(F, hls)
        exp = oracle.mmse_unified(C, ones, 1, inp["ow2"], t[f, 2], x[f, 2])
        assert normrel(H[f], exp) < TOL, f
