"""GPU parity for MATLAB semantics (wce_frames.semantics = WCE_SEM_MATLAB,
SURVEY 8(f)-3): proper conj in LT_LS, pilot estimators averaged over blocks
1-4, MATLAB's cubic divisors, MMSE averaged over the per-block solves.

Pinned directly by the reference's MATLAB workspace (matlab.mat, saved by
WiFi_RX.m:47-60): H_EST_{LT_LS,PS_Linear,PS_Cubic,PS_Sinc,PS_Third} and
eq_symbols.  matlab.mat holds no MMSE output, so PS_MMSE in this mode is
checked against the oracle's textbook solve averaged over blocks 1-4
(WiFi_channel_estimation_PS_MMSE.m:28-34) and its closed form."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu

TOL = 1e-10
TOL_LS = 1e-13


def _ow2(m):
    """WiFi_RX.m:30 (K = 64)."""
    d = m["rx_preamble2"] - m["rx_preamble1"]
    return float(np.sum((d * d.conj()).real) / (2 * 64))


@pytest.fixture(scope="module")
def ml(gpu_wce, golden):
    m = golden["matlab"]
    ctx = gpu_wce.Context(m["tx_preamble_fft"], m["rx_preamble_fft"], _ow2(m), gpu_wce.MMSE_TEXTBOOK)
    tx, rx = m["tx_symb"].T[None].copy(), m["rx_symb"].T[None].copy()   # MATLAB [53][15] -> [1][15][53]
    out = ctx.estimate_host(tx, rx, rx_pre=m["rx_preamble_fft"][None], mask=gpu_wce.ALL,
                            semantics=gpu_wce.SEM_MATLAB)
    return m, ctx, out


@pytest.mark.parametrize("name,key", [("lt_ls", "H_EST_LT_LS"), ("ps_linear", "H_EST_PS_Linear"),
                                      ("ps_cubic", "H_EST_PS_Cubic"), ("ps_sinc", "H_EST_PS_Sinc"),
                                      ("ps_cubic", "H_EST_PS_Third")])
def test_matlab_estimators_pinned(ml, name, key):
    m, _, out = ml
    assert normrel(out[name][0], m[key]) < TOL_LS
    if name == "lt_ls":
        assert out[name][0, 26] == 0


def test_matlab_equalization_pinned(ml):
    """WiFi_Equalization.m with the MATLAB LT_LS and PS_Linear estimates."""
    m, _, out = ml
    ref = m["eq_symbols"].T
    got = out["eq"][0]
    assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-13
    assert np.all(got[:, 26] == 0)


def test_matlab_shared_preamble_lt_ls(gpu_wce, ml):
    """Without a per-frame preamble the state's LT_LS is used (C quirk
    cancels: same estimate to rounding)."""
    m, ctx, _ = ml
    out = ctx.estimate_host(m["tx_symb"].T[None], m["rx_symb"].T[None], mask=gpu_wce.LT_LS,
                            semantics=gpu_wce.SEM_MATLAB)
    assert normrel(out["lt_ls"][0], m["H_EST_LT_LS"]) < 1e-14


def test_matlab_mmse_block_average(gpu_wce, golden, oracle, ml):
    """PS_MMSE.m: textbook solve per block 1-4, averaged.  Oracle: long double
    unified solve per block; closed form beta_b H_LT per block."""
    m, ctx, out = ml
    ow2 = _ow2(m)
    tx, rx = m["tx_symb"].T, m["rx_symb"].T
    hls = oracle.matlab_lt_ls(m["tx_preamble_fft"], m["rx_preamble_fft"])
    C = oracle.mmse_textbook_cmatrix(oracle.fmatrix(), hls)
    per = [oracle.mmse_unified(C, np.ones(N, np.uint8), 1, ow2, tx[b], rx[b]) for b in range(4)]
    ref = np.mean(np.stack(per), axis=0)
    assert normrel(out["ps_mmse"][0], ref) < TOL
    F = oracle.fmatrix()
    cvec = F @ (F.conj() @ hls / N)
    closed = np.mean([oracle.mmse_textbook_closed(cvec, tx[b], rx[b], ow2) for b in range(4)], axis=0)
    assert normrel(out["ps_mmse"][0], closed) < TOL


def test_matlab_batch_vs_oracle(gpu_wce, golden, oracle):
    """Device-generated frames with distinct blocks: every frame's LS family
    in MATLAB semantics matches the oracle's 4-block MATLAB functions; MMSE
    matches the oracle's block-averaged solve on sampled frames."""
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    hlt, C, a, b = ctx.shared()
    B = 512
    tx = gpu_wce.DeviceArray((B, NBLK, N), np.complex128)
    rx = gpu_wce.DeviceArray((B, NBLK, N), np.complex128)
    # frames carry the preamble's channel (as in WiFi_RX.m); with an unrelated
    # channel the textbook Ryy has cond ~4e6 and fp64 agrees only to ~1e-9
    ctx.synth(tx, rx, None, B, seed=0x5EED, h_shared=gpu_wce.DeviceArray.from_numpy(hlt))
    gpu_wce.synchronize()
    txh, rxh = tx.numpy(), rx.numpy()
    out = ctx.estimate_host(txh, rxh, mask=gpu_wce.LS_ALL | gpu_wce.PS_MMSE, semantics=gpu_wce.SEM_MATLAB)
    mask = np.ones(N, np.uint8)
    rng = np.random.default_rng(11)
    for f in np.concatenate([[0, B - 1], rng.choice(B, 14, replace=False)]):
        for name in ("ps_linear", "ps_cubic", "ps_sinc"):
            assert normrel(out[name][f], oracle.matlab(name, txh[f], rxh[f])) < TOL_LS, (f, name)
        per = [oracle.mmse_unified(C, mask, a, b, txh[f, k], rxh[f, k]) for k in range(4)]
        assert normrel(out["ps_mmse"][f], np.mean(np.stack(per), axis=0)) < TOL, f
    # blocks beyond 3 do not influence the MATLAB estimates
    txh2, rxh2 = txh.copy(), rxh.copy()
    txh2[:, 4:], rxh2[:, 4:] = 1.0, 0.0
    out2 = ctx.estimate_host(txh2, rxh2, mask=gpu_wce.LS_ALL | gpu_wce.PS_MMSE, semantics=gpu_wce.SEM_MATLAB)
    for name in ("ps_linear", "ps_cubic", "ps_sinc", "ps_mmse"):
        assert np.array_equal(out[name], out2[name]), name


def test_matlab_semantics_errors(gpu_wce, golden):
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_REF)
    tx = gpu_wce.DeviceArray((2, NBLK, N), np.complex128)
    rx = gpu_wce.DeviceArray((2, NBLK, N), np.complex128)
    h = gpu_wce.DeviceArray((2, N), zero=True)
    o = gpu_wce.Outputs(None, h.addr, None, None, None, None, N, 0, 0, 0, 0)
    with pytest.raises(gpu_wce.WceError):
        ctx.estimate(ctx.frames(tx, rx, 2, semantics=7), o, gpu_wce.PS_LINEAR)
    with pytest.raises(gpu_wce.WceError):   # MATLAB semantics reads 4 blocks: block stride >= 53
        ctx.estimate(ctx.frames(tx, rx, 2, block_stride=1, semantics=gpu_wce.SEM_MATLAB), o, gpu_wce.PS_LINEAR)
    with pytest.raises(gpu_wce.WceError):   # the profiling entry point takes C semantics only
        ctx.mmse_solve(ctx.frames(tx, rx, 2, semantics=gpu_wce.SEM_MATLAB), h, N)
