"""WCE_MMSE_COV on constant-modulus frames (wce_ctx_set_modulus, round 4;
WiFi_channel_estimation_PS_MMSE.m:29-32).

Ryy = a X C X^H + b I depends on a frame's symbols only through P = |x|^2 and
their phases; for PSK frames P is the batch's.  K = (a C P + b I)^-1 C is then
formed once (80 bits, host) and a matching frame takes H = K (conj x o rx)
(+ the correction for non-real x) on f64 MFMA (cm_real_kernel, cm_cplx_kernel); every other frame
runs the per-frame kernels, which skip the flagged ones.  Checked here:
  - every frame against the long double unified solve with C formed in 80
    bits (oracle_py.mmse_unified) at 1e-10, sampled;
  - matching frames against the per-frame path on the same frames (the
    switch wce_debug_set_cm), and non-matching frames bit for bit;
  - mixed batches (BPSK, QPSK, 16-QAM, a frame off the pattern by one
    symbol) and batch sizes past 131,072 frames, where the dense path's
    H = C W runs apply_kernel with the skip flags.
Parity unpinned against the reference itself (it holds no MMSE output); the
oracle is the restatement of the .m file's solve."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu
TOL = 1e-10
A = 8.8753


def pdp_rhh(L, decay):
    p = np.exp(-decay * np.arange(L))
    R = np.zeros((N, N), np.complex128)
    R[np.arange(L), np.arange(L)] = p / p.sum() * 1.1e-4
    return R


def channel_rx(rng, tx, ow2):
    B = tx.shape[0]
    p = np.exp(-0.5 * np.arange(6))
    ht = (0.0105 / np.sqrt(p.sum())) * np.exp(-0.25 * np.arange(6)) * 0.7071 * (
        rng.standard_normal((B, 6)) + 1j * rng.standard_normal((B, 6)))
    h = np.einsum("bt,tk->bk", ht, np.exp(-2j * np.pi * np.outer(np.arange(6), np.arange(N) - 26) / 64))
    noise = np.sqrt(ow2 / 2) * (rng.standard_normal(tx.shape) + 1j * rng.standard_normal(tx.shape))
    return h[:, None, :] * tx + noise


def mixed_frames(rng, B, kinds):
    """tx [B][1][53]: kinds[f] in {'bpsk', 'qpsk', 'qam16', 'off'} ('off': BPSK with one symbol at 2 A)"""
    tx = np.zeros((B, 1, N), np.complex128)
    lv = np.array([-3, -1, 1, 3], float) * (A / np.sqrt(10))
    for kind in ("bpsk", "qpsk", "qam16", "off"):
        sel = np.flatnonzero(kinds == kind)
        m = len(sel)
        if kind in ("bpsk", "off"):
            v = rng.choice([-A, A], (m, 1, N)).astype(np.complex128)
            if kind == "off":
                v[:, 0, 11] *= 2.0
        elif kind == "qpsk":
            v = A * (rng.choice([-1.0, 1.0], (m, 1, N)) + 1j * rng.choice([-1.0, 1.0], (m, 1, N))) / np.sqrt(2)
        else:
            v = lv[rng.integers(0, 4, (m, 1, N))] + 1j * lv[rng.integers(0, 4, (m, 1, N))]
        tx[sel] = v
    tx[:, :, 26] = 0
    return tx


def run(ctx, wce, tx, rx, cm):
    B = tx.shape[0]
    ctx.set_cm(cm)
    try:
        dtx, drx = wce.DeviceArray.from_numpy(tx), wce.DeviceArray.from_numpy(rx)
        H = wce.DeviceArray((B, N), zero=True)
        ctx.estimate(ctx.frames(dtx, drx, B, frame_stride=N, block_stride=N),
                     wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE)
        wce.synchronize()
        assert ctx.nonfinite_scan(H, B)[1] == 0
        return H.numpy()
    finally:
        ctx.set_cm(True)


def c_ld(oracle, R):
    F = oracle.fmatrix()
    return F @ oracle._ld(R) @ F.conj().T


# (taps, decay, per-frame kernel): quad (rank 16), two rows per lane (rank 24,
# round 6), Gram wave kernel (a full-rank spectrum wider than 1e5, K0 = 0),
# dense solve + H = C W
PROFILES = [(16, 0.5, "mmse_lr_quad_kernel<16, true>"), (24, 0.3, "mmse_lr_quad2_kernel<24>"),
            (53, 0.5, "mmse_lr_kernel<0, true>"), (53, 0.12, "")]


@pytest.mark.parametrize("L,decay,kern", PROFILES)
def test_constant_modulus_batch(gpu_wce, golden, oracle, L, decay, kern):
    """A mixed batch of 4,099 frames: 1/2 BPSK, 1/4 QPSK (non-real: the
    correction launch), 1/8 16-QAM and 1/8 BPSK off the pattern by one
    symbol (both: the per-frame path)."""
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(L, decay)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.lr_kernel(64) == kern
    rng = np.random.default_rng(L * 3 + int(decay * 100))
    B = 4099
    kinds = rng.choice(["bpsk", "bpsk", "bpsk", "bpsk", "qpsk", "qpsk", "qam16", "off"], B)
    kinds[:3] = ["bpsk", "qpsk", "qam16"]
    tx = mixed_frames(rng, B, kinds)
    rx = channel_rx(rng, tx, inp["ow2"])
    x_ref = np.full(N, A + 0j)
    x_ref[26] = 0
    ctx.set_modulus(x_ref)
    got = run(ctx, wce, tx, rx, True)
    per = run(ctx, wce, tx, rx, False)
    cmf = np.isin(kinds, ["bpsk", "qpsk"])
    assert np.array_equal(got[~cmf], per[~cmf])        # the per-frame kernels, unchanged
    d = normrel(got[cmf], per[cmf])
    C = c_ld(oracle, R)
    sel = np.concatenate([[0, 1, 2, B - 1], rng.choice(B, 36, replace=False)])
    exp = np.stack([oracle.mmse_unified(C, np.ones(N, np.uint8), 1.0, inp["ow2"], tx[f, 0], rx[f, 0]) for f in sel])
    err = normrel(got[sel], exp)
    errp = normrel(per[sel], exp)
    print(f"\nL={L} decay={decay}: constant-modulus vs long double max {err[cmf[sel]].max():.2e}, "
          f"per-frame path {errp.max():.2e}; CM vs per-frame max {d.max():.2e}")
    assert err.max() < TOL, (int(sel[err.argmax()]), err.max())
    assert d.max() < 5e-13                             # both within ~1e-13 of the long double solve
    # the long double reference itself is good to ~cond(Ryy) x 1.1e-19 ~ 4e-13
    # (tests/test_oracle.py::test_textbook_closed_form_vs_mp_literal); the two
    # GPU paths agree with each other to ~1e-15 (d above)
    assert err[cmf[sel]].max() < 5e-13


def test_constant_modulus_large_batch_apply_skip(gpu_wce, golden, oracle):
    """Dense C at 140,011 frames: the per-frame path's H = C W (apply_kernel,
    several tiles per wave at this size) must leave the constant-modulus
    frames' H alone (skip flags)."""
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(53, 0.12)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    rng = np.random.default_rng(77)
    B = 140011
    kinds = np.where(rng.random(B) < 0.9, "bpsk", "qam16")
    tx = mixed_frames(rng, B, kinds)
    rx = channel_rx(rng, tx, inp["ow2"])
    ctx.set_modulus(tx[np.flatnonzero(kinds == "bpsk")[0], 0])
    got = run(ctx, wce, tx, rx, True)
    per = run(ctx, wce, tx, rx, False)
    cmf = kinds == "bpsk"
    assert np.array_equal(got[~cmf], per[~cmf])
    assert normrel(got[cmf], per[cmf]).max() < 5e-13
    C = c_ld(oracle, R)
    sel = np.concatenate([[0, B - 1], rng.choice(B, 20, replace=False)])
    exp = np.stack([oracle.mmse_unified(C, np.ones(N, np.uint8), 1.0, inp["ow2"], tx[f, 0], rx[f, 0]) for f in sel])
    assert normrel(got[sel], exp).max() < TOL


def test_constant_modulus_off_and_rank8(gpu_wce, golden):
    """x_ref None switches the path off; a rank <= 8 state keeps the lane
    kernels (bit-identical with and without a pattern); a non-COV ctx
    rejects the call."""
    wce = gpu_wce
    inp = golden["inputs"]
    rng = np.random.default_rng(5)
    B = 777
    kinds = np.full(B, "bpsk")
    tx = mixed_frames(rng, B, kinds)
    rx = channel_rx(rng, tx, inp["ow2"])
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(8, 0.5))
    ref = run(ctx, wce, tx, rx, True)
    ctx.set_modulus(tx[0, 0])
    assert np.array_equal(run(ctx, wce, tx, rx, True), ref)
    ctx16 = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(16, 0.5))
    base = run(ctx16, wce, tx, rx, True)
    ctx16.set_modulus(tx[0, 0])
    assert not np.array_equal(run(ctx16, wce, tx, rx, True), base)   # the operator path runs ...
    ctx16.set_modulus(None)
    assert np.array_equal(run(ctx16, wce, tx, rx, True), base)       # ... and is off again
    plain = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    with pytest.raises(wce.WceError):
        plain.set_modulus(tx[0, 0])


def test_set_modulus_after_load_state(gpu_wce, golden):
    """create_cov -> load_state(another COV blob) -> set_modulus must not
    re-upload the ORIGINAL state over the loaded one: the ctx
    drops its host copy, set_modulus refuses, and estimates keep running the
    loaded state.  Loading the ctx's own state back keeps set_modulus usable."""
    wce = gpu_wce
    inp = golden["inputs"]
    rng = np.random.default_rng(9)
    B = 257
    tx = mixed_frames(rng, B, np.full(B, "bpsk"))
    rx = channel_rx(rng, tx, inp["ow2"])
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(16, 0.5))
    own = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(16, 0.5))
    other_blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(24, 0.3))
    other = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(24, 0.3))
    want = run(other, wce, tx, rx, True)
    ctx.load_state(other_blob)
    with pytest.raises(wce.WceError):
        ctx.set_modulus(tx[0, 0])
    assert np.array_equal(run(ctx, wce, tx, rx, True), want)     # still the loaded state
    ctx2 = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(16, 0.5))
    ctx2.load_state(own)                                          # its own state, byte for byte
    ctx2.set_modulus(tx[0, 0])
    ctx2.set_modulus(None)
