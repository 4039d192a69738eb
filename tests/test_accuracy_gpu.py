"""TEXTBOOK PS_MMSE accuracy outside the matched-channel regime
(WiFi_channel_estimation_PS_MMSE.m:28-32: a per-block solve for ANY rx).

Frames whose channel is independent of the preamble's are where Ryy
(cond ~4e6) loses the most digits: the round-1 kernel reached 1.7e-9 there
(profiles/r01_accuracy_probe.txt).  Every rank-1 read-out path -- the shared
TEXTBOOK headline, the config-5 fused kernel, per-frame covariance and MATLAB
block averaging -- is checked here against the long double closed form
(oracle_py.mmse_textbook_closed) at the north-star 1e-10 norm-relative.
Parity unpinned against the reference itself (matlab.mat holds no MMSE
output); the closed form is the restatement of the .m file."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu

TOL = 1e-10


def _cvec(oracle, F, tx_pre, rx_pre, matlab=False):
    """c = F ifft(H_LT) (WiFi_channel_estimation_PS_MMSE.m:20-27), long double."""
    hls = oracle.matlab_lt_ls(tx_pre, rx_pre) if matlab else oracle.lt_ls(tx_pre, rx_pre)
    return F @ (F.conj() @ hls / N)


def _frames(ctx, wce, B, seed, pre=False):
    tx = wce.DeviceArray((B, NBLK, N))
    rx = wce.DeviceArray((B, NBLK, N))
    p = wce.DeviceArray((B, N)) if pre else None
    ctx.synth(tx, rx, p, B, seed=seed)     # no h_shared: every frame draws its own channel
    wce.synchronize()
    return tx.numpy(), rx.numpy(), (p.numpy() if pre else None)


def _closed(oracle, c, tx0, rx0, ow2):
    return np.stack([oracle.mmse_textbook_closed(c, tx0[f], rx0[f], ow2) for f in range(tx0.shape[0])])


@pytest.fixture(scope="module")
def setup(gpu_wce, golden, oracle):
    inp = golden["inputs"]
    F = oracle.fmatrix()
    return inp, F


def test_shared_textbook_unrelated_channels(gpu_wce, setup, oracle):
    """The headline path (mmse_solve_fc_kernel): 1,024 frames with their own
    random channels plus the inputs.h frame, against the closed form."""
    inp, F = setup
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 1025
    tx, rx, _ = _frames(ctx, gpu_wce, B, seed=0xACC)
    tx[0], rx[0] = inp["tx_symb"], inp["rx_symb"]        # frame 0 = inputs.h
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    c = _cvec(oracle, F, inp["tx_pre"], inp["rx_pre"])
    err = normrel(out, _closed(oracle, c, tx[:, 0], rx[:, 0], inp["ow2"]))
    print(f"\nshared TEXTBOOK, unrelated channels: max {err.max():.2e} median {np.median(err):.2e}")
    assert err.max() < TOL, (int(err.argmax()), err.max())


def test_shared_textbook_matched_channels(gpu_wce, setup, oracle):
    inp, F = setup
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    hlt = ctx.shared()[0]
    B = 256
    tx = gpu_wce.DeviceArray((B, NBLK, N))
    rx = gpu_wce.DeviceArray((B, NBLK, N))
    ctx.synth(tx, rx, None, B, seed=5, h_shared=gpu_wce.DeviceArray.from_numpy(hlt))
    gpu_wce.synchronize()
    txh, rxh = tx.numpy(), rx.numpy()
    out = ctx.estimate_host(txh, rxh, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    c = _cvec(oracle, F, inp["tx_pre"], inp["rx_pre"])
    err = normrel(out, _closed(oracle, c, txh[:, 0], rxh[:, 0], inp["ow2"]))
    assert err.max() < TOL, err.max()


def test_pivot_on_faded_subcarrier(gpu_wce, setup, oracle):
    """A preamble whose channel fades by 80 dB on subcarrier 0: without the
    largest-pivot choice the first step would not absorb the rank-1 part."""
    inp, F = setup
    rx_pre = inp["rx_pre"].copy()
    rx_pre[0] *= 1e-4
    ctx = gpu_wce.Context(inp["tx_pre"], rx_pre, inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 256
    tx, rx, _ = _frames(ctx, gpu_wce, B, seed=0xFADE)
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    c = _cvec(oracle, F, inp["tx_pre"], rx_pre)
    err = normrel(out, _closed(oracle, c, tx[:, 0], rx[:, 0], inp["ow2"]))
    assert err.max() < TOL, err.max()


def test_complex_constellation(gpu_wce, setup, oracle):
    """QPSK-like complex tx (the exact row-54 update has a non-zero imaginary
    term only for non-real x)."""
    inp, F = setup
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 256
    tx, rx, _ = _frames(ctx, gpu_wce, B, seed=0x9e5)
    rng = np.random.default_rng(3)
    ph = np.exp(1j * np.pi / 4 * (1 + 2 * rng.integers(0, 4, size=tx.shape)))
    h = rx / np.where(tx == 0, 1, tx)             # the frame's channel (+ noise / tx)
    tx = np.abs(tx) * ph
    tx[:, :, 26] = 0
    rx = h * tx
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    c = _cvec(oracle, F, inp["tx_pre"], inp["rx_pre"])
    err = normrel(out, _closed(oracle, c, tx[:, 0], rx[:, 0], inp["ow2"]))
    assert err.max() < TOL, err.max()


def test_config5_fused_unrelated_channels(gpu_wce, setup, oracle):
    """configs[4]'s fused kernel (PS_MMSE with the LS family + equalization in
    its epilogue, mmse_solve_ls_kernel) on unrelated channels."""
    inp, F = setup
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 512
    tx, rx, pre = _frames(ctx, gpu_wce, B, seed=0xC5, pre=True)
    out = ctx.estimate_host(tx, rx, rx_pre=pre, mask=gpu_wce.ALL)
    c = _cvec(oracle, F, inp["tx_pre"], inp["rx_pre"])
    err = normrel(out["ps_mmse"], _closed(oracle, c, tx[:, 0], rx[:, 0], inp["ow2"]))
    assert err.max() < TOL, err.max()


def test_frame_cov_unrelated_preambles(gpu_wce, setup, oracle):
    """WCE_MMSE_FRAME_COV: each frame's C_f from a preamble whose channel is
    drawn independently of the frame's data channel."""
    inp, F = setup
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 384
    tx, rx, _ = _frames(ctx, gpu_wce, B, seed=0xF1)
    _, _, pre = _frames(ctx, gpu_wce, B, seed=0xF2, pre=True)
    ctx.reserve(B)
    out = ctx.estimate_host(tx, rx, rx_pre=pre, mask=gpu_wce.PS_MMSE | gpu_wce.FRAME_COV)["ps_mmse"]
    err = np.array([normrel(out[f], oracle.mmse_textbook_closed(_cvec(oracle, F, inp["tx_pre"], pre[f]),
                                                                 tx[f, 0], rx[f, 0], inp["ow2"]))
                    for f in range(B)])
    assert err.max() < TOL, err.max()


def test_matlab_semantics_unrelated_channels(gpu_wce, setup, oracle):
    """MATLAB semantics: the mean over blocks 1..4 of the per-block solves
    (split waves + averaging), each block against its closed form."""
    inp, F = setup
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], gpu_wce.MMSE_TEXTBOOK)
    B = 128
    tx, rx, _ = _frames(ctx, gpu_wce, B, seed=0x3A7)
    ctx.reserve(B)
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE, semantics=gpu_wce.SEM_MATLAB)["ps_mmse"]
    c = _cvec(oracle, F, inp["tx_pre"], inp["rx_pre"])   # the state's C (C-semantics LT_LS; equal to rounding)
    exp = np.mean(np.stack([_closed(oracle, c, tx[:, b], rx[:, b], inp["ow2"]) for b in range(4)]), axis=0)
    err = normrel(out, exp)
    assert err.max() < TOL, err.max()
