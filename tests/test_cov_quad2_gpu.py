"""WCE_MMSE_COV with a power-delay profile of 17..32 contiguous taps (rank
17..32) on mmse_lr_quad2_kernel (round 6): 16 lanes per (frame, block), two
rows of the R x R Toeplitz Gram system per lane, instantiated at 20 / 24 / 28
/ 32 rows (a smaller rank runs the next size up with the rows past it as
b I).  WiFi_channel_estimation_PS_MMSE.m:26-33 with Rhh = diag(PDP):
  - against the long double unified solve with C = F Rhh F^H formed from the
    reference's F (oracle_py.mmse_unified) at the north-star 1e-10 and at the
    ~1e-13 level the other tap-domain forms reach;
  - against the wave kernel (mmse_lr_kernel<K0, true>, variant 3 = 1) on the
    same frames (~1e-15: the same algebra summed in another order);
  - complex symbols (the correction term), null subcarriers, a frame without
    symbols, a ragged batch (not a multiple of the 16 units a workgroup holds),
    MATLAB block averaging (split launches), and a rank whose taps are not
    0..r-1 (kept on the wave kernel).
Parity unpinned against the reference itself (it holds no MMSE output)."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel
from test_cov_lowrank_gpu import c_ld, channel_frames, constellation, solve_ld, synth
from test_cov_taps_gpu import pdp_rhh, wave_kernel

pytestmark = pytest.mark.gpu
TOL = 1e-10


def size_of(L):
    return 20 if L <= 20 else 24 if L <= 24 else 28 if L <= 28 else 32


@pytest.mark.parametrize("L,decay", [(17, 0.4), (20, 0.3), (21, 0.3), (24, 0.3), (24, 0.05), (28, 0.2), (29, 0.2),
                                     (32, 0.15)])
def test_quad2_vs_long_double_and_wave_kernel(gpu_wce, golden, oracle, L, decay):
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(L, decay)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.cov_info()[:2] == (L, True)
    assert ctx.lr_kernel(65536) == f"mmse_lr_quad2_kernel<{size_of(L)}>"
    B = 1025
    tx, rx = synth(ctx, wce, B, seed=0x3A + L)
    tx[0], rx[0] = inp["tx_symb"], inp["rx_symb"]
    got = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"]
    wav = wave_kernel(wce, lambda: ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"])
    exp = solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"])
    err, d = normrel(got, exp), normrel(got, wav)
    print(f"\nL={L} decay={decay}: quad2 max {err.max():.2e} median {np.median(err):.2e}; vs wave kernel {d.max():.2e}")
    assert np.isfinite(got).all()
    assert err.max() < TOL, (int(err.argmax()), err.max())
    assert err.max() < 1e-12
    assert d.max() < 1e-12


@pytest.mark.parametrize("kind", ["qpsk", "qam16"])
def test_quad2_complex_symbols_and_nulls(gpu_wce, golden, oracle, kind):
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(24, 0.25)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.lr_kernel(4096) == "mmse_lr_quad2_kernel<24>"
    rng = np.random.default_rng(7 + len(kind))
    B = 301
    tx = constellation(rng, kind, (B, NBLK, N))
    tx[:, :, 26] = 0
    tx[1, 0, [3, 40]] = 0
    tx[2, 0, :] = 0
    rx = channel_frames(rng, tx, inp["ow2"])
    out = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"]
    wav = wave_kernel(wce, lambda: ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"])
    exp = solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"])
    assert not np.any(out[2])
    keep = np.arange(B) != 2
    err = normrel(out[keep], exp[keep])
    print(f"\n{kind}: quad2 max {err.max():.2e}; vs wave kernel {normrel(out[keep], wav[keep]).max():.2e}")
    assert err.max() < 1e-12, (int(err.argmax()), err.max())
    assert normrel(out[keep], wav[keep]).max() < 1e-12


def test_quad2_split_blocks_matlab(gpu_wce, golden, oracle):
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(27, 0.2)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 37
    assert ctx.lr_kernel(4 * B) == "mmse_lr_quad2_kernel<28>"
    tx, rx = synth(ctx, wce, B, seed=98)
    out = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE, semantics=wce.SEM_MATLAB)["ps_mmse"]
    C = c_ld(oracle, R)
    per = [solve_ld(oracle, C, tx[:, b], rx[:, b], inp["ow2"]) for b in range(4)]   # blocks 0..3 (.m:28-35)
    exp = (((per[0] + per[1]) + per[2]) + per[3]) / 4
    err = normrel(out, exp)
    assert err.max() < 1e-12, err.max()


def test_scattered_rank24_taps_keep_wave_kernel(gpu_wce, golden, oracle):
    """Taps not at 0..r-1: no Toeplitz Gram, so the wave kernel's tap-domain form."""
    wce = gpu_wce
    inp = golden["inputs"]
    perm = np.random.default_rng(24).permutation(N)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(24, 0.3, perm))
    assert ctx.lr_kernel(4096) == "mmse_lr_kernel<3, true>"


def test_quad2_batch_edges(gpu_wce, golden):
    """Batches of 1, 15, 16, 17 and 4,097 units: the last workgroup's spare
    16-lane rows return early; every frame equals the same frame run alone."""
    wce = gpu_wce
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(22, 0.3))
    tx, rx = synth(ctx, wce, 4097, seed=5)
    full = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"]
    assert np.isfinite(full).all()
    for B in (1, 15, 16, 17):
        part = ctx.estimate_host(tx[:B], rx[:B], mask=wce.PS_MMSE)["ps_mmse"]
        assert np.array_equal(part, full[:B]), B


@pytest.mark.parametrize("L,kernel", [(12, "mmse_lr_quad_kernel<12, true>"), (22, "mmse_lr_quad2_kernel<24>")])
def test_quad_kernels_complex_symbols_split_matlab(gpu_wce, golden, oracle, L, kernel):
    """Round 6's tap-domain correction (lrq_cplx_taps: U t as the read-out DFT,
    U^H v as the beta DFT) on 16-QAM frames with nulls, in MATLAB semantics
    (one unit per (frame, block), blocks 0..3 averaged): against the long
    double per-block solves and the wave kernel on the same frames."""
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(L, 0.3)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 45
    assert ctx.lr_kernel(4 * B) == kernel
    rng = np.random.default_rng(1200 + L)
    tx = constellation(rng, "qam16", (B, NBLK, N))
    tx[:, :, 26] = 0
    tx[1, 2, [5, 33]] = 0
    rx = channel_frames(rng, tx, inp["ow2"])
    run = lambda: ctx.estimate_host(tx, rx, mask=wce.PS_MMSE, semantics=wce.SEM_MATLAB)["ps_mmse"]
    out = run()
    wav = wave_kernel(wce, run)
    C = c_ld(oracle, R)
    per = [solve_ld(oracle, C, tx[:, b], rx[:, b], inp["ow2"]) for b in range(4)]   # blocks 0..3 (.m:28-35)
    exp = (((per[0] + per[1]) + per[2]) + per[3]) / 4
    err = normrel(out, exp)
    print(f"\nL={L} 16-QAM MATLAB: max {err.max():.2e}; vs wave kernel {normrel(out, wav).max():.2e}")
    assert np.isfinite(out).all()
    assert err.max() < 1e-12, (int(err.argmax()), err.max())
    assert normrel(out, wav).max() < 1e-12
