"""WCE_MMSE_COV with a diagonal Rhh (a power-delay profile) on the Gram wave
kernel's tap-domain form (mmse_lr_kernel<K0, true>, round 4):
U^H P U = s_i s_j Q(t_i - t_j) from one DFT of |x|^2 per frame, the border
from one DFT of x o conj(rx), the read-out and the complex-symbol correction
as DFTs over the taps.  It evaluates the exact DFT where the product Gram
(mmse_lr_kernel<K0>, variant 5) uses the state's U, built from main.c's F
(main.c:18-26; phase error up to ~6e-14): the two models differ by ~1e-13
(tools/cov_full_rank_probe.py, profiles/r04_accuracy_probe.txt).  Checked:
  - every profile that runs the wave kernel against the long double unified
    solve with the reference's F (oracle_py.mmse_unified) at 1e-10 -- the
    round-3 bound of test_pdp_rank_sweep -- and at the measured ~1e-13 level;
  - the tap form against the product Gram on the same frames;
  - complex symbols (correction), nulls, a frame without symbols, split
    (MATLAB block averaging) launches, taps not at 0..L-1.
Parity unpinned against the reference itself (it holds no MMSE output)."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel
from test_cov_lowrank_gpu import c_ld, channel_frames, constellation, solve_ld, synth

pytestmark = pytest.mark.gpu
TOL = 1e-10


def pdp_rhh(L, decay, perm=None):
    p = np.exp(-decay * np.arange(L))
    R = np.zeros((N, N), np.complex128)
    R[np.arange(L), np.arange(L)] = p / p.sum() * 1.1e-4
    if perm is not None:
        R = R[np.ix_(perm, perm)]
    return R


def product_gram(wce, fn):
    lib = wce.load()
    assert lib.wce_debug_set_variant(3, 5) == 0
    try:
        return fn()
    finally:
        assert lib.wce_debug_set_variant(3, 0) == 0


def wave_kernel(wce, fn, on=True):
    """Ranks 17..32 with taps 0..r-1 run mmse_lr_quad2_kernel by default
    (round 6); variant 3 = 1 keeps them on the wave kernel tested here."""
    if not on:
        return fn()
    lib = wce.load()
    assert lib.wce_debug_set_variant(3, 1) == 0
    try:
        return fn()
    finally:
        assert lib.wce_debug_set_variant(3, 0) == 0


# (taps, decay, K0): the wave kernel's ranks (> 16) and a spectrum wider than 1e5 at full rank
PROFILES = [(53, 0.5, 0), (46, 0.1, 0), (40, 0.1, 1), (33, 0.2, 2), (24, 0.3, 3), (17, 0.4, 4)]


@pytest.mark.parametrize("L,decay,k0", PROFILES)
def test_taps_vs_long_double_and_product_gram(gpu_wce, golden, oracle, L, decay, k0):
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(L, decay)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    wv = L <= 32
    assert wave_kernel(wce, lambda: ctx.lr_kernel(1 << 20), wv) == f"mmse_lr_kernel<{k0}, true>"
    assert product_gram(wce, lambda: ctx.lr_kernel(1 << 20)) == f"mmse_lr_kernel<{k0}>"
    B = 1025
    tx, rx = synth(ctx, wce, B, seed=0x7A + L)
    tx[0], rx[0] = inp["tx_symb"], inp["rx_symb"]
    got = wave_kernel(wce, lambda: ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"], wv)
    prod = product_gram(wce, lambda: ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"])
    exp = solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"])
    err, errp, d = normrel(got, exp), normrel(prod, exp), normrel(got, prod)
    print(f"\nL={L} decay={decay}: taps max {err.max():.2e} median {np.median(err):.2e}; "
          f"product Gram max {errp.max():.2e}; taps vs product {d.max():.2e}")
    assert err.max() < TOL, (int(err.argmax()), err.max())
    assert err.max() < 1e-12                 # measured ~1e-13 (the exact-DFT model's own distance included)
    assert d.max() < 1e-12


@pytest.mark.parametrize("kind", ["qpsk", "qam16"])
def test_taps_complex_symbols_nulls_and_spread_taps(gpu_wce, golden, oracle, kind):
    """Non-real symbols (the correction DFTs), null subcarriers, a frame with no
    symbols (H = 0) and a PDP whose taps are scattered over 0..52."""
    wce = gpu_wce
    inp = golden["inputs"]
    perm = np.random.default_rng(11).permutation(N)
    R = pdp_rhh(45, 0.25, perm)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.lr_kernel(4096) == "mmse_lr_kernel<1, true>"
    rng = np.random.default_rng(len(kind))
    B = 300
    tx = constellation(rng, kind, (B, NBLK, N))
    tx[:, :, 26] = 0
    tx[1, 0, [3, 40]] = 0
    tx[2, 0, :] = 0
    rx = channel_frames(rng, tx, inp["ow2"])
    out = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"]
    exp = solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"])
    assert not np.any(out[2])
    keep = np.arange(B) != 2
    err = normrel(out[keep], exp[keep])
    print(f"\n{kind} spread taps: max {err.max():.2e}")
    assert err.max() < 1e-12, (int(err.argmax()), err.max())


def test_taps_split_blocks_matlab(gpu_wce, golden, oracle):
    """MATLAB semantics (one wave per (frame, block), then the block mean)
    run the tap form per block: the mean of the per-block long double solves."""
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(53, 0.5)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 24
    tx, rx = synth(ctx, wce, B, seed=99)
    out = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE, semantics=wce.SEM_MATLAB)["ps_mmse"]
    C = c_ld(oracle, R)
    per = [solve_ld(oracle, C, tx[:, b], rx[:, b], inp["ow2"]) for b in range(4)]   # blocks 0..3 (.m:28-35)
    exp = (((per[0] + per[1]) + per[2]) + per[3]) / 4
    err = normrel(out, exp)
    assert err.max() < 1e-12, err.max()


def test_non_diagonal_rhh_keeps_product_gram(gpu_wce, golden):
    wce = gpu_wce
    inp = golden["inputs"]
    R = pdp_rhh(24, 0.3)
    R[2, 5] = R[5, 2] = 1e-9
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.lr_kernel(4096) == "mmse_lr_kernel<3>"


@pytest.mark.parametrize("L", [8, 12])
def test_scattered_taps_keep_product_lane_and_quad(gpu_wce, golden, oracle, L):
    """A PDP whose kept taps are not 0..L-1 has no Toeplitz Gram at i - j: the
    lane / quad kernels run their product Gram (State::taps_contig = 0), within
    1e-10 of the long double solve; the contiguous profile of the same powers
    runs the Toeplitz form."""
    wce = gpu_wce
    inp = golden["inputs"]
    perm = np.random.default_rng(40 + L).permutation(N)
    R = pdp_rhh(L, 0.5, perm)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    prod = "mmse_lr_lane_staged_kernel<8>" if L == 8 else "mmse_lr_quad_kernel<12>"
    assert ctx.lr_kernel(4096) == prod
    B = 300
    tx, rx = synth(ctx, wce, B, seed=0x5C + L)
    out = ctx.estimate_host(tx, rx, mask=wce.PS_MMSE)["ps_mmse"]
    exp = solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"])
    err = normrel(out, exp)
    assert err.max() < TOL, err.max()
    ctc = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(L, 0.5))
    assert ctc.lr_kernel(4096) == ("mmse_lr_lane_staged_kernel<8, 1, true>" if L == 8 else "mmse_lr_quad_kernel<12, true>")
