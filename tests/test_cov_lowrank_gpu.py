"""WCE_MMSE_COV on the covariances a channel model actually produces
(WiFi_channel_estimation_PS_MMSE.m:26-33, main.c:189-205 with C = F Rhh F^H).

A power-delay profile of L taps gives Rhh = diag(p_0..p_{L-1}, 0, ...): C has
rank L, and at the synthetic frames' SNR Ryy = X C X^H + ow2 I has cond ~4e6.
The dense form C X (Ryy^-1 rx) loses ~eps cond(Ryy) there (2e-10 .. 1e-8 in
profiles/r03_accuracy_probe.txt); the low-rank Gram path (mmse_lr_kernel, H =
U s) is checked here at every rank the state can choose, on 1,025 frames per
profile with channels of their own (frame 0 = the inputs.h frame), against
the long double unified solve (oracle_py.mmse_unified) with C = F Rhh F^H
formed in 80 bits from the same Rhh -- never the fp64-rounded C, whose
rounding alone moves a rank-deficient answer by ~1e-10.  Parity unpinned
against the reference itself (it holds no MMSE output); the oracle is the
restatement of the .m file's solve."""
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


def c_ld(oracle, R):
    F = oracle.fmatrix()
    return F @ oracle._ld(R) @ F.conj().T


def solve_ld(oracle, C, tx0, rx0, b):
    ones = np.ones(N, np.uint8)
    return np.stack([oracle.mmse_unified(C, ones, 1.0, b, tx0[f], rx0[f]) for f in range(tx0.shape[0])])


def synth(ctx, wce, B, seed):
    tx, rx = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N))
    ctx.synth(tx, rx, None, B, seed=seed)   # every frame draws its own 6-tap channel
    wce.synchronize()
    return tx.numpy(), rx.numpy()


def constellation(rng, kind, shape):
    if kind == "qpsk":
        return A * (rng.choice([-1.0, 1.0], shape) + 1j * rng.choice([-1.0, 1.0], shape)) / np.sqrt(2)
    lv = np.array([-3, -1, 1, 3], float) * (A / np.sqrt(10))
    return lv[rng.integers(0, 4, shape)] + 1j * lv[rng.integers(0, 4, shape)]


def channel_frames(rng, tx, ow2):
    """rx = h o tx + CN(0, ow2): per-frame 6-tap channels, like synth_kernel's."""
    B = tx.shape[0]
    k = np.arange(N)
    p = np.exp(-0.5 * np.arange(6))
    ht = (0.0105 / np.sqrt(p.sum())) * np.exp(-0.25 * np.arange(6)) * 0.7071 * (
        rng.standard_normal((B, 6)) + 1j * rng.standard_normal((B, 6)))
    h = np.einsum("bt,tk->bk", ht, np.exp(-2j * np.pi * np.outer(np.arange(6), k - 26) / 64))
    noise = np.sqrt(ow2 / 2) * (rng.standard_normal(tx.shape) + 1j * rng.standard_normal(tx.shape))
    return h[:, None, :] * tx + noise


# (taps, decay, low-rank path expected): ranks 1..40 take the Gram path at K0 = 6..1;
# a full-rank spectrum within 1e5 takes the dense solve; one wider than 1e5 the Gram path at K0 = 0
PROFILES = [(1, 0.5, True), (4, 0.5, True), (6, 0.5, True), (8, 0.5, True), (16, 0.5, True), (24, 0.3, True),
            (40, 0.1, True), (53, 0.12, False), (53, 0.5, True)]


@pytest.mark.parametrize("L,decay,lowrank", PROFILES)
def test_pdp_rank_sweep(gpu_wce, golden, oracle, L, decay, lowrank):
    inp = golden["inputs"]
    R = pdp_rhh(L, decay)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    r, lr, lmax, lmin = ctx.cov_info()
    assert (r, lr) == (L, lowrank)
    B = 1025
    tx, rx = synth(ctx, gpu_wce, B, seed=0xC0 + L)
    tx[0], rx[0] = inp["tx_symb"], inp["rx_symb"]          # frame 0 = inputs.h
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    err = normrel(out, solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"]))
    print(f"\nL={L} decay={decay} rank={r} {'low-rank' if lr else 'dense'}: max {err.max():.2e} "
          f"median {np.median(err):.2e}")
    assert err.max() < TOL, (int(err.argmax()), err.max())


@pytest.mark.parametrize("L", [1, 6, 16, 45])
@pytest.mark.parametrize("kind", ["qpsk", "qam16"])
def test_complex_symbols_and_nulls(gpu_wce, golden, oracle, L, kind):
    """Non-real symbols take the correction term U^H [(x - conj x) o rho] / b;
    null subcarriers (DC, extra nulls, a frame without symbols) drop out of G."""
    inp = golden["inputs"]
    R = pdp_rhh(L, 0.3)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.cov_info()[1]
    rng = np.random.default_rng(L * 7 + len(kind))
    B = 256
    tx = constellation(rng, kind, (B, NBLK, N))
    tx[:, :, 26] = 0
    tx[1, 0, [3, 40]] = 0
    tx[2, 0, :] = 0                                        # no symbols at all: H = 0
    tx[3, 0, 7] = 1e-90                                    # tiny, kept
    rx = channel_frames(rng, tx, inp["ow2"])
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    exp = solve_ld(oracle, c_ld(oracle, R), tx[:, 0], rx[:, 0], inp["ow2"])
    assert not np.any(out[2]) and not np.any(exp[2])
    keep = np.ones(B, bool)
    keep[2] = False
    err = normrel(out[keep], exp[keep])
    print(f"\n{kind} L={L}: max {err.max():.2e}")
    assert err.max() < TOL, (int(err.argmax()), err.max())


def test_rotated_low_rank_rhh(gpu_wce, golden, oracle):
    """A non-diagonal Rhh (rank 5 in a random basis, formed in fp64): the 80-bit
    Jacobi eigendecomposition finds the rank; checked against the solve with
    the same factor's C = U U^H in long double (the fp64 input's null-space
    rounding, ~1e-16 of lambda_max, is below the rank tolerance)."""
    inp = golden["inputs"]
    rng = np.random.default_rng(5)
    Q, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    d = np.zeros(N)
    d[:5] = np.exp(-0.4 * np.arange(5))
    R = (Q * (d / d.sum() * 1.1e-4)) @ Q.conj().T
    blob = gpu_wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    U, r, k0, _, _ = gpu_wce.cov_factor(blob)
    assert (r, k0) == (5, 6)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 512
    tx, rx = synth(ctx, gpu_wce, B, seed=77)
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    Uld = oracle._ld(U)
    err = normrel(out, solve_ld(oracle, Uld @ Uld.conj().T, tx[:, 0], rx[:, 0], inp["ow2"]))
    print(f"\nrotated rank-5 Rhh: max {err.max():.2e}")
    assert err.max() < TOL


def test_matlab_block_average_lowrank(gpu_wce, golden, oracle):
    """MATLAB semantics (WiFi_channel_estimation_PS_MMSE.m:28-35): one Gram
    solve per block 0..3, then the mean (avg_blocks_kernel)."""
    inp = golden["inputs"]
    R = pdp_rhh(8, 0.5)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 200
    tx, rx = synth(ctx, gpu_wce, B, seed=99)
    out = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE, semantics=gpu_wce.SEM_MATLAB)["ps_mmse"]
    C = c_ld(oracle, R)
    per = [solve_ld(oracle, C, tx[:, b], rx[:, b], inp["ow2"]) for b in range(4)]
    exp = (((per[0] + per[1]) + per[2]) + per[3]) / 4
    err = normrel(out, exp)
    assert err.max() < TOL, err.max()


def test_paths_agree_where_both_are_accurate(gpu_wce, golden):
    """Full rank, spectrum within 1e5 (the dense form's home ground): forcing the
    Gram path (K0 = 0) on BPSK frames gives the dense answer to ~1e-12."""
    inp = golden["inputs"]
    R = pdp_rhh(53, 0.12)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 300
    tx, rx = synth(ctx, gpu_wce, B, seed=3)
    dense = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    ctx.set_cov_path(2)
    lowr = ctx.estimate_host(tx, rx, mask=gpu_wce.PS_MMSE)["ps_mmse"]
    assert normrel(lowr, dense).max() < 1e-11


def test_lowrank_batch_shards_and_ls_outputs(gpu_wce, golden, oracle):
    """65,537 frames: non-finite scan clean, sampled frames vs the oracle, the
    batch equals its shards bit for bit, and LS outputs requested in the same
    call (no fusion on this path) equal an LS-only call."""
    import importlib
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    inp = golden["inputs"]
    R = pdp_rhh(6, 0.5)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    wce = gpu_wce
    B = 65537
    tx, rx = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N))
    ctx.synth(tx, rx, None, B, seed=0x5EED)
    H = wce.DeviceArray((B, N), zero=True)
    L1 = wce.DeviceArray((B, N), zero=True)
    ctx.estimate(ctx.frames(tx, rx, B), wce.Outputs(None, L1.addr, None, None, H.addr, None, N, 0, 0, 0, 0),
                 wce.PS_MMSE | wce.PS_LINEAR)
    wce.synchronize()
    assert ctx.nonfinite_scan(H, B)[1] == 0
    C = c_ld(oracle, R)
    rng = np.random.default_rng(1)
    for f in np.concatenate([[0, B - 1], rng.choice(B, 30, replace=False)]):
        t, r = tx.rows(f)[0], rx.rows(f)[0]
        exp = oracle.mmse_unified(C, np.ones(N, np.uint8), 1.0, inp["ow2"], t[0], r[0])
        assert normrel(H.rows(f)[0], exp) < TOL, f
    L2 = wce.DeviceArray((B, N), zero=True)
    ctx.estimate(ctx.frames(tx, rx, B), wce.Outputs(None, L2.addr, None, None, None, None, N, 0, 0, 0, 0),
                 wce.PS_LINEAR)
    wce.synchronize()
    assert np.array_equal(L1.numpy(), L2.numpy())
    whole = H.numpy()
    for rank in range(4):
        first, count = multi.native_shard(wce, B, 4, rank)
        fr = ctx.frames(tx.addr + first * NBLK * N * 16, rx.addr + first * NBLK * N * 16, count)
        Hs = wce.DeviceArray((count, N), zero=True)
        ctx.estimate(fr, wce.Outputs(None, None, None, None, Hs.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE)
        wce.synchronize()
        assert np.array_equal(Hs.numpy(), whole[first:first + count]), rank


def test_profiling_entry_rejects_lowrank(gpu_wce, golden):
    inp = golden["inputs"]
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh(4, 0.5))
    B = 4
    tx, rx = gpu_wce.DeviceArray((B, NBLK, N)), gpu_wce.DeviceArray((B, NBLK, N))
    W = gpu_wce.DeviceArray((B, N))
    with pytest.raises(gpu_wce.WceError):
        ctx.mmse_solve(ctx.frames(tx, rx, B), W)


@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 6, 7, 8])
def test_lane_kernel_every_small_rank(gpu_wce, golden, oracle, L):
    """Ranks 1..8 run one frame per lane (mmse_lr_lane_staged_kernel): BPSK and
    QPSK frames against the long double solve, and against the wave-per-frame
    Gram kernel (variant WCE_VARIANT_LR = 1) on the same frames, C and MATLAB
    semantics, 515 frames (a partial last wave of lanes).  The product at this
    size is the staged one-workgroup-per-CU build in the Toeplitz form (a PDP
    with taps 0..L-1: Gamma = S Q S, round 4; variant 3 forces the same build:
    bit for bit); the two-workgroups build (variant 4; ranks 7, 8) computes the
    same sums (bit for bit); variant 5 runs the product Gram (sum_k |x_k|^2 P_k)
    in the same staged build, and the direct form (variant 2: per-lane loads,
    no LDS staging, product Gram) is the independent check of the staging (to
    rounding)."""
    inp = golden["inputs"]
    lib = gpu_wce.load()
    R = pdp_rhh(L, 0.4)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.cov_info()[:2] == (L, True)
    B = 515
    assert ctx.lr_kernel(B) == f"mmse_lr_lane_staged_kernel<{L}, 1, true>"
    tx, rx = synth(ctx, gpu_wce, B, seed=0x1A0 + L)
    rng = np.random.default_rng(L)
    txq = constellation(rng, "qpsk", tx.shape)
    txq[:, :, 26] = 0
    rxq = channel_frames(rng, txq, inp["ow2"])
    C = c_ld(oracle, R)
    names = {2: f"mmse_lr_lane_kernel<{L}>", 3: f"mmse_lr_lane_staged_kernel<{L}, 1, true>",
             4: f"mmse_lr_lane_staged_kernel<{L}, 2, true>" if L >= 7 else f"mmse_lr_lane_staged_kernel<{L}, 1, true>",
             5: f"mmse_lr_lane_staged_kernel<{L}>"}
    try:
        for t, r in ((tx, rx), (txq, rxq)):
            got = {}
            for v in (0, 1, 2, 3, 4, 5):
                assert lib.wce_debug_set_variant(3, v) == 0
                if v in names:
                    assert ctx.lr_kernel(B) == names[v]
                got[v] = ctx.estimate_host(t, r, mask=gpu_wce.PS_MMSE)["ps_mmse"]
                got[v, "m"] = ctx.estimate_host(t, r, mask=gpu_wce.PS_MMSE, semantics=gpu_wce.SEM_MATLAB)["ps_mmse"]
            for v in (3, 4):
                assert np.array_equal(got[v], got[0]) and np.array_equal(got[v, "m"], got[0, "m"]), v
            # direct vs LDS-staged form of the product Gram: same sums in the same order (the
            # compiler may contract a product into an FMA differently in the two instantiations)
            dd = max(normrel(got[5], got[2]).max(), normrel(got[5, "m"], got[2, "m"]).max())
            assert dd < 1e-12, dd
            # Toeplitz vs product Gram: the same Gamma summed two ways
            dt = max(normrel(got[0], got[5]).max(), normrel(got[0, "m"], got[5, "m"]).max())
            assert dt < 1e-11, dt
            sel = np.r_[0:30, B - 10:B]
            err = normrel(got[0][sel], solve_ld(oracle, C, t[sel, 0], r[sel, 0], inp["ow2"]))
            assert err.max() < TOL, err.max()
            per = [solve_ld(oracle, C, t[sel, b], r[sel, b], inp["ow2"]) for b in range(4)]
            errm = normrel(got[0, "m"][sel], (((per[0] + per[1]) + per[2]) + per[3]) / 4)
            assert errm.max() < TOL, errm.max()
            # the two kernels: the same algebra summed in another order (rank 1
            # carries the most rounding, ~1e-11 from the long double solve, r03 probe)
            d = max(normrel(got[0], got[1]).max(), normrel(got[0, "m"], got[1, "m"]).max())
            print(f"\nrank {L}: vs long double {max(err.max(), errm.max()):.2e}, lane vs wave kernel {d:.2e}, "
                  f"direct vs staged {dd:.2e}, Toeplitz vs product {dt:.2e}")
            assert d < TOL
    finally:
        assert lib.wce_debug_set_variant(3, 0) == 0


@pytest.mark.parametrize("L", [7, 8])
@pytest.mark.parametrize("matlab", [False, True])
def test_lane_two_workgroup_build_at_size(gpu_wce, golden, oracle, L, matlab):
    """Ranks 7 and 8 past one 64-unit wave per SIMD (> 65,536 (frame, block)
    units on 256 CUs) run the two-workgroups-per-CU build
    mmse_lr_lane_staged_kernel<R, 2, true> (launch_mmse_lr; the product
    Gram's build, variant 5, spills at rank 8):
    70,001 frames in C semantics, 17,001 frames = 68,004 units in MATLAB split
    mode.  The first half of the batch is BPSK, the second QPSK (the
    correction pass).  Non-finite scan clean; the first, the last and 30
    random frames against the long double solve with C formed in 80 bits
    (WiFi_channel_estimation_PS_MMSE.m:26-33); the whole batch bit-equal to
    the one-workgroup build forced through variant 3."""
    wce = gpu_wce
    inp = golden["inputs"]
    lib = wce.load()
    R = pdp_rhh(L, 0.5)
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    B = 17001 if matlab else 70001
    units = 4 * B if matlab else B
    NB = 4                                             # blocks 0..3 held per frame
    rng = np.random.default_rng(0x7E0 + L + 16 * matlab)
    tx = np.where(rng.random((B, NB, N)) < 0.5, -A, A).astype(np.complex128)
    tx[B // 2:] = constellation(rng, "qpsk", (B - B // 2, NB, N))
    tx[:, :, 26] = 0
    rx = channel_frames(rng, tx, inp["ow2"])
    dtx, drx = wce.DeviceArray.from_numpy(tx), wce.DeviceArray.from_numpy(rx)
    fr = ctx.frames(dtx, drx, B, frame_stride=NB * N, semantics=wce.SEM_MATLAB if matlab else wce.SEM_C)

    def run(v):
        assert lib.wce_debug_set_variant(3, v) == 0
        H = wce.DeviceArray((B, N), zero=True)
        ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE)
        wce.synchronize()
        return H

    try:
        assert ctx.lr_kernel(units) == f"mmse_lr_lane_staged_kernel<{L}, 2, true>"
        H = run(0)
        assert ctx.nonfinite_scan(H, B)[1] == 0
        got = H.numpy()
        assert lib.wce_debug_set_variant(3, 3) == 0
        assert ctx.lr_kernel(units) == f"mmse_lr_lane_staged_kernel<{L}, 1, true>"
        assert np.array_equal(run(3).numpy(), got)
        assert lib.wce_debug_set_variant(3, 5) == 0              # the product Gram's MW = 2 build
        assert ctx.lr_kernel(units) == f"mmse_lr_lane_staged_kernel<{L}, 2>"
        prod = run(5).numpy()
        assert normrel(prod, got).max() < 1e-11
    finally:
        assert lib.wce_debug_set_variant(3, 0) == 0
    C = c_ld(oracle, R)
    sel = np.concatenate([[0, B - 1], rng.choice(B, 30, replace=False)])
    if matlab:
        per = [solve_ld(oracle, C, tx[sel, b], rx[sel, b], inp["ow2"]) for b in range(4)]
        exp = (((per[0] + per[1]) + per[2]) + per[3]) / 4
    else:
        exp = solve_ld(oracle, C, tx[sel, 0], rx[sel, 0], inp["ow2"])
    err = normrel(got[sel], exp)
    print(f"\nrank {L} {'MATLAB' if matlab else 'C'} {B} frames ({units} units): max {err.max():.2e}")
    assert err.max() < TOL, (int(sel[err.argmax()]), err.max())


@pytest.mark.parametrize("L", [9, 10, 12, 13, 16])
def test_quad_kernel_mid_ranks(gpu_wce, golden, oracle, L):
    """Ranks 9..16 run 16 lanes per frame (mmse_lr_quad_kernel; a PDP with taps
    0..L-1 in the Toeplitz form, round 4): BPSK and 16-QAM frames against the
    long double solve, against the wave-per-frame Gram kernel (variant
    WCE_VARIANT_LR = 1) and against the quad kernel's product Gram (variant
    5), C and MATLAB semantics, 515 frames (a partial last row group of the
    last wave)."""
    inp = golden["inputs"]
    lib = gpu_wce.load()
    R = pdp_rhh(L, 0.3)
    ctx = gpu_wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    assert ctx.cov_info()[:2] == (L, True)
    B = 515
    tx, rx = synth(ctx, gpu_wce, B, seed=0x2B0 + L)
    rng = np.random.default_rng(L)
    txq = constellation(rng, "qam16", tx.shape)
    txq[:, :, 26] = 0
    rxq = channel_frames(rng, txq, inp["ow2"])
    C = c_ld(oracle, R)
    try:
        for t, r in ((tx, rx), (txq, rxq)):
            got = {}
            for v in (0, 1, 5):
                assert lib.wce_debug_set_variant(3, v) == 0
                if v != 1:
                    assert ctx.lr_kernel(B) == f"mmse_lr_quad_kernel<{L}{', true' if v == 0 else ''}>"
                got[v] = ctx.estimate_host(t, r, mask=gpu_wce.PS_MMSE)["ps_mmse"]
                got[v, "m"] = ctx.estimate_host(t, r, mask=gpu_wce.PS_MMSE, semantics=gpu_wce.SEM_MATLAB)["ps_mmse"]
            dp = max(normrel(got[0], got[5]).max(), normrel(got[0, "m"], got[5, "m"]).max())
            assert dp < 1e-11, dp
            sel = np.r_[0:30, B - 10:B]
            err = normrel(got[0][sel], solve_ld(oracle, C, t[sel, 0], r[sel, 0], inp["ow2"]))
            per = [solve_ld(oracle, C, t[sel, b], r[sel, b], inp["ow2"]) for b in range(4)]
            errm = normrel(got[0, "m"][sel], (((per[0] + per[1]) + per[2]) + per[3]) / 4)
            d = max(normrel(got[0], got[1]).max(), normrel(got[0, "m"], got[1, "m"]).max())
            print(f"\nrank {L}: vs long double {max(err.max(), errm.max()):.2e}, quad vs wave kernel {d:.2e}, "
                  f"Toeplitz vs product {dp:.2e}")
            assert err.max() < TOL and errm.max() < TOL and d < TOL
    finally:
        assert lib.wce_debug_set_variant(3, 0) == 0
