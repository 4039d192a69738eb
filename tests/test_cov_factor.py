"""WCE_MMSE_COV host state (CPU, no device): Rhh validation and the 80-bit
low-rank factor C = F Rhh F^H = U U^H that the Gram path (mmse_lr_kernel)
applies, plus a numpy restatement of that path's algebra against the long
double unified solve -- the formulation checked without a GPU."""
import numpy as np
import pytest

from oracle_py import N, normrel


CM_TAIL = 64 * 64 * 16 + 64 * 8 + 16               # State: Kcm, pcm, cm_on (+ 12 B)
TAPS_TAIL = 16 + 2 * 64 * 4 + 2 * 64 * 8 + 64 * 16   # State: cov_taps, taps_contig (+ 8 B), tap_of, col_of, col_s, tap_s, dft


def taps_tables(blob):
    """State's tap-domain tables (the blob's last TAPS_TAIL bytes)."""
    t = blob[len(blob) - TAPS_TAIL:]
    on = int(t[:4].view(np.int32)[0])
    tap_of = t[16:272].view(np.int32)
    col_of = t[272:528].view(np.int32)
    col_s = t[528:1040].view(np.float64)
    tap_s = t[1040:1552].view(np.float64)
    dft = t[1552:2576].view(np.complex128)
    return on, tap_of, col_of, col_s, tap_s, dft


def pdp_rhh(L, decay):
    p = np.exp(-decay * np.arange(L))
    R = np.zeros((N, N), np.complex128)
    R[np.arange(L), np.arange(L)] = p / p.sum() * 1.1e-4
    return R


@pytest.fixture(scope="module")
def inp(golden):
    return golden["inputs"]


@pytest.mark.parametrize("L,decay,k0", [(1, 0.5, 6), (5, 0.5, 6), (6, 0.5, 5), (13, 0.5, 5), (16, 0.5, 4),
                                        (29, 0.2, 3), (40, 0.1, 1), (45, 0.1, 1), (46, 0.1, 0), (52, 0.12, 0),
                                        (53, 0.12, -1), (53, 0.5, 0)])
def test_factor_rank_and_path(wce, oracle, inp, L, decay, k0):
    R = pdp_rhh(L, decay)
    U, r, kk, lmax, lmin = wce.cov_factor(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R))
    assert (r, kk) == (L, k0)
    F = oracle.fmatrix()
    C = np.asarray(F @ oracle._ld(R) @ F.conj().T, np.complex128)
    assert np.max(np.abs(U @ U.conj().T - C)) < 4e-15 * np.max(np.abs(C))
    pd = np.diag(R).real * N                 # eigenvalues of C = F diag(p) F^H (F^H F = 53 I)
    assert abs(lmax - pd.max()) < 1e-13 * pd.max() and abs(lmin - pd[:L].min()) < 1e-13 * pd[:L].min()


def test_rotated_rhh_rank(wce, oracle, inp):
    """Rank 5 in a random unitary basis, formed in fp64: the null space carries
    only rounding (~1e-16 lambda_max), below the 2^-46 rank tolerance."""
    rng = np.random.default_rng(5)
    Q, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    d = np.zeros(N)
    d[:5] = np.exp(-0.4 * np.arange(5))
    R = (Q * d) @ Q.conj().T
    U, r, k0, _, _ = wce.cov_factor(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R))
    assert (r, k0) == (5, 6)
    F = oracle.fmatrix()
    C = np.asarray(F @ oracle._ld(R) @ F.conj().T, np.complex128)
    assert np.max(np.abs(U @ U.conj().T - C)) < 1e-14 * np.max(np.abs(C))


def test_invalid_rhh_rejected(wce, inp):
    R = pdp_rhh(8, 0.5)
    bad = {
        "not Hermitian": R + 1e-9 * np.triu(np.ones((N, N)), 1),
        "imaginary diagonal": R + 1e-9j * np.eye(N),
        "indefinite": R - 1e-6 * np.eye(N),
        "NaN": np.where(np.eye(N) > 0, np.nan, R),
        "Inf": np.where(np.eye(N) > 0, np.inf, R),
        "negative definite": -R,
    }
    for what, M in bad.items():
        with pytest.raises(wce.WceError):
            wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=M)
        assert what


def test_accepts_rounding_level_asymmetry_and_zero(wce, inp):
    R = pdp_rhh(8, 0.5)
    R2 = R.copy()
    R2[0, 3] += 1e-14 * R.max()          # 1e-14 relative: within the 1e-12 Hermitian tolerance
    U, r, k0, _, _ = wce.cov_factor(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R2))
    assert r >= 8
    U, r, k0, lmax, lmin = wce.cov_factor(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"],
                                                         Rhh=np.zeros((N, N))))
    assert (r, k0, lmax, lmin) == (0, 6, 0.0, 0.0)    # C = 0: H = 0 (Gram system b I, zero border)


def _lowrank_np(U, tx, rx, a, b):
    """The Gram path's algebra in fp64 (mmse_lr_kernel without its register layout)."""
    G = tx[:, None] * U
    M = a * (G.conj().T @ G) + b * np.eye(U.shape[1])
    L = np.linalg.cholesky(M)
    t = np.linalg.solve(L.conj().T, np.linalg.solve(L, G.conj().T @ rx))
    y = U @ t
    if np.any(tx.imag != 0):
        v = (tx - tx.conj()) * (rx - a * tx * y)
        y = y + U @ (U.conj().T @ v) / b
    return y


@pytest.mark.parametrize("L", [1, 4, 16, 40])
def test_lowrank_algebra_vs_long_double(wce, oracle, inp, L):
    R = pdp_rhh(L, 0.3)
    U, r, _, _, _ = wce.cov_factor(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R))
    F = oracle.fmatrix()
    C = F @ oracle._ld(R) @ F.conj().T
    rng = np.random.default_rng(L)
    ow2 = inp["ow2"]
    worst = 0.0
    for i in range(24):
        if i % 3 == 0:
            tx = 8.8753 * rng.choice([-1.0, 1.0], N).astype(complex)
        else:
            tx = 8.8753 * (rng.choice([-1.0, 1.0], N) + 1j * rng.choice([-1.0, 1.0], N)) / np.sqrt(2)
        tx[26] = 0
        h = (rng.standard_normal(N) + 1j * rng.standard_normal(N)) * 0.007
        h = np.fft.fft(np.fft.ifft(h) * (np.arange(N) < 6))       # a 6-tap channel of its own
        rx = h * tx + np.sqrt(ow2 / 2) * (rng.standard_normal(N) + 1j * rng.standard_normal(N))
        got = _lowrank_np(U, tx, rx, 1.0, ow2)
        exp = oracle.mmse_unified(C, np.ones(N, np.uint8), 1.0, ow2, tx, rx)
        worst = max(worst, float(normrel(got, exp)))
    assert worst < 1e-11, worst


@pytest.mark.parametrize("L,rot", [(1, False), (5, False), (8, False), (5, True), (13, False)])
def test_lane_gram_factors(wce, oracle, inp, L, rot):
    """State::Pk, the rank <= 8 lane kernel's per-subcarrier Gram factors
    P_k[i][j] = conj(U_ki) U_kj (i >= j, packed at i (i + 1) / 2 + j, formed
    from the 80-bit U and rounded once): consistent with the state's own U to
    rounding, real on the diagonal, and all zero past rank 8."""
    R = pdp_rhh(L, 0.5)
    if rot:
        rng = np.random.default_rng(9)
        Q, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
        R = (Q * np.diag(R).real) @ Q.conj().T
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    U, r, _, _, _ = wce.cov_factor(blob)
    assert r == L
    end = len(blob) - CM_TAIL - TAPS_TAIL   # the round-4 members after P_k
    P = blob[end - N * 36 * 16:end].view(np.complex128).reshape(N, 36)
    if L > 8:
        assert not np.any(P)
        return
    ref = np.zeros((N, 36), np.complex128)
    for i in range(L):
        for j in range(i + 1):
            ref[:, i * (i + 1) // 2 + j] = np.conj(U[:, i]) * U[:, j]
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(P - ref)) < 4e-16 * scale * 4
    assert not np.any(P[:, [i * (i + 1) // 2 + i for i in range(8)]].imag)
    assert not np.any(P[:, L * (L + 1) // 2:])


def _cm_operator(wce, blob, R, x_ref):
    """wce_state_set_modulus on a host blob -> (K 53 x 53, pattern p, on)."""
    import ctypes
    lib = wce.load()
    x = np.ascontiguousarray(x_ref, np.complex128)
    Rc = np.ascontiguousarray(R, np.complex128)
    rc = lib.wce_state_set_modulus(blob.ctypes.data_as(ctypes.c_void_p), blob.nbytes, Rc.ctypes.data_as(ctypes.c_void_p),
                                   x.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    tail = blob[len(blob) - (CM_TAIL + TAPS_TAIL):len(blob) - TAPS_TAIL]
    K = tail[:64 * 64 * 16].view(np.complex128).reshape(64, 64)[:N, :N]
    p = tail[64 * 64 * 16:64 * 64 * 16 + 64 * 8].view(np.float64)[:N]
    on = int(tail[-16:-12].view(np.int32)[0])
    return K, p, on


@pytest.mark.parametrize("L,decay", [(16, 0.5), (24, 0.3), (53, 0.5), (53, 0.12)])
@pytest.mark.parametrize("kind", ["bpsk", "qpsk"])
def test_constant_modulus_operator(wce, oracle, inp, L, decay, kind):
    """K = (a C P + b I)^-1 C, formed in 80 bits through the eigen-decomposition
    of a U^H P U + b I (wce_state.cpp host_build_cm), applied as the GPU's
    constant-modulus path does -- H1 = K (conj x o rx), plus for non-real x
    the correction C ((x - conj x) o (rx - a x o H1)) / b -- in fp64 numpy,
    against the long double unified solve with C formed in 80 bits
    (WiFi_channel_estimation_PS_MMSE.m:26-33) on frames whose symbols share
    x_ref's moduli (DC null)."""
    R = pdp_rhh(L, decay)
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    rng = np.random.default_rng(L + 100 * (kind == "qpsk"))
    A = 8.8753

    def symbols(m):
        if kind == "bpsk":
            x = rng.choice([-A, A], (m, N)).astype(np.complex128)
        else:
            x = A * (rng.choice([-1.0, 1.0], (m, N)) + 1j * rng.choice([-1.0, 1.0], (m, N))) / np.sqrt(2)
        x[:, 26] = 0
        return x
    x = symbols(33)
    K, p, on = _cm_operator(wce, blob, R, x[0])
    assert on == 1 and p[26] == 0.0 and np.all(p[np.arange(N) != 26] == np.abs(x[0, 0]) ** 2 * 0 + p[0])
    F = oracle.fmatrix()
    C_ld = F @ oracle._ld(R) @ F.conj().T
    C = np.asarray(C_ld, np.complex128)
    h = (rng.standard_normal((33, N)) + 1j * rng.standard_normal((33, N))) * 0.01
    rx = h * x + np.sqrt(inp["ow2"] / 2) * (rng.standard_normal((33, N)) + 1j * rng.standard_normal((33, N)))
    ow2 = float(inp["ow2"])
    worst = 0.0
    for f in range(33):
        H = K @ (np.conj(x[f]) * rx[f])
        if kind == "qpsk":
            H = H + (C @ ((x[f] - np.conj(x[f])) * (rx[f] - x[f] * H))) / ow2
        exp = oracle.mmse_unified(C_ld, np.ones(N, np.uint8), 1.0, ow2, x[f], rx[f])
        worst = max(worst, float(normrel(H, exp)))
    print(f"\nL={L} decay={decay} {kind}: max {worst:.2e}")
    assert worst < 1e-11


def test_constant_modulus_rejects_mismatch(wce, inp):
    import ctypes
    lib = wce.load()
    R = pdp_rhh(16, 0.5)
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    x = np.full(N, 8.8753 + 0j)
    R2 = pdp_rhh(12, 0.5)                       # not the Rhh of this state (rank differs)
    rc = lib.wce_state_set_modulus(blob.ctypes.data_as(ctypes.c_void_p), blob.nbytes,
                                   R2.ctypes.data_as(ctypes.c_void_p), x.ctypes.data_as(ctypes.c_void_p))
    assert rc != 0
    x[3] = np.nan
    rc = lib.wce_state_set_modulus(blob.ctypes.data_as(ctypes.c_void_p), blob.nbytes,
                                   R.ctypes.data_as(ctypes.c_void_p), x.ctypes.data_as(ctypes.c_void_p))
    assert rc != 0


@pytest.mark.parametrize("case", ["scaled", "permuted_taps", "dense_offdiag"])
def test_constant_modulus_rejects_same_rank_mismatch(wce, inp, case):
    """A different Rhh of the SAME rank must not pass: K would be
    built for another C than the state's C / U that the per-frame path and the
    non-real correction use.  Same power profile scaled, the same taps in
    another order of power, and a non-diagonal Rhh of equal rank."""
    import ctypes
    lib = wce.load()
    R = pdp_rhh(16, 0.5)
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    if case == "scaled":
        R2 = R * 1.5
    elif case == "permuted_taps":
        d = np.diag(R).copy()
        R2 = np.diag(np.r_[d[:16][::-1], np.zeros(N - 16)]).astype(np.complex128)   # taps 0..15, powers reversed
    else:
        R2 = R.copy()
        R2[1, 2] = R2[2, 1] = 0.1 * R[2, 2]
    assert wce.cov_factor(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R2))[1] == 16
    x = np.full(N, 8.8753 + 0j)
    x[26] = 0
    before = blob.copy()
    rc = lib.wce_state_set_modulus(blob.ctypes.data_as(ctypes.c_void_p), blob.nbytes,
                                   R2.ctypes.data_as(ctypes.c_void_p), x.ctypes.data_as(ctypes.c_void_p))
    assert rc != 0
    rc = lib.wce_state_set_modulus(before.ctypes.data_as(ctypes.c_void_p), before.nbytes,
                                   R.ctypes.data_as(ctypes.c_void_p), x.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0                                    # the state's own Rhh still passes


@pytest.mark.parametrize("L,decay,spread", [(53, 0.5, False), (24, 0.3, False), (20, 0.2, True)])
def test_tap_tables(wce, oracle, inp, L, decay, spread):
    """A diagonal Rhh sets State's tap-domain tables (mmse_lr_kernel<K0, true>):
    column j <-> tap t_j in descending power, sqrt(lambda) by column and by
    tap, and the exact DFT E[m] = exp(-2 pi i m / 53); U[:, j] of the same
    state is s_j F[:, t_j] with the reference's F (main.c:18-26), which the
    exact DFT matches to the reference F's own phase error (<= 1e-13)."""
    R = pdp_rhh(L, decay)
    if spread:                                   # taps not at 0..L-1, not in power order
        perm = np.random.default_rng(3).permutation(N)
        R = R[np.ix_(perm, perm)]
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    U, r, _, _, _ = wce.cov_factor(blob)
    on, tap_of, col_of, col_s, tap_s, dft = taps_tables(blob)
    assert on == 1 and r == L
    lam = np.diag(R).real
    t = tap_of[:r]
    assert np.all(np.diff(lam[t]) <= 0) and len(set(t)) == r        # descending power, distinct taps
    assert np.array_equal(col_of[t], np.arange(r)) and np.sum(col_of >= 0) == r
    assert np.allclose(col_s[:r], np.sqrt(lam[t]), rtol=1e-15, atol=0) and not np.any(col_s[r:])
    assert np.array_equal(tap_s[t], col_s[:r]) and np.sum(tap_s != 0) == r
    m = np.arange(N)
    ang = np.longdouble(-2) * np.longdouble("3.14159265358979323846264338327950288") * m / N
    ex = np.cos(ang) + 1j * np.sin(ang)
    assert np.max(np.abs(dft[:N] - ex.astype(np.complex128))) <= 1.6e-16 and not np.any(dft[N:])   # rounded once
    E = dft[:N]
    Ut = E[np.outer(m, t) % N] * col_s[:r]      # the kernel's U
    assert np.max(np.abs(Ut - U[:, :r])) <= 1e-13 * np.max(col_s)


def test_tap_tables_off_for_non_diagonal(wce, inp):
    R = pdp_rhh(24, 0.3)
    R[2, 5] = R[5, 2] = 1e-9
    on, tap_of, col_of, _, _, _ = taps_tables(wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R))
    assert on == 0 and not np.any(tap_of) and np.all(col_of == -1)


def _taps_np(blob, tx, rx, a, b):
    """The tap-domain Gram path's algebra in fp64 (mmse_lr_kernel<K0, true>
    without its register layout): Q / D DFTs, Gram s_i s_j Q(t_i - t_j), the
    read-out and correction as DFTs over the taps."""
    on, tap_of, col_of, col_s, tap_s, dft = taps_tables(blob)
    r = int(np.sum(col_of >= 0))
    E = dft[:N]
    k = np.arange(N)
    Ekm = E[np.outer(k, k) % N]                       # E[k m]
    p = np.abs(tx) ** 2
    Q = (p[:, None] * Ekm.conj()).sum(0)              # Q(d) = sum_k p_k conj(E[k d])
    D = ((tx * rx.conj())[:, None] * Ekm).sum(0)      # D(m) = sum_k v_k E[k m]
    t, s = tap_of[:r], col_s[:r]
    G = a * np.outer(s, s) * Q[(t[:, None] - t[None, :]) % N] + b * np.eye(r)
    beta = np.conj(s * D[t])                          # G^H rx (the border row is its conjugate)
    L = np.linalg.cholesky(G)
    tt = np.linalg.solve(L.conj().T, np.linalg.solve(L, beta))
    c = np.zeros(N, complex)
    c[t] = s * tt
    y = Ekm @ c
    if np.any(tx.imag != 0):
        v = (tx - tx.conj()) * (rx - a * tx * y)
        w = Ekm.conj().T @ v
        y = y + Ekm @ (tap_s ** 2 * np.pad(w, (0, 64 - N)))[:N] / b
    return y


@pytest.mark.parametrize("L,decay", [(53, 0.5), (46, 0.1), (24, 0.3), (16, 0.5)])
def test_taps_algebra_vs_long_double(wce, oracle, inp, L, decay):
    """The tap-domain form runs the exact DFT, not main.c's F: its answers
    stay within ~1e-13 of the long double solve with the reference's F
    (profiles/r04_accuracy_probe.txt: 1.3e-13 on the widest PDP); fp64 numpy
    here adds its own ~eps cond rounding."""
    R = pdp_rhh(L, decay)
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    F = oracle.fmatrix()
    C = F @ oracle._ld(R) @ F.conj().T
    rng = np.random.default_rng(L)
    ow2 = inp["ow2"]
    worst = 0.0
    for i in range(12):
        if i % 3 == 0:
            tx = 8.8753 * rng.choice([-1.0, 1.0], N).astype(complex)
        else:
            lv = np.array([-3, -1, 1, 3]) * 8.8753 / np.sqrt(10)
            tx = lv[rng.integers(0, 4, N)] + 1j * lv[rng.integers(0, 4, N)]
        tx[26] = 0
        h = (rng.standard_normal(N) + 1j * rng.standard_normal(N)) * 0.007
        h = np.fft.fft(np.fft.ifft(h) * (np.arange(N) < 6))
        rx = h * tx + np.sqrt(ow2 / 2) * (rng.standard_normal(N) + 1j * rng.standard_normal(N))
        got = _taps_np(blob, tx, rx, 1.0, ow2)
        exp = oracle.mmse_unified(C, np.ones(N, np.uint8), 1.0, ow2, tx, rx)
        worst = max(worst, float(normrel(got, exp)))
    assert worst < 1e-11, worst


def test_taps_contig_orders_columns_by_tap(wce, inp):
    """A PDP whose kept taps are exactly 0..L-1 (any powers, not necessarily
    decreasing) orders U's columns by tap index (State::taps_contig: the lane and
    quad kernels' Toeplitz Gram reads Q(i - j)); scattered taps keep the
    descending-power order and taps_contig = 0."""
    L = 6
    p = np.array([0.5, 1.0, 0.25, 0.8, 0.1, 0.3]) * 1e-5
    R = np.zeros((N, N), np.complex128)
    R[np.arange(L), np.arange(L)] = p
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    on, tap_of, col_of, col_s, tap_s, dft = taps_tables(blob)
    contig = int(blob[len(blob) - TAPS_TAIL + 4:len(blob) - TAPS_TAIL + 8].view(np.int32)[0])
    assert on == 1 and contig == 1
    assert np.array_equal(tap_of[:L], np.arange(L)) and np.allclose(col_s[:L], np.sqrt(p), rtol=1e-15, atol=0)
    R2 = np.zeros((N, N), np.complex128)
    R2[[0, 2, 5], [0, 2, 5]] = [1e-5, 3e-5, 2e-5]
    blob2 = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R2)
    on2, tap2, _, s2, _, _ = taps_tables(blob2)
    contig2 = int(blob2[len(blob2) - TAPS_TAIL + 4:len(blob2) - TAPS_TAIL + 8].view(np.int32)[0])
    assert on2 == 1 and contig2 == 0 and list(tap2[:3]) == [2, 5, 0]


@pytest.mark.parametrize("L,decay", [(53, 0.12), (53, 0.5), (6, 0.5)])
def test_circulant_C_for_diagonal_rhh(wce, oracle, inp, L, decay):
    """A diagonal Rhh's State::C is the exact-DFT circulant C_ij = c((i - j) mod 53)
    -- the model U (and the constant-modulus K) of the same state factor: within
    the reference F's own phase error of F Rhh F^H in long double, equal to U U^H."""
    R = pdp_rhh(L, decay)
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    C = blob[:64 * 64 * 16].view(np.complex128).reshape(64, 64)[:N, :N]
    k = np.arange(N)
    assert np.array_equal(C, C[(k[:, None] - k[None, :]) % N, 0])
    F = oracle.fmatrix()
    Cref = np.asarray(F @ oracle._ld(R) @ F.conj().T, np.complex128)
    assert np.max(np.abs(C - Cref)) < 2e-13 * np.max(np.abs(Cref))
    U, r, _, _, _ = wce.cov_factor(blob)
    if r == N or L < N:
        assert np.max(np.abs(U @ U.conj().T - C)) < 4e-15 * np.max(np.abs(C))
