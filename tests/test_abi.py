"""C-ABI boundary checks that need no GPU: libwce.so loads, exports every
symbol include/*.h declares, its 80-bit host precompute (F, the reference's
cofactor invF, the MMSE covariance) matches the reference bit for bit, and
device entry points fail loudly without a gfx950 device."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle_py import N, from_split

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in ("wce.h", "wce_compat.h", "wce_debug.h"):
        src = open(os.path.join(REPO, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", src, flags=re.M):
            if m.group(1) not in ("if", "defined"):
                names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol(wce):
    lib = wce.load()
    syms = declared_symbols()
    assert {"wce_estimate", "wce_ctx_create", "WiFi_channel_estimation_PS_MMSE"} <= syms
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing
    # the Python mirror binds the whole public ABI
    public = declared_symbols() - {s for s in syms if s.startswith("wce_debug")}
    assert public <= set(wce.wce.ABI), sorted(public - set(wce.wce.ABI))


def test_version_string(wce):
    assert b"gfx950" in wce.load().wce_version()


def _ld_pairs(fn):
    out = np.zeros(N * N * 2, np.longdouble)
    assert fn(out.ctypes.data_as(ctypes.c_void_p)) == 0
    return out[0::2] + 1j * out[1::2].astype(np.clongdouble)


def test_host_F_and_invF_bit_exact(wce, golden):
    lib = wce.load()
    F = _ld_pairs(lib.wce_debug_reference_F).reshape(N, N)
    invF = _ld_pairs(lib.wce_debug_reference_invF).reshape(N, N)
    gF, ginv = from_split(golden["ref"]["F"]), from_split(golden["ref"]["invF"])
    assert np.array_equal(F.real, gF.real) and np.array_equal(F.imag, gF.imag)
    assert np.array_equal(invF.real, ginv.real) and np.array_equal(invF.imag, ginv.imag)


def build_state(wce, tx_pre, rx_pre, ow2, mode):
    lib = wce.load()
    tp = np.ascontiguousarray(tx_pre, np.complex128)
    rp = np.ascontiguousarray(rx_pre, np.complex128)
    C = np.zeros((N, N), np.complex128)
    h = np.zeros(N, np.complex128)
    s = np.zeros((4, N))
    ab = np.zeros(2)
    xm = ctypes.c_ulonglong()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.wce_debug_build_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_int] + \
        [ctypes.c_void_p] * 4 + [ctypes.POINTER(ctypes.c_ulonglong)]
    rc = lib.wce_debug_build_state(p(tp), p(rp), float(ow2), mode, p(C), p(h), p(s), p(ab), ctypes.byref(xm))
    assert rc == 0
    return C, h, s, ab, xm.value


@pytest.mark.parametrize("case", [0, 1])
def test_ref_state_bit_exact(wce, oracle, golden, case):
    """C_ref = F (Rhh FH) from the reference's invF, H_LT from LT_LS: bit-exact
    against the oracle's long double pipeline rounded to fp64."""
    r = golden["ref"]
    C, h, s, ab, xm = build_state(wce, r["pre_tx"][case], r["pre_rx"][case], r["ow2"], wce.MMSE_REF)
    hls = from_split(r["pre_lt_ls"][case])
    assert np.array_equal(h, hls.astype(np.complex128))
    Co = oracle.mmse_ref_cmatrix(from_split(r["F"]), from_split(r["invF"]), hls).astype(np.complex128)
    assert np.array_equal(C, Co)
    assert ab[0] == 0.0 and ab[1] == 2 * r["ow2"]
    assert xm == sum(1 << k for k in (5, 19, 33, 47))


def test_textbook_state(wce, oracle, golden):
    r = golden["ref"]
    C, h, s, ab, xm = build_state(wce, r["pre_tx"][0], r["pre_rx"][0], r["ow2"], wce.MMSE_TEXTBOOK)
    Co = oracle.mmse_textbook_cmatrix(from_split(r["F"]), from_split(r["pre_lt_ls"][0])).astype(np.complex128)
    assert np.abs(C - Co).max() / np.abs(Co).max() < 1e-15
    assert np.allclose(C, C.conj().T, rtol=0, atol=1e-20)      # Hermitian
    assert ab[0] == 1.0 and ab[1] == r["ow2"] and xm == (1 << N) - 1


def test_sinc_table(wce, golden):
    r = golden["ref"]
    _, _, s, _, _ = build_state(wce, r["pre_tx"][0], r["pre_rx"][0], r["ow2"], wce.MMSE_REF)
    for p, P in enumerate((5, 19, 33, 47)):
        a = (np.arange(N) - P) / 14.0
        ref = np.where(a == 0, 1.0, np.sin(np.pi * a) / np.where(a == 0, 1, np.pi * a))
        assert np.allclose(s[p], ref, rtol=1e-15, atol=1e-17)
        assert s[p][P] == 1.0


def test_no_device_fails_loudly(wce):
    if wce.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(wce.WceError) as e:
        wce.Context(np.ones(N), np.ones(N), 1e-7)
    assert e.value.code in (-5, -2)
    with pytest.raises(wce.WceError):
        wce.WiFi_channel_estimation_PS_Linear(np.ones(N), np.ones(N))


CM_TAIL = 64 * 64 * 16 + 64 * 8 + 16     # State's constant-modulus operator Kcm, pattern pcm, cm_on (+ 12 B)
TAPS_TAIL = 16 + 2 * 64 * 4 + 2 * 64 * 8 + 64 * 16   # cov_taps, taps_contig (+ 8 B), tap_of, col_of, col_s, tap_s, dft


def _pdp_cov(L=53, decay=0.12):
    """Exponential power-delay-profile channel covariance (time domain, full rank)."""
    p = np.exp(-decay * np.arange(L))
    return np.diag(p / p.sum()).astype(np.complex128) * 1e-4


def test_cov_state_C_is_F_Rhh_FH(wce, golden):
    """WCE_MMSE_COV: State::C = F Rhh F' (80-bit products), a = 1, b = ow2."""
    inp = golden["inputs"]
    R = _pdp_cov()
    R[3, 7] = R[7, 3] = 2e-6 + 0j       # not diagonal: exercise the full product
    R[5, 11], R[11, 5] = 1e-6 + 3e-7j, 1e-6 - 3e-7j
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    C = blob[:64 * 64 * 16].view(np.complex128).reshape(64, 64)[:53, :53]
    t = np.arange(53)
    F = np.exp(-2j * np.pi * np.outer(t, t).astype(np.longdouble) / 53).astype(np.clongdouble)
    ref = (F @ R.astype(np.clongdouble) @ F.conj().T).astype(np.complex128)
    assert np.max(np.abs(C - ref)) / np.max(np.abs(ref)) < 1e-14
    # State tail: a, b, ow2, xmask, mode, magic, then the low-rank factor
    # U, UT (64 x 64 complex each), cov_lmax, cov_lmin, cov_rank, cov_k0,
    # the layout version and size (+ 8 B reserved), the lane kernel's P_k
    # (53 x 36 complex), the constant-modulus operator (CM_TAIL) and the
    # tap-domain tables (TAPS_TAIL)
    t = blob[:len(blob) - (2 * 64 * 64 * 16 + 16 + 8 + 16 + 53 * 36 * 16 + CM_TAIL + TAPS_TAIL)]
    a, b, ow2 = t[-40:-16].view(np.float64)
    mode, magic = t[-8:].view(np.int32)
    assert (a, b, ow2, mode, magic) == (1.0, inp["ow2"], inp["ow2"], wce.MMSE_COV, 0x80211)
    assert t[-16:-8].view(np.uint64)[0] == (1 << 53) - 1    # X = diag(tx) over all 53
    assert wce.state_mode(blob) == wce.MMSE_COV


def _state_field_offset(blob):
    """byte offset of (cov_rank, cov_k0, layout, bytes) in a state blob"""
    return len(blob) - (53 * 36 * 16 + 24 + CM_TAIL + TAPS_TAIL)


def test_state_validation_rejects_foreign_blobs(wce, golden):
    """wce_state_validate / wce_ctx_load_state accept only a state of this
    build: magic, layout version, size, mode, and a COV rank / solve form in
    range (a larger blob from another build used to pass)."""
    inp = golden["inputs"]
    R = np.zeros((N, N), np.complex128)
    R[:8, :8] = _pdp_cov(8, 0.5)                                  # 8 taps: rank 8, Gram path
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    o = _state_field_offset(blob)
    rank, k0, layout, nbytes = blob[o:o + 16].view(np.int32)
    assert (rank, nbytes) == (8, len(blob)) and k0 == (53 - 8) // 8 and layout >= 4
    assert wce.state_mode(blob) == wce.MMSE_COV
    for field, bad in ((0, 54), (0, -1), (1, 7), (1, -2), (2, layout + 1), (3, len(blob) + 16)):
        b2 = blob.copy()
        b2[o + 4 * field:o + 4 * field + 4] = np.array([bad], np.int32).view(np.uint8)
        with pytest.raises(wce.WceError):
            wce.state_mode(b2)
    b2 = blob.copy()
    b2[o + 4:o + 8] = np.array([-1], np.int32).view(np.uint8)   # dense form needs full rank
    with pytest.raises(wce.WceError):
        wce.state_mode(b2)
    with pytest.raises(wce.WceError):
        wce.state_mode(blob[:-16].copy())                          # short blob


def test_state_validation_rank_within_gram_rows(wce, golden):
    """cov_rank <= 53 - 8 cov_k0 (the Gram kernels' RMAX): a blob
    whose k0 is in range but leaves fewer Gram rows than its rank is refused
    before any kernel indexes LDS with it."""
    inp = golden["inputs"]
    R = np.zeros((N, N), np.complex128)
    R[:8, :8] = _pdp_cov(8, 0.5)                                  # rank 8, k0 = 5: 13 rows
    blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
    o = _state_field_offset(blob)
    assert wce.state_mode(blob) == wce.MMSE_COV
    b2 = blob.copy()
    b2[o + 4:o + 8] = np.array([6], np.int32).view(np.uint8)     # k0 = 6 <= COV_K0_MAX, but 53 - 48 = 5 < 8
    with pytest.raises(wce.WceError):
        wce.state_mode(b2)
    R16 = np.zeros((N, N), np.complex128)
    R16[:16, :16] = _pdp_cov(16, 0.5)
    b3 = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R16)
    k0 = b3[o + 4:o + 8].view(np.int32)[0]
    assert 16 <= 53 - 8 * k0                                      # the builder keeps the invariant
    b3[o + 4:o + 8] = np.array([k0 + 1], np.int32).view(np.uint8)
    with pytest.raises(wce.WceError):
        wce.state_mode(b3)


@pytest.mark.gpu
def test_c_host_cli_runs():
    """tools/wce_cli.c, a C host using only include/wce.h, runs every
    configuration (including the DC spot check) and exits 0."""
    import subprocess
    cli = os.path.join(REPO, "tools", "wce_cli")
    if not os.path.exists(cli):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "80211parallelestimation_amd", "csrc"), "cli"])
    r = subprocess.run([cli, "4096", "textbook", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "frames/s" in r.stdout and "front end" in r.stdout and "bit-identical to the C casts" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("65536", "textbook", "5"), ("1001", "ref", "3")])
def test_c_host_multi_device_runs(args):
    """tools/wce_multi.c, one C process over every visible GPU through the C
    ABI (RCCL state broadcast, wce_shard, nonfinite guard, shard-boundary
    frames recomputed on device 0): exits 0."""
    import subprocess
    exe = os.path.join(REPO, "tools", "wce_multi")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "80211parallelestimation_amd", "csrc"), "multi"])
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "frames/s aggregate" in r.stdout and "non-finite frames (max over devices): 0;" in r.stdout
    assert "mismatching device 0: 0" in r.stdout


def test_ref_pilot_row_map(wce, golden, oracle):
    """State::Wp (round 5): w at the pilots of REF's per-frame covariance,
    folded into one real map of (re h, im h), against main.c's chain in long
    double (main.c:186-203: g = invF h, q = re g - im g, w = FH^T q with FH[c][r]
    = re F[r][c] - im F[r][c]) on random h: within 1e-15 of the chain's scale."""
    r = golden["ref"]
    blob = wce.state_blob(r["pre_tx"][0], r["pre_rx"][0], r["ow2"], wce.MMSE_REF)
    off = 2 * 64 * 64 * 16                                   # past C, Mu
    Wp = blob[off:off + 4 * 64 * 16].view(np.float64).reshape(4, 64, 2)
    assert not np.any(Wp[:, N:])
    F, invF = from_split(r["F"]), from_split(r["invF"])
    Mw = (F.real.astype(np.float64) - F.imag.astype(np.float64)).astype(np.longdouble)   # rounded through double
    rng = np.random.default_rng(4)
    for _ in range(8):
        h = (rng.standard_normal(N) + 1j * rng.standard_normal(N)) * 0.01
        g = invF @ h.astype(np.clongdouble)
        q = g.real - g.imag
        w_ref = np.array([np.sum(Mw[p] * q) for p in (5, 19, 33, 47)])
        w = Wp[:, :N, 0] @ h.real + Wp[:, :N, 1] @ h.imag
        scale = np.abs(Mw[[5, 19, 33, 47]]) @ np.abs(q)
        assert np.all(np.abs(w - w_ref.astype(np.float64)) <= 1e-15 * scale), (w, w_ref)
