"""The CPU oracle pinned against the reference's own outputs (golden vectors
produced by the compiled reference, tests/golden/make_golden.py) and against
the MATLAB workspace matlab.mat.  No GPU needed."""
import os

import numpy as np
import pytest

from oracle_py import N, NBLK, PILOTS, from_split, normrel


def bits_equal(a, b):
    a = np.asarray(a, np.clongdouble)
    b = np.asarray(b, np.clongdouble)
    return np.array_equal(a.real, b.real) and np.array_equal(a.imag, b.imag)


def test_fmatrix_bit_exact(oracle, golden):
    assert bits_equal(oracle.fmatrix(), from_split(golden["ref"]["F"]))


@pytest.mark.parametrize("name", ["ps_linear", "ps_cubic", "ps_sinc"])
def test_ps_estimators_bit_exact(oracle, golden, name):
    r = golden["ref"]
    for f in range(r["frames_tx"].shape[0]):
        H = getattr(oracle, name)(r["frames_tx"][f], r["frames_rx"][f])
        assert bits_equal(H, from_split(r[name][f])), (name, f)


def test_lt_ls_bit_exact(oracle, golden):
    r = golden["ref"]
    for f in range(r["frames_tx"].shape[0]):
        H = oracle.lt_ls(r["pre_tx"][f % 2], r["pre_rx"][f % 2])
        assert bits_equal(H, from_split(r["lt_ls"][f]))
        assert H[26] == 0


def test_inverse_cofactor_bit_exact(oracle, golden):
    invF = oracle.inverse_cofactor(oracle.fmatrix())
    assert bits_equal(invF, from_split(golden["ref"]["invF"]))
    # and it is only ~1.5e-7 accurate: exact F^-1 = F^H / 53
    exact = oracle.fmatrix().conj().T / 53
    err = np.abs((invF - exact).astype(np.complex128)).max() * 53
    assert 1e-8 < err < 1e-6


def test_mmse_ref_repaired_bit_exact(oracle, golden):
    r = golden["ref"]
    F = from_split(r["F"])
    invF = from_split(r["invF"])
    for c in range(2):
        hls = from_split(r["pre_lt_ls"][c])
        for f in range(r["frames_tx"].shape[0]):
            H = oracle.mmse_ref_repaired(r["frames_tx"][f], r["frames_rx"][f], F, r["ow2"], hls, invF)
            assert bits_equal(H, from_split(r["ps_mmse_ref"][c, f])), (c, f)


def test_mmse_golden_values(golden):
    # values quoted in SURVEY 8(c)(i): inputs.h frame
    r = golden["ref"]
    m = from_split(r["ps_mmse_ref"][0, 0]).astype(np.complex128)
    assert abs(m[0] - (1.115539799734874443549e03 - 1.364070362604641952875e03j)) < 1e-9
    lin = from_split(r["ps_linear"][0]).astype(np.complex128)
    assert abs(lin[0] - (9.253895176911212610829e-03 - 1.592455267909223567380e-04j)) < 1e-17


def test_literal_inverse_is_nan(oracle, golden):
    """Known answer: the reference's cofactor inverse of a diagonal Ryy divides
    0/0 in its unpivoted Schur determinant (utils.c:557) -> NaN."""
    R = np.diag(np.full(6, 2 * golden["ref"]["ow2"]))
    Ri = oracle.inverse_cofactor(R)
    nan = np.isnan(Ri.real.astype(float)) | np.isnan(Ri.imag.astype(float))
    assert np.array_equal(nan, golden["ref"]["literal_inv_diag6_nan"])
    assert nan.sum() > 0


def test_mmse_unified_matches_ref_formula(oracle, golden):
    """The unified kernel formula in REF mode (C_ref, pilots, a=0, b=2 ow2)
    reproduces the repaired reference pipeline."""
    r = golden["ref"]
    F, invF = from_split(r["F"]), from_split(r["invF"])
    for c in range(2):
        hls = from_split(r["pre_lt_ls"][c])
        C = oracle.mmse_ref_cmatrix(F, invF, hls)
        for f in range(r["frames_tx"].shape[0]):
            H = oracle.mmse_unified(C, oracle.pilot_mask(), 0, 2 * np.longdouble(r["ow2"]), r["frames_tx"][f],
                                    r["frames_rx"][f])
            assert normrel(H, from_split(r["ps_mmse_ref"][c, f])) < 1e-15


def test_mmse_textbook_closed_form(oracle, golden):
    """TEXTBOOK (MATLAB per-block) MMSE: long double Cholesky vs closed form.
    Parity unpinned against the reference (no MMSE output in matlab.mat)."""
    r = golden["ref"]
    F = from_split(r["F"])
    for c in range(2):
        hls = from_split(r["pre_lt_ls"][c])
        C = oracle.mmse_textbook_cmatrix(F, hls)
        # C = c c^H with c = F ifft(H_LT) (= H_LT up to the rounding of the double-precision F)
        cvec = F @ (F.conj() @ hls / 53)
        assert normrel(C.reshape(-1), np.outer(cvec, cvec.conj()).reshape(-1)) < 1e-17
        assert normrel(cvec, hls) < 1e-13
        for f in range(r["frames_tx"].shape[0]):
            tx, rx = r["frames_tx"][f], r["frames_rx"][f]
            H = oracle.mmse_unified(C, np.ones(N, np.uint8), 1, r["ow2"], tx, rx)
            Hc = oracle.mmse_textbook_closed(cvec, tx, rx, r["ow2"])
            assert normrel(H, Hc) < 1e-11   # Ryy has cond ~4e6; frames 1-7 carry channels unrelated to H_LT


@pytest.mark.parametrize("name,key", [("ps_linear", "H_EST_PS_Linear"), ("ps_sinc", "H_EST_PS_Sinc"),
                                      ("ps_cubic", "H_EST_PS_Cubic")])
def test_matlab_pins(oracle, golden, name, key):
    """Per-block interpolators, averaged over blocks 1-4 as WiFi_channel_estimation_PS_*.m do,
    reproduce matlab.mat (pins the per-block formula the C code shares; cubic with MATLAB divisors)."""
    m = golden["matlab"]
    tx, rx = m["tx_symb"].T, m["rx_symb"].T   # MATLAB [53][15] -> [15][53]
    H = oracle.matlab(name, tx, rx)
    assert normrel(H, m[key]) < 1e-13


def test_matlab_lt_ls_and_c_quirk(oracle, golden):
    m = golden["matlab"]
    H = oracle.matlab_lt_ls(m["tx_preamble_fft"], m["rx_preamble_fft"])
    assert normrel(H, m["H_EST_LT_LS"]) < 1e-14
    # the C "conj" quirk (a real scale factor) cancels: same estimate to rounding
    Hc = oracle.lt_ls(m["tx_preamble_fft"], m["rx_preamble_fft"])
    assert normrel(Hc, m["H_EST_LT_LS"]) < 1e-14


def test_equalization_matlab_pin(oracle, golden):
    m = golden["matlab"]
    eq = oracle.equalize(m["rx_symb"].T, m["H_EST_LT_LS"], m["H_EST_PS_Linear"])
    ref = m["eq_symbols"].T
    assert np.max(np.abs((eq - ref).astype(np.complex128))) / np.max(np.abs(ref)) < 1e-13
    assert np.all(eq[:, 26] == 0)


def test_cubic_c_vs_matlab_divisors_differ(oracle, golden):
    """Documented quirk: main.c divides every difference by 14 (main.c:116-118)."""
    m = golden["matlab"]
    tx, rx = m["tx_symb"].T, m["rx_symb"].T
    c_quirk = np.mean([oracle.ps_cubic(tx[b], rx[b]) for b in range(4)], axis=0)
    assert normrel(c_quirk, m["H_EST_PS_Cubic"]) > 0.1


def test_pilots_through_interpolants(oracle, golden):
    r = golden["ref"]
    for f in range(r["frames_tx"].shape[0]):
        tx, rx = r["frames_tx"][f], r["frames_rx"][f]
        hp = rx[list(PILOTS)] / tx[list(PILOTS)]
        for name in ("ps_linear", "ps_sinc"):
            H = getattr(oracle, name)(tx, rx).astype(np.complex128)
            assert np.allclose(H[list(PILOTS)], hp, rtol=1e-14, atol=0), name
        # the divisor quirk keeps the C cubic on the first two pilots only
        H = oracle.ps_cubic(tx, rx).astype(np.complex128)
        assert np.allclose(H[list(PILOTS[:2])], hp[:2], rtol=1e-14, atol=0)


def test_cpu_port_matches_oracle(oracle, golden):
    """The fp64 OpenMP port (bench cpu_baseline) agrees with the long double oracle."""
    r = golden["ref"]
    F, invF = from_split(r["F"]), from_split(r["invF"])
    hls = from_split(r["pre_lt_ls"][0])
    C = oracle.mmse_ref_cmatrix(F, invF, hls).astype(np.complex128)
    tx = np.ascontiguousarray(r["frames_tx"].reshape(-1))
    rx = np.ascontiguousarray(r["frames_rx"].reshape(-1))
    H, _ = oracle.bench_mmse_f64(C, oracle.pilot_mask(), 0.0, 2 * r["ow2"], tx, rx, N, 2)
    for f in range(r["frames_tx"].shape[0]):
        assert normrel(H[f], from_split(r["ps_mmse_ref"][0, f])) < 1e-13


def test_front_end_blocks_matlab_pin(oracle, golden):
    """WiFi_blocks_extraction.m: packet -> 80-sample blocks -> CP drop -> fft64
    -> circshift 26 -> 53 bins; matlab.mat's tx/rx_symb reproduced."""
    m = golden["matlab"]
    for pk, sk in (("rx_packet", "rx_symb"), ("tx_packet", "tx_symb")):
        sym = oracle.front_blocks(m[pk], NBLK)
        ref = m[sk].T
        assert np.max(np.abs((sym - ref).astype(np.complex128))) / np.max(np.abs(ref)) < 1e-14, pk


def test_front_end_preamble_matlab_pin(oracle, golden):
    """WiFi_RX.m:18-30: preamble copies, averaged FFT, sigma^2."""
    m = golden["matlab"]
    assert np.array_equal(m["rx_preamble1"], m["rx_lptot"][-64:])
    assert np.array_equal(m["rx_preamble2"], m["rx_lptot"][-128:-64])
    for lk, fk in (("rx_lptot", "rx_preamble_fft"), ("tx_lptot", "tx_preamble_fft")):
        pre, ow2 = oracle.front_preamble(m[lk])
        assert normrel(pre, m[fk]) < 1e-14, lk
    _, ow2 = oracle.front_preamble(m["rx_lptot"])
    d = m["rx_preamble2"] - m["rx_preamble1"]
    assert abs(float(ow2) - np.sum(np.abs(d) ** 2) / 128) < 1e-15 * abs(float(ow2))
    assert 0 < float(ow2) < 1e-3


def test_mmse_formula_pins_vs_oracle(oracle, golden):
    """WiFi_channel_estimation_PS_MMSE.m's formula computed by the reference's
    own multiply() and cofactor inverse() (tests/golden/make_mmse_pins.py,
    oracle/ref_harness.cpp:refh_mmse_formula) pins the oracle's restatements:
    the TEXTBOOK closed form and the long double unified solve (WCE_MMSE_COV
    with a rank-6 and a full-rank power-delay profile), at the noise powers
    where the cofactor inverse is itself accurate (cond(Ryy) <= ~4e4)."""
    import os
    pins = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "mmse_formula_pins.npz")))
    F = from_split(golden["ref"]["F"])
    hls = from_split(pins["h_ls"])
    assert normrel(hls, oracle.lt_ls(golden["inputs"]["tx_pre"], golden["inputs"]["rx_pre"])) == 0
    c = F @ (F.conj() @ hls / N)
    ones = np.ones(N, np.uint8)
    worst = 0.0
    for wi, ow2 in enumerate(pins["ow2"]):
        for f in range(pins["frames_tx"].shape[0]):
            t, r = pins["frames_tx"][f], pins["frames_rx"][f]
            checks = [(pins["H_textbook"][wi, f], oracle.mmse_textbook_closed(c, t, r, ow2))]
            for kind in ("pdp6", "pdp53"):
                C = F @ oracle._ld(pins["rhh_" + kind]) @ F.conj().T
                checks.append((pins["H_" + kind][wi, f], oracle.mmse_unified(C, ones, 1.0, ow2, t, r)))
            for pin, want in checks:
                worst = max(worst, float(normrel(from_split(pin), want)))
    assert worst < 5e-12, worst   # measured 2.0e-12 (rank 6 at ow2 = 1e-5: the cofactor inverse's own error)


def test_textbook_closed_form_vs_mp_literal(oracle, golden):
    """The oracle's long double closed form of the headline (TEXTBOOK) mode
    against WiFi_channel_estimation_PS_MMSE.m:26-32 evaluated literally in
    mpmath at 50 digits (tests/golden/make_textbook_mp.py) at the operating
    ow2 = 9.6172e-8.  Measured max 2.9e-13 over the 13 frames: the closed
    form's cancellation (uH rx - (uH v)(vH rx)/(s + vH v)) costs cond(Ryy) ~ 4e6
    times long double's 1.1e-19, i.e. ~4e-13 is its floor -- the same with an
    exact c, so it is not F's or H_LT's rounding; hence 1e-12 here."""
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "textbook_mp_pins.npz"))
    inp = golden["inputs"]
    assert float(d["ow2"]) == float(inp["ow2"])
    F = oracle.fmatrix()
    c = F @ (F.conj() @ oracle.lt_ls(inp["tx_pre"], inp["rx_pre"]) / N)
    errs = [oracle.normrel(oracle.mmse_textbook_closed(c, d["tx"][i], d["rx"][i], d["ow2"]),
                           d["H_hi"][i].astype(np.clongdouble) + d["H_lo"][i]) for i in range(len(d["tx"]))]
    assert len(errs) == 13 and max(errs) < 1e-12, errs


def test_textbook_mp_fixture_inputs_regenerate():
    """The fixture's bench frames are the Python restatement of synth_kernel
    (make_textbook_mp.synth_block0) of the bench's seed and H_LT: rerunning it
    gives the stored inputs bit for bit (the GPU test ties them to the
    device's own frames)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_textbook_mp as m
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "textbook_mp_pins.npz"))
    for i in np.nonzero(d["kind"] == "bench")[0]:
        t, r = m.synth_block0(int(d["bench_frame"][i]), d["h_shared"], float(d["ow2"]))
        assert np.array_equal(t, d["tx"][i]) and np.array_equal(r, d["rx"][i])


def test_cov_unified_solve_vs_mp_literal(oracle, golden):
    """The oracle's long double unified solve with C = F Rhh F^H (the
    reference's F) against the .m formula evaluated literally in mpmath with a
    model Rhh (tests/golden/make_cov_mp.py), 7 profiles x 4 frames at the
    operating ow2: measured <= 9.1e-14."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cov_lowrank_gpu import c_ld, solve_ld
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cov_mp_pins.npz"))
    inp = golden["inputs"]
    worst = 0.0
    for pi in range(len(d["taps"])):
        exp = solve_ld(oracle, c_ld(oracle, np.diag(d["pdp"][pi]).astype(np.complex128)), d["tx"], d["rx"], inp["ow2"])
        Hm = d["H_hi"][pi].astype(np.clongdouble) + d["H_lo"][pi]
        worst = max(worst, max(float(oracle.normrel(exp[f], Hm[f])) for f in range(len(d["tx"]))))
    assert worst < 2e-13, worst
