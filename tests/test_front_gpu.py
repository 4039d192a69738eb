"""GPU parity for the time-domain front end:
WiFi_blocks_extraction.m:1-11 and WiFi_RX.m:18-30 on the device, pinned by
matlab.mat (tx/rx_packet -> tx/rx_symb, tx/rx_lptot -> *_preamble_fft) and
checked against the oracle's long double direct DFT; then the whole
WiFi_RX.m receive chain (front end -> MATLAB-semantics estimators ->
equalization) from time-domain samples to matlab.mat's H_EST_* and eq_symbols."""
import numpy as np
import pytest

from oracle_py import N, NBLK, normrel

pytestmark = pytest.mark.gpu

TOL_FE = 1e-14


def _rel(a, ref):
    a, ref = np.asarray(a, np.complex128), np.asarray(ref, np.complex128)
    return np.max(np.abs(a - ref)) / np.max(np.abs(ref))


@pytest.fixture(scope="module")
def fe_ctx(gpu_wce):
    """The front end needs no shared state: an empty ctx only binds the device."""
    return gpu_wce.Context(empty=True)


@pytest.mark.parametrize("side", ["rx", "tx"])
def test_front_end_matlab_pins(gpu_wce, golden, fe_ctx, side):
    m = golden["matlab"]
    sym, pre, ow2 = fe_ctx.front_end_host(m[side + "_packet"][None], m[side + "_lptot"][None])
    assert _rel(sym[0], m[side + "_symb"].T) < TOL_FE
    assert _rel(pre[0], m[side + "_preamble_fft"]) < TOL_FE
    if side == "rx":
        d = m["rx_preamble2"] - m["rx_preamble1"]
        ref = np.sum(np.abs(d) ** 2) / 128     # WiFi_RX.m:30
        assert abs(ow2[0] - ref) <= 1e-14 * ref
        assert abs(ow2[0] - 9.6172e-08) < 1e-11   # inputs.h:18 OW2 is its 4-digit rounding
    else:
        assert ow2[0] == 0.0   # the transmitted LTF copies are identical


def test_front_end_batch_vs_oracle(gpu_wce, oracle, fe_ctx):
    """Random packets with padded strides: every block of every frame vs numpy's
    FFT; sampled frames vs the oracle's long double direct DFT."""
    rng = np.random.default_rng(5)
    B, nb, pstride, L, lstride = 777, NBLK, NBLK * 80 + 9, 160, 171
    pk = (rng.standard_normal((B, pstride)) + 1j * rng.standard_normal((B, pstride))) * 0.01
    lp = (rng.standard_normal((B, lstride)) + 1j * rng.standard_normal((B, lstride))) * 0.01
    dpk, dlp = gpu_wce.DeviceArray.from_numpy(pk), gpu_wce.DeviceArray.from_numpy(lp)
    fs, bs = nb * 64 + 3, 60                       # padded output strides
    dsym = gpu_wce.DeviceArray((B, fs), zero=True)
    dpre = gpu_wce.DeviceArray((B, 56), zero=True)
    dow2 = gpu_wce.DeviceArray((B,), np.float64, zero=True)
    fe_ctx.front_end_blocks(dpk, B, nb, dsym, packet_stride=pstride, frame_stride=fs, block_stride=bs)
    fe_ctx.front_end_preamble(dlp, B, L, dpre, dow2, lptot_stride=lstride, pre_stride=56)
    gpu_wce.synchronize()
    sym, pre, ow2 = dsym.numpy(), dpre.numpy(), dow2.numpy()
    blocks = pk[:, :nb * 80].reshape(B, nb, 80)[:, :, 16:]
    ref = np.roll(np.fft.fft(blocks, axis=-1), 26, axis=-1)[..., :N]
    got = np.stack([sym[:, b * bs:b * bs + N] for b in range(nb)], axis=1)
    assert _rel(got, ref) < TOL_FE
    # untouched padding stays zero
    for b in range(nb):
        assert np.all(sym[:, b * bs + N:(b + 1) * bs] == 0) if b < nb - 1 else True
    assert np.all(pre[:, N:] == 0)
    p1, p2 = lp[:, L - 64:L], lp[:, L - 128:L - 64]
    ref_pre = np.roll(np.fft.fft((p1 + p2) / 2, axis=-1), 26, axis=-1)[:, :N]
    assert _rel(pre[:, :N], ref_pre) < TOL_FE
    assert np.max(np.abs(ow2 - np.sum(np.abs(p2 - p1) ** 2, axis=1) / 128) / ow2) < 1e-14
    for f in (0, B - 1, 333):
        o = oracle.front_blocks(pk[f], nb)
        assert _rel(got[f], o) < TOL_FE, f
        op, ow = oracle.front_preamble(lp[f, :L])
        assert _rel(pre[f, :N], op) < TOL_FE
        assert abs(ow2[f] - float(ow)) <= 1e-14 * float(ow)


def test_receive_chain_time_domain_to_matlab(gpu_wce, golden):
    """WiFi_RX.m:17-60 on the device: time-domain tx/rx packets and LTFs ->
    front end -> estimators in MATLAB semantics -> equalization; compared
    with matlab.mat's H_EST_* and eq_symbols."""
    m = golden["matlab"]
    boot = gpu_wce.Context(empty=True)
    tx_sym, tx_pre, _ = boot.front_end_host(m["tx_packet"][None], m["tx_lptot"][None])
    rx_sym, rx_pre, ow2 = boot.front_end_host(m["rx_packet"][None], m["rx_lptot"][None])
    ctx = gpu_wce.Context(tx_pre[0], rx_pre[0], float(ow2[0]), gpu_wce.MMSE_TEXTBOOK)
    out = ctx.estimate_host(tx_sym, rx_sym, rx_pre=rx_pre, mask=gpu_wce.ALL, semantics=gpu_wce.SEM_MATLAB)
    for name, key in (("lt_ls", "H_EST_LT_LS"), ("ps_linear", "H_EST_PS_Linear"), ("ps_cubic", "H_EST_PS_Cubic"),
                      ("ps_sinc", "H_EST_PS_Sinc")):
        assert normrel(out[name][0], m[key]) < 1e-13, name
    assert _rel(out["eq"][0], m["eq_symbols"].T) < 1e-13
    assert np.all(np.isfinite(out["ps_mmse"]))


def test_front_end_errors(gpu_wce, fe_ctx):
    d = gpu_wce.DeviceArray((4, 1200), zero=True)
    o = gpu_wce.DeviceArray((4, NBLK * N), zero=True)
    with pytest.raises(gpu_wce.WceError):   # packet stride shorter than 15 blocks of 80
        fe_ctx.front_end_blocks(d, 4, NBLK, o, packet_stride=1199)
    with pytest.raises(gpu_wce.WceError):
        fe_ctx.front_end_blocks(d, 4, 0, o)
    with pytest.raises(gpu_wce.WceError):   # output block stride < 53
        fe_ctx.front_end_blocks(d, 4, NBLK, o, block_stride=52)
    with pytest.raises(gpu_wce.WceError):   # LTF shorter than two 64-sample copies
        fe_ctx.front_end_preamble(d, 4, 127, o)
    fe_ctx.front_end_blocks(d, 0, NBLK, o)   # empty batch: no-op
    gpu_wce.synchronize()
