"""Generate the committed golden fixtures from the reference itself.

Runs only where /root/reference is mounted (never on the GPU box):
  1. builds oracle/_ref/libref.so from the reference's own main.c/utils.c
     (oracle/Makefile, target `ref`);
  2. calls the reference's functions through it and stores inputs + outputs
     as data (npz): tests/golden/{inputs_h,ref_vectors,matlab_pins}.npz.

Long double outputs are stored exactly as (hi, lo) float64 pairs with
hi = fp64(x), lo = x - hi.

Usage: python tests/golden/make_golden.py
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("WCE_REFERENCE", "/root/reference")
N, NBLK = 53, 15
PILOTS = (5, 19, 33, 47)
LD = np.clongdouble


def p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def split(x):
    x = np.asarray(x, dtype=np.clongdouble)
    re, im = x.real, x.imag
    hr, hi_ = re.astype(np.float64), im.astype(np.float64)
    lr = (re - hr.astype(np.longdouble)).astype(np.float64)
    li = (im - hi_.astype(np.longdouble)).astype(np.float64)
    return np.stack([hr, hi_, lr, li], axis=-1)   # [..., 4] = re_hi, im_hi, re_lo, im_lo


def synth_frames(rng, n, A=8.8753, ow2=9.6172e-08):
    """Synthetic block-0 frames (BPSK, 802.11 pilots, 6-tap channel, AWGN)."""
    tx = np.where(rng.random((n, N)) < 0.5, -A, A).astype(np.complex128)
    tx[:, 26] = 0
    for i, k in enumerate(PILOTS):
        tx[:, k] = A * (1, 1, 1, -1)[i]
    taps = (rng.standard_normal((n, 6)) + 1j * rng.standard_normal((n, 6))) * 0.0105 / np.sqrt(2 * 6)
    taps *= np.exp(-0.25 * np.arange(6))
    kk = np.arange(N) - 26
    H = taps @ np.exp(-2j * np.pi * np.outer(np.arange(6), kk) / 64)
    noise = (rng.standard_normal((n, N)) + 1j * rng.standard_normal((n, N))) * np.sqrt(ow2 / 2)
    return tx, H * tx + noise, H


def main():
    subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "ref", f"REF={REF}"])
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref.so"))
    lib.refh_ow2.restype = ctypes.c_double
    ow2 = lib.refh_ow2()
    txp, rxp = np.zeros(N, LD), np.zeros(N, LD)
    txs, rxs = np.zeros(N * NBLK, LD), np.zeros(N * NBLK, LD)
    lib.refh_inputs(p(txp), p(rxp), p(txs), p(rxs))
    for a in (txp, rxp, txs, rxs):   # inputs.h literals are doubles: complex128 is exact
        assert np.array_equal(a, a.astype(np.complex128).astype(LD))
    np.savez_compressed(os.path.join(HERE, "inputs_h.npz"), ow2=np.float64(ow2),
                        tx_pre=txp.astype(np.complex128), rx_pre=rxp.astype(np.complex128),
                        tx_symb=txs.reshape(NBLK, N).astype(np.complex128),
                        rx_symb=rxs.reshape(NBLK, N).astype(np.complex128))

    F = np.zeros((N, N), LD)
    lib.refh_fmatrix(p(F))
    invF = np.zeros((N, N), LD)
    lib.refh_inverse(p(F.copy()), N, p(invF))

    # frames: 0 = inputs.h block 0, 1..7 synthetic
    rng = np.random.default_rng(0x80211)
    stx, srx, _ = synth_frames(rng, 7)
    ftx = np.concatenate([txs[:N].astype(np.complex128)[None], stx])
    frx = np.concatenate([rxs[:N].astype(np.complex128)[None], srx])
    # preamble cases: 0 = inputs.h, 1 = synthetic preamble of a different channel
    _, _, Hp = synth_frames(rng, 1)
    rxp2 = Hp[0] * txp.astype(np.complex128) + (rng.standard_normal(N) + 1j * rng.standard_normal(N)) * np.sqrt(ow2 / 4)
    pres = [(txp, rxp), (txp, rxp2.astype(LD))]

    out = {"F": split(F), "invF": split(invF), "frames_tx": ftx, "frames_rx": frx, "ow2": np.float64(ow2),
           "pre_tx": np.stack([a.astype(np.complex128) for a, _ in pres]),
           "pre_rx": np.stack([b.astype(np.complex128) for _, b in pres])}
    for name in ("lt_ls", "ps_linear", "ps_cubic", "ps_sinc"):
        rows = []
        for f in range(len(ftx)):
            H = np.zeros(N, LD)
            if name == "lt_ls":
                getattr(lib, "refh_" + name)(p(txp.copy()), p(pres[f % 2][1].copy()), p(H))
            else:
                getattr(lib, "refh_" + name)(p(ftx[f].astype(LD)), p(frx[f].astype(LD)), p(H))
            rows.append(split(H))
        out[name] = np.stack(rows)
    hlt = []
    mm = []
    for c, (tp, rp) in enumerate(pres):
        H = np.zeros(N, LD)
        lib.refh_lt_ls(p(tp.copy()), p(rp.copy()), p(H))
        hlt.append(split(H))
        rows = []
        for f in range(len(ftx)):
            Hm = np.zeros(N, LD)
            lib.refh_mmse_repaired(p(ftx[f].astype(LD)), p(frx[f].astype(LD)), p(F.copy()), ctypes.c_double(ow2),
                                   p(H.copy()), p(invF.copy()), p(Hm), None)
            rows.append(split(Hm))
        mm.append(np.stack(rows))
    out["pre_lt_ls"] = np.stack(hlt)         # [case][53][4]
    out["ps_mmse_ref"] = np.stack(mm)        # [case][frame][53][4]

    # literal inverse(Ryy) known answer on a 6x6 diagonal (same bug as 53x53)
    R = np.diag(np.full(6, 2 * ow2)).astype(LD)
    Ri = np.zeros((6, 6), LD)
    lib.refh_inverse(p(R), 6, p(Ri))
    out["literal_inv_diag6_nan"] = np.isnan(Ri.real.astype(np.float64)) | np.isnan(Ri.imag.astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "ref_vectors.npz"), **out)

    import scipy.io as sio   # MAT v5: plain numeric arrays, no code execution
    m = sio.loadmat(os.path.join(REF, "matlab.mat"))
    keep = ["tx_symb", "rx_symb", "tx_preamble_fft", "rx_preamble_fft", "H_EST_LT_LS", "H_EST_PS_Linear",
            "H_EST_PS_Cubic", "H_EST_PS_Sinc", "H_EST_PS_Third", "eq_symbols", "tx_packet", "rx_packet",
            "tx_lptot", "rx_lptot", "rx_symb_long", "tx_symb_long", "rx_preamble1", "rx_preamble2"]
    np.savez_compressed(os.path.join(HERE, "matlab_pins.npz"),
                        **{k: np.asarray(m[k]).astype(np.complex128).squeeze() for k in keep})
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
