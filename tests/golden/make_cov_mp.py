"""Independent pins of WCE_MMSE_COV (a caller's channel covariance Rhh) at the
operating noise power, one per solve form the library selects.

WiFi_channel_estimation_PS_MMSE.m:26-32 with the model Rhh in place of
ifft(H_EST) ifft(H_EST)', evaluated LITERALLY in mpmath at 50 digits exactly
as tests/golden/make_textbook_mp.py does for the headline:
    Rhy = Rhh*F'*X4,  Ryy = X4*F*Rhh*F'*X4' + ow2*eye(53),  H = F*Rhy*pinv(Ryy)*rx
(full 53 x 53 products, pinv by mpmath's LU inverse).  Rhh = diag(p) with
p_t = exp(-d t) / sum * 1.1e-4 for t < L (bench.py bench_cov_lowrank's
profiles): L = 4, 8 (one frame per lane), 12, 16 (16 lanes per frame), 24
(two Gram rows per lane), 53 taps (the tap-domain wave kernel) and the
full-rank exp(-0.12 t) profile of the dense COV solve (bench cov_mode).
Frames (block 0): the inputs.h frame, frames 0 and 65,535 of the bench's
batch (make_textbook_mp.synth_block0), and one QPSK frame with its own
channel.  ow2 = inputs.h's 9.6172e-8.

Output tests/golden/cov_mp_pins.npz (data only).  CPU only, ~1 min on 8 cores.
Usage: python tests/golden/make_cov_mp.py
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_textbook_mp as tb  # noqa: E402

N = 53
PROFILES = [(4, 0.5), (8, 0.5), (12, 0.5), (16, 0.5), (24, 0.5), (53, 0.5), (53, 0.12)]


def pdp(L, decay):
    p = np.zeros(N)
    p[:L] = np.exp(-decay * np.arange(L))
    return p / p.sum() * 1.1e-4


def cov_literal(args):
    tx, rx, p, ow2 = args
    import mpmath as mp
    mp.mp.dps = tb.DPS
    c = lambda z: mp.mpc(float(z.real), float(z.imag))
    F = mp.matrix(N, N)
    for t in range(N):
        for f in range(N):
            F[t, f] = mp.expjpi(-2 * mp.mpf(t * f) / N)
    FH = F.transpose_conj()
    Rhh = mp.diag([mp.mpf(float(v)) for v in p])
    X4 = mp.diag([c(v) for v in tx])
    Rhy = Rhh * FH * X4
    Ryy = X4 * F * Rhh * FH * X4.transpose_conj() + mp.mpf(float(ow2)) * mp.eye(N)
    H = F * Rhy * mp.inverse(Ryy) * mp.matrix([c(v) for v in rx])
    hi = np.array([complex(float(H[k].real), float(H[k].imag)) for k in range(N)])
    lo = np.array([complex(float(H[k].real - mp.mpf(hi[k].real)), float(H[k].imag - mp.mpf(hi[k].imag)))
                   for k in range(N)])
    return hi, lo


def main():
    inp = dict(np.load(os.path.join(HERE, "inputs_h.npz")))
    ow2 = float(inp["ow2"])
    hlt = tb.h_lt_fp64(inp["tx_pre"], inp["rx_pre"], ow2)
    frames = [(inp["tx_symb"][0].copy(), inp["rx_symb"][0].copy())]
    frames += [tb.synth_block0(f, hlt, ow2) for f in (0, 65535)]
    frames += [tb.unrelated_frames(ow2)[3]]          # the QPSK frame of the TEXTBOOK pins
    jobs = [(t, r, pdp(L, d), ow2) for (L, d) in PROFILES for (t, r) in frames]
    with Pool(8) as pool:
        res = pool.map(cov_literal, jobs)
    nf = len(frames)
    np.savez_compressed(os.path.join(HERE, "cov_mp_pins.npz"),
                        tx=np.array([t for t, _ in frames]), rx=np.array([r for _, r in frames]),
                        taps=np.array([L for L, _ in PROFILES]), decay=np.array([d for _, d in PROFILES]),
                        pdp=np.array([pdp(L, d) for L, d in PROFILES]),
                        H_hi=np.array([h for h, _ in res]).reshape(len(PROFILES), nf, N),
                        H_lo=np.array([lo for _, lo in res]).reshape(len(PROFILES), nf, N), ow2=np.float64(ow2))
    print("wrote cov_mp_pins.npz:", len(PROFILES), "profiles x", nf, "frames")


if __name__ == "__main__":
    main()
