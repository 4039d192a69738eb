"""Golden MMSE outputs from the reference's OWN matrix routines (round 3).

The reference holds no MMSE output for WiFi_channel_estimation_PS_MMSE.m's
formula (matlab.mat has none, and main.c's PS_MMSE is NaN).  Its
utils.c does hold the routines that formula needs: multiply() and the cofactor
inverse().  oracle/ref_harness.cpp:refh_mmse_formula composes
    H = F (Rhh F' X4) inv(X4 F Rhh F' X4' + ow2 I) rx
from them in the reference's long double complex, with Rhh = ifft(H_LS)
ifft(H_LS)' (TEXTBOOK) or a model covariance (WCE_MMSE_COV).

The cofactor inverse (unpivoted Schur determinants of every minor) is only as
good as Ryy's conditioning allows: at the frames' own noise power (cond(Ryy)
~4e6) it is 4e-9 away from the long double closed form, so the pins use
ow2 = 1e-3, 1e-4, 1e-5 (cond ~4e2 .. 4e4), where it agrees with
oracle_py's closed form / unified solve to <= 2.0e-12
(tests/test_oracle.py::test_mmse_formula_pins_vs_oracle).

Runs only where /root/reference is mounted (never on the GPU box); writes
tests/golden/mmse_formula_pins.npz (data only).
Usage: python tests/golden/make_mmse_pins.py
"""
import ctypes
import os
import subprocess
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
REF = os.environ.get("WCE_REFERENCE", "/root/reference")
N = 53
LD = np.clongdouble
OW2S = (1e-3, 1e-4, 1e-5)


def pdp(L, decay):
    p = np.zeros(N)
    p[:L] = np.exp(-decay * np.arange(L))
    return np.diag(p / p.sum() * 1.1e-4).astype(np.complex128)


COVS = {"textbook": None, "pdp6": pdp(6, 0.5), "pdp53": pdp(53, 0.12)}


def _one(args):
    kind, f, ow2, tx, rx, F, hls = args
    from make_golden import p
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref.so"))
    H = np.zeros(N, LD)
    R = COVS[kind]
    lib.refh_mmse_formula(p(tx.astype(LD)), p(rx.astype(LD)), p(F.copy()), ctypes.c_double(ow2),
                          p(hls.copy()), p(R.astype(LD)) if R is not None else None, p(H))
    return kind, f, ow2, H


def main():
    from make_golden import split, synth_frames, p
    subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle", ), "ref", f"REF={REF}"])
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref.so"))
    inp = dict(np.load(os.path.join(HERE, "inputs_h.npz")))
    F = np.zeros((N, N), LD)
    lib.refh_fmatrix(p(F))
    hls = np.zeros(N, LD)
    lib.refh_lt_ls(p(inp["tx_pre"].astype(LD)), p(inp["rx_pre"].astype(LD)), p(hls))   # main.c:66-75
    rng = np.random.default_rng(0x3A55)
    stx, srx, _ = synth_frames(rng, 3)     # channels of their own (not the preamble's)
    tx = np.concatenate([inp["tx_symb"][:1], stx])
    rx = np.concatenate([inp["rx_symb"][:1], srx])
    jobs = [(k, f, w, tx[f], rx[f], F, hls) for k in COVS for w in OW2S for f in range(len(tx))]
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(_one, jobs)
    out = {"frames_tx": tx, "frames_rx": rx, "ow2": np.array(OW2S), "h_ls": split(hls),
           "rhh_pdp6": COVS["pdp6"], "rhh_pdp53": COVS["pdp53"]}
    for kind in COVS:
        out["H_" + kind] = np.stack([np.stack([split(next(H for k, ff, ww, H in res if k == kind and ff == f
                                                         and ww == w)) for f in range(len(tx))]) for w in OW2S])
    np.savez_compressed(os.path.join(HERE, "mmse_formula_pins.npz"), **out)   # H_*: [ow2][frame][53][4]
    print("written", os.path.join(HERE, "mmse_formula_pins.npz"))


if __name__ == "__main__":
    sys.exit(main())
