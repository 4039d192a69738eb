"""The COV low-rank kernels on complex symbols: the bench's BPSK frames against
the same frames turned QPSK (tx and rx times one unit phase per symbol, so the
channel and the noise statistics are unchanged), HIP-event timing.
usage: python tools/ab_cplx.py [--taps 16 24] [--frames 65536] [--lib path/libwce.so]"""
import argparse
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
N, NBLK = 53, 15


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--taps", type=int, nargs="+", default=[16, 24])
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lib", default=None, help="libwce.so to load (default: the in-tree build)")
    args = ap.parse_args()
    wce = importlib.import_module("80211parallelestimation_amd")
    if args.lib:
        sys.modules["80211parallelestimation_amd.wce"]._lib = None
        wce.load(os.path.abspath(args.lib))
    import bench
    import prof_leg
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    n = args.frames
    stream = wce.Stream()
    s = stream.handle
    c0 = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
    c0.synth(tx, rx, None, n, seed=0x80211)
    wce.synchronize()
    ph = np.exp(1j * np.pi / 4 * (2 * np.random.default_rng(5).integers(0, 4, (n, NBLK, N)) + 1))
    txq = wce.DeviceArray.from_numpy(tx.numpy() * ph)
    rxq = wce.DeviceArray.from_numpy(rx.numpy() * ph)
    H = wce.DeviceArray((n, N), zero=True)
    o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    for L in args.taps:
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=prof_leg.pdp_rank(L))
        res = {}
        for name, (t, r) in (("bpsk", (tx, rx)), ("qpsk", (txq, rxq))):
            fr = ctx.frames(t, r, n)
            run = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
            for _ in range(3):
                run()
            res[name] = bench.time_events(wce, stream, run, args.reps)
        print(f"L={L} {ctx.lr_kernel(n)}: BPSK {res['bpsk'] * 1e3:.1f} us, QPSK {res['qpsk'] * 1e3:.1f} us "
              f"({res['qpsk'] / res['bpsk']:.2f}x)")


if __name__ == "__main__":
    main()
