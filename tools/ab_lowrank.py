"""Interleaved A/B of the WCE_MMSE_COV low-rank forms at one rank: the
library's default selection (round 6: mmse_lr_quad2_kernel for ranks 17..32
with taps 0..r-1) against the wave kernel on the same frames and buffers
(wce_debug_set_variant(3, 1)), HIP-event timing, outputs compared.
usage: python tools/ab_lowrank.py [--taps 17 20 24 28 32] [--frames 65536] [--rounds 5]"""
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
    ap.add_argument("--taps", type=int, nargs="+", default=[17, 20, 24, 28, 32])
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    wce = importlib.import_module("80211parallelestimation_amd")
    import bench
    lib = wce.load()
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    n = args.frames
    stream = wce.Stream()
    s = stream.handle
    c0 = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
    c0.synth(tx, rx, None, n, seed=0x80211, h_shared=wce.DeviceArray.from_numpy(c0.shared()[0]))   # the bench's frames
    fr = wce.Context.frames(tx, rx, n)
    H = wce.DeviceArray((n, N), zero=True)
    o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    for L in args.taps:
        p = np.exp(-0.5 * np.arange(L))
        R = np.zeros((N, N), np.complex128)
        R[np.arange(L), np.arange(L)] = p / p.sum() * 1.1e-4     # bench.py bench_cov_lowrank's profile
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R)
        run = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
        vs = (0, 7, 6, 1) if 20 < L <= 24 else (0, 6, 1) if L == 16 else (0, 7, 1)   # 6: quad2's Cholesky broadcasts as separate movs; 7: 1 wave/SIMD
        names, times, outs = {}, {v: [] for v in vs}, {}
        for r in range(args.rounds):
            for v in vs:
                assert lib.wce_debug_set_variant(3, v) == 0
                names[v] = ctx.lr_kernel(n)
                for _ in range(3):
                    run()
                times[v].append(bench.time_events(wce, stream, run, args.reps))
                if r == 0:
                    outs[v] = H.numpy()
        assert lib.wce_debug_set_variant(3, 0) == 0
        d = np.max(np.abs(outs[0] - outs[1]), axis=1) / np.maximum(np.max(np.abs(outs[1]), axis=1), 1e-300)
        if 6 in outs:
            print(f"L={L} fused-DPP Cholesky bit-identical to the separate movs: {bool(np.array_equal(outs[0], outs[6]))}")
        if 7 in outs:
            print(f"L={L} 1-wave/SIMD build bit-identical: {bool(np.array_equal(outs[0], outs[7]))}")
        fl = bench.flop_lr_taps(L)
        for v in vs:
            t = float(np.median(times[v]))
            print(f"L={L} v{v} {names[v]:28s} median {t * 1e3:7.1f} us  {fl * n / (t * 1e-3) / 1e12:5.1f} TF "
                  f"({100 * fl * n / (t * 1e-3) / 1e12 / bench.PEAK_FP64_TFLOPS:4.1f}% of FP64 peak)  "
                  f"({', '.join(f'{x * 1e3:.0f}' for x in times[v])})")
        print(f"L={L} outputs: max norm-rel diff {d.max():.2e}, finite {bool(np.isfinite(outs[0]).all())}")


if __name__ == "__main__":
    main()
