"""Interleaved A/B of kernel variants (wce_debug_set_variant) on the same
buffers in one process: rounds x (variant a, variant b, ...), HIP-event
timing per launch, outputs compared bit for bit across variants.
usage: python tools/ab_variant.py {ref,ls,dense} [--variants 0 1] [--rounds 5] [--reps 20]"""
import argparse
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
N, NBLK = 53, 15
WHICH = {"ref": 0, "ls": 1, "dense": 2, "headline": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("leg", choices=sorted(WHICH))
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--floor", action="store_true",
                    help="ref: also time PS_Linear alone on the same frames (ls_elem_kernel: the same 8 pilot "
                         "sectors in and 848 B out per frame, i.e. the REF read-out's traffic shape)")
    args = ap.parse_args()
    wce = importlib.import_module("80211parallelestimation_amd")
    import bench
    lib = wce.load()
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    n = args.frames
    stream = wce.Stream()
    s = stream.handle
    if args.leg == "ref":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        tx, rx, fr = bench.ref_frames(wce, ctx, n)
        H = wce.DeviceArray((n, N), zero=True)
        outs = [H]
        o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
        run = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
        alg, unit = bench.BYTES_REF_ALG, "alg"
    elif args.leg == "headline":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
        hlt = ctx.shared()[0]
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211, h_shared=wce.DeviceArray.from_numpy(hlt))
        fr = ctx.frames(tx, rx, n)
        H = wce.DeviceArray((n, N), zero=True)
        outs = [H]
        o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
        run = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
        alg, unit = bench.FLOP_SOLVE_TXT / 1000.0 + bench.FLOP_APPLY / 1000.0, "(= PF/s of F_alg)"
    elif args.leg == "dense":
        # COV mode (full-rank PDP covariance): the dense solve alone (W = X z)
        import prof_leg
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=prof_leg.pdp_rhh())
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211)
        fr = ctx.frames(tx, rx, n)
        W = wce.DeviceArray((n, N), zero=True)
        outs = [W]
        run = lambda: ctx.mmse_solve(fr, W, N, s)
        alg, unit = bench.FLOP_SOLVE_TXT / 1000.0, "(= PF/s of F_alg solve flops)"
    else:
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        bufs, fr = bench.ls_frames(wce, ctx, n)
        hlt, hlin = wce.DeviceArray((n, N)), wce.DeviceArray((n, N))
        outs = [hlt, hlin]
        o = wce.Outputs(hlt.addr, hlin.addr, None, None, None, None, N, 0, 0, 0, 0)
        run = lambda: ctx.estimate(fr, o, wce.LT_LS | wce.PS_LINEAR, s)
        alg, unit = bench.BYTES_LS_CFG2, "alg"
    ref_out = None
    times = {v: [] for v in args.variants}
    for r in range(args.rounds):
        for v in args.variants:
            assert lib.wce_debug_set_variant(WHICH[args.leg], v) == 0
            for _ in range(3):
                run()
            t = bench.time_events(wce, stream, run, args.reps)
            times[v].append(t)
            if r == 0:
                got = [x.numpy() for x in outs]
                if ref_out is None:
                    ref_out = got
                else:
                    same = all(np.array_equal(a, b) for a, b in zip(got, ref_out))
                    dif = max(float(np.max(np.abs(a - b), axis=-1).max() / max(np.abs(b).max(), 1e-300))
                              for a, b in zip(got, ref_out))
                    print(f"variant {v}: outputs bit-identical to variant {args.variants[0]}: {same} "
                          f"(max |diff| / max |ref| = {dif:.2e})")
    if args.floor and args.leg == "ref":
        hl = wce.DeviceArray((n, N), zero=True)
        ol = wce.Outputs(None, hl.addr, None, None, None, None, N, 0, 0, 0, 0)
        lin = lambda: ctx.estimate(fr, ol, wce.PS_LINEAR, s)
        for _ in range(3):
            lin()
        tl = [bench.time_events(wce, stream, lin, args.reps) for _ in range(args.rounds)]
        t = float(np.median(tl))
        print(f"same traffic shape, PS_Linear alone (ls_elem_kernel): median {t * 1e3:.1f} us  "
              f"{(bench.BYTES_PILOT_SECTORS + N * 16) * n / (t * 1e-3) / 1e12:.2f} TB/s on the sector floor "
              f"({', '.join(f'{x * 1e3:.0f}' for x in tl)})")
    for v, ts in times.items():
        t = float(np.median(ts))
        print(f"{args.leg} variant {v}: median {t * 1e3:.1f} us  min {min(ts) * 1e3:.1f}  "
              f"{alg * n / (t * 1e-3) / 1e12:.2f} TB/s {unit}  ({', '.join(f'{x * 1e3:.0f}' for x in ts)})")


if __name__ == "__main__":
    main()
