"""Interleaved A/B of whole libwce.so builds (tools/variants.sh) on one leg,
one process: rounds x libraries, HIP-event timing per launch.
legs: config5 (all 5 estimators + equalization fused, fp32 LS/eq outputs,
per-frame preambles), headline (PS_MMSE TEXTBOOK), dense (COV mmse_solve), apply (COV H = C W).
usage: python tools/ab_libs.py build_variants/A build_variants/B [--leg config5] [--frames 262144]"""
import argparse
import importlib.util
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--leg", choices=["config5", "headline", "dense", "apply", "r1dense", "lowrank", "cm", "cmq", "fcref", "c5ref_fc",
                                 "refmm", "fctb"],
                default="config5")
ap.add_argument("--taps", type=int, default=8, help="lowrank: L-tap PDP covariance (rank L; 53 = decay 0.5)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--frames", type=int, default=262144)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
N, NB, n = 53, 15, args.frames
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
runs = []
for d in args.dirs:
    spec = importlib.util.spec_from_file_location("wce_" + os.path.basename(d.rstrip("/")),
                                                  os.path.join(REPO, "80211parallelestimation_amd", "wce.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m._lib = None
    m.load(os.path.join(d, "libwce.so"))
    st = m.Stream()
    if args.leg in ("dense", "apply"):
        import prof_leg
        ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=prof_leg.pdp_rhh())
    elif args.leg in ("lowrank", "cm", "cmq"):   # cm(q): the same ctx on the constant-modulus operator (wce_ctx_set_modulus)
        import prof_leg
        ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=prof_leg.pdp_rank(args.taps))
    elif args.leg in ("fcref", "c5ref_fc", "refmm"):
        ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m.MMSE_REF)
    else:
        ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m.MMSE_TEXTBOOK)
    if args.leg == "cmq":   # QPSK frames (non-real symbols of one modulus: cm_real_kernel flags, cm_cplx_kernel solves)
        rng = np.random.default_rng(7)
        A = 8.8753
        xq = A * (rng.choice([-1.0, 1.0], (n, 1, N)) + 1j * rng.choice([-1.0, 1.0], (n, 1, N))) / np.sqrt(2)
        xq[:, :, 26] = 0
        hq = 1e-2 * np.exp(1j * rng.uniform(0, 2 * np.pi, (n, 1, 1)))
        rq = hq * xq + np.sqrt(inp["ow2"] / 2) * (rng.standard_normal(xq.shape) + 1j * rng.standard_normal(xq.shape))
        tx, rx = m.DeviceArray.from_numpy(xq), m.DeviceArray.from_numpy(rq)
        pre = None
        keep = [tx, rx]
    else:
        tx, rx, pre = m.DeviceArray((n, NB, N)), m.DeviceArray((n, NB, N)), m.DeviceArray((n, N))
        ctx.synth(tx, rx, pre, n, seed=0x80211)
        keep = [tx, rx, pre]
    m.synchronize()   # synth runs on the null stream; the legs on st
    if args.leg == "config5":
        outs = [m.DeviceArray((n, N), np.complex64) for _ in range(4)] + [m.DeviceArray((n, N))]
        eq = m.DeviceArray((n, NB, N), np.complex64)
        o = m.Outputs(*(x.addr for x in outs), eq.addr, N, NB * N, N, 0, m.OUT_LS_F32)
        fr = ctx.frames(tx, rx, n, rx_pre=pre)
        f = (lambda c, fr, o, st, m: lambda: c.estimate(fr, o, m.ALL, st.handle))(ctx, fr, o, st, m)
        keep += outs + [eq]
        check = outs[4]
    elif args.leg in ("fcref", "c5ref_fc", "fctb"):   # REF / TEXTBOOK (fctb) + FRAME_COV: PS_MMSE alone / all 5 + eq (fp64)
        ctx.reserve(n)
        fr = ctx.frames(tx, rx, n, rx_pre=pre)
        if args.leg in ("fcref", "fctb"):
            H = m.DeviceArray((n, N))
            o = m.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
            mk = m.PS_MMSE | m.FRAME_COV
            keep.append(H)
        else:
            outs = [m.DeviceArray((n, N)) for _ in range(5)]
            eq = m.DeviceArray((n, NB, N))
            o = m.Outputs(*(x.addr for x in outs), eq.addr, N, NB * N, N, 0, 0)
            mk = m.ALL | m.FRAME_COV
            keep += outs + [eq]
            H = outs[4]
        f = (lambda c, fr, o, st, mk: lambda: c.estimate(fr, o, mk, st.handle))(ctx, fr, o, st, mk)
        check = H
    elif args.leg in ("headline", "lowrank", "cm", "cmq", "refmm"):   # refmm: REF PS_MMSE (mmse_ref_flat_kernel)
        if args.leg == "cm":
            ctx.set_modulus(tx.rows(0)[0, 0])
        if args.leg == "cmq":
            ctx.set_modulus(xq[0, 0])
        H = m.DeviceArray((n, N))
        fr = ctx.frames(tx, rx, n, frame_stride=N, block_stride=N) if args.leg == "cmq" else ctx.frames(tx, rx, n)
        o = m.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
        f = (lambda c, fr, o, st, m: lambda: c.estimate(fr, o, m.PS_MMSE, st.handle))(ctx, fr, o, st, m)
        keep.append(H)
        check = H
    elif args.leg == "apply":   # H = C W alone, on the solve's W
        W, H = m.DeviceArray((n, N)), m.DeviceArray((n, N))
        ctx.mmse_solve(ctx.frames(tx, rx, n), W, N, st.handle)
        f = (lambda c, W, H, st: lambda: c.mmse_apply(W, H, n, N, st.handle))(ctx, W, H, st)
        keep += [W, H]
        check = H
    else:   # dense: COV mmse_solve_kernel<false>; r1dense: TEXTBOOK through the same back-substitution kernel (<true>)
        if args.leg == "r1dense":
            ctx.set_border_dot(False)
        W = m.DeviceArray((n, N))
        fr = ctx.frames(tx, rx, n)
        f = (lambda c, fr, W, st: lambda: c.mmse_solve(fr, W, N, st.handle))(ctx, fr, W, st)
        keep.append(W)
        check = W
    runs.append((os.path.basename(d.rstrip("/")), m, st, f, check, keep, ctx))
times = {r[0]: [] for r in runs}
for rd in range(args.rounds):
    for name, m, st, f, check, keep, ctx in runs:
        for _ in range(3):
            f()
        e0, e1 = m.Event(), m.Event()
        e0.record(st.handle)
        for _ in range(args.reps):
            f()
        e1.record(st.handle)
        times[name].append(e0.elapsed_ms(e1) / args.reps)
outs = [r[4].numpy() for r in runs]
if args.leg == "apply":   # each library's H against its own W: H = C W exactly as numpy forms it (to rounding)
    for name, m, st, f, check, keep, ctx in runs:
        Wh = keep[3].numpy()
        C = ctx.shared()[1]
        ref = Wh @ C.T
        o = check.numpy()
        den = np.abs(ref).max(1)
        err = np.abs(o - ref).max(1) / np.where(den > 0, den, 1)
        print(f"apply {name}: W all-zero frames {int(np.sum(~Wh.any(1)))}, max norm-rel |H - W C^T| {err.max():.2e}")
for (name, *_), o in zip(runs, outs):
    print(f"{args.leg} {name}: median {np.median(times[name]) * 1e3:.1f} us  "
          f"({', '.join(f'{t * 1e3:.0f}' for t in times[name])})  same output as {runs[0][0]}: "
          f"{bool(np.array_equal(o, outs[0], equal_nan=True))}  max norm-rel diff "
          f"{float(np.nanmax(np.abs(o - outs[0]).reshape(n, -1).max(1) / np.abs(outs[0]).reshape(n, -1).max(1))):.2e}"
          f"  non-finite frames {int(np.sum(~np.isfinite(o.reshape(n, -1)).all(1)))}"
          f"  all-zero frames {int(np.sum(~o.reshape(n, -1).any(1)))}")
