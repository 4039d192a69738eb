"""Interleaved A/B timing of the LS path (config 2: LT_LS + PS_Linear, per-frame
preamble) across libwce.so variants, one process.
usage: python tools/ab_ls.py build_variants/A build_variants/B ... [--frames 1048576]"""
import argparse
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--frames", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--mask", type=int, default=3)
ap.add_argument("--ostride", type=int, default=53, help="output row stride (complex); 64 = 1 KiB-aligned rows")
ap.add_argument("--sets", type=int, default=1, help="independently allocated buffer sets, each timed with every variant")
args = ap.parse_args()
N = 53
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
rng = np.random.default_rng(1)
chunk = 65536
txh = np.where(rng.random((chunk, N)) < 0.5, -8.8753, 8.8753).astype(np.complex128)
rxh = txh * (0.01 + 0.001j) + 1e-4 * rng.standard_normal((chunk, N))
preh = np.repeat(((0.01 + 0.001j) * inp["tx_pre"])[None], chunk, axis=0) + 1e-4 * rng.standard_normal((chunk, N))
state = []
for d in args.dirs:
    spec = importlib.util.spec_from_file_location("w" + os.path.basename(d.rstrip("/")),
                                                  os.path.join(REPO, "80211parallelestimation_amd", "wce.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m._lib = None
    lib = m.load(os.path.join(d, "libwce.so"))
    ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m.MMSE_REF)
    n = args.frames
    if not state:
        # buffer sets shared by every variant: HBM placement moves the timing by
        # up to ~15% between allocations, more than most variants differ
        bsets = []
        for _ in range(args.sets):
            tx, rx, pre = m.DeviceArray((n, N)), m.DeviceArray((n, N)), m.DeviceArray((n, N))
            for off in range(0, n, chunk):
                k = min(chunk, n - off)
                for dst, h in ((tx, txh), (rx, rxh), (pre, preh)):
                    assert lib.wce_memcpy_htod(dst.addr + off * N * 16, h[:k].ctypes.data, k * N * 16) == 0
            bsets.append((tx, rx, pre, [m.DeviceArray((n, args.ostride)) for _ in range(4)]))
    for si, (tx, rx, pre, outs) in enumerate(bsets):
        o = m.Outputs(*(x.addr for x in outs), None, None, args.ostride, 0, 0, 0, 0)
        fr = ctx.frames(tx.addr, rx.addr, n, frame_stride=N, block_stride=N, rx_pre=pre.addr, pre_stride=N)
        name = os.path.basename(d.rstrip("/")) + (f"@set{si}" if args.sets > 1 else "")
        state.append((name, m, ctx, fr, o, m.Stream(), bsets))
res = {s[0]: [] for s in state}
for rnd in range(args.rounds + 1):
    for name, m, ctx, fr, o, st, _ in state:
        ctx.estimate(fr, o, args.mask, st.handle)
        e0, e1 = m.Event(), m.Event()
        e0.record(st)
        for _ in range(args.reps):
            ctx.estimate(fr, o, args.mask, st.handle)
        e1.record(st)
        if rnd:
            res[name].append(e0.elapsed_ms(e1) / args.reps)
for name, v in res.items():
    med = float(np.median(v))
    print(f"{name:12s} median {med * 1e3:8.1f} us  min {min(v) * 1e3:8.1f}  {2672 * args.frames / (med * 1e-3) / 1e9:7.0f} GB/s (alg, config 2)")
