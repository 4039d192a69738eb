"""Interleaved A/B timing of mmse_solve across libwce.so variants, one process
(MI355X_MICROARCH / cdna_hip_programming 5.4 rule 24).
usage: python tools/ab_solve.py build_variants/A build_variants/B ... [--rounds 7] [--frames 65536]"""
import argparse
import ctypes
import importlib.util
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--frames", type=int, default=65536)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--mode", type=int, default=1)
ap.add_argument("--entry", choices=["solve", "estimate"], default="solve",
                help="estimate: the headline wce_estimate(PS_MMSE) (rank-1 bordered-dot kernel)")
args = ap.parse_args()

mods = []
for d in args.dirs:
    spec = importlib.util.spec_from_file_location("wce_" + os.path.basename(d.rstrip("/")),
                                                  os.path.join(REPO, "80211parallelestimation_amd", "wce.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m._lib = None
    m.load(os.path.join(d, "libwce.so"))
    mods.append((os.path.basename(d.rstrip("/")), m))

inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
B, N, NB = args.frames, 53, 15
state = []
for name, m in mods:
    ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], args.mode)
    hlt, _, _, _ = ctx.shared()
    tx, rx = m.DeviceArray((B, NB, N)), m.DeviceArray((B, NB, N))
    hs = m.DeviceArray.from_numpy(hlt)
    ctx.synth(tx, rx, None, B, h_shared=hs)
    W = m.DeviceArray((B, N), zero=True)
    st = m.Stream()
    fr = ctx.frames(tx, rx, B)
    if args.entry == "estimate":
        outs = m.Outputs(None, None, None, None, W.addr, None, N, 0, 0, 0, 0)
        ctx.mmse_solve = lambda fr, W, n, s, c=ctx, o=outs, mm=m: c.estimate(fr, o, mm.PS_MMSE, s)
    state.append((name, m, ctx, fr, W, st, tx, rx, hs))
import time
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:   # clock ramp before the first timed round
    for name, m, ctx, fr, W, st, *_ in state:
        ctx.mmse_solve(fr, W, N, st.handle)
    state[0][5].synchronize()
res = {name: [] for name, *_ in state}
outs = {}
for rnd in range(args.rounds + 1):
    for name, m, ctx, fr, W, st, *_ in state:
        e0, e1 = m.Event(), m.Event()
        ctx.mmse_solve(fr, W, N, st.handle)
        e0.record(st)
        for _ in range(args.reps):
            ctx.mmse_solve(fr, W, N, st.handle)
        e1.record(st)
        ms = e0.elapsed_ms(e1) / args.reps
        if rnd > 0:
            res[name].append(ms)
        outs[name] = W.numpy()[:64]
base = None
for name, v in res.items():
    med = float(np.median(v))
    base = base or med
    fl = (4 / 3 * N ** 3 + 20 * N * N) * B
    print(f"{name:24s} median {med:.4f} ms  min {min(v):.4f}  {fl / med / 1e9:.2f} TFLOP/s  x{base / med:.3f}")
ref = outs[state[0][0]]
for name, o in outs.items():
    err = np.max(np.abs(o - ref)) / np.max(np.abs(ref))
    print(f"  {name:22s} max rel diff vs {state[0][0]}: {err:.2e}")
