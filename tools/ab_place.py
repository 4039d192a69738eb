"""HBM placement probe for the LS path (config 2: LT_LS + PS_Linear, per-frame
preamble).  One device allocation holds the five streams (tx, rx, rx_pre in;
LT_LS, PS_Linear out); each layout places them at different relative offsets.
Interleaved rounds, same kernel: only the placement differs.
usage: python tools/ab_place.py [--frames 1048576]"""
import argparse
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
wce = importlib.import_module("80211parallelestimation_amd")
lib = wce.load()
N, n = 53, args.frames
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
A = n * N * 16
MiB = 1 << 20
# layouts: gap (bytes) inserted after each of the 5 arrays, in order tx, rx, pre, lt, lin
layouts = {
    "packed": [0, 0, 0, 0, 0],
    "gap4K": [4096] * 5,
    "gap64K": [65536] * 5,
    "gap1M": [MiB] * 5,
    "gap2M+4K": [2 * MiB + 4096] * 5,
    "gap2M": [2 * MiB] * 5,
    "stagger": [0, 1 * MiB + 256, 2 * MiB + 512, 3 * MiB + 768, 0],
    "rnd1": list(np.random.default_rng(1).integers(0, 64, 5) * 4096),
    "rnd2": list(np.random.default_rng(2).integers(0, 64, 5) * 4096),
}
total = 5 * A + max(sum(v) for v in layouts.values()) + 5 * 32 * MiB + 4 * MiB
buf = wce.DeviceArray((total,), dtype=np.uint8)
base = (buf.addr + 2 * MiB - 1) // (2 * MiB) * (2 * MiB)
rng = np.random.default_rng(1)
chunk = 65536
txh = np.where(rng.random((chunk, N)) < 0.5, -8.8753, 8.8753).astype(np.complex128)
rxh = txh * (0.01 + 0.001j) + 1e-4 * rng.standard_normal((chunk, N))
preh = np.repeat(((0.01 + 0.001j) * inp["tx_pre"])[None], chunk, axis=0) + 1e-4 * rng.standard_normal((chunk, N))
st = wce.Stream()
res = {}
plans = {}
for name, gaps in layouts.items():
    addrs, p = [], base
    for g in gaps:
        addrs.append(p)
        p += A + int(g)
    plans[name] = addrs
    res[name] = []
# every stream start rounded up to an alignment (inside the same allocation)
for al in (64 * 1024, 2 * MiB, 32 * MiB):
    addrs, p = [], base
    for _ in range(5):
        p = (p + al - 1) // al * al
        addrs.append(p)
        p += A
    name = f"align{al // 1024}K"
    plans[name] = addrs
    res[name] = []
    assert p <= buf.addr + total
for rnd in range(args.rounds + 1):
    for name, (tx, rx, pre, lt, lin) in plans.items():
        if rnd == 0:
            for off in range(0, n, chunk):
                k = min(chunk, n - off)
                for d, h in ((tx, txh), (rx, rxh), (pre, preh)):
                    assert lib.wce_memcpy_htod(d + off * N * 16, h[:k].ctypes.data, k * N * 16) == 0
        o = wce.Outputs(lt, lin, None, None, None, None, N, 0, 0, 0, 0)
        fr = ctx.frames(tx, rx, n, frame_stride=N, block_stride=N, rx_pre=pre, pre_stride=N)
        ctx.estimate(fr, o, 3, st.handle)
        e0, e1 = wce.Event(), wce.Event()
        e0.record(st)
        for _ in range(args.reps):
            ctx.estimate(fr, o, 3, st.handle)
        e1.record(st)
        if rnd:
            res[name].append(e0.elapsed_ms(e1) / args.reps)
for name, v in res.items():
    med = float(np.median(v))
    offs = [(a - base) % (64 * MiB) // 4096 for a in plans[name]]
    print(f"{name:10s} median {med * 1e3:7.1f} us  min {min(v) * 1e3:7.1f}  {2672 * n / (med * 1e-3) / 1e9:6.0f} GB/s  "
          f"4K-page offsets mod 64 MiB {offs}")
