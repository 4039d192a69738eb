"""LS config 2 over several independently allocated buffer sets (5 separate
hipMallocs each), interleaved: how much of the run-to-run spread of the
1,048,576-frame LS line is which allocation the buffers got.
usage: python tools/ab_alloc.py [--sets 6]"""
import argparse
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ap = argparse.ArgumentParser()
ap.add_argument("--sets", type=int, default=6)
ap.add_argument("--frames", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=7)
args = ap.parse_args()
wce = importlib.import_module("80211parallelestimation_amd")
lib = wce.load()
N, n = 53, args.frames
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
rng = np.random.default_rng(1)
chunk = 65536
txh = np.where(rng.random((chunk, N)) < 0.5, -8.8753, 8.8753).astype(np.complex128)
rxh = txh * (0.01 + 0.001j) + 1e-4 * rng.standard_normal((chunk, N))
preh = np.repeat(((0.01 + 0.001j) * inp["tx_pre"])[None], chunk, axis=0) + 1e-4 * rng.standard_normal((chunk, N))
sets = []
for i in range(args.sets):
    arrs = [wce.DeviceArray((n, N)) for _ in range(5)]
    for off in range(0, n, chunk):
        k = min(chunk, n - off)
        for d, h in zip(arrs[:3], (txh, rxh, preh)):
            lib.wce_memcpy_htod(d.addr + off * N * 16, h[:k].ctypes.data, k * N * 16)
    sets.append(arrs)
st = wce.Stream()
res = [[] for _ in sets]
for rnd in range(args.rounds + 1):
    for i, (tx, rx, pre, lt, lin) in enumerate(sets):
        fr = ctx.frames(tx, rx, n, frame_stride=N, block_stride=N, rx_pre=pre, pre_stride=N)
        o = wce.Outputs(lt.addr, lin.addr, None, None, None, None, N, 0, 0, 0, 0)
        ctx.estimate(fr, o, 3, st.handle)
        e0, e1 = wce.Event(), wce.Event()
        e0.record(st)
        for _ in range(10):
            ctx.estimate(fr, o, 3, st.handle)
        e1.record(st)
        if rnd:
            res[i].append(e0.elapsed_ms(e1) / 10)
for i, v in enumerate(res):
    med = float(np.median(v))
    addrs = " ".join(f"{a.addr >> 20:#x}" for a in sets[i])
    print(f"set {i}: median {med * 1e3:7.1f} us  min {min(v) * 1e3:7.1f}  {2672 * n / (med * 1e-3) / 1e9:6.0f} GB/s  "
          f"VA MiB {addrs}")
