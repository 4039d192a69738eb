"""Where does a headline step's time go?  Event-timed solve, apply, and whole
wce_estimate(PS_MMSE) step vs the host wall clock (bench.py's timing)."""
import importlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
wce = importlib.import_module("80211parallelestimation_amd")
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
B, N, NB = 65536, 53, 15
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
hlt = ctx.shared()[0]
st = wce.Stream()
s = st.handle
tx, rx = wce.DeviceArray((B, NB, N)), wce.DeviceArray((B, NB, N))
ctx.synth(tx, rx, None, B, h_shared=wce.DeviceArray.from_numpy(hlt), stream=s)
H = wce.DeviceArray((B, N))
fr = ctx.frames(tx, rx, B)
o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)


def ev(fn, reps=20):
    e0, e1 = wce.Event(), wce.Event()
    fn()
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    return e0.elapsed_ms(e1) / reps


step = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
print("solve  ms", ev(lambda: ctx.mmse_solve(fr, H, N, s)))
print("apply  ms", ev(lambda: ctx.mmse_apply(H, H, B, N, s)))
print("step   ms (events)", ev(step))
st.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    step()
st.synchronize()
print("step   ms (wall)", (time.perf_counter() - t0) / 20 * 1e3)
t0 = time.perf_counter()
for _ in range(200):
    ctx.estimate(fr, o, wce.PS_MMSE, s) if False else None
t0 = time.perf_counter()
for _ in range(1000):
    wce.load().wce_version()
print("ctypes call us", (time.perf_counter() - t0) / 1000 * 1e6)
