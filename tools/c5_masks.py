"""configs[4] fused kernel cost by output mask (1,048,576 frames, fp32 LS / eq
outputs, per-frame preambles): where the epilogue's time goes."""
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
N, NBLK = 53, 15
wce = importlib.import_module("80211parallelestimation_amd")
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
n = 1 << 20
st = wce.Stream()
tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
ctx.synth(tx, rx, pre, n, seed=0x80211, stream=st.handle)
outs = [wce.DeviceArray((n, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((n, N))]
eq = wce.DeviceArray((n, NBLK, N), np.complex64)
o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
fr = ctx.frames(tx, rx, n, rx_pre=pre)
masks = {"ALL": wce.ALL, "MMSE": wce.PS_MMSE, "MMSE+EQ": wce.PS_MMSE | wce.EQUALIZE,
         "MMSE+LT+LIN": wce.PS_MMSE | wce.LT_LS | wce.PS_LINEAR,
         "MMSE+LS4": wce.PS_MMSE | wce.LS_ALL, "MMSE+LT+LIN+EQ": wce.PS_MMSE | wce.LT_LS | wce.PS_LINEAR | wce.EQUALIZE}
res = {}
for rnd in range(2):
    for name, m in masks.items():
        f = lambda: ctx.estimate(fr, o, m, st.handle)
        for _ in range(2):
            f()
        st.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            f()
        st.synchronize()
        res.setdefault(name, []).append((time.perf_counter() - t0) / 5 * 1e3)
print(json.dumps({k: min(v) for k, v in res.items()}))
