"""Where config 5's time goes: MMSE alone vs + LS family (fused epilogue) vs
+ equalization, per-frame preamble, 131,072 frames, event-timed after a clock
pre-warm.  usage: python tools/config5_breakdown.py [lib_dir ...]"""
import importlib.util
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dirs = sys.argv[1:] or [os.path.join(REPO, "80211parallelestimation_amd")]
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
B, N, NB = 131072, 53, 15
for d in dirs:
    spec = importlib.util.spec_from_file_location("w" + os.path.basename(d.rstrip("/")),
                                                  os.path.join(REPO, "80211parallelestimation_amd", "wce.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m._lib = None
    m.load(os.path.join(d, "libwce.so"))
    ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m.MMSE_TEXTBOOK)
    st = m.Stream()
    tx, rx, pre = m.DeviceArray((B, NB, N)), m.DeviceArray((B, NB, N)), m.DeviceArray((B, N))
    ctx.synth(tx, rx, pre, B, stream=st.handle)
    outs = [m.DeviceArray((B, N)) for _ in range(5)]
    eq = m.DeviceArray((B, NB, N))
    o = m.Outputs(*(x.addr for x in outs), eq.addr, N, NB * N, N, 0, 0)
    fr = m.Context.frames(tx, rx, B, rx_pre=pre)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        ctx.estimate(fr, o, m.ALL, st.handle)
        st.synchronize()
    for label, mask in (("MMSE", m.PS_MMSE), ("MMSE+LS4", m.PS_MMSE | m.LS_ALL), ("MMSE+LS4+EQ", m.ALL),
                        ("LS4+EQ alone", m.LS_ALL | m.EQUALIZE)):
        e0, e1 = m.Event(), m.Event()
        ctx.estimate(fr, o, mask, st.handle)
        e0.record(st)
        for _ in range(10):
            ctx.estimate(fr, o, mask, st.handle)
        e1.record(st)
        ms = e0.elapsed_ms(e1) / 10
        print(f"{os.path.basename(d.rstrip('/')):14s} {label:14s} {ms:7.3f} ms  {B / (ms * 1e-3):.3e} frames/s")
