"""Phase shares of mmse_solve from the WCE_STAMPS diagnostic build."""
import ctypes, importlib.util, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = sys.argv[1]
spec = importlib.util.spec_from_file_location("w", os.path.join(REPO, "80211parallelestimation_amd", "wce.py"))
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m); m.load(os.path.join(d, "libwce.so"))
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
B, N = 65536, 53
ctx = m.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], 1)
hlt = ctx.shared()[0]
tx, rx = m.DeviceArray((B, 15, N)), m.DeviceArray((B, 15, N))
ctx.synth(tx, rx, None, B, h_shared=m.DeviceArray.from_numpy(hlt))
W = m.DeviceArray((B, N))
for _ in range(3):
    ctx.mmse_solve(ctx.frames(tx, rx, B), W)
m.synchronize()
st = np.zeros(B * 10, np.uint64)
m._lib.wce_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert m._lib.wce_debug_stamps(st.ctypes.data, st.size) == 0
st = st.reshape(B, 10)[:, :9].astype(np.int64)
d = np.diff(st, axis=1)
tot = d.sum(axis=1)
names = [f"panel{k}" for k in range(7)] + ["backsolve"]
print("median wave cycles (s_memtime) per phase; share of stamped span")
for i, n in enumerate(names):
    print(f"  {n:10s} {np.median(d[:, i]):9.0f}  {np.median(d[:, i] / tot) * 100:5.1f}%")
print(f"  total      {np.median(tot):9.0f}")
