"""PCIe-inclusive headline (frames in pinned host memory) across chunking
choices: chunks, streams, and one merged H2D copy per chunk (tx and rx of a
chunk adjacent in host memory) vs two.  usage: python tools/ab_pcie.py"""
import importlib
import itertools
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
wce = importlib.import_module("80211parallelestimation_amd")
lib = wce.load()
N, NBLK, B = 53, 15, 65536
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
tx, rx = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N))
hlt, _, _, _ = ctx.shared()
ctx.synth(tx, rx, None, B, h_shared=wce.DeviceArray.from_numpy(hlt))
wce.synchronize()
t0h, r0h = tx.numpy()[:, 0], rx.numpy()[:, 0]


def run(nchunks, nstreams, merged, reps=5):
    c = B // nchunks
    nb = c * N * 16
    if merged:    # [chunk][tx c x 53 | rx c x 53]
        host = wce.PinnedArray((nchunks, 2, c, N))
        host.array[:, 0] = t0h.reshape(nchunks, c, N)
        host.array[:, 1] = r0h.reshape(nchunks, c, N)
    else:
        txh, rxh = wce.PinnedArray((B, N)), wce.PinnedArray((B, N))
        txh.array[:] = t0h
        rxh.array[:] = r0h
    hh = wce.PinnedArray((B, N))
    streams = [wce.Stream() for _ in range(nstreams)]
    bufs = [(wce.DeviceArray((2, c, N)), wce.DeviceArray((c, N))) for _ in range(nstreams)]

    def one():
        for i in range(nchunks):
            s = streams[i % nstreams].handle
            din, dH = bufs[i % nstreams]
            if merged:
                lib.wce_memcpy_htod_async(din.addr, host.addr + i * 2 * nb, 2 * nb, s)
            else:
                lib.wce_memcpy_htod_async(din.addr, txh.addr + i * nb, nb, s)
                lib.wce_memcpy_htod_async(din.addr + nb, rxh.addr + i * nb, nb, s)
            fr = ctx.frames(din.addr, din.addr + nb, c, frame_stride=N, block_stride=N)
            ctx.estimate(fr, wce.Outputs(None, None, None, None, dH.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE, s)
            lib.wce_memcpy_dtoh_async(hh.addr + i * nb, dH.addr, nb, s)
        for st in streams:
            st.synchronize()

    one()
    t = time.perf_counter()
    for _ in range(reps):
        one()
    dt = (time.perf_counter() - t) / reps
    return dt


# copy-only ceilings
def copy_rate(direction, nbytes=B * N * 16 * 2):
    h = wce.PinnedArray((nbytes // 16,))
    d = wce.DeviceArray((nbytes // 16,))
    s = wce.Stream()
    f = lib.wce_memcpy_htod_async if direction == "h2d" else lib.wce_memcpy_dtoh_async
    args = (d.addr, h.addr) if direction == "h2d" else (h.addr, d.addr)
    f(*args, nbytes, s.handle)
    s.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        f(*args, nbytes, s.handle)
    s.synchronize()
    return nbytes * 5 / (time.perf_counter() - t) / 1e9


print(f"copy ceilings: H2D {copy_rate('h2d'):.1f} GB/s, D2H {copy_rate('d2h'):.1f} GB/s (one stream, 111 MB)")
for nchunks, nstreams, merged in itertools.product((8, 16, 32, 64), (2, 3, 4), (False, True)):
    dt = run(nchunks, nstreams, merged)
    print(f"chunks {nchunks:3d} streams {nstreams} merged {int(merged)}: {dt * 1e3:6.2f} ms  "
          f"{B / dt:.3e} frames/s  {2544 * B / dt / 1e9:5.1f} GB/s", flush=True)
