"""Sweep of the PCIe-inclusive headline pipeline (bench.bench_host_pipeline):
streams x chunks, continuous streaming, same frames.
usage: python tools/ab_hostpipe.py"""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

wce = importlib.import_module("80211parallelestimation_amd")
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
B, N, NB = 65536, 53, 15
tx, rx = wce.DeviceArray((B, NB, N)), wce.DeviceArray((B, NB, N))
ctx.synth(tx, rx, None, B, seed=0x80211)
H = wce.DeviceArray((B, N), zero=True)
for ns, nc in ((3, 16), (4, 16), (4, 32), (6, 32), (8, 64), (2, 8)):
    r = bench.bench_host_pipeline(wce, ctx, tx, rx, H, B, 8, nstreams=ns, nchunks=nc)
    print(f"streams {ns} chunks {nc}: {r['frames_per_s']:.3e} frames/s, {r['pcie_GBs']:.1f} GB/s, "
          f"{100 * r['frac_of_h2d_bound']:.1f}% of the H2D bound, identical {r['bit_identical_to_device_path']}")
