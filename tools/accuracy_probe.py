"""Accuracy of the two TEXTBOOK MMSE paths (second bordered row vs
back-substitution + C W) against the long double closed form, for frames
whose channel matches the preamble (well conditioned) and for unrelated
channels (Ryy cond ~4e6).  Prints max / median norm-relative errors."""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
wce = importlib.import_module("80211parallelestimation_amd")
import oracle_py as orc

inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
hlt = ctx.shared()[0]
F = orc.fmatrix()
hls = orc.lt_ls(inp["tx_pre"], inp["rx_pre"])
cvec = F @ (F.conj() @ hls / 53)
B = 400
for label, hs in (("matched channel", hlt), ("unrelated channel", None)):
    tx, rx = wce.DeviceArray((B, 15, 53)), wce.DeviceArray((B, 15, 53))
    ctx.synth(tx, rx, None, B, seed=77, h_shared=wce.DeviceArray.from_numpy(hs) if hs is not None else None)
    wce.synchronize()
    txh, rxh = tx.numpy(), rx.numpy()
    ref = np.stack([orc.mmse_textbook_closed(cvec, txh[f, 0], rxh[f, 0], inp["ow2"]) for f in range(B)])
    for on in (True, False):
        ctx.set_border_dot(on)
        out = ctx.estimate_host(txh, rxh, mask=wce.PS_MMSE)["ps_mmse"]
        err = orc.normrel(out, ref)
        print(f"{label:18s} {'bordered row' if on else 'back-subst + CW':16s} max {err.max():.2e}  median {np.median(err):.2e}")
