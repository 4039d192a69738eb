"""bench.py's cov_lowrank section alone (same frames, same timing), for a
short GPU call while iterating on the low-rank kernels.
usage: python tools/quick_lowrank.py [reps]"""
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

N, NBLK = 53, 15


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    wce = importlib.import_module("80211parallelestimation_amd")
    assert wce.device_count() > 0
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    stream = wce.Stream()
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    hlt = ctx.shared()[0]
    B = 65536
    tx, rx = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N))
    ctx.synth(tx, rx, None, B, seed=0x80211, h_shared=wce.DeviceArray.from_numpy(hlt), stream=stream.handle)
    out = bench.bench_cov_lowrank(wce, lambda R: wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=R),
                                  stream, tx, rx, B, reps)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
