"""Time selected bench.py legs alone (quick A/B on the GPU box): prints one
JSON object per leg.  Legs: frame_cov, config5_ref, config5, config5_sharded,
cov_lowrank, cov_mode (the headline ctx's dense-C leg is bench.main's)."""
import argparse
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("legs", nargs="+")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    wce = importlib.import_module("80211parallelestimation_amd")
    wce.load().wce_set_device(0)
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    stream = wce.Stream()
    mk = lambda m: wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m, device=0)
    dist = bench.Dist()
    for leg in args.legs:
        if leg == "frame_cov":
            r = bench.bench_frame_cov(wce, mk, stream, 65536, args.reps)
        elif leg == "config5_ref":
            r = bench.bench_config5_ref(wce, mk(wce.MMSE_REF), stream, 1 << 20, args.reps)
        elif leg == "config5":
            r = bench.bench_config5(wce, mk(wce.MMSE_TEXTBOOK), stream, 131072, args.reps)
        elif leg == "config5_sharded":
            r = bench.bench_config5_sharded(wce, mk(wce.MMSE_TEXTBOOK), dist, stream, 10)
        elif leg == "cov_lowrank":
            c = mk(wce.MMSE_TEXTBOOK)
            B = 65536
            tx, rx = wce.DeviceArray((B, 15, 53)), wce.DeviceArray((B, 15, 53))
            hs = wce.DeviceArray.from_numpy(c.shared()[0])
            c.synth(tx, rx, None, B, seed=0x80211, h_shared=hs, stream=stream.handle)
            r = bench.bench_cov_lowrank(
                wce, lambda R: wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], device=0, Rhh=R), stream,
                tx, rx, B, args.reps)
        elif leg == "small_batch":
            r = bench.bench_small_batch(wce, mk(wce.MMSE_TEXTBOOK), stream)
        else:
            raise SystemExit(f"unknown leg {leg}")
        print(json.dumps({leg: r}), flush=True)


if __name__ == "__main__":
    main()
