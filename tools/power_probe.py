"""Board power and shader clock while a kernel runs back to back.

Runs one leg (headline TEXTBOOK solve by default, 65,536 frames) in a loop on
one thread for --seconds, and samples `amd-smi metric` (power, clocks) from
the main thread.  Read-only SMI queries; nothing is set.
usage: python tools/power_probe.py [--leg headline|ls|config5|cov|lowrank|idle] [--taps 24] [--seconds 8]"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
N, NBLK = 53, 15


def smi():
    for cmd in (["amd-smi", "metric", "-g", "0", "-p", "-c", "--json"],
                ["rocm-smi", "-d", "0", "--showpower", "--showclocks", "--json"]):
        try:
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=10)
            if out.returncode == 0 and out.stdout.strip():
                return cmd[0], out.stdout.strip()
        except Exception as e:   # noqa: BLE001 -- report and try the other tool
            last = repr(e)
    return "none", last if "last" in dir() else "no output"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", default="headline", choices=["headline", "ls", "config5", "cov", "lowrank", "idle"])
    ap.add_argument("--taps", type=int, default=24, help="lowrank: an L-tap power-delay profile (taps 0..L-1)")
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--lib", default=None, help="libwce.so to load (default: the in-tree build)")
    args = ap.parse_args()
    import importlib
    wce = importlib.import_module("80211parallelestimation_amd")
    if args.lib:
        sys.modules["80211parallelestimation_amd.wce"]._lib = None
        wce.load(os.path.abspath(args.lib))
    import bench
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    n = args.frames
    stream = wce.Stream()
    s = stream.handle
    run = None
    if args.leg == "headline":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211)
        fr = ctx.frames(tx, rx, n)
        H = wce.DeviceArray((n, N), zero=True)
        o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
        run = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
    elif args.leg == "config5":   # all 5 + eq fused, fp32 LS/eq outputs, per-frame preambles
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
        tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
        ctx.synth(tx, rx, pre, n, seed=0x80211)
        outs = [wce.DeviceArray((n, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((n, N))]
        eq = wce.DeviceArray((n, NBLK, N), np.complex64)
        o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
        fr = ctx.frames(tx, rx, n, rx_pre=pre)
        run = lambda: ctx.estimate(fr, o, wce.ALL, s)
    elif args.leg == "cov":   # dense-C solve alone (WCE_MMSE_COV, full-rank PDP covariance)
        import prof_leg
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=prof_leg.pdp_rhh())
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211)
        fr = ctx.frames(tx, rx, n)
        W = wce.DeviceArray((n, N), zero=True)
        run = lambda: ctx.mmse_solve(fr, W, N, s)
    elif args.leg == "lowrank":   # WCE_MMSE_COV with an L-tap PDP (the bench's cov_lowrank legs)
        import prof_leg
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=prof_leg.pdp_rank(args.taps))
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211)
        fr = ctx.frames(tx, rx, n)
        H = wce.DeviceArray((n, N), zero=True)
        o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
        run = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
    elif args.leg == "ls":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        bufs, fr = bench.ls_frames(wce, ctx, n)
        hlt, hlin = wce.DeviceArray((n, N)), wce.DeviceArray((n, N))
        o = wce.Outputs(hlt.addr, hlin.addr, None, None, None, None, N, 0, 0, 0, 0)
        run = lambda: ctx.estimate(fr, o, wce.LT_LS | wce.PS_LINEAR, s)
    stop = threading.Event()
    stats = {"launches": 0, "secs": 0.0}

    def loop():
        if run is None:
            return
        t0 = time.perf_counter()
        while not stop.is_set():
            for _ in range(50):
                run()
            stream.synchronize()
            stats["launches"] += 50
        stats["secs"] = time.perf_counter() - t0

    th = threading.Thread(target=loop)
    th.start()
    samples = []
    t_end = time.time() + args.seconds
    while time.time() < t_end:
        samples.append((round(time.time(), 2),) + smi())
        time.sleep(0.3)
    stop.set()
    th.join()
    per = stats["secs"] / stats["launches"] * 1e3 if stats["launches"] else None
    print(json.dumps({"leg": args.leg, "frames": n, "launches": stats["launches"],
                      "ms_per_launch_wall": per}))
    for t, tool, out in samples:
        print(f"--- t={t} {tool}")
        print(out)


if __name__ == "__main__":
    main()
