"""Energy bound of BASELINE configs[4] as named (all 5 estimators + per-symbol
equalization fused, fp64 solve / fp32 LS and eq outputs, per-frame preambles,
1,048,576 frames on one GPU): is the fused kernel's time set by the board's
power cap?

Three runs on the same frames, each back to back for --seconds while
`amd-smi metric` samples socket power and shader clock (read-only):
  fused   wce.ALL (mmse_solve_ls_kernel: the solve + the LS/eq epilogue)
  solve   PS_MMSE alone (mmse_solve_fc_kernel)
  lseq    LT_LS + PS_Linear + PS_Cubic + PS_Sinc + equalization without PS_MMSE
          (the epilogue's HBM work as its own pass)
plus an idle window (no kernel) for the board's floor.  Per run: ms per step
(HIP events), mean power, clock, J per frame = P t / frames, and the dynamic
energy (P - P_idle) t / frames.

Bound: at a socket power cap P_cap, a kernel that must spend the solve's
and the epilogue's dynamic energy takes at least
    t_min = frames (E_dyn_solve + E_dyn_lseq) / (P_cap - P_idle)
-- if the fused time sits at this bound (and its power at the cap) the
remaining gap to a time target is the board's energy budget, not the code.
usage: python tools/energy_bound.py [--frames 1048576] [--seconds 4] > gpurun_out/energy_bound.json
"""
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
N, NBLK = 53, 15


def sample_smi(stop, out, skip_s=0.5):
    t0 = time.perf_counter()
    while not stop.is_set():
        try:
            r = subprocess.run(["amd-smi", "metric", "-g", "0", "-p", "-c", "--json"], capture_output=True,
                               text=True, timeout=5)
            g = json.loads(r.stdout)
            g = g["gpu_data"][0] if isinstance(g, dict) and "gpu_data" in g else (g[0] if isinstance(g, list) else g)
            clk = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_")
                   and isinstance(v, dict) and isinstance(v.get("clk"), dict)]
            if time.perf_counter() - t0 >= skip_s:
                out.append((float(g["power"]["socket_power"]["value"]), sum(clk) / max(1, len(clk))))
        except Exception:   # noqa: BLE001 -- best effort sampling, reported by the sample count
            pass
        time.sleep(0.1)


def measure(stream, fn, seconds):
    """(mean W, mean MHz, samples) while fn runs back to back (fn None: idle)"""
    stop, samples = threading.Event(), []
    th = threading.Thread(target=sample_smi, args=(stop, samples))
    th.start()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        if fn is None:
            time.sleep(0.05)
            continue
        for _ in range(4):
            fn()
        stream.synchronize()
    stop.set()
    th.join()
    if not samples:
        return None, None, 0
    p = np.array(samples)
    return float(p[:, 0].mean()), float(p[:, 1].mean()), len(samples)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--cap-w", type=float, default=None, help="socket power cap (default: the max power seen)")
    args = ap.parse_args()
    import importlib
    wce = importlib.import_module("80211parallelestimation_amd")
    import bench
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    n = args.frames
    stream = wce.Stream()
    s = stream.handle
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
    tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx.synth(tx, rx, pre, n, seed=0x80211, stream=s)
    outs = [wce.DeviceArray((n, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((n, N))]
    eq = wce.DeviceArray((n, NBLK, N), np.complex64)
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
    fr = ctx.frames(tx, rx, n, rx_pre=pre)
    lseq_mask = wce.ALL & ~wce.PS_MMSE
    runs = {"fused": lambda: ctx.estimate(fr, o, wce.ALL, s),
            "solve": lambda: ctx.estimate(fr, o, wce.PS_MMSE, s),
            "lseq": lambda: ctx.estimate(fr, o, lseq_mask, s)}
    res = {"frames": n, "workload": "BASELINE configs[4] at 1,048,576 frames on one GPU (bench config5_sharded N=1)",
           "runs": {}}
    for name in ("fused", "solve", "lseq", "fused"):   # fused twice: first and last (drift check)
        f = runs[name]
        for _ in range(3):
            f()
        stream.synchronize()
        t = bench.time_events(wce, stream, f, 5)
        w, mhz, ns = measure(stream, f, args.seconds)
        key = name if name not in res["runs"] else name + "_again"
        res["runs"][key] = {"ms_per_step": t, "socket_power_W": w, "gfx_clock_MHz": mhz, "samples": ns,
                            "J_per_frame": (w * t * 1e-3 / n) if w else None}
        print(f"{key}: {t:.3f} ms, {w} W, {mhz} MHz ({ns} samples)", file=sys.stderr, flush=True)
    time.sleep(1.0)
    w0, mhz0, ns0 = measure(stream, None, args.seconds)
    res["idle"] = {"socket_power_W": w0, "gfx_clock_MHz": mhz0, "samples": ns0}
    if w0:
        cap = args.cap_w or max(r["socket_power_W"] for r in res["runs"].values() if r["socket_power_W"])
        for r in res["runs"].values():
            r["J_dyn_per_frame"] = (r["socket_power_W"] - w0) * r["ms_per_step"] * 1e-3 / n if r["socket_power_W"] else None
        R = res["runs"]
        e_dyn = R["solve"]["J_dyn_per_frame"] + R["lseq"]["J_dyn_per_frame"]
        t_min = n * e_dyn / (cap - w0) * 1e3
        fused = min(R["fused"]["ms_per_step"], R.get("fused_again", R["fused"])["ms_per_step"])
        res["bound"] = {"P_cap_W": cap, "P_idle_W": w0,
                        "E_dyn_solve_plus_lseq_J_per_frame": e_dyn,
                        "t_min_ms": t_min, "fused_ms": fused, "fused_over_bound": fused / t_min,
                        "target_ms": 9.1, "target_reachable_at_cap": t_min <= 9.1,
                        "model": "t_min = frames (E_dyn_solve + E_dyn_lseq) / (P_cap - P_idle), E_dyn = (P - P_idle) t"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
