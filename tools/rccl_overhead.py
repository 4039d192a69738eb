"""Does an initialised process group slow the headline kernel?  Times three
back-to-back regions of K headline steps (65,536 frames, TEXTBOOK) after a
clock pre-warm, with --pg none | nccl | gloo (world size 1), and with RCCL
optionally torn down again before timing (--destroy).
usage: python tools/rccl_overhead.py --pg nccl [--steps 100] [--destroy]"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ap = argparse.ArgumentParser()
ap.add_argument("--pg", choices=["none", "nccl", "gloo"], default="none")
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--destroy", action="store_true")
ap.add_argument("--barrier", action="store_true", help="dist.barrier(device_ids=[0]) before each region, as bench.py")
ap.add_argument("--bcast", action="store_true", help="the state broadcast bench.py's make_ctx does")
args = ap.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29551")
if args.pg != "none":
    import torch
    import torch.distributed as dist
    if args.pg == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        t = torch.zeros(1, device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    if args.destroy:
        dist.destroy_process_group()
wce = importlib.import_module("80211parallelestimation_amd")
inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
if args.bcast:
    importlib.import_module("80211parallelestimation_amd.multi").broadcast_state_device(dist, wce, ctx, src=0)
st = wce.Stream()
B, N = 65536, 53
tx, rx = wce.DeviceArray((B, 15, N)), wce.DeviceArray((B, 15, N))
hlt, _, _, _ = ctx.shared()
hs = wce.DeviceArray.from_numpy(hlt)
ctx.synth(tx, rx, None, B, seed=0x80211, h_shared=hs, stream=st.handle)
H = wce.DeviceArray((B, N), zero=True)
fr = ctx.frames(tx, rx, B)
o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
step = lambda: ctx.estimate(fr, o, wce.PS_MMSE, st.handle)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for _ in range(10):
        step()
    st.synchronize()
res = []
for _ in range(3):
    e0, e1 = wce.Event(), wce.Event()
    st.synchronize()
    if args.barrier:
        dist.barrier(device_ids=[0])
        st.synchronize()
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(args.steps):
        step()
    e1.record(st)
    st.synchronize()
    res.append(((time.perf_counter() - t0) * 1e3 / args.steps, e0.elapsed_ms(e1) / args.steps))
print(f"pg={args.pg}{' (destroyed)' if args.destroy else ''}{' barrier' if args.barrier else ''}{' bcast' if args.bcast else ''}: ms/step wall, events: "
      + "  ".join(f"{a:.4f} {b:.4f}" for a, b in res), flush=True)
