"""Interleaved A/B timing of the front-end kernels across libwce.so variants
(tools/variants.sh), one process; outputs must be bit-identical.
usage: python tools/ab_front.py build_variants/A build_variants/B ... [--rounds 7] [--frames 65536]"""
import argparse
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--frames", type=int, default=65536)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()

mods = []
for d in args.dirs:
    spec = importlib.util.spec_from_file_location("wce_" + os.path.basename(d.rstrip("/")),
                                                  os.path.join(REPO, "80211parallelestimation_amd", "wce.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m._lib = None
    m.load(os.path.join(d, "libwce.so"))
    mods.append((os.path.basename(d.rstrip("/")), m))

B, N, NB = args.frames, 53, 15
rng = np.random.default_rng(0)
chunk = 4096
pk_h = (rng.standard_normal((chunk, NB * 80)) + 1j * rng.standard_normal((chunk, NB * 80))) * 0.01
lt_h = (rng.standard_normal((chunk, 160)) + 1j * rng.standard_normal((chunk, 160))) * 0.01
state = []
for name, m in mods:
    ctx = m.Context(empty=True)
    pk, lt = m.DeviceArray((B, NB * 80)), m.DeviceArray((B, 160))
    lib = m.load()
    for off in range(0, B, chunk):
        k = min(chunk, B - off)
        lib.wce_memcpy_htod(pk.addr + off * NB * 80 * 16, pk_h[:k].ctypes.data, k * NB * 80 * 16)
        lib.wce_memcpy_htod(lt.addr + off * 160 * 16, lt_h[:k].ctypes.data, k * 160 * 16)
    sym, pre, ow2 = m.DeviceArray((B, NB, N)), m.DeviceArray((B, N)), m.DeviceArray((B,), np.float64)
    state.append((name, m, ctx, pk, lt, sym, pre, ow2, m.Stream()))
res = {(name, k): [] for name, *_ in state for k in ("blocks", "preamble")}
outs = {}
for rnd in range(args.rounds + 1):
    for name, m, ctx, pk, lt, sym, pre, ow2, st in state:
        for kind in ("blocks", "preamble"):
            if kind == "blocks":
                f = lambda: ctx.front_end_blocks(pk, B, NB, sym, stream=st.handle)
            else:
                f = lambda: ctx.front_end_preamble(lt, B, 160, pre, ow2, stream=st.handle)
            f()
            e0, e1 = m.Event(), m.Event()
            e0.record(st)
            for _ in range(args.reps):
                f()
            e1.record(st)
            if rnd > 0:
                res[(name, kind)].append(e0.elapsed_ms(e1) / args.reps)
        outs[name] = (sym.numpy()[:256], pre.numpy()[:256], ow2.numpy()[:256])
bytes_ = {"blocks": B * NB * (1024 + 848), "preamble": B * (2048 + 848 + 8)}
first = next(iter(outs.values()))
for (name, kind), v in res.items():
    med = float(np.median(v))
    same = all(np.array_equal(a, b) for a, b in zip(outs[name], first))
    print(f"{name:14s} {kind:9s} median {med * 1e3:8.1f} us  min {min(v) * 1e3:8.1f}  "
          f"{bytes_[kind] / (med * 1e-3) / 1e9:7.0f} GB/s  identical={same}")
