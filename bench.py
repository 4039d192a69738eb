#!/usr/bin/env python3
"""Benchmark: MMSE-estimated 802.11 frames/s on MI355X (BASELINE.json metric).

Workload (N=1 = BASELINE configs[2]): PS_MMSE over 65,536 synthetic frames
per GPU (53 subcarriers x 15 OFDM blocks, complex fp64, resident in HBM
before timing), 53x53 solve per frame + batched f64-MFMA product.  The timed
step is one wce_estimate(PS_MMSE) over the whole batch.  Headline mode is
TEXTBOOK (dense Ryy = X C X' + ow2 I, WiFi_channel_estimation_PS_MMSE.m); the
REF-repaired main.c mode (same kernels, Ryy = 2 ow2 I) is reported beside it.

Multi-GPU: one process per GPU (torch.distributed.run); frames are sharded
(weak scaling, frames_per_gpu each), the shared state (C, H_LT, tx_pre, ...)
is built on rank 0 and sent with ONE RCCL broadcast; no other collective on
the data path.  Timing: barrier + device sync on both sides, max over ranks.

Extra JSON fields: roofline of the dominant kernel (mmse_solve) measured with
HIP events on the launch stream, the MFMA apply kernel, the LS/HBM path
(config 2), and a CPU baseline (the oracle's fp64 OpenMP port, rank 0 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

N, NBLK = 53, 15
# algorithmic work per frame (DESIGN.md "Rooflines")
FLOP_CHOL = 4.0 / 3.0 * N ** 3           # n^3/6 complex MACs x 8
FLOP_RYY = 12.0 * N * N                  # a x_i C_ij conj(x_j) + b
FLOP_TRSV = 8.0 * N * N                  # forward (bordered row) + back substitution
FLOP_APPLY = 8.0 * N * N                 # H = C w
FLOP_SOLVE_TXT = FLOP_CHOL + FLOP_RYY + FLOP_TRSV
FLOP_SOLVE_REF = FLOP_CHOL + FLOP_TRSV   # REF: a = 0, Ryy is the diagonal 2 ow2 I (no build term)
# what the rank-1 kernel (mmse_solve_fc_kernel) executes per frame: the LDL^H,
# the rank-1 Ryy build (one complex product per lower-triangle element), the
# two bordered forward solves; no back-substitution, no C W product
# (round 2: pivot 0 is eliminated exactly from the rank-1 factors, the
# Cholesky runs over the 52 x 52 trailing matrix)
FLOP_EXEC_R1 = 4.0 / 3.0 * (N - 1) ** 3 + 6.0 * N * (N + 1) / 2 + FLOP_TRSV
BYTES_FE_BLOCK = 64 * 16 + N * 16        # front end: 64 useful samples in (CP skipped) + 53 bins out
BYTES_FE_PRE = 128 * 16 + N * 16 + 8     # two LTF copies in, preamble FFT + sigma^2 out
BYTES_LS_CFG2 = 2672                     # LT_LS + PS_Linear: rx_pre 848 + pilots 128 + 2 x 848 out
BYTES_REF_ALG = 8 * 16 + N * 16          # REF PS_MMSE: 4 tx + 4 rx pilots in, H out = 976
BYTES_PILOT_SECTORS = 8 * 64             # the 8 pilot reads of a frame each fetch a whole 64-B sector
PEAK_FP64_TFLOPS = 78.6                  # MI355X FP64 vector = FP64 matrix (spec)
PEAK_HBM_GBS = 8000.0                    # MI355X HBM3E spec (MI355X_MICROARCH.md)
KSTEPS_MFMA = 14                         # 4-deep f64 MFMA k-steps over 56 >= 53 subcarriers
METRIC = "MMSE-estimated 802.11 frames/sec (53 subcarriers) at 1/2/4/8 MI355X; % roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--prewarm-s", type=float, default=0.3, help="untimed clock ramp before the warmup steps")
    ap.add_argument("--frames-per-gpu", type=int, default=65536)
    ap.add_argument("--mode", choices=["textbook", "ref"], default="textbook")
    ap.add_argument("--ls-frames", type=int, default=1 << 20, help="config-2 LS batch (past the 256 MiB MALL)")
    ap.add_argument("--c5-frames", type=int, default=131072, help="config-5 frames per GPU (1,048,576 / 8)")
    ap.add_argument("--no-extras", action="store_true", help="headline only (for profiling runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU work budget of the baseline sample")
    ap.add_argument("--extras-out", default=os.path.join("gpurun_out", "bench_extras.json"),
                    help="full per-leg JSON (the stdout line carries one-number summaries)")
    ap.add_argument("--dry-run", action="store_true",
                    help="control path only: start the ranks, form the process group, barrier, max over ranks, "
                         "print the line; no device is touched (with WCE_DIST_BACKEND=gloo)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start the N
    ranks here, one process per GPU, as the reference's mpirun does for
    main_mpi.c (MPI_Init / MPI_Comm_size / MPI_Comm_rank, main_mpi.c:16-27,
    687-688), through torch.distributed.run on 127.0.0.1.  This parent never
    touches the GPU (no torch import, no HIP call), so no process that has
    initialised a device is replaced or forked.  The children's stdout is
    relayed line by line to stderr as it arrives (progress stays visible);
    rank 0's final JSON line is checked -- n_gpus and the process group both
    span N ranks -- and printed last on stdout.  Exit status: the launcher's
    when any rank failed, 3 when the line is missing or does not span N."""
    import subprocess
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, WCE_BENCH_LAUNCHER="bench.py --gpus %d" % n)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    print("bench: launching %d ranks: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    import signal

    def forward(sig, _frame):   # a SIGTERM / SIGINT to this parent reaches the ranks (torch.distributed.run
        p.send_signal(sig)      # tears its workers down on it) instead of orphaning them
    for sg in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sg, forward)
    last = None
    for ln in p.stdout:
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            last = s
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = p.wait()
    if rc != 0:
        print(f"bench: a rank failed (launcher exit {rc})", file=sys.stderr, flush=True)
        return rc
    try:
        res = json.loads(last) if last else None
    except ValueError:
        res = None
    if res is None:
        print("bench: no result line from rank 0", file=sys.stderr, flush=True)
        return 3
    dc = res.get("dist_check") or {}
    if res.get("n_gpus") != n or dc.get("group_size") != n or not dc.get("all_ranks_agree"):
        print(f"bench: line does not span {n} ranks: n_gpus={res.get('n_gpus')} dist_check={dc}",
              file=sys.stderr, flush=True)
        return 3
    print(last, flush=True)
    return 0


def check_world(gpus: int):
    """None when this process should run the bench itself, else the exit
    status: with a launcher (WORLD_SIZE set) the world must be --gpus ranks;
    without one, --gpus N > 1 starts the N ranks (launch_ranks)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"bench: WORLD_SIZE={ws} but --gpus {gpus}; refusing to report a {ws}-rank run as {gpus}",
                  file=sys.stderr, flush=True)
            return 2
        return None
    if gpus < 1:
        print(f"bench: --gpus {gpus}", file=sys.stderr, flush=True)
        return 2
    if gpus > 1:
        return launch_ranks(gpus, sys.argv[1:])
    return None


def dry_run(args, dist):
    """--dry-run: the N-rank control path without a device -- the process
    group, the barriers and the max over ranks every timed leg uses -- and a
    contract-shaped line (value null) from rank 0.  WCE_DRY_FAIL_RANK=r makes
    rank r exit 1 after the group forms (the launcher's failure path);
    WCE_DRY_HOLD_S=t keeps every rank alive t seconds (its signal path)."""
    dist.barrier()
    if os.environ.get("WCE_DRY_FAIL_RANK") == str(dist.rank):
        print(f"bench: dry run: rank {dist.rank} failing on request", file=sys.stderr, flush=True)
        sys.exit(1)
    if os.environ.get("WCE_DRY_HOLD_S"):   # tests: ranks that stay alive until stopped
        time.sleep(float(os.environ["WCE_DRY_HOLD_S"]))
    t0 = time.perf_counter()
    dist.barrier()
    el = dist.max(time.perf_counter() - t0)
    res = {"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": dist.world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f64", "data": "dry-run (no device)", "dry_run": True,
           "launcher": os.environ.get("WCE_BENCH_LAUNCHER", "external" if "WORLD_SIZE" in os.environ else None),
           "barrier_ms_max": el * 1e3,
           "config": {"workload": "dry run", "frames_per_gpu": args.frames_per_gpu,
                      "global_frames": args.frames_per_gpu * dist.world,
                      "parallelism": f"dp{dist.world} (frames sharded, 1 RCCL state broadcast)"},
           "dist_check": dist.group_check()}
    if dist.rank == 0:
        print(json.dumps(res, separators=(",", ":")), flush=True)
    dist.close()


class Dist:
    """torch.distributed only when launched with WORLD_SIZE > 1.  Backend
    "nccl" (= RCCL over xGMI, the default) or, for rehearsing the control path
    on a one-GPU box, WCE_DIST_BACKEND=gloo (ranks then share devices)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = os.environ.get("WCE_DIST_BACKEND", "nccl")
        self.torch = None
        self.device = self.local
        # WCE_FORCE_DIST=1: run the distributed path at world size 1 too (a
        # one-rank RCCL group), so a one-GPU box exercises exactly the code the
        # N>1 runs take: device broadcast, device barrier, max all-reduce.
        if self.world > 1 or os.environ.get("WCE_FORCE_DIST") == "1":
            import torch
            import torch.distributed as dist
            self.torch, self.dist = torch, dist
            # ranks > 0 wait in the barriers of the sharded legs while rank 0 runs
            # its single-GPU legs (minutes at N = 1's sizes): an explicit,
            # generous process-group timeout instead of the watchdog default
            import datetime
            tmo = datetime.timedelta(minutes=int(os.environ.get("WCE_DIST_TIMEOUT_MIN", "30")))
            if self.backend == "nccl":
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local), timeout=tmo)
                # first all-reduce now, long before any timed region: the
                # first one in a process sets RCCL up lazily
                self.barrier()
            else:
                self.device = self.local % max(1, torch.cuda.device_count())
                dist.init_process_group("gloo", timeout=tmo)

    def barrier(self):
        if self.torch is None:
            return
        if self.backend == "nccl":
            self.dist.barrier(device_ids=[self.local])
        else:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.torch is None:
            return x
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([x], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def group_check(self) -> dict:
        """Every rank's process group must span WORLD_SIZE ranks with this
        rank at RANK (main_mpi.c:687-688's communicator, here the RCCL one):
        each rank checks its own view, the verdict is the min over ranks."""
        if self.torch is None:
            return {"backend": None, "world_size_env": self.world, "group_size": 1, "all_ranks_agree": True}
        ok = float(self.dist.get_world_size() == self.world and self.dist.get_rank() == self.rank)
        agree = -self.max(-ok) == 1.0      # min over ranks
        return {"backend": self.dist.get_backend(), "world_size_env": self.world,
                "group_size": self.dist.get_world_size(), "all_ranks_agree": bool(agree)}

    def broadcast_state(self, wce, ctx):
        """One broadcast of the packed shared state from rank 0 (RCCL, device
        to device; host-staged under gloo)."""
        if self.torch is None:
            return
        import importlib
        multi = importlib.import_module("80211parallelestimation_amd.multi")
        if self.backend == "nccl":
            multi.broadcast_state_device(self.dist, wce, ctx, src=0)
        else:
            ptr, n = ctx.state()
            blob = np.zeros(n, np.uint8)
            if self.rank == 0:
                assert wce.load().wce_memcpy_dtoh(blob.ctypes.data, ptr, n) == 0
            blob = multi.broadcast_state_host(self.dist, blob, n, src=0)
            if self.rank != 0:
                ctx.load_state(blob)

    def close(self):
        if self.torch is not None:
            self.dist.destroy_process_group()


def pmc_leg(leg: str, frames: int, write_bytes: float, tol: float = 0.02, waves: int = None):
    """Per-dispatch PMC counters of one bench leg's dominant kernel from the
    committed profiles/*_pmc_legs.json (tools/pmc_legs.sh: rocprofv3 --pmc over
    tools/prof_leg.py, which launches ONLY that kernel, at exactly the bench's
    launch size).  Used only if the profiled launches are this launch: the
    recorded frames must equal `frames`, and either SQ_WAVES must equal
    `waves` (when the caller knows the launch's wave count) or WRITE_SIZE
    (exact for 16-B/lane streaming stores, MI355X_MICROARCH.md HBM) must equal
    the launch's algorithmic output bytes `write_bytes` within `tol`.
    Returns (counters, source file) or (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_legs.json")), reverse=True)
    if not files:
        return None, "no profiles/*_pmc_legs.json"
    # the newest legs file that profiled this leg's CURRENT kernel (a round
    # re-profiles only the legs whose kernel changed)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from prof_leg import LEGS
    want = LEGS.get(leg, (None,))[0]
    d, src = None, None
    for f in files:
        c = json.load(open(f)).get(leg)
        if c and c.get("kernel") == want:
            d, src = c, f
            break
    if not d:
        return None, f"leg {leg} ({want}) not profiled"
    files = [src]
    if d["frames"] != frames:
        return None, f"profiled at {d['frames']} frames, bench launch is {frames}"
    k = d["counters"]
    if waves is not None:
        if abs(k.get("SQ_WAVES", -1) - waves) > 0.5:
            return None, f"SQ_WAVES {k.get('SQ_WAVES')} is not this launch's {waves} waves"
    elif "WRITE_SIZE" not in k or abs(k["WRITE_SIZE"] * 1024.0 - write_bytes) > tol * write_bytes:
        return None, f"WRITE_SIZE {k.get('WRITE_SIZE')} KiB is not this launch's {write_bytes:.0f} B of outputs"
    return k, os.path.basename(files[-1])


def hbm_bytes(k, narrow_fetch_kib: float = 0.0):
    """HBM bytes of one dispatch from its counters: FETCH_SIZE counts a wide
    coalesced streaming read (16 B/lane) at half its bytes on gfx950 (x2, the
    guide's correction), but a narrow scattered read's 64-B sectors in full --
    calibrated by the pilot-only leg (tools/prof_leg.py ls_pilots: 8 sectors
    = 512 B per frame measured as FETCH_SIZE).  narrow_fetch_kib = the part of
    FETCH_SIZE that is such sector reads; WRITE_SIZE is exact."""
    return (2.0 * (k["FETCH_SIZE"] - narrow_fetch_kib) + narrow_fetch_kib + k["WRITE_SIZE"]) * 1024.0


def mfma_flops(k):
    """Executed f64 MFMA flops of one dispatch: SQ_INSTS_VALU_MFMA_MOPS_F64
    counts 512-flop units (4 per v_mfma_f64_16x16x4, 1 per v_mfma_f64_4x4x4_4b;
    r02_pmc_legs.json apply1m: 58.72 M MOPS for 14.68 M 16x16x4)."""
    return k["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512.0


def power_clock(stream, step, seconds=2.5):
    """Board power and shader clock while the headline kernel runs back to
    back (untimed, after the timed region): `amd-smi metric` sampled from a
    second thread, read only.  The FP64 solve is power-capped on MI355X
    (DESIGN.md s6), so the clock it holds is part of its roofline story.
    None when amd-smi is unavailable."""
    import shutil
    import subprocess
    import threading
    if not shutil.which("amd-smi"):
        return None
    stop, samples = threading.Event(), []

    def sample():
        time.sleep(0.4)   # past the ramp
        while not stop.is_set():
            try:
                out = subprocess.run(["amd-smi", "metric", "-g", "0", "-p", "-c", "--json"], capture_output=True,
                                     text=True, timeout=5)
                g = json.loads(out.stdout)["gpu_data"][0]
                clk = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_")]
                samples.append((float(g["power"]["socket_power"]["value"]), sum(clk) / len(clk)))
            except Exception:   # noqa: BLE001 -- best effort, informational
                pass
            time.sleep(0.2)

    th = threading.Thread(target=sample)
    th.start()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            step()
        stream.synchronize()
    stop.set()
    th.join()
    if not samples:
        return None
    return {"socket_power_W": sum(p for p, _ in samples) / len(samples),
            "gfx_clock_MHz": sum(c for _, c in samples) / len(samples), "samples": len(samples),
            "note": "amd-smi metric during back-to-back headline launches (untimed); the spec peak assumes 2,400 MHz"}


def time_events(wce, stream, fn, reps):
    e0, e1 = wce.Event(), wce.Event()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    return e0.elapsed_ms(e1) / reps


def main():
    args = parse()
    rc = check_world(args.gpus)
    if rc is not None:
        sys.exit(rc)
    dist = Dist()
    if args.dry_run:
        return dry_run(args, dist)
    import importlib
    wce = importlib.import_module("80211parallelestimation_amd")
    dev = dist.device if dist.world > 1 else 0
    assert wce.device_count() > 0, "bench needs an MI355X"
    wce.load().wce_set_device(dev)
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    mode = wce.MMSE_TEXTBOOK if args.mode == "textbook" else wce.MMSE_REF
    stream = wce.Stream()

    def make_ctx(m):
        if dist.world > 1 and dist.rank != 0:
            c = wce.Context(empty=True, device=dev)
        else:
            c = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m, device=dev)
        dist.broadcast_state(wce, c)
        return c

    ctx = make_ctx(mode)
    hlt, _, _, _ = ctx.shared()
    B = args.frames_per_gpu
    first = dist.rank * B
    tx = wce.DeviceArray((B, NBLK, N))
    rx = wce.DeviceArray((B, NBLK, N))
    hs = wce.DeviceArray.from_numpy(hlt)     # frames share the preamble's channel (physically consistent)
    ctx.synth(tx, rx, None, B, first_frame=first, seed=0x80211, h_shared=hs, stream=stream.handle)
    H = wce.DeviceArray((B, N), zero=True)
    frames = ctx.frames(tx, rx, B)
    outs = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    s = stream.handle

    def step(c=ctx):
        c.estimate(frames, outs, wce.PS_MMSE, s)

    # Bring the GPU to its steady-state clock before the W warmup steps: a
    # cold MI355X ramps over tens of ms, longer than W steps of ~1 ms, and
    # the timed region would otherwise mix ramp and steady state.  Untimed.
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < args.prewarm_s:
        for _ in range(10):
            step()
        stream.synchronize()
    for _ in range(args.warmup):
        step()
    stream.synchronize()
    dist.barrier()
    stream.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_enq = time.perf_counter()
    stream.synchronize()
    t_done = time.perf_counter()
    dist.barrier()
    t1 = time.perf_counter()
    elapsed = dist.max(t1 - t0)
    # the headline output must be all finite (wce_nonfinite_scan, untimed);
    # max over ranks is an 8-byte all-reduce outside the timed region
    _, bad = ctx.nonfinite_scan(H, B, stream=s)
    nonfinite = int(dist.max(float(bad)))
    total_frames = B * dist.world * args.steps
    value = total_frames / elapsed
    res = {"metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": dist.world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "prewarm_s": args.prewarm_s, "nonfinite_frames": nonfinite,
           "launcher": os.environ.get("WCE_BENCH_LAUNCHER", "external" if "WORLD_SIZE" in os.environ else None),
           # where this rank's timed region went: host enqueue of the K steps,
           # the wait for the stream, the closing barrier (rank 0's view)
           "timed_region_ms": {"enqueue": (t_enq - t0) * 1e3, "stream_sync": (t_done - t_enq) * 1e3,
                               "barrier": (t1 - t_done) * 1e3},
           "config": {"workload": f"PS_MMSE {args.mode} (53x53 per-frame Hermitian solve of Ryy = X C X' + ow2 I, bordered read-out H = u s), BASELINE configs[2]",
                      "frames_per_gpu": B, "global_frames": B * dist.world, "subcarriers": N, "ofdm_blocks": NBLK,
                      "parallelism": f"dp{dist.world} (frames sharded, 1 RCCL state broadcast)"}}

    if not args.no_extras:
        # Dominant kernel = the whole step: for the rank-1 covariances (TEXTBOOK,
        # REF) one launch of mmse_solve_fc_kernel does the MMSE (Cholesky with two
        # bordered rows, H = u s).  HIP events on the launch stream.  The kernel
        # runs on the FP64 VALU (no MFMA: DESIGN.md s6), so the bound is the FP64
        # vector peak, 78.6 TF -- numerically the same as the FP64 MFMA peak.
        reps = max(5, args.steps)
        t_step = time_events(wce, stream, step, reps)
        fl_alg = FLOP_SOLVE_TXT + FLOP_APPLY if mode == wce.MMSE_TEXTBOOK else FLOP_SOLVE_REF + FLOP_APPLY
        ach = fl_alg * B / (t_step * 1e-3) / 1e12
        kname = "mmse_solve_fc_kernel"
        k, tsrc = pmc_leg("headline", B, N * 16.0 * B, waves=B) if mode == wce.MMSE_TEXTBOOK else (None, "REF headline")
        ach_x = FLOP_EXEC_R1 * B / (t_step * 1e-3) / 1e12
        res["roofline"] = {"bound": "fp64-valu", "kernel": f"{kname} (fp64 VALU Cholesky, row-per-lane panels, bordered by conj(rx) and (w o x)^T)",
                           "achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                           "frac": ach / PEAK_FP64_TFLOPS, "traffic": hbm_bytes(k) if k else None,
                           "traffic_unit": "HBM bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, same-size launches)",
                           "traffic_source": tsrc,
                           "algorithmic_bytes": 3 * 848 * B,
                           "flop_per_frame": fl_alg, "frames_per_launch": B, "avg_launch_ms": t_step,
                           "flop_per_frame_executed": FLOP_EXEC_R1 if mode == wce.MMSE_TEXTBOOK else None,
                           "achieved_executed": ach_x if mode == wce.MMSE_TEXTBOOK else None,
                           "frac_executed": ach_x / PEAK_FP64_TFLOPS if mode == wce.MMSE_TEXTBOOK else None,
                           "valu_insts_per_frame": (k["SQ_INSTS_VALU"] / B) if k and "SQ_INSTS_VALU" in k else None,
                           "note": "frac = SURVEY 8(d) F_alg (4/3 n^3 + 28 n^2, the generic dense MMSE) per the "
                                   "measurement contract; frac_executed = the flops this kernel runs (exact first "
                                   "step, Cholesky over pivots 1..52, rank-1 Ryy build, two bordered forward "
                                   "solves; no back-substitution, no C W product). peak = MI355X FP64 vector "
                                   "(= FP64 matrix), spec, 2.4 GHz"}
        res["mmse_frac_of_roofline"] = value / dist.world * fl_alg / (PEAK_FP64_TFLOPS * 1e12)
        if dist.rank == 0:
            pc = power_clock(stream, step)
            if pc:
                res["roofline"]["board"] = pc

    if not args.no_extras and dist.rank == 0:
        try:
            # the general path: dense C (WCE_MMSE_COV, full-rank model Rhh): solve with
            # back-substitution, then H = C W on the f64 MFMA (apply_kernel).
            # Rank 0 only; no collective.
            reps = max(5, args.steps)
            pdp = np.exp(-0.12 * np.arange(N))
            Rhh = np.diag(pdp / pdp.sum()).astype(np.complex128) * 1.1e-4
            ctx3 = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], device=dev, Rhh=Rhh)
            for _ in range(2):
                step(ctx3)
            t_cov = time_events(wce, stream, lambda: step(ctx3), reps)
            W = H
            t_cs = time_events(wce, stream, lambda: ctx3.mmse_solve(frames, W, N, s), reps)
            t_apply = time_events(wce, stream, lambda: ctx3.mmse_apply(W, H, B, N, s), reps)
            ach_apply = FLOP_APPLY * B / (t_apply * 1e-3) / 1e12
            ctx3.set_modulus(tx.rows(0)[0, 0])       # constant-modulus frames: the shared operator (round 4)
            for _ in range(2):
                step(ctx3)
            t_cm = time_events(wce, stream, lambda: step(ctx3), reps)
            _, bad_cm = ctx3.nonfinite_scan(H, B, stream=s)
            ctx3.set_modulus(None)
            res["cov_mode"] = {"workload": "WCE_MMSE_COV: full-rank PDP covariance, dense C (BASELINE configs[2] shape)",
                               "constant_modulus": {
                                   "kernel": "cm_real_kernel: H = K (conj x o rx) on f64 MFMA (persistent, K in LDS), K = (a C P + b I)^-1 C",
                                   "ms_per_step": t_cm, "frames_per_s_per_gpu": B / (t_cm * 1e-3),
                                   "speedup_vs_per_frame": t_cov / t_cm,
                                   "achieved_GBs": 3 * N * 16 * B / (t_cm * 1e-3) / 1e9,
                                   "hbm_frac": 3 * N * 16 * B / (t_cm * 1e-3) / 1e9 / PEAK_HBM_GBS,
                                   "nonfinite_frames": int(bad_cm),
                                   "note": "BPSK frames share |x|^2, so Ryy's factorisation is frame-independent "
                                           "(wce_ctx_set_modulus); not the headline, not credited F_alg"},
                               "frames_per_s_per_gpu": B / (t_cov * 1e-3), "ms_per_step": t_cov,
                               "solve_kernel": "mmse_solve_kernel<false> (dense C, back-substitution)",
                               "solve_ms": t_cs, "solve_tflops": FLOP_SOLVE_TXT * B / (t_cs * 1e-3) / 1e12,
                               "solve_frac_fp64_peak": FLOP_SOLVE_TXT * B / (t_cs * 1e-3) / 1e12 / PEAK_FP64_TFLOPS}
            kc, csrc = pmc_leg("cov_solve", B, N * 16.0 * B, waves=B)
            if kc:
                res["cov_mode"]["solve_pmc_per_wave"] = {
                    c: kc[c] / B for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS",
                                           "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES") if c in kc}
                res["cov_mode"]["solve_pmc_source"] = csrc
            # MFMA counters of exactly this launch (65,536 frames = 4,096 waves of 16
            # frames): the 'apply' leg of tools/pmc_legs.sh
            # its counters from same-size launches (tools/pmc_legs.sh 'apply'); the
            # grid is capped at 2 workgroups per CU, so check the output bytes
            ka, asrc = pmc_leg("apply", B, N * 16.0 * B, tol=0.12)
            app = {"kernel": "apply_kernel = H = C W (v_mfma_f64_16x16x4 + 4x4x4_4b tail rows, C in LDS), COV mode",
                   "avg_launch_ms": t_apply, "achieved_tflops": ach_apply,
                   "frac_fp64_peak": ach_apply / PEAK_FP64_TFLOPS, "pmc_source": asrc,
                   "algorithmic_bytes": 2 * N * 16 * B}
            if ka:
                tiles = (B + 15) // 16
                mfma = ka["SQ_INSTS_VALU_MFMA_F64"]             # wave-level f64 MFMA instructions per launch
                app.update({"tiles": tiles, "mfma_insts_per_tile": mfma / tiles,
                            "traffic": hbm_bytes(ka),
                            "executed_tflops": mfma_flops(ka) / (t_apply * 1e-3) / 1e12,
                            "mfma_busy_frac_pmc": ka["SQ_VALU_MFMA_BUSY_CYCLES"] / (ka["GRBM_GUI_ACTIVE"] / 8.0 * 256 * 4),
                            "note": "executed = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 flop; 3M (Gauss) form, three real "
                                    "products per complex one: per 16-frame tile rows 0..47 3 x 14 x 3 "
                                    "v_mfma_f64_16x16x4, rows 48..52 14 x 6 v_mfma_f64_4x4x4_4b (56 x 56 executed, "
                                    "53 x 53 useful); achieved counts the 4-product 8 n^2 flop of the contract; busy = "
                                    "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs)"})
            # the same product at 1,048,576 frames (the configs[3] batch): apply_kernel
            # (C staged in LDS, each wave streaming 16-frame tiles with the next
            # tile's W loaded under the MFMAs), 16 tiles per wave.
            # W = the 65,536 solved frames tiled 16 times (device copies), so the
            # operands are real solutions, not zeros.
            nbig = 16 * B
            Wb, Hb = wce.DeviceArray((nbig, N)), wce.DeviceArray((nbig, N))
            for t in range(16):
                assert wce.load().wce_memcpy_dtod(Wb.addr + t * B * N * 16, W.addr, B * N * 16, s) == 0
            for _ in range(2):
                ctx3.mmse_apply(Wb, Hb, nbig, N, s)
            t_big = time_events(wce, stream, lambda: ctx3.mmse_apply(Wb, Hb, nbig, N, s), reps)
            ach_big = FLOP_APPLY * nbig / (t_big * 1e-3) / 1e12
            app["frames_1M"] = {"kernel": "apply_kernel (streaming, C in LDS, 3M form)", "frames": nbig,
                                "avg_launch_ms": t_big,
                                "achieved_tflops": ach_big, "frac_fp64_peak": ach_big / PEAK_FP64_TFLOPS,
                                "achieved_GBs": 2 * N * 16 * nbig / (t_big * 1e-3) / 1e9,
                                "frac_hbm_peak": 2 * N * 16 * nbig / (t_big * 1e-3) / 1e9 / PEAK_HBM_GBS,
                                "memory_floor_note": "the same loads and stores without the MFMAs take 0.380 ms "
                                                     "(4.68 TB/s, profiles/r03_ab_apply_3m.txt)",
                                "algorithmic_bytes": 2 * N * 16 * nbig}
            # its MFMA counters from same-size launches (tools/pmc_legs.sh apply1m);
            # the grid is capped at 2 workgroups per CU, so check the output bytes:
            # WRITE_SIZE runs ~9% over them (the 5-row last output tile writes
            # partial 64-B sectors)
            kb, bsrc = pmc_leg("apply1m", nbig, N * 16.0 * nbig, tol=0.12)
            app["frames_1M"]["pmc_source"] = bsrc
            if kb:
                mf = kb["SQ_INSTS_VALU_MFMA_F64"]
                app["frames_1M"].update({
                    "traffic": hbm_bytes(kb),
                    "mfma_insts": mf,
                    "executed_tflops": mfma_flops(kb) / (t_big * 1e-3) / 1e12,
                    "mfma_busy_frac_pmc": kb["SQ_VALU_MFMA_BUSY_CYCLES"] / (kb["GRBM_GUI_ACTIVE"] / 8.0 * 256 * 4)})
            del Wb, Hb
            res["apply_kernel"] = app
            del ctx3
        except Exception as e:  # noqa: BLE001 -- recorded in the leg's slot
            res.setdefault("cov_mode", {})["error"] = f"{type(e).__name__}: {e}"[:240]

    if not args.no_extras:
        reps = max(5, args.steps)
        # the other MMSE mode, same kernels
        other = wce.MMSE_REF if mode == wce.MMSE_TEXTBOOK else wce.MMSE_TEXTBOOK
        ctx2 = make_ctx(other)
        for _ in range(2):
            step(ctx2)
        t_other = time_events(wce, stream, lambda: step(ctx2), reps)
        res["ref_mode" if other == wce.MMSE_REF else "textbook_mode"] = {
            "frames_per_s_per_gpu": B / (t_other * 1e-3), "ms_per_step": t_other}
        del ctx2

        # PCIe-inclusive headline from pinned host memory (rank 0).  Runs before
        # the 1,048,576-frame leg: after that leg's 27 GB come and go, this
        # leg's overlap measured 30% lower
        if dist.rank == 0:
            guarded(res, "host_pipeline", lambda: bench_host_pipeline(wce, ctx, tx, rx, H, B, 8))

        # rank-0 single-GPU legs first: the 1,048,576-frame strong-scaling legs
        # below allocate and free ~37 GB, which moves later legs' placement
        # (LS spread is physical placement)
        if dist.rank == 0:
            # rank 0 only: contexts built locally (make_ctx would broadcast: a collective)
            local_ctx = lambda m: wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], m, device=dev)
            # LS path (config 2: LT_LS + PS_Linear), HBM-bound
            guarded(res, "ls_config2", lambda: bench_ls(wce, ctx, stream, args.ls_frames, reps))
            guarded(res, "front_end", lambda: bench_front(wce, ctx, stream, B, reps))
            guarded(res, "frame_cov", lambda: bench_frame_cov(wce, local_ctx, stream, B, reps))
            guarded(res, "config5", lambda: bench_config5(wce, ctx, stream, args.c5_frames, reps))
            guarded(res, "cov_lowrank", lambda: bench_cov_lowrank(
                wce, lambda R: wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], device=dev, Rhh=R), stream,
                tx, rx, B, reps))
            guarded(res, "small_batch", lambda: bench_small_batch(wce, ctx, stream))
            guarded(res, "ldc_convert", lambda: bench_ldc_convert(wce, stream, reps))
            # REF past the MALL: 1,048,576 full frames (27 GB), last of the rank-0 legs
            ctx_ref = local_ctx(wce.MMSE_REF)
            guarded(res.setdefault("ref_mode", {}), "b%d" % args.ls_frames,
                    lambda: bench_ref_large(wce, ctx_ref, stream, args.ls_frames, reps))
            # BASELINE configs[4] in main.c semantics at its full 1,048,576 frames (45 GB)
            guarded(res, "config5_ref", lambda: bench_config5_ref(wce, ctx_ref, stream, args.ls_frames, reps))
            del ctx_ref

        # BASELINE configs[3]: 1,048,576 frames in total, sharded over the
        # ranks (strong scaling), same kernel; all ranks, barrier + max
        # steps scale with the world size so every N times about the same
        # per-rank work (at N=8 a shard is 131,072 frames, ~1 ms per step)
        res["config4"] = bench_config4(wce, ctx, dist, stream, hs, max(5, args.steps // 5) * dist.world,
                                       prewarm_s=args.prewarm_s)
        res["config5_sharded"] = bench_config5_sharded(wce, ctx, dist, stream, max(3, args.steps // 20) * dist.world,
                                                       prewarm_s=args.prewarm_s)


    if not args.no_cpu_baseline and dist.rank == 0 and dist.world == 1:
        guarded(res, "cpu_baseline", lambda: cpu_baseline(wce, ctx, frames, tx, rx, B, mode, args.cpu_seconds))
        if "error" not in res["cpu_baseline"]:
            refc = guarded({}, "r", lambda: cpu_reference(args.cpu_seconds / 2))
            if refc is not None:
                res["cpu_baseline"]["reference_code"] = refc

    res["dist_check"] = dist.group_check()
    if dist.rank == 0:
        emit(res, args.extras_out)
    dist.close()


def guarded(res, key, fn):
    """Run one extra leg; a failure is recorded in its slot instead of
    losing the headline line (rank-0-only legs: no collective can be left
    half-entered by it).  Returns the leg's result."""
    try:
        res[key] = fn()
    except Exception as e:  # noqa: BLE001 -- reported, never swallowed silently
        res[key] = {"error": f"{type(e).__name__}: {e}"[:240]}
    return res[key]


COMPACT_LIMIT = 8192


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def compact(res, extras_path):
    """The driver-facing line: the contract keys, the dominant kernel's
    roofline, the CPU baseline and one-number summaries of every extra leg.
    Everything else (notes, per-wave PMC, board samples, sub-legs) lives in
    the extras file written beside it.  Must stay under COMPACT_LIMIT bytes
    (the driver keeps the last 8 KB of stdout; tests/test_bench_contract.py)."""
    out = _pick(res, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                      "scaling", "vs_baseline", "dtype", "data", "prewarm_s", "nonfinite_frames", "timed_region_ms",
                      "launcher"))
    cfg = res.get("config", {})
    out["config"] = {"workload": "PS_MMSE %s, BASELINE configs[2]" % ("textbook" if "textbook" in cfg.get("workload", "")
                                                                     else "ref"),
                     **_pick(cfg, ("frames_per_gpu", "global_frames", "subcarriers", "ofdm_blocks", "parallelism"))}
    r = res.get("roofline")
    if r:
        out["roofline"] = _pick(r, ("bound", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes",
                                    "flop_per_frame", "frames_per_launch", "avg_launch_ms", "frac_executed",
                                    "traffic_source"))
        out["roofline"]["kernel"] = "mmse_solve_fc_kernel"
        if isinstance(r.get("board"), dict):
            out["roofline"]["board"] = _pick(r["board"], ("socket_power_W", "gfx_clock_MHz"))
    c = res.get("cpu_baseline")
    if isinstance(c, dict):
        out["cpu_baseline"] = _pick(c, ("value", "unit", "cores", "kind", "sample", "max_normrel_err_vs_gpu", "error"))
        if "sample" in out["cpu_baseline"]:
            out["cpu_baseline"]["sample"] = out["cpu_baseline"]["sample"][:120]
        rc = c.get("reference_code")
        if isinstance(rc, dict):
            out["cpu_baseline"]["reference_code"] = {
                k: {"value": v["value"], "cores": v.get("cores", 1)} for k, v in rc.items()
                if isinstance(v, dict) and "value" in v}
    legs = {}

    def leg(name, d, keys):
        if isinstance(d, dict) and d:
            legs[name] = _pick(d, keys + ("error",))

    t1 = ("ms_per_step", "frames_per_s")
    leg("config4", res.get("config4"), t1 + ("global_frames", "n_gpus", "scaling", "frames_per_s_per_gpu"))
    leg("config5_sharded", res.get("config5_sharded"),
        t1 + ("global_frames", "n_gpus", "scaling", "nonfinite_outputs", "solve_only_ms", "epilogue_ms", "frac_hbm"))
    ls = res.get("ls_config2", {})
    big = next((v for k, v in ls.items() if k.startswith("b") and k != "b65536" and isinstance(v, dict)), None)
    leg("ls_config2", big, ("frames", "avg_launch_ms", "achieved_GBs", "frac", "traffic"))
    cm = res.get("cov_mode", {})
    leg("cov_mode", cm, ("ms_per_step", "solve_ms", "solve_frac_fp64_peak"))
    if "constant_modulus" in cm:
        legs.setdefault("cov_mode", {})["constant_modulus_ms"] = cm["constant_modulus"].get("ms_per_step")
    app = res.get("apply_kernel", {})
    leg("apply_kernel", app, ("avg_launch_ms", "achieved_tflops", "executed_tflops", "mfma_busy_frac_pmc"))
    if isinstance(app.get("frames_1M"), dict):
        legs.setdefault("apply_kernel", {})["frames_1M_ms"] = app["frames_1M"].get("avg_launch_ms")
    rm = res.get("ref_mode", {})
    leg("ref_mode", rm, ("ms_per_step",))
    rb = next((v for k, v in rm.items() if k.startswith("b") and isinstance(v, dict)), None)
    if rb and "roofline" in rb:
        legs.setdefault("ref_mode", {})["b1M"] = {"ms": rb.get("avg_launch_ms"), "frac": rb["roofline"].get("frac")}
    fc = res.get("frame_cov", {})
    for m in ("textbook", "ref"):
        if isinstance(fc.get(m), dict):
            legs["frame_cov_" + m] = _pick(fc[m], ("ms_per_step", "nonfinite_frames"))
            if "roofline" in fc[m]:
                legs["frame_cov_" + m].update(_pick(fc[m]["roofline"], ("frac", "traffic", "algorithmic_bytes")))
    c5r = res.get("config5_ref", {})
    for m in ("fp64", "mixed_fp64_solve_fp32_ls", "frame_cov_fp64", "frame_cov_mixed_fp32_ls"):
        if isinstance(c5r.get(m), dict):
            legs["config5_ref_" + m] = {"ms": c5r[m].get("ms_per_step"),
                                        "frac": c5r[m].get("roofline", {}).get("frac")}
    c5 = res.get("config5", {})
    for m in ("fp64", "mixed_fp64_solve_fp32_ls"):
        if isinstance(c5.get(m), dict):
            legs["config5_" + m] = {"ms": c5[m].get("ms_per_step")}
    lr = res.get("cov_lowrank", {})
    for k, v in lr.items():
        if isinstance(v, dict) and k.startswith("L"):
            legs["lowrank_" + k] = {"ms": v.get("ms_per_step"), "kernel": str(v.get("kernel", ""))[:40]}
            if "roofline" in v:
                legs["lowrank_" + k]["frac"] = v["roofline"].get("frac")
    fe = res.get("front_end", {})
    for m in ("blocks", "preamble"):
        if isinstance(fe.get(m), dict):
            legs["front_" + m] = {"ms": fe[m].get("avg_launch_ms"), "frac": fe[m].get("frac")}
    hp = res.get("host_pipeline")
    leg("host_pipeline", hp, ("frames_per_s", "bit_identical_to_device_path", "frac_of_h2d_bound"))
    for k in ("small_batch", "ldc_convert"):
        if isinstance(res.get(k), dict) and "error" in res[k]:
            legs[k] = {"error": res[k]["error"]}
    # the driver's record keeps the last 2,000 characters of stdout: the legs a
    # reader checks first (configs[3] and [4], REF past the MALL, the dense and
    # tap-domain COV solves, configs[1]) go last, so they are the ones it keeps
    last = ("ls_config2", "cov_mode", "lowrank_L24", "lowrank_L53", "ref_mode", "config5_sharded", "config4")
    ordered = {k: v for k, v in legs.items() if k not in last}
    ordered.update({k: legs[k] for k in last if k in legs})
    out["dist_check"] = res.get("dist_check")
    out["extras_file"] = extras_path
    out["legs"] = _round_sig(ordered)
    return out


def _round_sig(x, sig=5):
    """floats of the leg summaries to `sig` significant digits (the line is
    read from a 2,000-character tail; the full values are in the extras file)"""
    if isinstance(x, dict):
        return {k: _round_sig(v, sig) for k, v in x.items()}
    if isinstance(x, float) and x == x and x not in (float("inf"), float("-inf")) and x != 0.0:
        return float(f"{x:.{sig}g}")
    return x


def emit(res, extras_path):
    """Write the full result to the extras file, then print the compact line
    LAST on stdout (the driver parses the final line of an 8 KB tail)."""
    if extras_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(extras_path)), exist_ok=True)
            with open(extras_path, "w") as f:
                json.dump(res, f)
        except OSError as e:
            print(f"bench: extras not written: {e}", file=sys.stderr)
            extras_path = None
    line = json.dumps(compact(res, extras_path), separators=(",", ":"))
    if len(line) > COMPACT_LIMIT:      # never lose the headline: drop the leg summaries first
        c = compact(res, extras_path)
        c["legs"] = {"dropped": f"{len(line)} B line"}
        line = json.dumps(c, separators=(",", ":"))
    print(line, flush=True)


def prewarm_sync(dist, stream, fn, seconds):
    """Untimed clock ramp on every rank right before a sharded leg's timed
    region.  Ranks > 0 reach these legs while rank 0 still runs its
    single-GPU legs, and sit idle in the barrier meanwhile: without this their
    GPUs start the timed steps cold, and the max over ranks is a cold rank's
    time.  Barrier first so all ranks ramp together."""
    stream.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(4):
            fn()
        stream.synchronize()


def bench_config5_sharded(wce, ctx, dist, stream, steps, total=1 << 20, prewarm_s=0.3):
    """BASELINE configs[4] as the config names it: all 5 estimators +
    per-symbol equalization, fused, mixed precision (fp64 solve, LS family and
    equalized symbols stored fp32), per-frame preambles, `total` frames
    sharded over the ranks (strong scaling).  Timed like config4."""
    import importlib
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    first, count = multi.shard(total, dist.world, dist.rank)
    s = stream.handle
    tx, rx, pre = wce.DeviceArray((count, NBLK, N)), wce.DeviceArray((count, NBLK, N)), wce.DeviceArray((count, N))
    ctx.synth(tx, rx, pre, count, first_frame=first, seed=0x80211, stream=s)
    outs = [wce.DeviceArray((count, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((count, N))]
    eq = wce.DeviceArray((count, NBLK, N), np.complex64)
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
    fr = ctx.frames(tx, rx, count, rx_pre=pre)
    for _ in range(3):
        ctx.estimate(fr, o, wce.ALL, s)
    prewarm_sync(dist, stream, lambda: ctx.estimate(fr, o, wce.ALL, s), prewarm_s)
    stream.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.estimate(fr, o, wce.ALL, s)
    stream.synchronize()
    dist.barrier()
    dt = dist.max(time.perf_counter() - t0) / steps
    # untimed: every output of the last step must be finite (the 4 fp32 LS
    # outputs, the fp64 MMSE, the 15 fp32 equalized blocks); max over ranks
    bad = sum(ctx.nonfinite_scan(h, count, f32=(i < 4), stream=s)[1] for i, h in enumerate(outs))
    bad += ctx.nonfinite_scan(eq, count * NBLK, f32=True, stream=s)[1]
    res = {"workload": "BASELINE configs[4]: all 5 estimators + equalization fused, fp64 solve / fp32 LS and eq "
                       "outputs, per-frame preambles, 1,048,576 frames sharded over the ranks",
           "global_frames": total, "frames_per_gpu": count, "n_gpus": dist.world, "steps": steps,
           "ms_per_step": dt * 1e3, "frames_per_s": total / dt, "scaling": "strong",
           "nonfinite_outputs": int(dist.max(float(bad))),
           **config5_traffic(count, dt)}
    if dist.world == 1:
        # where the time goes (untimed, N = 1 only): the same frames' PS_MMSE
        # alone (the fused kernel's solve), and board power / shader clock
        # under each -- the FP64 solve holds the board at its power cap, and
        # the epilogue's HBM stream shares that budget
        Hm = wce.DeviceArray((count, N))
        om = wce.Outputs(None, None, None, None, Hm.addr, None, N, 0, 0, 0, 0)
        solo = lambda: ctx.estimate(fr, om, wce.PS_MMSE, s)
        for _ in range(3):
            solo()
        t_solo = time_events(wce, stream, solo, 5)
        res["solve_only_ms"] = t_solo
        res["epilogue_ms"] = dt * 1e3 - t_solo
        res["board_fused"] = power_clock(stream, lambda: ctx.estimate(fr, o, wce.ALL, s), seconds=2.0)
        res["board_solve_only"] = power_clock(stream, solo, seconds=2.0)
        del Hm
    return res


def config5_traffic(count, dt):
    """HBM traffic of the fused configs[4] kernel from the 'config5' PMC leg
    (1,048,576 frames: only the N=1 launch size is profiled)."""
    wbytes = (4 * N * 8 + N * 16 + NBLK * N * 8) * count
    k, src = pmc_leg("config5", count, wbytes, waves=count)   # one wave per frame
    if not k:
        return {"pmc_source": src}
    alg = (NBLK * N + N + N) * 16 * count + wbytes     # rx 15 blocks + tx block 0 + rx_pre in
    return {"algorithmic_bytes": alg, "traffic": hbm_bytes(k), "achieved_GBs": alg / dt / 1e9,
            "frac_hbm": alg / dt / 1e9 / PEAK_HBM_GBS, "pmc_source": src,
            "valu_insts_per_frame": k.get("SQ_INSTS_VALU", 0) / count}


def bench_config4(wce, ctx, dist, stream, hs, steps, total=1 << 20, prewarm_s=0.3):
    """BASELINE configs[3]: `total` frames sharded contiguously over the
    ranks (wce_shard's partition), each rank generating its shard from the
    global frame index; timed like the headline (barrier + device sync on
    both sides, max over ranks).  Strong scaling: total work fixed."""
    import importlib
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    first, count = multi.shard(total, dist.world, dist.rank)
    tx, rx = wce.DeviceArray((count, NBLK, N)), wce.DeviceArray((count, NBLK, N))
    ctx.synth(tx, rx, None, count, first_frame=first, seed=0x80211, h_shared=hs, stream=stream.handle)
    H = wce.DeviceArray((count, N))
    fr = ctx.frames(tx, rx, count)
    o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    for _ in range(3):
        ctx.estimate(fr, o, wce.PS_MMSE, stream.handle)
    prewarm_sync(dist, stream, lambda: ctx.estimate(fr, o, wce.PS_MMSE, stream.handle), prewarm_s)
    stream.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.estimate(fr, o, wce.PS_MMSE, stream.handle)
    stream.synchronize()
    dist.barrier()
    dt = dist.max(time.perf_counter() - t0) / steps
    return {"workload": "BASELINE configs[3]: PS_MMSE over 1,048,576 frames sharded over the ranks",
            "global_frames": total, "frames_per_gpu": count, "n_gpus": dist.world, "steps": steps,
            "ms_per_step": dt * 1e3, "frames_per_s": total / dt, "frames_per_s_per_gpu": total / dt / dist.world,
            "scaling": "strong"}


def ls_frames(wce, ctx, n, pilots_only=False):
    """configs[1] input: n frames holding block 0 only (frame_stride = 53: the
    PS path reads 4 pilots of block 0, LT_LS the frame's own preamble), plus
    per-frame preambles.  Returns (buffers, wce.Frames)."""
    lib = wce.load()
    tx, rx, pre = wce.DeviceArray((n, N)), wce.DeviceArray((n, N)), wce.DeviceArray((n, N))
    rng = np.random.default_rng(1)
    chunk = min(n, 65536)
    txh = np.where(rng.random((chunk, N)) < 0.5, -8.8753, 8.8753).astype(np.complex128)
    rxh = txh * (0.01 + 0.001j) + 1e-4 * rng.standard_normal((chunk, N))
    tp = np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz"))["tx_pre"]
    preh = np.repeat(((0.01 + 0.001j) * tp)[None], chunk, axis=0) + 1e-4 * rng.standard_normal((chunk, N))
    for off in range(0, n, chunk):
        m = min(chunk, n - off)
        for d, h in ((tx, txh), (rx, rxh), (pre, preh)):
            assert lib.wce_memcpy_htod(d.addr + off * N * 16, h[:m].ctypes.data, m * N * 16) == 0
    fr = ctx.frames(tx, rx, n, frame_stride=N, block_stride=N, rx_pre=None if pilots_only else pre, pre_stride=N)
    return (tx, rx, pre), fr


def bench_ls(wce, ctx, stream, n, reps):
    """LT_LS (per-frame preamble) + PS_Linear over n frames; algorithmic bytes
    2,672 B/frame (ls_frames' layout)."""
    s = stream.handle
    bufs, fr_n = ls_frames(wce, ctx, n)
    tx, rx, pre = bufs
    hlt, hlin = wce.DeviceArray((n, N)), wce.DeviceArray((n, N))
    o = wce.Outputs(hlt.addr, hlin.addr, None, None, None, None, N, 0, 0, 0, 0)
    out = {"workload": "LT_LS + PS_Linear (config 2), per-frame preamble, algorithmic 2672 B/frame"}
    for label, nb in (("b%d" % n, n), ("b65536", min(n, 65536))):
        fr = ctx.frames(tx, rx, nb, frame_stride=N, block_stride=N, rx_pre=pre, pre_stride=N)
        f = lambda: ctx.estimate(fr, o, wce.LT_LS | wce.PS_LINEAR, s)
        for _ in range(3):
            f()
        t = time_events(wce, stream, f, reps)
        gbs = BYTES_LS_CFG2 * nb / (t * 1e-3) / 1e9
        out[label] = {"frames": nb, "avg_launch_ms": t, "frames_per_s": nb / (t * 1e-3), "achieved_GBs": gbs,
                      "peak_GBs": PEAK_HBM_GBS, "frac": gbs / PEAK_HBM_GBS}
    # non-finite guard over the LT_LS output of the big batch: 848 B/frame read
    bm = wce.DeviceArray(((n + 31) // 32,), dtype=np.uint32)
    cnt = wce.DeviceArray((1,), dtype=np.uint64)
    t = time_events(wce, stream, lambda: ctx.nonfinite_scan(hlt, n, bitmap=bm, n_bad=cnt, stream=s), reps)
    gbs = 848 * n / (t * 1e-3) / 1e9
    out["nonfinite_scan"] = {"kernel": "nonfinite_scan_kernel<false>", "frames": n, "avg_launch_ms": t,
                             "algorithmic_bytes_per_frame": 848, "achieved_GBs": gbs, "frac": gbs / PEAK_HBM_GBS}
    # HBM bytes from counters of same-size launches (tools/pmc_legs.sh 'ls';
    # the pilot-sector reads calibrated by the pilot-only leg 'ls_pilots')
    key = "b%d" % n
    k, src = pmc_leg("ls", n, 2 * N * 16.0 * n)
    kp, _ = pmc_leg("ls_pilots", n, N * 16.0 * n)
    out[key]["pmc_source"] = src
    if k and kp:
        traffic = hbm_bytes(k, narrow_fetch_kib=kp["FETCH_SIZE"])
        out[key].update({"traffic": traffic, "traffic_bytes_per_frame": traffic / n,
                         "real_GBs": traffic / (out[key]["avg_launch_ms"] * 1e-3) / 1e9,
                         "pilot_fetch_bytes_per_frame": kp["FETCH_SIZE"] * 1024.0 / n,
                         "traffic_note": "FETCH_SIZE x2 for the streamed rx_pre reads, pilot sectors counted in "
                                         "full (the pilot-only leg measures them at ~512 B = 8 x 64-B sectors "
                                         "per frame), WRITE_SIZE exact"})
    return out


def ref_frames(wce, ctx, n, stream=None):
    """REF-mode input: n full frames (15 x 53 blocks, 12,720 B of tx and of rx
    each), synthesised on the device.  Returns (tx, rx, wce.Frames)."""
    tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
    ctx.synth(tx, rx, None, n, seed=0x80211, stream=stream)
    return tx, rx, ctx.frames(tx, rx, n)


def bench_ref_large(wce, ctx, stream, n, reps):
    """PS_MMSE in REF (main.c) semantics past the 256 MiB MALL: n full frames,
    one mmse_ref_flat_kernel launch.  Algorithmic bytes 976 per frame (4 tx + 4
    rx pilots in, 53 out); the pilot reads cost a 64-B sector each, so the
    sector floor is 8 x 64 + 848 = 1,360 B per frame."""
    s = stream.handle
    tx, rx, fr = ref_frames(wce, ctx, n, s)
    H = wce.DeviceArray((n, N))
    o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    f = lambda: ctx.estimate(fr, o, wce.PS_MMSE, s)
    for _ in range(3):
        f()
    t = time_events(wce, stream, f, reps)
    alg = BYTES_REF_ALG * n / (t * 1e-3) / 1e9
    sec = (BYTES_PILOT_SECTORS + N * 16) * n / (t * 1e-3) / 1e9
    k, src = pmc_leg("ref", n, N * 16.0 * n)
    traffic = hbm_bytes(k, narrow_fetch_kib=k["FETCH_SIZE"]) if k else None
    _, bad = ctx.nonfinite_scan(H, n, stream=s)
    return {"frames": n, "avg_launch_ms": t, "frames_per_s": n / (t * 1e-3),
            "roofline": {"bound": "hbm", "kernel": "mmse_ref_flat_kernel", "achieved": alg, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": alg / PEAK_HBM_GBS, "traffic": traffic,
                         "algorithmic_bytes": BYTES_REF_ALG * n, "sector_floor_bytes": (BYTES_PILOT_SECTORS + N * 16) * n,
                         "achieved_sector_GBs": sec, "frac_sector": sec / PEAK_HBM_GBS, "pmc_source": src,
                         "traffic_note": "FETCH_SIZE (pilot sectors, counted in full) + WRITE_SIZE"},
            "nonfinite_frames": bad}


def front_frames(wce, n):
    """n time-domain packets (15 blocks of 80 samples) and 160-sample LTFs."""
    rng = np.random.default_rng(2)
    chunk = min(n, 8192)
    pk = wce.DeviceArray((n, NBLK * 80))
    lt = wce.DeviceArray((n, 160))
    lib = wce.load()
    src = (rng.standard_normal((chunk, NBLK * 80)) + 1j * rng.standard_normal((chunk, NBLK * 80))) * 0.01
    srcl = (rng.standard_normal((chunk, 160)) + 1j * rng.standard_normal((chunk, 160))) * 0.01
    for off in range(0, n, chunk):
        m = min(chunk, n - off)
        assert lib.wce_memcpy_htod(pk.addr + off * NBLK * 80 * 16, src[:m].ctypes.data, m * NBLK * 80 * 16) == 0
        assert lib.wce_memcpy_htod(lt.addr + off * 160 * 16, srcl[:m].ctypes.data, m * 160 * 16) == 0
    return pk, lt


def bench_front(wce, ctx, stream, n, reps):
    """Time-domain front end over n frames of 15 x 80-sample
    blocks + a 160-sample LTF each: HBM-bound, algorithmic bytes per block
    1,872 (64 samples in, 53 bins out), per LTF 2,904."""
    s = stream.handle
    pk, lt = front_frames(wce, n)
    sym = wce.DeviceArray((n, NBLK, N))
    pre = wce.DeviceArray((n, N))
    ow2 = wce.DeviceArray((n,), np.float64)
    fb = lambda: ctx.front_end_blocks(pk, n, NBLK, sym, stream=s)
    fp = lambda: ctx.front_end_preamble(lt, n, 160, pre, ow2, stream=s)
    out = {"workload": f"{n} frames x 15 blocks of 80 samples + 160-sample LTF (WiFi_blocks_extraction.m, WiFi_RX.m:18-30)"}
    for label, f, per, units in (("blocks", fb, BYTES_FE_BLOCK, n * NBLK), ("preamble", fp, BYTES_FE_PRE, n)):
        for _ in range(3):
            f()
        t = time_events(wce, stream, f, reps)
        gbs = per * units / (t * 1e-3) / 1e9
        kn = f"front_kernel<{'true' if label == 'preamble' else 'false'}>"
        k, _ = pmc_leg("front_" + label, n, (N * 16.0 + (8 if label == "preamble" else 0)) * units,
                       tol=0.1 if label == "preamble" else 0.02)   # sigma^2: one 8-B store per frame
        traffic = hbm_bytes(k) if k else None
        out[label] = {"kernel": kn, "avg_launch_ms": t,
                      "frames_per_s": n / (t * 1e-3), "algorithmic_bytes_per_unit": per, "achieved_GBs": gbs,
                      "peak_GBs": PEAK_HBM_GBS, "frac": gbs / PEAK_HBM_GBS,
                      "algorithmic_bytes": per * units, "traffic": traffic}
    return out


def bench_ldc_convert(wce, stream, reps, frames=65536):
    """The reference's data format on the device (wce_ldconv.hip): frames
    held as long double complex (x87, 32 B per value) converted to complex
    double and back, 15 x 53 values per frame.  HBM-bound: 48 B per value
    either way."""
    s = stream.handle
    n = frames * NBLK * N
    ld = wce.DeviceArray((n,), np.clongdouble, zero=True)
    c = wce.DeviceArray((n,), zero=True)
    out = {"workload": f"{frames} frames x 15 x 53 values, long double complex <-> complex double"}
    for label, f in (("to_complex", lambda: wce.ldc_to_complex(ld, c, n, s)),
                     ("to_ldc", lambda: wce.complex_to_ldc(c, ld, n, s))):
        for _ in range(3):
            f()
        t = time_events(wce, stream, f, reps)
        gbs = 48.0 * n / (t * 1e-3) / 1e9
        out[label] = {"avg_launch_ms": t, "frames_per_s": frames / (t * 1e-3), "achieved_GBs": gbs,
                      "peak_GBs": PEAK_HBM_GBS, "frac": gbs / PEAK_HBM_GBS}
    return out


def bench_small_batch(wce, ctx, stream, n=1024, calls=200):
    """Serving-style small batches (all 5 estimators + equalization, per-frame
    preamble, 1,024 frames per call): direct wce_estimate calls vs one
    captured HIP-graph plan replayed (wce_plan), host wall clock per call."""
    s = stream.handle
    tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx.synth(tx, rx, pre, n, seed=5, stream=s)
    outs = [wce.DeviceArray((n, N)) for _ in range(5)]
    eq = wce.DeviceArray((n, NBLK, N))
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, 0)
    fr = ctx.frames(tx, rx, n, rx_pre=pre)
    # a multi-kernel call: MATLAB semantics + per-frame covariance (LT_LS,
    # the factor matvec, 4 solve waves per frame, the block average)
    frm = ctx.frames(tx, rx, n, rx_pre=pre, semantics=wce.SEM_MATLAB)
    om = wce.Outputs(None, None, None, None, outs[4].addr, None, N, 0, 0, 0, 0)
    mm = wce.PS_MMSE | wce.FRAME_COV
    ctx.reserve(n)
    plan, planm = ctx.plan(fr, o, wce.ALL), ctx.plan(frm, om, mm)
    res = {"workload": f"{n} frames per call, all 5 estimators + equalization, per-frame preamble (one fused "
                       f"kernel); matlab_frame_cov: PS_MMSE with MATLAB semantics and per-frame covariance "
                       f"(several kernels per call)", "calls": calls}
    cases = (("direct", lambda: ctx.estimate(fr, o, wce.ALL, s)), ("plan", lambda: plan.launch(s)),
             ("matlab_frame_cov_direct", lambda: ctx.estimate(frm, om, mm, s)),
             ("matlab_frame_cov_plan", lambda: planm.launch(s)))
    for label, f in cases:
        for _ in range(20):
            f()
        stream.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            f()
        stream.synchronize()
        dt = (time.perf_counter() - t0) / calls
        res[label] = {"us_per_call": dt * 1e6, "frames_per_s": n / dt}
    plan.close()
    planm.close()
    return res


def bench_host_pipeline(wce, ctx, tx, rx, H_dev, B, reps, nstreams=3, nchunks=16):
    """PCIe-inclusive rate (never `value`): the headline PS_MMSE
    with frames in pinned HOST memory -- block 0 of tx and rx in (2 x 848 B),
    H out (848 B) -- in nchunks chunks round-robin over nstreams streams, so
    the H2D copies, the solves and the D2H copies of different chunks overlap.
    Host wall clock over the whole batch; the result must equal the
    device-resident path's H bit for bit."""
    c = B // nchunks
    # host layout [chunk][tx c x 53 | rx c x 53]: one H2D copy per chunk
    # (tools/ab_pcie.py: one copy beats two, 16 chunks over 3 streams is best)
    host = wce.PinnedArray((nchunks, 2, c, N))
    hh = wce.PinnedArray((B, N))
    host.array[:, 0] = tx.numpy()[:c * nchunks, 0].reshape(nchunks, c, N)
    host.array[:, 1] = rx.numpy()[:c * nchunks, 0].reshape(nchunks, c, N)
    streams = [wce.Stream() for _ in range(nstreams)]
    bufs = [(wce.DeviceArray((2, c, N)), wce.DeviceArray((c, N))) for _ in range(nstreams)]
    lib = wce.load()
    nb = c * N * 16

    frs = [ctx.frames(din.addr, din.addr + nb, c, frame_stride=N, block_stride=N) for din, _ in bufs]
    outs = [wce.Outputs(None, None, None, None, dH.addr, None, N, 0, 0, 0, 0) for _, dH in bufs]

    def one_pass(sync=True):
        for i in range(nchunks):
            j = i % nstreams
            s = streams[j].handle
            din, dH = bufs[j]
            assert lib.wce_memcpy_htod_async(din.addr, host.addr + 2 * i * nb, 2 * nb, s) == 0
            ctx.estimate(frs[j], outs[j], wce.PS_MMSE, s)
            assert lib.wce_memcpy_dtoh_async(hh.addr + i * nb, dH.addr, nb, s) == 0
        if sync:
            for st in streams:
                st.synchronize()

    for _ in range(4):      # the first passes in a process pay queue / copy-engine setup (~30%)
        one_pass()
    # the device-resident path on the same frames (the headline H buffer has
    # been reused by the COV leg since)
    ctx.estimate(ctx.frames(tx, rx, B), wce.Outputs(None, None, None, None, H_dev.addr, None, N, 0, 0, 0, 0),
                 wce.PS_MMSE, streams[0].handle)
    streams[0].synchronize()
    same = bool(np.array_equal(hh.array[:c * nchunks], H_dev.numpy()[:c * nchunks]))
    # continuous streaming: the passes queue back to back (a host feeding frames
    # does not drain the pipeline between batches); one sync at the end
    t0 = time.perf_counter()
    for _ in range(reps):
        one_pass(sync=False)
    for st in streams:
        st.synchronize()
    dt = (time.perf_counter() - t0) / reps
    frames = c * nchunks
    # copy-only ceiling of the H2D direction (the larger one: 1,696 of the
    # 2,544 B per frame), one stream, the whole input buffer
    dst = wce.DeviceArray((host.nbytes // 16,))
    assert lib.wce_memcpy_htod_async(dst.addr, host.addr, host.nbytes, streams[0].handle) == 0
    streams[0].synchronize()
    tc = time.perf_counter()
    for _ in range(3):
        assert lib.wce_memcpy_htod_async(dst.addr, host.addr, host.nbytes, streams[0].handle) == 0
    streams[0].synchronize()
    h2d = 3 * host.nbytes / (time.perf_counter() - tc) / 1e9
    bound = h2d * 1e9 / (2 * N * 16)
    return {"workload": f"headline PS_MMSE, {frames} frames in pinned host memory, {nchunks} chunks over "
                        f"{nstreams} streams (one H2D of tx/rx block 0, solve, D2H H per chunk, overlapped)",
            "ms_per_batch": dt * 1e3, "frames_per_s": frames / dt, "pcie_bytes_per_frame": 3 * N * 16,
            "pcie_GBs": 3 * N * 16 * frames / dt / 1e9, "bit_identical_to_device_path": same,
            "h2d_ceiling_GBs": h2d, "h2d_bound_frames_per_s": bound, "frac_of_h2d_bound": frames / dt / bound,
            "note": "host-to-host rate including PCIe; bench value is device-resident"}


def bench_config5(wce, ctx, stream, n, reps):
    """BASELINE configs[4] per GPU: all 5 estimators + per-symbol equalization,
    per-frame preamble, 1,048,576 / 8 frames on this GPU.  Algorithmic bytes
    per frame: rx 15x53 + tx block 0 + rx_pre in, 5 H + eq out.  Reported in
    fp64 and in the config's mixed precision (fp64 solve, LS family + eq
    stored fp32: WCE_OUT_LS_F32)."""
    s = stream.handle
    tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx.synth(tx, rx, pre, n, seed=0x80211, stream=s)
    fr = ctx.frames(tx, rx, n, rx_pre=pre)
    res = {"workload": "BASELINE configs[4] share of one GPU: LT_LS + PS_Linear/Cubic/Sinc + PS_MMSE + "
                       "equalization, per-frame preamble, fused (LS family in the MMSE solve epilogue)",
           "frames": n}
    for label, f32 in (("fp64", False), ("mixed_fp64_solve_fp32_ls", True)):
        dt = np.complex64 if f32 else np.complex128
        outs = [wce.DeviceArray((n, N), dt) for _ in range(4)] + [wce.DeviceArray((n, N))]
        eq = wce.DeviceArray((n, NBLK, N), dt)
        o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32 if f32 else 0)
        f = lambda: ctx.estimate(fr, o, wce.ALL, s)
        for _ in range(3):
            f()
        t = time_events(wce, stream, f, reps)
        ob = 8 if f32 else 16
        bytes_frame = (NBLK * N + N + N) * 16 + N * 16 + (4 * N + NBLK * N) * ob
        res[label] = {"ms_per_step": t, "frames_per_s": n / (t * 1e-3), "algorithmic_bytes_per_frame": bytes_frame,
                      "achieved_GBs": bytes_frame * n / (t * 1e-3) / 1e9}
        del outs, eq
    return res


def bench_config5_ref(wce, ctx_ref, stream, n, reps):
    """BASELINE configs[4] in main.c semantics (round 3): REF PS_MMSE + LT_LS /
    PS_Linear / PS_Cubic / PS_Sinc + equalization over n frames with per-frame
    preambles, one HBM pass (ref_ls_elem_kernel: one (frame, subcarrier)
    element per thread).  frame_cov_*: the same with WCE_MMSE_FRAME_COV, i.e.
    each frame's PS_MMSE from its own LT_LS as main.c:37-53 / 148 chain them
    (round 5: ref_fc_kernel writes each frame's PS_MMSE itself -- LT_LS, w
    at the pilots from the folded map, u = Mu h on f64 MFMA, H = u s -- and
    the one-pass kernel writes the LS family + eq; the factor kernel's extra
    rx_pre read, 848 B per frame, shows in `traffic`).  Bytes per frame, SURVEY 8(d): rx 15x53 + tx block 0 +
    rx_pre in, 5 H + eq out = 31,376 (fp64) / 23,320 (LS + eq stored fp32); the
    kernel reads only tx's 4 pilots of block 0, so it moves 784 B less
    (30,592 / 22,536: its minimum I/O, the rate quoted as `achieved`)."""
    s = stream.handle
    tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx_ref.synth(tx, rx, pre, n, seed=0x80211, stream=s)
    fr = ctx_ref.frames(tx, rx, n, rx_pre=pre)
    res = {"workload": f"BASELINE configs[4], main.c semantics: REF PS_MMSE + LT_LS + PS_Linear/Cubic/Sinc + "
                       f"equalization, per-frame preambles, {n} frames, one HBM pass (ref_ls_elem_kernel)",
           "frames": n}
    ctx_ref.reserve(n)   # FRAME_COV: the per-frame factor rows (u, w) live in the ctx's workspace
    for label, f32, leg, fc in (("fp64", False, "config5_ref", False),
                                ("mixed_fp64_solve_fp32_ls", True, "config5_ref_f32", False),
                                ("frame_cov_fp64", False, "config5_ref_fc", True),
                                ("frame_cov_mixed_fp32_ls", True, "config5_ref_fc_f32", True)):
        dt = np.complex64 if f32 else np.complex128
        outs = [wce.DeviceArray((n, N), dt) for _ in range(4)] + [wce.DeviceArray((n, N))]
        eq = wce.DeviceArray((n, NBLK, N), dt)
        o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32 if f32 else 0)
        mask = wce.ALL | (wce.FRAME_COV if fc else 0)
        f = lambda: ctx_ref.estimate(fr, o, mask, s)
        for _ in range(3):
            f()
        t = time_events(wce, stream, f, reps)
        ob = 8 if f32 else 16
        out_b = (4 * N + NBLK * N) * ob + N * 16
        survey = (NBLK * N + N + N) * 16 + out_b            # 31,376 / 23,320
        minimal = (NBLK * N + N + 4) * 16 + out_b            # tx: 4 pilots
        ach = minimal * n / (t * 1e-3) / 1e9
        # WRITE_SIZE runs 5% (fp64) / 11% (fp32) over the output bytes: 53-element
        # rows end in partial 64-B sectors; FETCH_SIZE = streamed rx / rx_pre (x2,
        # the gfx950 correction) + the 8 pilot sectors per frame (counted in full)
        ls_b = out_b - (N * 16 if fc else 0)   # FRAME_COV: PS_MMSE leaves from ref_fc_kernel
        k, src = pmc_leg(leg, n, ls_b * n, tol=0.12) if leg != "config5_ref_fc_f32" else (None, "fp32 FRAME_COV leg not profiled")
        traffic = hbm_bytes(k, narrow_fetch_kib=BYTES_PILOT_SECTORS * n / 1024.0) if k else None
        if fc and traffic is not None:   # + ref_fc_kernel: rx_pre and the pilots in, H out
            kf, _ = pmc_leg("config5_ref_fc_factors", n, N * 16.0 * n, tol=0.12)
            traffic = traffic + hbm_bytes(kf, narrow_fetch_kib=BYTES_PILOT_SECTORS * n / 1024.0) if kf else None
        bad = sum(ctx_ref.nonfinite_scan(h, n, f32=(f32 and i < 4), stream=s)[1] for i, h in enumerate(outs))
        bad += ctx_ref.nonfinite_scan(eq, n * NBLK, f32=f32, stream=s)[1]
        res[label] = {"ms_per_step": t, "frames_per_s": n / (t * 1e-3),
                      "kernels": "ref_fc_kernel (PS_MMSE) + ref_ls_elem_kernel<true> (LS family + eq)" if fc else
                                 "ref_ls_elem_kernel<true>",
                      "roofline": {"bound": "hbm", "kernel": "ref_ls_elem_kernel", "achieved": ach,
                                   "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                                   "traffic": traffic, "pmc_source": src,
                                   "bytes_per_frame": minimal, "survey_bytes_per_frame": survey,
                                   "achieved_on_survey_bytes": survey * n / (t * 1e-3) / 1e9},
                      "nonfinite_outputs": bad}
        del outs, eq
    return res


def tile_block0(wce, tx, rx, B, n):
    """n frames holding block 0 only (frame_stride = 53), block 0 of the B
    frames in tx / rx tiled n / B times: a 1,048,576-frame low-rank batch in
    1.8 GB instead of 27 GB (the per-frame MMSE reads block 0 only)."""
    lib = wce.load()
    out = []
    for src in (tx, rx):
        h = np.ascontiguousarray(src.numpy()[:, 0])
        d = wce.DeviceArray((n, N))
        for off in range(0, n, B):
            m = min(B, n - off)
            assert lib.wce_memcpy_htod(d.addr + off * N * 16, h.ctypes.data, m * N * 16) == 0
        out.append(d)
    return out[0], out[1], wce.Context.frames(out[0], out[1], n, frame_stride=N, block_stride=N)


def bench_cov_lowrank(wce, make_ctx, stream, tx, rx, B, reps, big=1 << 20):
    """WCE_MMSE_COV with a power-delay profile of L taps (rank L, the channel
    model of SURVEY 8(d)): the low-rank Gram path, which meets 1e-10 where
    the dense Ryy solve cannot.  Ranks 1..8 run one frame per
    lane (mmse_lr_lane_staged_kernel: frames staged through LDS, P_k / U
    shared per workgroup in LDS; 2,544 B per frame move: tx + rx block in, H
    out), ranks 9..16 16 lanes per frame (mmse_lr_quad_kernel), higher ranks
    one frame per wave (mmse_lr_kernel).  Per-frame rate on the headline's
    frames, beside the wave kernel (ranks <= 16) and the dense path forced on
    the same ctx (wce_debug_set_variant / wce_debug_set_cov_path).  Rank 8
    also at 1,048,576 frames (configs[3]'s batch), where ranks 7 and 8 run
    the two-workgroups-per-CU build.  Kernel names come from the library's
    own selection (wce_debug_lr_kernel); every leg's H is scanned."""
    s = stream.handle
    lib = wce.load()
    H = wce.DeviceArray((B, N))
    fr = wce.Context.frames(tx, rx, B)
    o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    out = {"workload": f"{B} frames, PS_MMSE, Rhh = L-tap exponential PDP (rank L)"}
    for L in (4, 8, 16, 24, 53):
        p = np.exp(-0.5 * np.arange(L))
        Rhh = np.zeros((N, N), np.complex128)
        Rhh[np.arange(L), np.arange(L)] = p / p.sum() * 1.1e-4
        c = make_ctx(Rhh)
        r, lr, _, _ = c.cov_info()
        f = lambda: c.estimate(fr, o, wce.PS_MMSE, s)
        for _ in range(2):
            f()
        t = time_events(wce, stream, f, reps)
        lane = lr and 1 <= r <= 8
        quad = lr and 9 <= r <= 32      # mmse_lr_quad_kernel (9..16), mmse_lr_quad2_kernel (17..32, taps 0..r-1)
        leg = {"rank": r, "path": "low-rank" if lr else "dense",
               "kernel": c.lr_kernel(B) if lr else "mmse_solve_kernel<false> + H = C W",
               "ms_per_step": t, "frames_per_s": B / (t * 1e-3),
               "nonfinite_frames": ctx_scan(c, H, B, s)}
        if lane or quad:
            leg["achieved_GBs"] = 3 * N * 16 * B / (t * 1e-3) / 1e9
            leg["hbm_frac"] = leg["achieved_GBs"] / PEAK_HBM_GBS
            assert lib.wce_debug_set_variant(3, 1) == 0    # the same ranks one frame per wave
            try:
                for _ in range(2):
                    f()
                tw = time_events(wce, stream, f, reps)
                leg.update({"wave_kernel": c.lr_kernel(B), "wave_kernel_ms_per_step": tw})
            finally:
                assert lib.wce_debug_set_variant(3, 0) == 0
        if lr:
            # the tap-domain forms (a diagonal Rhh, round 4: the Toeplitz Gram of the
            # lane / quad kernels, the DFT Gram of the wave kernel) against the
            # product Gram on the same ctx (variant 5)
            assert lib.wce_debug_set_variant(3, 5) == 0
            try:
                for _ in range(2):
                    f()
                tp = time_events(wce, stream, f, reps)
                leg.update({"product_gram_kernel": c.lr_kernel(B), "product_gram_ms_per_step": tp,
                            "taps_speedup": tp / t})
            finally:
                assert lib.wce_debug_set_variant(3, 0) == 0
        if lr and r > 16:
            # FP64-VALU bound, priced at the tap form's algorithmic flops (DESIGN.md
            # s2): r x r Cholesky + triangular solves + the Q / D / read-out DFTs (20 N^2)
            fl = flop_lr_taps(r)
            ach = fl * B / (t * 1e-3) / 1e12
            kn = c.lr_kernel(B)
            kw, wsrc = pmc_leg("lowrank%d" % L, B, N * 16.0 * B,
                               waves=4 * ((B + 15) // 16) if "quad" in kn else B)   # quad forms: 16 units per 4-wave group
            leg["roofline"] = {"bound": "valu-f64", "achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                               "frac": ach / PEAK_FP64_TFLOPS, "flops_per_frame": fl,
                               "traffic": hbm_bytes(kw) if kw else None, "pmc_source": wsrc}
            if kw:
                # per frame (= per wave for the wave kernel; a quad-form wave holds 4 frames)
                leg["pmc_per_frame"] = {k: kw[k] / B for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_LDS",
                                                               "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT",
                                                               "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES")
                                        if k in kw}
        if L in (16, 53):
            # constant-modulus frames (the synthetic BPSK: +-A, DC null) on the shared
            # operator K = (a C P + b I)^-1 C (wce_ctx_set_modulus): two f64-MFMA
            # launches instead of the per-frame solve; HBM roofline on the 2,544 B
            # per frame; never the headline, never credited F_alg
            c.set_modulus(tx.rows(0)[0, 0])
            for _ in range(2):
                f()
            tc = time_events(wce, stream, f, reps)
            gbs = 3 * N * 16 * B / (tc * 1e-3) / 1e9
            kc, srcc = pmc_leg("cm%d" % L, B, N * 16.0 * B, tol=0.12)   # persistent grid: check the output bytes
            leg["constant_modulus"] = {
                "kernel": "cm_real_kernel (+ cm_cplx_kernel for non-real symbols: none here)",
                "ms_per_step": tc, "frames_per_s": B / (tc * 1e-3), "speedup_vs_per_frame": t / tc,
                "roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": gbs / PEAK_HBM_GBS, "algorithmic_bytes": 3 * N * 16 * B,
                             "traffic": hbm_bytes(kc) if kc else None, "pmc_source": srcc},
                # per 16-frame tile: rows 0..47 3 x 14 x 3 v_mfma_f64_16x16x4 (2,048 flop), rows 48..52
                # 14 x 6 v_mfma_f64_4x4x4_4b (512 flop)
                "mfma_executed_tflops": (3 * KSTEPS_MFMA * 3 * 2048 + KSTEPS_MFMA * 6 * 512) * ((B + 15) // 16)
                / (tc * 1e-3) / 1e12,
                "nonfinite_frames": ctx_scan(c, H, B, s),
                "note": "frames whose |x|^2 pattern matches the ctx's (all synthetic frames): "
                        "H = K (conj x o rx), K formed once in 80 bits"}
            c.set_modulus(None)
        if L == 8:
            txb, rxb, frb = tile_block0(wce, tx, rx, B, big)
            Hb = wce.DeviceArray((big, N))
            ob = wce.Outputs(None, None, None, None, Hb.addr, None, N, 0, 0, 0, 0)
            fb = lambda: c.estimate(frb, ob, wce.PS_MMSE, s)
            for _ in range(2):
                fb()
            tb = time_events(wce, stream, fb, max(3, reps // 4))
            gbs = 3 * N * 16 * big / (tb * 1e-3) / 1e9
            kb, src = pmc_leg("lowrank8_1m", big, N * 16.0 * big, tol=0.05)
            leg[f"frames_{big}"] = {
                "kernel": c.lr_kernel(big), "frames": big, "ms_per_step": tb, "frames_per_s": big / (tb * 1e-3),
                "roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": gbs / PEAK_HBM_GBS, "algorithmic_bytes": 3 * N * 16 * big,
                             "traffic": hbm_bytes(kb) if kb else None, "pmc_source": src},
                "nonfinite_frames": ctx_scan(c, Hb, big, s)}
            del txb, rxb, Hb
        c.set_cov_path(1)
        for _ in range(2):
            f()
        td = time_events(wce, stream, f, reps)
        leg.update({"dense_forced_ms_per_step": td, "dense_forced_frames_per_s": B / (td * 1e-3)})
        out[f"L{L}"] = leg
        del c
    return out


def flop_lr_taps(r):
    """Algorithmic flops of one frame on the tap-domain Gram path: the r x r
    Cholesky and the bordered / back substitutions (as the dense solve's, at
    size r) plus the three 53-point DFTs of the Gram row Q (real weights,
    4 N^2), the border D and the read-out (8 N^2 each); real symbols (no
    correction DFTs), as the bench's BPSK frames."""
    return 4.0 / 3.0 * r ** 3 + 8.0 * r * r + 20.0 * N * N


def ctx_scan(c, H, n, s):
    """non-finite frames of an fp64 output (wce_nonfinite_scan, untimed)"""
    return int(c.nonfinite_scan(H, n, stream=s)[1])


def bench_frame_cov(wce, make_ctx, stream, n, reps):
    """PS_MMSE with each frame's own preamble covariance (WCE_MMSE_FRAME_COV,
    SURVEY 8(f)-4), C semantics.  TEXTBOOK: LT_LS per frame and the rank-1
    factor u = Mu h on f64 MFMA in one launch (ref_fc_kernel<UOUT>), then the
    dense per-frame solve; REF: LT_LS, the factors and the read-out in one
    launch (ref_fc_kernel)."""
    s = stream.handle
    out = {"workload": f"{n} frames, per-frame preamble, PS_MMSE | FRAME_COV"}
    for label, m in (("textbook", wce.MMSE_TEXTBOOK), ("ref", wce.MMSE_REF)):
        c = make_ctx(m)
        tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
        c.synth(tx, rx, pre, n, seed=0x80211, stream=s)
        H = wce.DeviceArray((n, N))
        c.reserve(n)
        fr = c.frames(tx, rx, n, rx_pre=pre)
        o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
        f = lambda: c.estimate(fr, o, wce.PS_MMSE | wce.FRAME_COV, s)
        for _ in range(3):
            f()
        t = time_events(wce, stream, f, reps)
        out[label] = {"ms_per_step": t, "frames_per_s": n / (t * 1e-3), "nonfinite_frames": ctx_scan(c, H, n, s)}
        if m == wce.MMSE_TEXTBOOK:
            out[label]["kernels"] = "ref_fc_kernel<UOUT> (LT_LS, u = Mu h) + mmse_solve_fc_kernel"
        if m == wce.MMSE_REF:
            # one launch (ref_fc_kernel): rx_pre 848 + 8 pilots 128 in, H 848 out
            alg = (N * 16 + 8 * 16 + N * 16) * n
            k, src = pmc_leg("frame_cov_ref", n, N * 16.0 * n, tol=0.12)   # persistent grid: check the output bytes
            gbs = alg / (t * 1e-3) / 1e9
            out[label].update({"kernel": "ref_fc_kernel (LT_LS, w at the pilots from the folded map, u = Mu h on "
                                         "f64 MFMA, H = u s)",
                               "roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                            "frac": gbs / PEAK_HBM_GBS, "algorithmic_bytes": alg,
                                            "traffic": hbm_bytes(k, narrow_fetch_kib=BYTES_PILOT_SECTORS * n / 1024.0)
                                            if k else None, "pmc_source": src,
                                            # executed: per 16-frame tile u = Mu h in the 3M form, rows 0..47
                                            # 3 x 14 x 3 v_mfma_f64_16x16x4 (2,048 flop), rows 48..52 14 x 6
                                            # v_mfma_f64_4x4x4_4b (512 flop)
                                            "mfma_executed_tflops": (3 * KSTEPS_MFMA * 3 * 2048 + KSTEPS_MFMA * 6 * 512)
                                            * ((n + 15) // 16) / (t * 1e-3) / 1e12}})
        del c
    return out


def cpu_reference(budget_s):
    """The reference's OWN sequential code (oracle/_ref/libref.so, compiled
    from its main.c/utils.c by oracle/Makefile; 1 core), when that library was
    built and travelled with the snapshot: LT_LS + PS_Linear (config 2) and
    REF-mode PS_MMSE through its matrix routines (NaN inverse(Ryy) repaired,
    per-frame inverse(F) hoisted)."""
    import ctypes
    lib_path = os.path.join(REPO, "oracle", "_ref", "libref.so")
    if not os.path.exists(lib_path):
        return None
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py
    lib = ctypes.CDLL(lib_path)
    P = ctypes.c_void_p
    lib.refh_bench_ls.restype = ctypes.c_double
    lib.refh_bench_ls.argtypes = [ctypes.c_int] + [P] * 6
    lib.refh_bench_mmse.restype = ctypes.c_double
    lib.refh_bench_mmse.argtypes = [ctypes.c_int, P, P, P, ctypes.c_double, P, P, P]
    has_omp = hasattr(lib, "refh_bench_ls_omp")
    if has_omp:
        lib.refh_bench_ls_omp.restype = ctypes.c_double
        lib.refh_bench_ls_omp.argtypes = [ctypes.c_int, ctypes.c_int] + [P] * 6
        lib.refh_bench_mmse_omp.restype = ctypes.c_double
        lib.refh_bench_mmse_omp.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_double, P, P, P]
    try:
        cores = max(1, min(len(os.sched_getaffinity(0)), 16))
    except AttributeError:  # pragma: no cover
        cores = max(1, min(os.cpu_count() or 1, 16))
    LD = np.clongdouble
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    ref = dict(np.load(os.path.join(REPO, "tests", "golden", "ref_vectors.npz")))
    rng = np.random.default_rng(0)
    p = lambda a: a.ctypes.data_as(P)
    out = {"kind": "reference", "cores": 1,
           "source": "oracle/_ref/libref.so = /root/reference main.c + utils.c, g++ -O2 (oracle/Makefile)"}
    n = 100000
    tx = np.ascontiguousarray(np.repeat(inp["tx_symb"][0][None], n, 0).astype(LD))
    rx = np.ascontiguousarray((np.repeat(inp["rx_symb"][0][None], n, 0)
                               * (1 + 0.01 * rng.standard_normal((n, 1)))).astype(LD))
    pre = np.ascontiguousarray((np.repeat(inp["rx_pre"][None], n, 0)
                                * (1 + 0.01 * rng.standard_normal((n, 1)))).astype(LD))
    tpre = np.ascontiguousarray(inp["tx_pre"].astype(LD))
    h1, h2 = np.zeros((n, N), LD), np.zeros((n, N), LD)
    t = lib.refh_bench_ls(n, p(tpre), p(pre), p(tx), p(rx), p(h1), p(h2))
    out["ls_config2"] = {"value": n / t, "unit": "frames/s", "sample": f"{n} frames, {t:.2f} s"}
    if has_omp:
        t = lib.refh_bench_ls_omp(n, cores, p(tpre), p(pre), p(tx), p(rx), p(h1), p(h2))
        out["ls_config2_omp"] = {"value": n / t, "unit": "frames/s", "cores": cores,
                                 "sample": f"{n} frames, {t:.3f} s, the reference's functions in a "
                                           f"frames-parallel OpenMP loop (its own OpenMP driver crashes)"}
    F = np.ascontiguousarray(oracle_py.from_split(ref["F"]))
    invF = np.ascontiguousarray(oracle_py.from_split(ref["invF"]))
    hls = np.ascontiguousarray(oracle_py.lt_ls(inp["tx_pre"], inp["rx_pre"]).astype(LD))
    H = np.zeros((n, N), LD)
    t1 = lib.refh_bench_mmse(1, p(tx), p(rx), p(F), float(inp["ow2"]), p(hls), p(invF), p(H))
    m = int(max(1, min(n, 0.5 * budget_s / max(t1, 1e-6))))
    t = lib.refh_bench_mmse(m, p(tx), p(rx), p(F), float(inp["ow2"]), p(hls), p(invF), p(H))
    if has_omp:
        mo = int(max(cores, min(n, 0.5 * budget_s * cores / max(t1, 1e-6))))
        to = lib.refh_bench_mmse_omp(mo, cores, p(tx), p(rx), p(F), float(inp["ow2"]), p(hls), p(invF), p(H))
        out["mmse_ref_mode_omp"] = {"value": mo / to, "unit": "frames/s", "cores": cores,
                                    "sample": f"{mo} frames, {to:.2f} s, frames-parallel OpenMP loop over the "
                                              f"reference's per-frame MMSE"}
    out["mmse_ref_mode"] = {"value": m / t, "unit": "frames/s", "sample": f"{m} frames, {t:.2f} s",
                            "note": "the reference's literal PS_MMSE also spends ~4 s per frame inverting F "
                                    "and returns NaN; both are removed here"}
    if hasattr(lib, "refh_bench_mmse_formula"):
        # the headline (TEXTBOOK) mode through the reference's own arithmetic:
        # WiFi_channel_estimation_PS_MMSE.m:26-33 composed from multiply()
        # (utils.c:16-31) and the cofactor inverse() (utils.c:141-170) of each
        # frame's 52 x 52 Ryy, ~4 s per frame; the inputs.h frame and channel
        # variations of it, 1 frame on 1 core, then `cores` frames on `cores`
        lib.refh_bench_mmse_formula.restype = ctypes.c_double
        lib.refh_bench_mmse_formula.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_double, P, P]
        t1 = lib.refh_bench_mmse_formula(1, 1, p(tx), p(rx), p(F), float(inp["ow2"]), p(hls), p(H))
        tc = lib.refh_bench_mmse_formula(cores, cores, p(tx), p(rx), p(F), float(inp["ow2"]), p(hls), p(H))
        out["mmse_textbook"] = {
            "value": 1.0 / t1, "unit": "frames/s", "cores": 1, "sample": f"1 frame, {t1:.2f} s",
            "frames_parallel": {"value": cores / tc, "unit": "frames/s", "cores": cores,
                                "sample": f"{cores} frames, {tc:.2f} s, frames-parallel OpenMP loop"},
            "routine": "refh_mmse_formula: the .m formula from the reference's multiply() and cofactor inverse()",
            "note": "the headline mode; the GPU runs the same formula as a bordered Cholesky (DESIGN.md s2)"}
    return out


def cpu_baseline(wce, ctx, frames, tx, rx, B, mode, budget_s):
    """The oracle's fp64 OpenMP port of the same unified MMSE (kind "port"),
    on a bounded sample of the benchmark's own frames; its H is compared with
    the GPU's H of the same frames (max norm-relative error)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    hlt, C, a, b = ctx.shared()
    mask = oracle_py.pilot_mask() if mode == 0 else np.ones(N, np.uint8)
    m = min(B, 4096)
    txh = tx.numpy()[:m, 0].copy()
    rxh = rx.numpy()[:m, 0].copy()
    Hc, t = oracle_py.bench_mmse_f64(C, mask, a, b, txh.reshape(-1), rxh.reshape(-1), N, cores)
    rate = m / t
    Hg = wce.DeviceArray((B, N), zero=True)
    ctx.estimate(frames, wce.Outputs(None, None, None, None, Hg.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE)
    wce.synchronize()
    err = oracle_py.normrel(Hg.rows(0, m), Hc)
    target = int(min(max(rate * budget_s / cores, m), 2_000_000))
    reps = max(1, target // m)
    t_tot = 0.0
    for _ in range(reps):
        _, t = oracle_py.bench_mmse_f64(C, mask, a, b, txh.reshape(-1), rxh.reshape(-1), N, cores)
        t_tot += t
    frames = reps * m
    return {"value": frames / t_tot, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{frames} frames ({m} distinct bench frames x {reps}): the unified dense MMSE in fp64 "
                      f"(LDL^H + back-substitution + C w, the GPU's dense-C path), OpenMP over frames, "
                      f"{t_tot:.2f} s wall",
            "max_normrel_err_vs_gpu": float(err.max()), "median_normrel_err_vs_gpu": float(np.median(err)),
            "err_frames": m,
            "reference_main_c_seconds_per_frame": 232.6,
            "reference_note": "main.c PS_MMSE itself: ~200-233 s/frame on 1 core, output NaN (SURVEY 0-1); "
                              "its OpenMP path segfaults"}


if __name__ == "__main__":
    main()
