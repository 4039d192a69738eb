"""Run ONE bench leg's dominant kernel at exactly the bench's launch size,
`--reps` times, and nothing else but its setup (synth / one solve): the
workload for rocprofv3 --pmc passes (tools/pmc_legs.sh), so that a per-kernel
average over the dispatches of a pass is an average over same-size launches.

legs (bench.py field -> kernel, frames per launch):
  headline   roofline            mmse_solve_fc_kernel             65,536 (TEXTBOOK, 1 wave/frame)
  apply      apply_kernel        apply_kernel                     65,536 (COV H = C W, persistent since round 5)
  cov_solve  cov_mode            mmse_solve_kernel<false>         65,536 (COV dense solve)
  ref        ref_mode.b1048576   mmse_ref_elem_kernel          1,048,576 (REF, main.c semantics)
  ls         ls_config2          ls_flat_kernel                1,048,576 (LT_LS + PS_Linear)
  ls_pilots  (calibration)       ls_flat_kernel                1,048,576 (PS_Linear only: pilot reads)
  front_*    front_end           front_kernel<false/true>         65,536 frames (x 15 blocks / 1 LTF)
  config5    config5_sharded     mmse_solve_ls_kernel<true,true,true>  1,048,576 (all 5 + eq, fp32 LS)
  config5_ref(_f32) config5_ref   ref_ls_elem_kernel<true>      1,048,576 (REF + LS family + eq, fp64 / fp32 LS)
  config5_ref_fc(_factors)       ref_ls_elem_kernel<true> / ref_fc_kernel<false>  1,048,576 (the same | FRAME_COV)
  frame_cov_ref frame_cov.ref    ref_fc_kernel<false>             65,536 (REF PS_MMSE | FRAME_COV: one launch)
  lowrank<L> cov_lowrank.L<L>    mmse_lr_lane_staged_kernel<L, 1, true> (L <= 8) / mmse_lr_quad_kernel<L, true> (L <= 16) /
                                 mmse_lr_quad2_kernel<24> (L = 24, round 6) / mmse_lr_kernel<0, true> (53, tap-domain Gram)
                                 65,536 (COV, L-tap PDP: rank L)
  lowrank8_1m cov_lowrank.L8.frames_1048576  mmse_lr_lane_staged_kernel<8, 2, true>  1,048,576 (block 0 only)
"""
import argparse
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
N, NBLK = 53, 15

LEGS = {
    "headline": ("mmse_solve_fc_kernel", 65536),
    "apply": ("apply_kernel", 65536),                # round 5: the streaming kernel at every size
    "apply1m": ("apply_kernel", 1 << 20),             # the same at configs[3]'s batch
    "cov_solve": ("mmse_solve_kernel<false>", 65536),
    "ref": ("mmse_ref_elem_kernel", 1 << 20),          # round 6: one element per thread past the MALL
    "ls": ("ls_elem_kernel", 1 << 20),
    "ls_pilots": ("ls_elem_kernel", 1 << 20),      # PS_Linear only: calibrates the pilot-sector reads
    "front_blocks": ("front_kernel<false>", 65536),
    "front_preamble": ("front_kernel<true>", 65536),
    "config5": ("mmse_solve_ls_kernel<true, true, true>", 1 << 20),
    "config5_ref": ("ref_ls_elem_kernel<true>", 1 << 20),
    "config5_ref_f32": ("ref_ls_elem_kernel<true>", 1 << 20),
    "config5_ref_fc": ("ref_ls_elem_kernel<true>", 1 << 20),          # REF + FRAME_COV, all 5 + eq (round 4) ...
    "config5_ref_fc_factors": ("ref_fc_kernel<false>", 1 << 20),     # ... and its PS_MMSE kernel (same workload, round 5)
    "frame_cov_ref": ("ref_fc_kernel<false>", 65536),        # REF + FRAME_COV, PS_MMSE only: the whole step
    "lowrank4": ("mmse_lr_lane_staged_kernel<4, 1, true>", 65536),     # Toeplitz Gram (taps 0..3, round 4)
    "lowrank8": ("mmse_lr_lane_staged_kernel<8, 1, true>", 65536),
    "lowrank16": ("mmse_lr_quad_kernel<16, true, true>", 65536),   # round 6: fused-DPP Cholesky, pair-form DFTs
    "lowrank24": ("mmse_lr_quad2_kernel<24, true, 2>", 65536),    # round 6: two Gram rows per lane (taps 0..23)
    "lowrank53": ("mmse_lr_kernel<0, true>", 65536),     # the same at full rank, spectrum 2e11
    "lowrank8_1m": ("mmse_lr_lane_staged_kernel<8, 2, true>", 1 << 20),   # block 0 only, frame_stride 53
    "cm16": ("cm_real_kernel", 65536),         # constant-modulus operator path, 16-tap PDP (round 4)
    "cm53": ("cm_real_kernel", 65536),         # the same, 53-tap exp(-0.5 k) (wide spectrum)
}


def pdp_rank(L):
    p = np.exp(-0.5 * np.arange(L))
    R = np.zeros((N, N), np.complex128)
    R[np.arange(L), np.arange(L)] = p / p.sum() * 1.1e-4
    return R


def pdp_rhh():
    p = np.exp(-0.12 * np.arange(N))
    return np.diag(p / p.sum()).astype(np.complex128) * 1.1e-4


def same_kernel(label, full):
    """the library's label (default template arguments left out) names LEGS' full demangled name"""
    return label == full or full.startswith(label[:-1] + ", ")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", choices=sorted(LEGS), required=True)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    wce = importlib.import_module("80211parallelestimation_amd")
    import bench
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    leg = args.leg
    n = LEGS[leg][1]
    if leg in ("headline", "apply", "apply1m", "cov_solve"):
        if leg == "headline":
            ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
        else:
            ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rhh())
        hlt = ctx.shared()[0]
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211, h_shared=wce.DeviceArray.from_numpy(hlt))
        H = wce.DeviceArray((n, N), zero=True)
        fr = ctx.frames(tx, rx, n)
        if leg == "headline":
            run = lambda: ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                                       wce.PS_MMSE)
        elif leg == "cov_solve":
            run = lambda: ctx.mmse_solve(fr, H, N)
        else:
            W = wce.DeviceArray((n, N), zero=True)
            ctx.mmse_solve(fr, W, N)
            run = lambda: ctx.mmse_apply(W, H, n, N)
    elif leg == "lowrank8_1m":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rank(8))
        B = 65536
        tx0, rx0 = wce.DeviceArray((B, NBLK, N)), wce.DeviceArray((B, NBLK, N))
        ctx.synth(tx0, rx0, None, B, seed=0x80211)
        tx, rx, fr = bench.tile_block0(wce, tx0, rx0, B, n)
        del tx0, rx0
        assert same_kernel(ctx.lr_kernel(n), LEGS[leg][0])
        H = wce.DeviceArray((n, N), zero=True)
        run = lambda: ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                                   wce.PS_MMSE)
    elif leg.startswith("cm"):
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rank(int(leg[2:])))
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211)
        wce.synchronize()
        ctx.set_modulus(tx.rows(0)[0, 0])
        H = wce.DeviceArray((n, N), zero=True)
        fr = ctx.frames(tx, rx, n)
        run = lambda: ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                                   wce.PS_MMSE)
    elif leg.startswith("lowrank"):
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], Rhh=pdp_rank(int(leg[7:])))
        tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
        ctx.synth(tx, rx, None, n, seed=0x80211)
        H = wce.DeviceArray((n, N), zero=True)
        fr = ctx.frames(tx, rx, n)
        assert same_kernel(ctx.lr_kernel(n), LEGS[leg][0])
        run = lambda: ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                                   wce.PS_MMSE)
    elif leg == "frame_cov_ref":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
        ctx.synth(tx, rx, pre, n, seed=0x80211)
        ctx.reserve(n)
        H = wce.DeviceArray((n, N), zero=True)
        fr = ctx.frames(tx, rx, n, rx_pre=pre)
        run = lambda: ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                                   wce.PS_MMSE | wce.FRAME_COV)
    elif leg.startswith("config5_ref"):
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        ctx.reserve(n)
        f32 = leg.endswith("f32")
        dt = np.complex64 if f32 else np.complex128
        tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
        ctx.synth(tx, rx, pre, n, seed=0x80211)
        outs = [wce.DeviceArray((n, N), dt) for _ in range(4)] + [wce.DeviceArray((n, N))]
        eq = wce.DeviceArray((n, NBLK, N), dt)
        o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32 if f32 else 0)
        fr = ctx.frames(tx, rx, n, rx_pre=pre)
        mask = wce.ALL | (wce.FRAME_COV if leg.startswith("config5_ref_fc") else 0)
        run = lambda: ctx.estimate(fr, o, mask)
    elif leg == "ref":
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        tx, rx, fr = bench.ref_frames(wce, ctx, n)
        H = wce.DeviceArray((n, N), zero=True)
        run = lambda: ctx.estimate(fr, wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                                   wce.PS_MMSE)
    elif leg in ("ls", "ls_pilots"):
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        bufs, fr = bench.ls_frames(wce, ctx, n, pilots_only=leg == "ls_pilots")
        hlt, hlin = wce.DeviceArray((n, N)), wce.DeviceArray((n, N))
        if leg == "ls":
            o = wce.Outputs(hlt.addr, hlin.addr, None, None, None, None, N, 0, 0, 0, 0)
            run = lambda: ctx.estimate(fr, o, wce.LT_LS | wce.PS_LINEAR)
        else:
            o = wce.Outputs(None, hlin.addr, None, None, None, None, N, 0, 0, 0, 0)
            run = lambda: ctx.estimate(fr, o, wce.PS_LINEAR)
    elif leg.startswith("front_"):
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF)
        pk, lt = bench.front_frames(wce, n)
        sym, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
        ow2 = wce.DeviceArray((n,), np.float64)
        if leg == "front_blocks":
            run = lambda: ctx.front_end_blocks(pk, n, NBLK, sym)
        else:
            run = lambda: ctx.front_end_preamble(lt, n, 160, pre, ow2)
    else:
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
        tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
        ctx.synth(tx, rx, pre, n, seed=0x80211)
        outs = [wce.DeviceArray((n, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((n, N))]
        eq = wce.DeviceArray((n, NBLK, N), np.complex64)
        o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
        fr = ctx.frames(tx, rx, n, rx_pre=pre)
        run = lambda: ctx.estimate(fr, o, wce.ALL)
    wce.synchronize()
    for _ in range(args.reps):
        run()
    wce.synchronize()
    print(f"{leg}: {args.reps} launches of {LEGS[leg][0]} at {n} frames")


if __name__ == "__main__":
    main()
