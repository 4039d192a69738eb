"""configs[4] as named (bench_config5_sharded at N = 1): the fused launch
(solve + LS family + equalization in the solve's epilogue) against a
two-stream form -- PS_MMSE alone on one stream, the LS family + equalization
pass (mask LS_ALL | EQUALIZE) on a second, concurrently -- on the same
1,048,576 frames, fp32 LS / eq outputs.  Host wall per step over `steps`
steps, both streams drained at the end; outputs of the two forms compared."""
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
N, NBLK = 53, 15


def main():
    wce = importlib.import_module("80211parallelestimation_amd")
    wce.load().wce_set_device(0)
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    steps = 10
    s1, s2 = wce.Stream(), wce.Stream()
    tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx.synth(tx, rx, pre, n, seed=0x80211, stream=s1.handle)
    outs = [wce.DeviceArray((n, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((n, N))]
    eq = wce.DeviceArray((n, NBLK, N), np.complex64)
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
    fr = ctx.frames(tx, rx, n, rx_pre=pre)
    outs2 = [wce.DeviceArray((n, N), np.complex64) for _ in range(4)] + [wce.DeviceArray((n, N))]
    eq2 = wce.DeviceArray((n, NBLK, N), np.complex64)
    o_ls = wce.Outputs(*(x.addr for x in outs2[:4]), None, eq2.addr, N, NBLK * N, N, 0, wce.OUT_LS_F32)
    o_mm = wce.Outputs(None, None, None, None, outs2[4].addr, None, N, 0, 0, 0, 0)

    def fused():
        ctx.estimate(fr, o, wce.ALL, s1.handle)

    def split():
        ctx.estimate(fr, o_ls, wce.LS_ALL | wce.EQUALIZE, s2.handle)
        ctx.estimate(fr, o_mm, wce.PS_MMSE, s1.handle)

    def solve_only():
        ctx.estimate(fr, o_mm, wce.PS_MMSE, s1.handle)

    def ls_only():
        ctx.estimate(fr, o_ls, wce.LS_ALL | wce.EQUALIZE, s2.handle)

    res = {"frames": n}
    for name, f in (("fused", fused), ("split_two_streams", split), ("solve_only", solve_only),
                    ("ls_eq_only", ls_only), ("fused_again", fused)):
        for _ in range(3):
            f()
        s1.synchronize(); s2.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            f()
        s1.synchronize(); s2.synchronize()
        res[name + "_ms"] = (time.perf_counter() - t0) / steps * 1e3
    fused(); split()
    s1.synchronize(); s2.synchronize()
    same = {}
    for i, nm in enumerate(("lt_ls", "ps_linear", "ps_cubic", "ps_sinc", "ps_mmse")):
        a, b = outs[i].numpy(), outs2[i].numpy()
        same[nm] = bool(np.array_equal(a, b))
        if not same[nm]:
            same[nm + "_maxrel"] = float(np.max(np.abs(a - b)) / np.max(np.abs(a)))
    same["eq"] = bool(np.array_equal(eq.numpy(), eq2.numpy()))
    res["bitwise_same"] = same
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
