"""One rank of the two-process sharded-estimate test (tests/test_sharded_gpu.py),
launched by torch.distributed.run with WCE_DIST_BACKEND=gloo so that both
ranks share GPU 0.  It takes bench.py's distributed control path (bench.Dist):
rank 0 builds the 80-bit shared state, one broadcast delivers it, and each
rank synthesises and estimates its own wce_shard range of the global frames
(main_mpi.c:21-27,62-71 frame groups; main_mpi.c:687-688 the MPI_Bcast this
broadcast replaces).  Outputs go to $WCE_SHARD_OUT/rank<r>.npz."""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

N, NBLK = 53, 15


def main():
    import bench
    dist = bench.Dist()
    assert dist.world == 2 and dist.backend == "gloo", (dist.world, dist.backend)
    wce = importlib.import_module("80211parallelestimation_amd")
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    wce.load().wce_set_device(dist.device)
    total = int(os.environ["WCE_SHARD_TOTAL"])
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    if dist.rank == 0:
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=dist.device)
    else:
        ctx = wce.Context(empty=True, device=dist.device)
    dist.broadcast_state(wce, ctx)
    first, count = multi.native_shard(wce, total, dist.world, dist.rank)
    tx, rx, pre = wce.DeviceArray((count, NBLK, N)), wce.DeviceArray((count, NBLK, N)), wce.DeviceArray((count, N))
    ctx.synth(tx, rx, pre, count, first_frame=first, seed=0x5A4D)
    outs = [wce.DeviceArray((count, N), zero=True) for _ in range(5)]
    eq = wce.DeviceArray((count, NBLK, N), zero=True)
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, 0)
    ctx.estimate(ctx.frames(tx, rx, count, rx_pre=pre), o, wce.ALL)
    wce.synchronize()
    bad = sum(ctx.nonfinite_scan(h, count)[1] for h in outs)
    worst = dist.max(float(bad))
    names = ("lt_ls", "ps_linear", "ps_cubic", "ps_sinc", "ps_mmse")
    np.savez(os.path.join(os.environ["WCE_SHARD_OUT"], f"rank{dist.rank}.npz"), first=first, count=count,
             nonfinite_max=worst, eq=eq.numpy(), **{n: h.numpy() for n, h in zip(names, outs)})
    dist.barrier()
    dist.close()


if __name__ == "__main__":
    main()
