"""Two processes sharing GPU 0 estimate the two wce_shard halves of one
frame batch through bench.py's distributed control path (gloo backend: the
one-GPU stand-in for the driver's RCCL ranks).  The concatenated shard
outputs must equal a single-process run of the whole batch bit for bit --
the whole multi-rank data path (state broadcast, shard ranges, per-rank
synthesis from the global frame index, estimation) the 8-GPU run takes.
Reference analogue: the frame groups of main_mpi.c:21-27,62-71."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, NBLK = 53, 15
NAMES = ("lt_ls", "ps_linear", "ps_cubic", "ps_sinc", "ps_mmse")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_shards_equal_single_run(gpu_wce, golden, tmp_path):
    wce = gpu_wce
    total = 40001                    # odd: the shards differ by one frame
    env = dict(os.environ)
    port = _free_port()
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
               WCE_DIST_BACKEND="gloo", WCE_SHARD_TOTAL=str(total), WCE_SHARD_OUT=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "tests", "sharded_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    parts = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(2)]
    assert int(parts[0]["first"]) == 0 and int(parts[1]["first"]) == int(parts[0]["count"])
    assert int(parts[0]["count"]) + int(parts[1]["count"]) == total
    assert all(float(x["nonfinite_max"]) == 0 for x in parts)
    # the same frames in one process
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    tx, rx, pre = wce.DeviceArray((total, NBLK, N)), wce.DeviceArray((total, NBLK, N)), wce.DeviceArray((total, N))
    ctx.synth(tx, rx, pre, total, seed=0x5A4D)
    outs = [wce.DeviceArray((total, N), zero=True) for _ in range(5)]
    eq = wce.DeviceArray((total, NBLK, N), zero=True)
    o = wce.Outputs(*(x.addr for x in outs), eq.addr, N, NBLK * N, N, 0, 0)
    ctx.estimate(ctx.frames(tx, rx, total, rx_pre=pre), o, wce.ALL)
    wce.synchronize()
    for name, h in zip(NAMES, outs):
        assert np.array_equal(np.concatenate([x[name] for x in parts]), h.numpy()), name
    assert np.array_equal(np.concatenate([x["eq"] for x in parts]), eq.numpy())
