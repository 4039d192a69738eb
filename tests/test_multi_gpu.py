"""The N>1 path on one GPU: RCCL ("nccl" backend) in a one-rank group.

The driver's 2/4/8-GPU runs take bench.py's distributed branch (device
state broadcast over RCCL, device barrier, max all-reduce of the timing).  A
one-GPU box cannot hold two RCCL ranks, so these tests run that exact code
with world size 1: the broadcast buffer round trip into an empty context
(bit-identical estimates), and bench.py under torch.distributed.run with
WCE_FORCE_DIST=1.  Each runs in its own process, as the driver's ranks do.
The multi-rank exchange itself is covered on CPU (gloo, tests/test_multi.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    return env


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def test_rccl_state_broadcast_roundtrip(gpu_wce):
    p = subprocess.run([sys.executable, os.path.join(REPO, "tests", "multi_gpu_worker.py")], env=_env(),
                       capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    res = _last_json(p.stdout)
    for mode in ("textbook", "ref"):
        assert res[mode]["bit_identical"], res
        assert res[mode]["finite"], res
        assert res[mode]["bytes"] == gpu_wce.load().wce_state_size()
    assert res["allreduce_max"] == 3.5


def test_native_rccl_path(gpu_wce):
    """libwce's own RCCL path (wce_comm_*, no torch in the process): both
    launch models in their one-rank form, bit-identical estimates after the
    in-place state broadcast, the root's bytes untouched, the max all-reduce,
    and a root without state refused."""
    p = subprocess.run([sys.executable, os.path.join(REPO, "tests", "native_comm_worker.py")], env=_env(),
                       capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    res = _last_json(p.stdout)
    assert res["info"] == [0, 1, 0] and res["all_info"] == [0, 1, 0]
    for case in ("rank_textbook", "rank_ref", "all_ref"):
        r = res[case]
        assert r["bit_identical"] and r["finite"] and r["root_unchanged"], res
        assert r["bytes"] == gpu_wce.load().wce_state_size()
    assert res["max"] == 3.5
    assert res["empty_root_refused"]


def test_bench_distributed_path_one_rank(gpu_wce):
    env = _env()
    env["WCE_FORCE_DIST"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", env["MASTER_PORT"], os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "5", "--warmup", "2", "--no-extras", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    res = _last_json(p.stdout)
    assert res["n_gpus"] == 1 and res["steps"] == 5 and res["value"] > 0
    assert res["config"]["parallelism"].startswith("dp1")
