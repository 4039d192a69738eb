"""Multi-rank host logic on CPU (gloo, world size 2): frame sharding and the
single shared-state broadcast.  The GPU-side bit-identity of sharded frames
and estimates is in test_parity_gpu.py::test_full_size_properties."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("total,world", [(0, 2), (1, 2), (65536, 8), (1048576, 8), (1000003, 7), (5, 8)])
def test_shard_partitions_exactly(total, world):
    sys.path.insert(0, REPO)
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    seen = 0
    for r in range(world):
        first, count = multi.shard(total, world, r)
        assert first == seen
        seen += count
    assert seen == total
    counts = [multi.shard(total, world, r)[1] for r in range(world)]
    assert max(counts) - min(counts) <= 1


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    wce = importlib.import_module("80211parallelestimation_amd")
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
        n = wce.load().wce_state_size()
        blob = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK) if rank == 0 else None
        got = multi.broadcast_state_host(dist, blob, n, src=0)
        local = wce.state_blob(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK)
        mode = wce.state_mode(got)   # raises unless the bytes carry the state magic
        q.put((rank, bool(np.array_equal(got, local)), mode, multi.weak_shard(65536, rank)))
    finally:
        dist.destroy_process_group()


def test_state_broadcast_gloo_world2():
    """Rank 0 builds the 80-bit shared state on the host, one broadcast
    delivers it; rank 1 receives exactly the bytes it would have built."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == [0, 1]
    for rank, same, mode, (first, count) in res:
        assert same
        assert mode == 1   # WCE_MMSE_TEXTBOOK
        assert (first, count) == (rank * 65536, 65536)


@pytest.mark.parametrize("total,world", [(0, 2), (1, 2), (65536, 8), (1000003, 7), (5, 8)])
def test_native_shard_matches_host(wce, total, world):
    """wce_shard (C ABI) partitions exactly like multi.shard."""
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    for r in range(world):
        assert multi.native_shard(wce, total, world, r) == multi.shard(total, world, r)


def test_native_comm_fails_loudly_without_device(wce):
    """Bad arguments are rejected and, with no gfx950 device, a communicator
    cannot be created (an error code, never a silent CPU path)."""
    import ctypes

    multi = importlib.import_module("80211parallelestimation_amd.multi")
    lib = wce.load()
    f, c = ctypes.c_int64(), ctypes.c_int64()
    assert lib.wce_shard(10, 0, 0, ctypes.byref(f), ctypes.byref(c)) != 0
    assert lib.wce_shard(10, 2, 2, ctypes.byref(f), ctypes.byref(c)) != 0
    assert lib.wce_comm_info(None, None, None, None) != 0
    assert lib.wce_ctx_broadcast_state(None, None, 0, None) != 0
    assert lib.wce_comm_destroy(None) == 0
    if wce.device_count() == 0:
        with pytest.raises(wce.WceError):
            multi.NativeComm(wce, b"\0" * multi.COMM_ID_BYTES, 1, 0, 0)


class _NullStream:
    def synchronize(self):
        pass


def _bench_dist_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), WCE_DIST_BACKEND="gloo")
    sys.path.insert(0, REPO)
    bench = importlib.import_module("bench")
    d = bench.Dist()
    try:
        calls = []
        bench.prewarm_sync(d, _NullStream(), lambda: calls.append(1), 0.05)
        d.barrier()
        g = d.group_check()
        q.put((rank, d.world, d.max(1.5 + rank), len(calls) > 0, g["group_size"], g["all_ranks_agree"]))
    finally:
        d.close()


def test_bench_dist_control_path_gloo_world2():
    """bench.py's Dist over gloo at world size 2 (the N>1 launch's control
    path): the max over ranks every timed leg reports, the barriers, and the
    synchronised prewarm the sharded legs run before their timed region."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, 2, 2.5, True, 2, True), (1, 2, 2.5, True, 2, True)]
