"""BASELINE configs[3] size on one GPU: 1,048,576 frames (the 8-GPU batch),
estimated in one call and as the 8 shards wce_shard gives (each shard
generating its own frames from the global index, as each rank of the 8-GPU
run does).  The shards must reproduce the single batch bit for bit, every
frame must be finite, and the frames sampled against the oracle must agree.
This is the size-independent check of the sharded N>1 data path."""
import numpy as np
import pytest

from oracle_py import normrel

pytestmark = pytest.mark.gpu

N, NBLK = 53, 15
TOTAL, WORLD = 1 << 20, 8


def _head(wce, d, k):
    """the first k frames of a device frame array (without copying the rest)"""
    out = np.empty((k, NBLK, N), np.complex128)
    assert wce.load().wce_memcpy_dtoh(out.ctypes.data, d.addr, out.nbytes) == 0
    return out


@pytest.mark.parametrize("mode", [1, 0], ids=["textbook", "ref"])
def test_config4_batch_equals_its_shards(gpu_wce, golden, oracle, mode):
    import importlib
    wce = gpu_wce
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], mode, device=0)
    hlt, C, a, b = ctx.shared()
    hs = wce.DeviceArray.from_numpy(hlt) if mode == 1 else None
    tx, rx = wce.DeviceArray((TOTAL, NBLK, N)), wce.DeviceArray((TOTAL, NBLK, N))
    ctx.synth(tx, rx, None, TOTAL, seed=0x80211, h_shared=hs)
    H = wce.DeviceArray((TOTAL, N), zero=True)
    ctx.estimate(ctx.frames(tx, rx, TOTAL), wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0),
                 wce.PS_MMSE)
    wce.synchronize()
    _, bad = ctx.nonfinite_scan(H, TOTAL)
    assert bad == 0
    whole = H.numpy()
    del tx, rx
    for r in range(WORLD):
        first, count = multi.native_shard(wce, TOTAL, WORLD, r)
        stx, srx = wce.DeviceArray((count, NBLK, N)), wce.DeviceArray((count, NBLK, N))
        ctx.synth(stx, srx, None, count, first_frame=first, seed=0x80211, h_shared=hs)
        sH = wce.DeviceArray((count, N), zero=True)
        ctx.estimate(ctx.frames(stx, srx, count),
                     wce.Outputs(None, None, None, None, sH.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE)
        wce.synchronize()
        assert np.array_equal(sH.numpy(), whole[first:first + count]), r
        if r in (0, WORLD - 1):
            # a few frames of the shard against the long double oracle
            head = lambda d: _head(wce, d, 3)[:, 0]
            t0, r0 = head(stx), head(srx)
            mask = oracle.pilot_mask() if mode == 0 else np.ones(N, np.uint8)
            for j in range(3):
                want = oracle.mmse_unified(C, mask, a, b, t0[j], r0[j])
                assert normrel(sH.numpy()[j], want) < 1e-10
