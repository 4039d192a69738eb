"""The flat-index kernels split a batch into launches of 2^26 frames (so that
53 * frames < 2^32).  wce_debug_set_flat_chunk lowers that to a multiple of
32 so these tests reach the multi-launch path (frame offset f_begin > 0,
a ragged last launch) at small sizes: LT_LS + PS_Linear (configs[1]), REF
PS_MMSE, and the non-finite scan, each bit-identical to one launch, with
every output row written (outputs are pre-filled with NaN)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, NBLK = 53, 15


@pytest.fixture
def chunked(gpu_wce):
    lib = gpu_wce.load()
    assert lib.wce_debug_set_flat_chunk(1000) != 0        # not a multiple of 32
    assert lib.wce_debug_set_flat_chunk(16) != 0
    yield lambda c: lib.wce_debug_set_flat_chunk(c)
    assert lib.wce_debug_set_flat_chunk(0) == 0


def _nan_fill(wce, d):
    assert wce.load().wce_memset(d.addr, 0xFF, d.nbytes) == 0   # all-ones doubles are NaN


def _run(wce, ctx, n, mask, pre):
    tx, rx, rxp = pre
    outs = [wce.DeviceArray((n, N)) for _ in range(5)]
    for o in outs:
        _nan_fill(wce, o)
    o = wce.Outputs(*(x.addr for x in outs), None, N, 0, 0, 0, 0)
    ctx.estimate(ctx.frames(tx, rx, n, rx_pre=rxp), o, mask)
    wce.synchronize()
    return outs


@pytest.mark.parametrize("mode,mask,per_frame_pre,ref_form", [(0, 0b00011, True, 0), (0, 0b10000, False, 1),
                                                             (0, 0b10000, False, 3)],
                         ids=["ls_flat_config2", "ref_flat_mmse", "ref_elem_mmse"])
def test_multi_launch_bit_identical(gpu_wce, golden, chunked, mode, mask, per_frame_pre, ref_form):
    wce = gpu_wce
    assert wce.load().wce_debug_set_variant(0, ref_form) == 0   # REF read-out form (which 0)
    try:
        _multi_launch(wce, golden, chunked, mode, mask, per_frame_pre)
    finally:
        assert wce.load().wce_debug_set_variant(0, 0) == 0


def _multi_launch(wce, golden, chunked, mode, mask, per_frame_pre):
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], mode, device=0)
    n = 2500                                                   # 1024 + 1024 + 452 at chunk 1024
    tx, rx, rxp = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx.synth(tx, rx, rxp, n, seed=11)
    pre = (tx, rx, rxp if per_frame_pre else None)
    names = ["lt_ls", "ps_linear", "ps_cubic", "ps_sinc", "ps_mmse"]
    assert chunked(0) == 0
    one = [o.numpy() for o in _run(wce, ctx, n, mask, pre)]
    for c in (1024, 32, 2496):
        assert chunked(c) == 0
        outs = _run(wce, ctx, n, mask, pre)
        for i, name in enumerate(names):
            if mask & (1 << i):
                got = outs[i].numpy()
                assert np.isfinite(got.view(np.float64)).all(), (c, name)   # every row written
                assert np.array_equal(got, one[i]), (c, name)
                _, bad = ctx.nonfinite_scan(outs[i], n)
                assert bad == 0


def test_scan_multi_launch(gpu_wce, chunked):
    wce = gpu_wce
    n = 2500
    H = np.ones((n, N), np.complex128)
    bad = [0, 31, 1023, 1024, 2047, 2048, 2049, 2499]
    for f in bad:
        H[f, f % N] = np.nan
    d = wce.DeviceArray.from_numpy(H)
    ctx = wce.Context(empty=True, device=0)
    assert chunked(1024) == 0
    bits, count = ctx.nonfinite_scan(d, n)
    want = np.zeros((n + 31) // 32, np.uint32)
    for f in bad:
        want[f >> 5] |= np.uint32(1 << (f & 31))
    assert count == len(bad) and np.array_equal(bits, want)
