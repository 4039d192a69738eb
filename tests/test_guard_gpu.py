"""Non-finite guard (wce_nonfinite_scan, SURVEY 8(b)'s optional per-frame
non-finite bitmap) on the GPU, against numpy's isfinite on the same arrays.
The reference passes NaN/Inf through silently (main.c PS_MMSE returns NaN x 53;
a zero pilot makes PS_* divide by zero, main.c:82-84)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expect(H, n):
    bad = ~np.isfinite(H[:n, :53].view(np.float64 if H.dtype == np.complex128 else np.float32)).all(axis=1)
    bits = np.zeros((n + 31) // 32, np.uint32)
    for f in np.flatnonzero(bad):
        bits[f >> 5] |= np.uint32(1) << np.uint32(f & 31)
    return bits, int(bad.sum())


@pytest.mark.parametrize("n,stride,f32", [(1000, 53, False), (1000, 64, False), (64, 53, True), (1, 53, False),
                                          (70001, 53, False)])
def test_scan_bitmap_matches_numpy(gpu_wce, n, stride, f32):
    wce = gpu_wce
    rng = np.random.default_rng(n + stride)
    dt = np.complex64 if f32 else np.complex128
    H = (rng.standard_normal((n, stride)) + 1j * rng.standard_normal((n, stride))).astype(dt)
    # padding columns k >= 53 are not part of a frame: poison them, they must be ignored
    if stride > 53:
        H[:, 53:] = np.nan
    inj = [(0, 0, "re", np.nan), (n - 1, 52, "im", np.inf), (31 % n, 26, "re", -np.inf),
           (32 % n, 5, "im", np.nan), (32 % n, 47, "re", np.inf)]   # two bad entries in one frame
    inj += [(int(f), int(k), "re", np.nan) for f, k in zip(rng.integers(0, n, 20), rng.integers(0, 53, 20))]
    for f, k, part, v in inj:
        if part == "re":
            H[f, k] = v + 1j * H[f, k].imag
        else:
            H[f, k] = H[f, k].real + 1j * v
    d = wce.DeviceArray.from_numpy(H)
    ctx = wce.Context(empty=True, device=0)
    bits, count = ctx.nonfinite_scan(d, n, stride=stride, f32=f32)
    want_bits, want_count = _expect(H, n)
    assert np.array_equal(bits, want_bits)
    assert count == want_count


def test_scan_all_finite_and_reuse(gpu_wce):
    """Clean input: empty bitmap, count 0 -- also after a dirty scan into the
    same caller-owned buffers (the scan zeroes them itself)."""
    wce = gpu_wce
    n = 4096
    H = np.ones((n, 53), np.complex128)
    dirty = H.copy()
    dirty[::7, 3] = np.nan
    ctx = wce.Context(empty=True, device=0)
    bm = wce.DeviceArray(((n + 31) // 32,), dtype=np.uint32)
    cnt = wce.DeviceArray((1,), dtype=np.uint64)
    ctx.nonfinite_scan(wce.DeviceArray.from_numpy(dirty), n, bitmap=bm, n_bad=cnt)
    wce.synchronize()
    assert int(cnt.numpy()[0]) == len(range(0, n, 7))
    ctx.nonfinite_scan(wce.DeviceArray.from_numpy(H), n, bitmap=bm, n_bad=cnt)
    wce.synchronize()
    assert not bm.numpy().any() and int(cnt.numpy()[0]) == 0


def test_zero_pilot_frame_is_flagged(gpu_wce, golden):
    """A frame whose pilot tx[P0] is 0 makes PS_Linear divide by zero (as
    main.c:82-84 would); the guard flags exactly that frame."""
    wce = gpu_wce
    inp = golden["inputs"]
    B = 40
    tx = np.repeat(inp["tx_symb"][None], B, axis=0)
    rx = np.repeat(inp["rx_symb"][None], B, axis=0)
    tx[17, 0, 5] = 0
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_REF, device=0)
    out = ctx.estimate_host(tx, rx, mask=wce.PS_LINEAR)["ps_linear"]
    assert not np.isfinite(out[17].view(np.float64)).all()
    bits, count = ctx.nonfinite_scan(wce.DeviceArray.from_numpy(out), B)
    assert count == 1 and bits[0] == 1 << 17 and bits[1] == 0


def test_scan_argument_errors(gpu_wce):
    wce = gpu_wce
    ctx = wce.Context(empty=True, device=0)
    d = wce.DeviceArray((4, 53))
    lib = wce.load()
    bm = wce.DeviceArray((1,), dtype=np.uint32)
    assert lib.wce_nonfinite_scan(ctx.handle, d.addr, 52, 4, 0, bm.addr, None, None) == -1       # stride < 53
    assert lib.wce_nonfinite_scan(ctx.handle, d.addr, 53, 4, 2, bm.addr, None, None) != 0     # unknown flag
    assert lib.wce_nonfinite_scan(ctx.handle, None, 53, 4, 0, bm.addr, None, None) != 0
    assert lib.wce_nonfinite_scan(ctx.handle, d.addr, 53, 0, 0, None, None, None) == 0        # empty batch
