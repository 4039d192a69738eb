"""One context, several streams (include/wce.h "Threading"): the calls that
need scratch -- WCE_MMSE_FRAME_COV and MATLAB-semantics PS_MMSE -- keep it
per stream, so batches enqueued on different streams at once, or issued from
different host threads, give exactly the results of the same calls run one
after another.  Plans own their scratch and may replay beside direct calls."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, NBLK = 53, 15


def _batch(wce, ctx, n, seed):
    tx, rx, pre = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, N))
    ctx.synth(tx, rx, pre, n, seed=seed)
    H = wce.DeviceArray((n, N), zero=True)
    return tx, rx, pre, H


CASES = [("frame_cov", lambda wce: wce.PS_MMSE | wce.FRAME_COV, 0),
         ("matlab", lambda wce: wce.PS_MMSE, 1),
         ("matlab_frame_cov", lambda wce: wce.PS_MMSE | wce.FRAME_COV, 1),
         ("matlab_cov_lowrank", lambda wce: wce.PS_MMSE, 1)]   # mmse_lr_kernel split + block mean


def _call(wce, ctx, b, n, mask, sem, stream):
    tx, rx, pre, H = b
    fr = ctx.frames(tx, rx, n, rx_pre=pre, semantics=sem)
    o = wce.Outputs(None, None, None, None, H.addr, None, N, 0, 0, 0, 0)
    ctx.estimate(fr, o, mask, stream)


@pytest.mark.parametrize("name,maskf,sem", CASES, ids=[c[0] for c in CASES])
def test_streams_do_not_share_scratch(gpu_wce, golden, name, maskf, sem):
    wce = gpu_wce
    inp = golden["inputs"]
    if name == "matlab_cov_lowrank":
        p = np.zeros(N)
        p[:6] = np.exp(-0.5 * np.arange(6))
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], device=0,
                          Rhh=np.diag(p / p.sum()).astype(np.complex128) * 1.1e-4)
    else:
        ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    mask = maskf(wce)
    sizes = [8192, 6000, 8192, 3001]               # different sizes: a shared buffer's layout would differ too
    batches = [_batch(wce, ctx, n, 100 + i) for i, n in enumerate(sizes)]
    # serial reference, one stream
    for b, n in zip(batches, sizes):
        _call(wce, ctx, b, n, mask, sem, None)
    wce.synchronize()
    ref = [b[3].numpy() for b in batches]
    # all four at once, one stream each, no sync between them
    streams = [wce.Stream() for _ in sizes]
    for rep in range(3):
        for b in batches:
            assert wce.load().wce_memset(b[3].addr, 0, b[3].nbytes) == 0
        wce.synchronize()
        for b, n, s in zip(batches, sizes, streams):
            _call(wce, ctx, b, n, mask, sem, s.handle)
        for s in streams:
            s.synchronize()
        for b, r in zip(batches, ref):
            assert np.array_equal(b[3].numpy(), r), (name, rep)


def test_host_threads_share_one_context(gpu_wce, golden):
    """Four host threads, one stream each, 6 calls per thread on one ctx
    (FRAME_COV, growing batch sizes so the scratch is re-sized under load)."""
    wce = gpu_wce
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    mask = wce.PS_MMSE | wce.FRAME_COV
    sizes = [1024, 2048, 4096, 4096, 8192, 16384]
    big = max(sizes)
    batches = [_batch(wce, ctx, big, 200 + t) for t in range(4)]
    want = {}
    for t, b in enumerate(batches):
        for n in sizes:
            _call(wce, ctx, b, n, mask, 0, None)
            wce.synchronize()
            want[t, n] = b[3].numpy()[:n].copy()
    got, errors = {}, []

    def worker(t):
        try:
            s = wce.Stream()
            b = batches[t]
            out = []
            for n in sizes:
                _call(wce, ctx, b, n, mask, 0, s.handle)
                s.synchronize()
                out.append((n, b[3].numpy()[:n].copy()))
            got[t] = out
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=60)
    assert not errors, errors
    for t in range(4):
        for n, h in got[t]:
            assert np.array_equal(h, want[t, n]), (t, n)


def test_plan_replays_beside_direct_calls(gpu_wce, golden):
    wce = gpu_wce
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    mask = wce.PS_MMSE | wce.FRAME_COV
    n = 8192
    a, b = _batch(wce, ctx, n, 300), _batch(wce, ctx, n, 301)
    for x in (a, b):
        _call(wce, ctx, x, n, mask, 1, None)
    wce.synchronize()
    ra, rb = a[3].numpy(), b[3].numpy()
    fr = ctx.frames(a[0], a[1], n, rx_pre=a[2], semantics=1)
    plan = ctx.plan(fr, wce.Outputs(None, None, None, None, a[3].addr, None, N, 0, 0, 0, 0), mask)
    s1, s2 = wce.Stream(), wce.Stream()
    for _ in range(3):
        plan.launch(s1.handle)
        _call(wce, ctx, b, n, mask, 1, s2.handle)
    s1.synchronize()
    s2.synchronize()
    assert np.array_equal(a[3].numpy(), ra) and np.array_equal(b[3].numpy(), rb)
    plan.close()


def test_reserve_stream(gpu_wce, golden):
    wce = gpu_wce
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    s = wce.Stream()
    lib = wce.load()
    assert lib.wce_ctx_reserve_stream(ctx.handle, 4096, s.handle) == 0
    assert lib.wce_ctx_reserve_stream(ctx.handle, -1, s.handle) != 0
    assert lib.wce_ctx_reserve(ctx.handle, 2048) == 0
    b = _batch(wce, ctx, 4096, 7)
    _call(wce, ctx, b, 4096, wce.PS_MMSE | wce.FRAME_COV, 0, s.handle)
    s.synchronize()
    assert np.isfinite(b[3].numpy().view(np.float64)).all()


def test_pinned_host_pipeline(gpu_wce, golden):
    """Frames in pinned host memory, chunks round-robin over 2 streams
    (wce_memcpy_htod_async -> estimate -> wce_memcpy_dtoh_async): the host
    result equals the device-resident call bit for bit."""
    wce = gpu_wce
    inp = golden["inputs"]
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], wce.MMSE_TEXTBOOK, device=0)
    n, c = 4096, 1024
    tx, rx = wce.DeviceArray((n, NBLK, N)), wce.DeviceArray((n, NBLK, N))
    ctx.synth(tx, rx, None, n, seed=3)
    Hd = wce.DeviceArray((n, N), zero=True)
    ctx.estimate(ctx.frames(tx, rx, n), wce.Outputs(None, None, None, None, Hd.addr, None, N, 0, 0, 0, 0),
                 wce.PS_MMSE)
    wce.synchronize()
    txh, rxh, hh = wce.PinnedArray((n, N)), wce.PinnedArray((n, N)), wce.PinnedArray((n, N))
    txh.array[:] = tx.numpy()[:, 0]
    rxh.array[:] = rx.numpy()[:, 0]
    hh.array[:] = np.nan
    lib = wce.load()
    streams = [wce.Stream(), wce.Stream()]
    bufs = [[wce.DeviceArray((c, N)) for _ in range(3)] for _ in streams]
    nb = c * N * 16
    for i in range(n // c):
        s, (dt, dr, dh) = streams[i % 2].handle, bufs[i % 2]
        assert lib.wce_memcpy_htod_async(dt.addr, txh.addr + i * nb, nb, s) == 0
        assert lib.wce_memcpy_htod_async(dr.addr, rxh.addr + i * nb, nb, s) == 0
        ctx.estimate(ctx.frames(dt, dr, c, frame_stride=N, block_stride=N),
                     wce.Outputs(None, None, None, None, dh.addr, None, N, 0, 0, 0, 0), wce.PS_MMSE, s)
        assert lib.wce_memcpy_dtoh_async(hh.addr + i * nb, dh.addr, nb, s) == 0
    for st in streams:
        st.synchronize()
    assert np.array_equal(hh.array, Hd.numpy())
