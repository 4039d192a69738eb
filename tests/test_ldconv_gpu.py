"""The reference's long double complex format on the GPU (wce_ldconv.hip):
wce_ldc_to_complex must give exactly the bits of C's (double) cast and
wce_complex_to_ldc exactly C's (long double) cast (numpy's longdouble casts
on x86-64), over every branch: rounding ties, carry-out, overflow, fp64
subnormals, zeros, x87 denormals, Inf, NaN payloads, invalid encodings."""
import ctypes

import numpy as np
import pytest

import ldconv_ref as ref

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(np.finfo(np.longdouble).nmant != 63, reason="longdouble is not x87 extended here")]


def _c_cast_to_f64(ld: np.ndarray) -> np.ndarray:
    with np.errstate(all="ignore"):
        return ld.astype(np.complex128)


def test_ldc_to_complex_bit_exact(gpu_wce):
    wce = gpu_wce
    rng = np.random.default_rng(0xC0DE)
    m, se = ref.decode_cases(rng, 40000)
    ld = ref.raw_ld(m, se).view(np.clongdouble)           # 20000 complex, padding garbage
    n = ld.shape[0]
    src = wce.DeviceArray.from_numpy(ld)
    dst = wce.DeviceArray((n,), zero=True)
    wce.ldc_to_complex(src, dst, n)
    wce.synchronize()
    got = dst.numpy().view(np.uint64)
    want = _c_cast_to_f64(ld).view(np.uint64)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(i, hex(int(got[i])), hex(int(want[i]))) for i in bad[:5]]


def test_complex_to_ldc_bit_exact(gpu_wce):
    wce = gpu_wce
    rng = np.random.default_rng(0xC0DF)
    b = ref.encode_cases(rng, 40000)
    c = b.view(np.float64).view(np.complex128)
    n = c.shape[0]
    src = wce.DeviceArray.from_numpy(c)
    dst = wce.DeviceArray((n,), np.clongdouble)
    wce.complex_to_ldc(src, dst, n)
    wce.synchronize()
    got = dst.numpy().view(np.uint64).reshape(-1, 2)
    with np.errstate(all="ignore"):
        want = c.astype(np.clongdouble).view(np.uint64).reshape(-1, 2)
    assert np.array_equal(got[:, 0], want[:, 0])                                       # significands
    assert np.array_equal(got[:, 1] & np.uint64(0xFFFF), want[:, 1] & np.uint64(0xFFFF))   # sign + exponent
    assert not np.any(got[:, 1] >> np.uint64(16))                                     # padding zero


def test_round_trip_frames(gpu_wce, golden):
    """a batch of frames in the reference's format (the inputs.h frame and
    random ones) -> fp64 -> back: identity, and the fp64 values equal the C
    casts the compat shims apply one frame at a time"""
    wce = gpu_wce
    inp = golden["inputs"]
    rng = np.random.default_rng(7)
    B = 3000
    fr = (rng.standard_normal((B, 15 * 53)) + 1j * rng.standard_normal((B, 15 * 53))) * 8.8753
    ld = fr.astype(np.clongdouble)
    ld += (rng.standard_normal(ld.shape) * 2.0**-60).astype(np.longdouble) * ld   # bits below fp64
    ld[0, :53] = np.asarray(inp["tx_pre"], np.clongdouble)
    src = wce.DeviceArray.from_numpy(ld)
    mid = wce.DeviceArray(ld.shape, zero=True)
    back = wce.DeviceArray(ld.shape, np.clongdouble)
    wce.ldc_to_complex(src, mid, ld.size)
    wce.complex_to_ldc(mid, back, ld.size)
    wce.synchronize()
    f64 = mid.numpy()
    assert np.array_equal(f64.view(np.uint64), _c_cast_to_f64(ld).view(np.uint64))
    assert np.array_equal(back.numpy(), f64.astype(np.clongdouble))


def test_argument_errors(gpu_wce):
    wce = gpu_wce
    lib = wce.load()
    a = wce.DeviceArray((64,), np.clongdouble, zero=True)
    assert lib.wce_ldc_to_complex(a.ptr, ctypes.c_void_p(a.addr + 16), 4, None) != 0   # overlap
    assert lib.wce_ldc_to_complex(a.ptr, None, 4, None) != 0
    assert lib.wce_complex_to_ldc(a.ptr, a.ptr, -1, None) != 0
    assert lib.wce_ldc_to_complex(a.ptr, None, 0, None) == 0                          # empty: no-op
    b = wce.DeviceArray((64,), zero=True)
    assert lib.wce_ldc_to_complex(ctypes.c_void_p(a.addr + 8), b.ptr, 4, None) != 0   # misaligned
