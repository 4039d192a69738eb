"""The reference's long double complex format (wce_ldconv.hip), CPU side:
the Python restatement of the device decoder/encoder (tests/ldconv_ref.py)
against numpy's longdouble casts, which are the C casts of x86-64 (x87 80-bit
in a 16-byte slot, as main.c's arrays).  The GPU kernels are checked against
the same casts in test_ldconv_gpu.py."""
import numpy as np
import pytest

import ldconv_ref as ref

pytestmark = pytest.mark.skipif(np.finfo(np.longdouble).nmant != 63, reason="longdouble is not x87 extended here")


def test_decoder_restatement_matches_c_cast():
    rng = np.random.default_rng(0x87)
    m, se = ref.decode_cases(rng, 20000)
    ld = ref.raw_ld(m, se)
    with np.errstate(all="ignore"):
        want = ld.astype(np.float64).view(np.uint64)
    got = np.array([ref.x87_to_f64_bits(int(a), int(b)) for a, b in zip(m, se)], np.uint64)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(hex(int(m[i])), hex(int(se[i])), hex(int(got[i])), hex(int(want[i]))) for i in bad[:5]]


def test_encoder_restatement_matches_c_cast():
    rng = np.random.default_rng(0x88)
    b = ref.encode_cases(rng, 20000)
    with np.errstate(all="ignore"):
        raw = b.view(np.float64).astype(np.longdouble).view(np.uint64).reshape(-1, 2)
    for i, x in enumerate(b):
        mm, se = ref.f64_bits_to_x87(int(x))
        assert int(raw[i, 0]) == mm and int(raw[i, 1]) & 0xFFFF == se, (i, hex(int(x)))


def test_case_coverage():
    """the generated cases reach every branch of the decoder"""
    rng = np.random.default_rng(0x87)
    m, se = ref.decode_cases(rng, 20000)
    e = se & 0x7FFF
    E = e.astype(np.int64) - 16383
    jb = (m >> np.uint64(63)) == 1
    assert np.any(E > 1023) and np.any((E >= -1022) & (E <= 1023)) and np.any((E < -1022) & (E > -1076))
    assert np.any(E <= -1076) and np.any(e == 0) and np.any((e == 0x7FFF) & jb) and np.any((e == 0x7FFF) & ~jb)
    assert np.any(~jb & (e > 0) & (e < 0x7FFF))
    assert np.any((m & np.uint64(0x7FF)) == np.uint64(0x400))
