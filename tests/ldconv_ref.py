"""Test helpers for the reference's `long double complex` data format
(wce_ldconv.hip): bit patterns that exercise every branch of the x87 <-> fp64
conversions, and a pure-Python restatement of the device decoder, pinned on
the CPU against numpy's longdouble casts (the C casts of x86-64: numpy's
longdouble is the x87 80-bit format in a 16-byte slot)."""
import numpy as np

INDEFINITE = 0xFFF8000000000000


def x87_to_f64_bits(m: int, se: int) -> int:
    """Restatement of wce_ldconv.hip x87_to_f64_bits (test oracle only)."""
    sign = ((se >> 15) & 1) << 63
    e = se & 0x7FFF
    jbit = (m >> 63) & 1
    if e == 0x7FFF:
        if not jbit:
            return INDEFINITE
        if m & 0x7FFFFFFFFFFFFFFF == 0:
            return sign | 0x7FF0000000000000
        return sign | 0x7FF0000000000000 | (1 << 51) | ((m >> 11) & 0x000FFFFFFFFFFFFF)
    if e == 0:
        return sign
    if not jbit:
        return INDEFINITE
    E = e - 16383
    if E > 1023:
        return sign | 0x7FF0000000000000
    if E >= -1022:
        q, rem = m >> 11, m & 0x7FF
        if rem > 0x400 or (rem == 0x400 and q & 1):
            q += 1
        eb = E + 1023
        if q >> 53:
            q >>= 1
            eb += 1
            if eb >= 0x7FF:
                return sign | 0x7FF0000000000000
        return sign | (eb << 52) | (q & 0x000FFFFFFFFFFFFF)
    s = -1011 - E
    if s > 64:
        return sign
    q = m >> s
    half = 1 << (s - 1)
    rem = m & ((1 << s) - 1)
    return sign | (q + 1 if rem > half or (rem == half and q & 1) else q)


def f64_bits_to_x87(b: int):
    """Restatement of wce_ldconv.hip f64_bits_to_x87: (significand, sign/exponent)."""
    sign = (b >> 63) << 15
    e = (b >> 52) & 0x7FF
    f = b & 0x000FFFFFFFFFFFFF
    if e == 0x7FF:
        return ((1 << 63) if f == 0 else ((1 << 63) | (1 << 62) | (f << 11))), sign | 0x7FFF
    if e == 0:
        if f == 0:
            return 0, sign
        lz = 64 - f.bit_length()
        return f << lz, sign | (-1011 - lz + 16383)
    return (1 << 63) | (f << 11), sign | (e - 1023 + 16383)


def raw_ld(m: np.ndarray, se: np.ndarray) -> np.ndarray:
    """x87 values from significands and sign/exponent words, as a longdouble
    array (padding bytes set to garbage, as C leaves them)."""
    n = len(m)
    raw = np.zeros((n, 2), np.uint64)
    raw[:, 0] = m
    raw[:, 1] = (se.astype(np.uint64) & np.uint64(0xFFFF)) | np.uint64(0xA5A5_5A5A_0000_0000)
    return raw.view(np.longdouble).reshape(n)


def decode_cases(rng: np.random.Generator, n: int):
    """(m, se) pairs covering: normals across the whole fp64 range and past
    it, the rounding boundaries (ties at the 11 dropped bits, carry-out),
    fp64 subnormals (ties at every shift), zeros, x87 denormals, Inf, NaN
    payloads, unnormals, pseudo-Inf/NaN."""
    m = rng.integers(0, 2**63, n, dtype=np.uint64) | np.uint64(1 << 63)
    e = rng.integers(16383 - 1100, 16383 + 1030, n)
    sign = rng.integers(0, 2, n)
    k = n // 8
    # exact ties and near-ties of the 11 dropped bits
    m[:k] = (m[:k] & ~np.uint64(0x7FF)) | np.uint64(0x400)
    m[k:2 * k] = (m[k:2 * k] & ~np.uint64(0x7FF)) | rng.integers(0x3FF, 0x402, k, dtype=np.uint64)
    # carry out of the 53-bit significand (all ones, then round up)
    m[2 * k:2 * k + 16] = np.uint64(0xFFFFFFFFFFFFFC00)
    e[2 * k:2 * k + 8] = 16383 + 1023            # -> overflow to Inf by rounding
    # fp64 subnormal range with ties at the shifted position
    sub = slice(3 * k, 4 * k)
    e[sub] = rng.integers(16383 - 1090, 16383 - 1022, k)
    shift = (-1011 - (e[sub] - 16383)).astype(np.int64)
    for i, s in zip(range(sub.start, sub.stop), shift):
        if 12 <= s <= 63 and i % 2 == 0:
            mm = int(m[i]) & ~((1 << int(s)) - 1) | (1 << (int(s) - 1))
            m[i] = np.uint64(mm | (1 << 63))
    # zeros, x87 denormals, exponent extremes
    e[4 * k:4 * k + 8] = 0
    m[4 * k:4 * k + 4] = 0
    e[4 * k + 8:4 * k + 12] = 0x7FFE
    e[4 * k + 12:4 * k + 16] = 1
    # Inf and NaNs (quiet and signalling payloads)
    e[5 * k:5 * k + 32] = 0x7FFF
    m[5 * k:5 * k + 4] = np.uint64(1 << 63)
    m[5 * k + 4:5 * k + 16] = np.uint64(1 << 63) | rng.integers(1, 2**62, 12, dtype=np.uint64)
    m[5 * k + 16:5 * k + 28] = np.uint64(3 << 62) | rng.integers(0, 2**62, 12, dtype=np.uint64)
    # invalid encodings: pseudo-Inf/NaN (integer bit clear, e = 0x7fff), unnormals
    m[5 * k + 28:5 * k + 32] = rng.integers(0, 2**63, 4, dtype=np.uint64)
    m[6 * k:6 * k + 16] &= np.uint64((1 << 63) - 1)
    se = (sign << 15 | e).astype(np.uint64)
    return m, se


def encode_cases(rng: np.random.Generator, n: int) -> np.ndarray:
    """fp64 bit patterns: normals, subnormals, zeros, Inf, quiet and
    signalling NaNs."""
    b = rng.integers(0, 2**64, n, dtype=np.uint64)
    k = n // 8
    b[:k] &= np.uint64(0x800FFFFFFFFFFFFF)                     # subnormals (and zeros)
    b[k:k + 4] = np.array([0, 1 << 63, 0x7FF0000000000000, 0xFFF0000000000000], np.uint64)
    b[k + 4:k + 8] = np.array([0x7FF8000000000000, 0x7FF0000000000001, 0xFFF4000000000000, 1], np.uint64)
    return b
