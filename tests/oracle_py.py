"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline, never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")
N, NBLK = 53, 15
PILOTS = (5, 19, 33, 47)
LD = np.clongdouble

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            subprocess.check_call(["make", "-C", ORACLE_DIR, "liboracle.so"], stdout=subprocess.DEVNULL)
        _lib = ctypes.CDLL(ORACLE_LIB)
        _lib.orc_bench_mmse_f64.restype = ctypes.c_double
        _lib.orc_bench_mmse_f64.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                                            ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long,
                                            ctypes.c_long, ctypes.c_void_p]
        _lib.orc_bench_ls_f64.restype = ctypes.c_double
        _lib.orc_bench_ls_f64.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_void_p,
                                          ctypes.c_void_p]
        _lib.orc_mmse_ref_repaired.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_double] + [ctypes.c_void_p] * 3
        _lib.orc_mmse_unified.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longdouble,
                                          ctypes.c_longdouble, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_mmse_textbook_closed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_longdouble, ctypes.c_void_p]
        _lib.orc_inverse_cofactor.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ld(a):
    return np.ascontiguousarray(np.asarray(a, dtype=LD))


def from_split(s):
    """(hi, lo) float64 golden encoding -> clongdouble."""
    s = np.asarray(s)
    re = s[..., 0].astype(np.longdouble) + s[..., 2].astype(np.longdouble)
    im = s[..., 1].astype(np.longdouble) + s[..., 3].astype(np.longdouble)
    return (re + 1j * im).astype(LD)


def fmatrix():
    F = np.zeros((N, N), LD)
    load().orc_fmatrix(_p(F))
    return F


def inverse_cofactor(A):
    A = _ld(A)
    n = A.shape[0]
    Y = np.zeros((n, n), LD)
    load().orc_inverse_cofactor(_p(A), n, _p(Y))
    return Y


def _est(name, a, b):
    H = np.zeros(N, LD)
    getattr(load(), name)(_p(_ld(a)), _p(_ld(b)), _p(H))
    return H


def lt_ls(tx_pre, rx_pre):
    return _est("orc_lt_ls", tx_pre, rx_pre)


def ps_linear(tx, rx):
    return _est("orc_ps_linear", tx, rx)


def ps_cubic(tx, rx):
    return _est("orc_ps_cubic", tx, rx)


def ps_sinc(tx, rx):
    return _est("orc_ps_sinc", tx, rx)


def mmse_ref_repaired(tx, rx, F, ow2, H_LS, invF):
    H = np.zeros(N, LD)
    load().orc_mmse_ref_repaired(_p(_ld(tx)), _p(_ld(rx)), _p(_ld(F)), float(ow2), _p(_ld(H_LS)),
                                 _p(_ld(invF)) if invF is not None else None, _p(H))
    return H


def mmse_ref_cmatrix(F, invF, H_LS):
    C = np.zeros((N, N), LD)
    load().orc_mmse_ref_cmatrix(_p(_ld(F)), _p(_ld(invF)), _p(_ld(H_LS)), _p(C))
    return C


def mmse_textbook_cmatrix(F, H_LS):
    C = np.zeros((N, N), LD)
    load().orc_mmse_textbook_cmatrix(_p(_ld(F)), _p(_ld(H_LS)), _p(C))
    return C


def mmse_unified(C, mask, a, b, tx, rx):
    H = np.zeros(N, LD)
    m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8))
    load().orc_mmse_unified(_p(_ld(C)), _p(m), np.longdouble(a), np.longdouble(b), _p(_ld(tx)), _p(_ld(rx)), _p(H))
    return H


def mmse_textbook_closed(c, tx, rx, s):
    H = np.zeros(N, LD)
    load().orc_mmse_textbook_closed(_p(_ld(c)), _p(_ld(tx)), _p(_ld(rx)), np.longdouble(s), _p(H))
    return H


def equalize(rx_blocks, H_LT, H_PS):
    eq = np.zeros((NBLK, N), LD)
    load().orc_equalize(_p(_ld(rx_blocks)), _p(_ld(H_LT)), _p(_ld(H_PS)), _p(eq))
    return eq


def matlab(name, tx_blocks, rx_blocks):
    H = np.zeros(N, LD)
    getattr(load(), "orc_matlab_" + name)(_p(_ld(tx_blocks)), _p(_ld(rx_blocks)), _p(H))
    return H


def matlab_lt_ls(tx_pre, rx_pre):
    return _est("orc_matlab_lt_ls", tx_pre, rx_pre)


def front_blocks(samples, n_blocks):
    """time-domain packet -> [n_blocks][53] useful subcarriers (WiFi_blocks_extraction.m)."""
    out = np.zeros((n_blocks, N), LD)
    load().orc_front_blocks(_p(_ld(samples)), ctypes.c_int(n_blocks), _p(out))
    return out


def front_preamble(lptot):
    """long training field -> (preamble FFT [53], ow2) (WiFi_RX.m:24-30)."""
    x = _ld(lptot)
    out = np.zeros(N, LD)
    s = np.zeros(1, np.longdouble)
    load().orc_front_preamble(_p(x), ctypes.c_long(x.shape[0]), _p(out), _p(s))
    return out, s[0]


def pilot_mask():
    m = np.zeros(N, np.uint8)
    m[list(PILOTS)] = 1
    return m


def bench_mmse_f64(C, mask, a, b, tx, rx, frame_stride, nthreads):
    """fp64 OpenMP CPU port of the unified MMSE; tx/rx complex128 flat, returns (H, seconds)."""
    n = (tx.size - N) // frame_stride + 1
    H = np.zeros((n, N), np.complex128)
    Cc = np.ascontiguousarray(C, dtype=np.complex128)
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    t = load().orc_bench_mmse_f64(nthreads, _p(Cc), _p(m), a, b, _p(tx), _p(rx), n, frame_stride, _p(H))
    return H, t


def bench_ls_f64(tx_pre, rx_pre, tx, rx, frame_stride, nthreads):
    n = rx_pre.shape[0]
    H_LT = np.zeros((n, N), np.complex128)
    H_LIN = np.zeros((n, N), np.complex128)
    t = load().orc_bench_ls_f64(nthreads, _p(np.ascontiguousarray(tx_pre, np.complex128)), _p(rx_pre), _p(tx),
                                _p(rx), n, frame_stride, _p(H_LT), _p(H_LIN))
    return H_LT, H_LIN, t


def normrel(x, ref):
    """max_k |x_k - ref_k| / max_k |ref_k| (norm-relative per frame)."""
    x = np.asarray(x, dtype=np.clongdouble)
    ref = np.asarray(ref, dtype=np.clongdouble)
    num = np.max(np.abs(x - ref), axis=-1)
    den = np.max(np.abs(ref), axis=-1)
    return np.asarray(num / den, dtype=np.float64)
