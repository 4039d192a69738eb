"""Python host binding of libwce.so (the C ABI in include/wce.h).

Two layers, mirroring the C side:

* the reference's five entry points (main.c:4-8) with the same names and
  argument meaning -- one frame, host arrays, results written into H_EST --
  implemented by the compat shims in libwce.so (include/wce_compat.h);
* the batched engine: :class:`Context` (shared state on one device),
  :class:`DeviceArray` (HBM buffers), :meth:`Context.estimate` over B frames.

There is no CPU fallback: every compute call goes through the gfx950
kernels and raises :class:`WceError` if the library or the device is absent.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_double, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

import numpy as np

NSC = 53          # SAMPUTIL   (utils.h:13)
NBLK = 15         # OFDMBLK    (utils.h:15)
DC = 26           # main.c:74
PILOTS = (5, 19, 33, 47)   # utils.h:16-19

LT_LS = 1 << 0
PS_LINEAR = 1 << 1
PS_CUBIC = 1 << 2
PS_SINC = 1 << 3
PS_MMSE = 1 << 4
EQUALIZE = 1 << 5
LS_ALL = 0xF
ALL = 0x3F
OUT_LS_F32 = 1         # wce_outputs.flags: LS family + eq stored as complex float
FRAME_COV = 1 << 6   # WCE_MMSE_FRAME_COV: PS_MMSE covariance from each frame's own preamble

MMSE_REF = 0
MMSE_TEXTBOOK = 1
MMSE_COV = 2       # TEXTBOOK with a caller-supplied channel covariance Rhh
FFT_SIZE = 64            # front end: 64-point DFT per OFDM block (WiFi_RX.m:10)
SAMPLES_PER_BLOCK = 80   # 64 + 16-sample cyclic prefix (WiFi_RX.m:12)
SEM_C = 0          # main.c semantics
SEM_MATLAB = 1     # WiFi_channel_estimation_*.m semantics

STATUS = {0: "ok", -1: "invalid argument", -2: "HIP error", -3: "out of memory",
          -4: "context state not ready", -5: "no gfx950 device"}

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libwce.so")


class WceError(RuntimeError):
    def __init__(self, code, where=""):
        msg = STATUS.get(code, f"error {code}")
        detail = ""
        if _lib is not None:
            try:
                detail = _lib.wce_last_error().decode()
            except Exception:  # pragma: no cover
                detail = ""
        super().__init__(f"{where}: {msg}" + (f" ({detail})" if detail else ""))
        self.code = code


class Complex(ctypes.Structure):
    _fields_ = [("re", c_double), ("im", c_double)]


class Frames(ctypes.Structure):
    """struct wce_frames (include/wce.h)."""
    _fields_ = [("tx", c_void_p), ("rx", c_void_p), ("rx_pre", c_void_p), ("tx_pre", c_void_p),
                ("frame_stride", c_int64), ("block_stride", c_int64), ("pre_stride", c_int64),
                ("n_frames", c_int64), ("block", c_int32), ("semantics", c_int32)]


class Outputs(ctypes.Structure):
    """struct wce_outputs (include/wce.h)."""
    _fields_ = [("lt_ls", c_void_p), ("ps_linear", c_void_p), ("ps_cubic", c_void_p), ("ps_sinc", c_void_p),
                ("ps_mmse", c_void_p), ("eq", c_void_p), ("out_stride", c_int64),
                ("eq_frame_stride", c_int64), ("eq_block_stride", c_int64), ("eq_source", c_uint32),
                ("flags", c_uint32)]


_lib = None

# (name, argtypes) for every symbol include/wce.h and include/wce_compat.h declare
ABI = {
    "wce_ctx_create": [POINTER(c_void_p), c_int, c_void_p, c_void_p, c_double, c_int],
    "wce_ctx_create_empty": [POINTER(c_void_p), c_int],
    "wce_ctx_destroy": [c_void_p],
    "wce_ctx_reserve": [c_void_p, c_int64],
    "wce_ctx_reserve_stream": [c_void_p, c_int64, c_void_p],
    "wce_plan_create": [POINTER(c_void_p), c_void_p, c_void_p, c_void_p, c_uint32],
    "wce_plan_launch": [c_void_p, c_void_p],
    "wce_plan_destroy": [c_void_p],
    "wce_ctx_create_cov": [POINTER(c_void_p), c_int, c_void_p, c_void_p, c_void_p, c_double],
    "wce_state_build_cov": [c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_double],
    "wce_debug_set_fusion": [c_void_p, c_int],
    "wce_debug_set_border_dot": [c_void_p, c_int],
    "wce_debug_set_flat_chunk": [ctypes.c_int64],
    "wce_debug_set_variant": [c_int, c_int],
    "wce_debug_set_cov_path": [c_void_p, c_int],
    "wce_debug_lr_kernel": [c_void_p, c_int64],
    "wce_debug_cov_factor": [c_void_p, c_size_t, c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_double),
                             POINTER(c_double)],
    "wce_ctx_cov_info": [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_double), POINTER(c_double)],
    "wce_ctx_set_modulus": [c_void_p, c_void_p],
    "wce_state_set_modulus": [c_void_p, c_size_t, c_void_p, c_void_p],
    "wce_debug_set_cm": [c_void_p, c_int],
    "wce_debug_compat_state_builds": [],
    "wce_ctx_state": [c_void_p, POINTER(c_void_p), POINTER(c_size_t)],
    "wce_ctx_mark_ready": [c_void_p],
    "wce_state_size": [],
    "wce_state_build": [c_void_p, c_size_t, c_void_p, c_void_p, c_double, c_int],
    "wce_ctx_load_state": [c_void_p, c_void_p, c_size_t],
    "wce_state_validate": [c_void_p, c_size_t, POINTER(c_int)],
    "wce_ctx_get_shared": [c_void_p, c_void_p, c_void_p, POINTER(c_double), POINTER(c_double)],
    "wce_estimate": [c_void_p, POINTER(Frames), POINTER(Outputs), c_uint32, c_void_p],
    "wce_mmse_solve": [c_void_p, POINTER(Frames), c_void_p, c_int64, c_void_p],
    "wce_mmse_apply": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p],
    "wce_synth_frames": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                         c_uint64, c_void_p, c_double, c_double, c_void_p],
    "wce_front_end_blocks": [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_int64, c_void_p],
    "wce_front_end_preamble": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p,
                               c_void_p],
    "wce_nonfinite_scan": [c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int64, c_uint32, c_void_p, c_void_p,
                           c_void_p],
    "wce_comm_unique_id": [c_void_p],
    "wce_comm_init_rank": [POINTER(c_void_p), c_void_p, c_int, c_int, c_int],
    "wce_comm_init_all": [POINTER(c_void_p), c_int, POINTER(c_int)],
    "wce_comm_destroy": [c_void_p],
    "wce_comm_info": [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)],
    "wce_ctx_broadcast_state": [c_void_p, c_void_p, c_int, c_void_p],
    "wce_ctx_broadcast_state_all": [POINTER(c_void_p), POINTER(c_void_p), c_int, c_int, POINTER(c_void_p)],
    "wce_comm_max_f64": [c_void_p, POINTER(c_double), c_void_p],
    "wce_comm_max_f64_all": [POINTER(c_void_p), c_int, POINTER(c_double), POINTER(c_void_p)],
    "wce_shard": [ctypes.c_int64, c_int, c_int, POINTER(ctypes.c_int64), POINTER(ctypes.c_int64)],
    "wce_device_count": [POINTER(c_int)],
    "wce_set_device": [c_int],
    "wce_malloc": [POINTER(c_void_p), c_size_t],
    "wce_free": [c_void_p],
    "wce_memcpy_htod": [c_void_p, c_void_p, c_size_t],
    "wce_memcpy_dtoh": [c_void_p, c_void_p, c_size_t],
    "wce_memcpy_dtod": [c_void_p, c_void_p, c_size_t, c_void_p],
    "wce_ldc_to_complex": [c_void_p, c_void_p, ctypes.c_int64, c_void_p],
    "wce_complex_to_ldc": [c_void_p, c_void_p, ctypes.c_int64, c_void_p],
    "wce_memset": [c_void_p, c_int, c_size_t],
    "wce_host_alloc": [POINTER(c_void_p), c_size_t],
    "wce_host_free": [c_void_p],
    "wce_memcpy_htod_async": [c_void_p, c_void_p, c_size_t, c_void_p],
    "wce_memcpy_dtoh_async": [c_void_p, c_void_p, c_size_t, c_void_p],
    "wce_stream_create": [POINTER(c_void_p)],
    "wce_stream_destroy": [c_void_p],
    "wce_stream_synchronize": [c_void_p],
    "wce_event_create": [POINTER(c_void_p)],
    "wce_event_destroy": [c_void_p],
    "wce_event_record": [c_void_p, c_void_p],
    "wce_event_elapsed_ms": [POINTER(ctypes.c_float), c_void_p, c_void_p],
    "wce_last_error": [],
    "wce_version": [],
    "wce_compat_last_status": [],
    "WiFi_channel_estimation_LT_LS": [c_void_p, c_void_p, c_void_p],
    "WiFi_channel_estimation_PS_Linear": [c_void_p, c_void_p, c_void_p],
    "WiFi_channel_estimation_PS_Cubic": [c_void_p, c_void_p, c_void_p],
    "WiFi_channel_estimation_PS_Sinc": [c_void_p, c_void_p, c_void_p],
    "WiFi_channel_estimation_PS_MMSE": [c_void_p, c_void_p, c_void_p, c_double, c_void_p, c_void_p],
}
_VOID = {"WiFi_channel_estimation_LT_LS", "WiFi_channel_estimation_PS_Linear", "WiFi_channel_estimation_PS_Cubic",
         "WiFi_channel_estimation_PS_Sinc", "WiFi_channel_estimation_PS_MMSE"}
_STR = {"wce_last_error", "wce_version", "wce_debug_lr_kernel"}


def load(path: str = LIB_PATH):
    """Load libwce.so (in-tree build).  Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise WceError(-5, f"libwce.so not built at {path}; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, args in ABI.items():
        if name.startswith("wce_debug_") and not hasattr(lib, name):
            continue   # debug hooks are optional (older builds in A/B harnesses)
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = None if name in _VOID else (ctypes.c_char_p if name in _STR else c_int)
    lib.wce_state_size.restype = c_size_t
    if hasattr(lib, "wce_debug_compat_state_builds"):
        lib.wce_debug_compat_state_builds.restype = ctypes.c_ulonglong
    _lib = lib
    return lib


def _check(rc, where):
    if rc != 0:
        raise WceError(rc, where)


def device_count() -> int:
    n = c_int(0)
    _check(load().wce_device_count(byref(n)), "wce_device_count")
    return n.value


def _as_c128(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.complex128))


class PinnedArray:
    """Page-locked host memory (wce_host_alloc) with a numpy view, for
    stream-ordered copies that overlap estimation."""

    def __init__(self, shape, dtype=np.complex128):
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.ptr = c_void_p()
        _check(load().wce_host_alloc(byref(self.ptr), max(self.nbytes, 16)), "wce_host_alloc")
        buf = (ctypes.c_char * max(self.nbytes, 16)).from_address(self.ptr.value)
        self.array = np.frombuffer(buf, dtype=self.dtype, count=int(np.prod(self.shape))).reshape(self.shape)

    @property
    def addr(self) -> int:
        return self.ptr.value

    def free(self):
        if self.ptr is not None and self.ptr.value:
            self.array = None
            _lib.wce_host_free(self.ptr)
            self.ptr = c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:  # pragma: no cover
            pass


class DeviceArray:
    """A complex128 buffer in HBM (owned)."""

    def __init__(self, shape, dtype=np.complex128, zero=False):
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.ptr = c_void_p()
        _check(load().wce_malloc(byref(self.ptr), max(self.nbytes, 16)), "wce_malloc")
        if zero:
            _check(_lib.wce_memset(self.ptr, 0, max(self.nbytes, 16)), "wce_memset")

    @classmethod
    def from_numpy(cls, a):
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        if d.nbytes:
            _check(_lib.wce_memcpy_htod(d.ptr, a.ctypes.data_as(c_void_p), d.nbytes), "wce_memcpy_htod")
        return d

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        if self.nbytes:
            _check(_lib.wce_memcpy_dtoh(out.ctypes.data_as(c_void_p), self.ptr, self.nbytes), "wce_memcpy_dtoh")
        return out

    def rows(self, first, count=1) -> np.ndarray:
        """rows [first, first + count) of the leading axis, without copying the rest"""
        first, count = int(first), int(count)
        if first < 0 or count < 0 or first + count > self.shape[0]:
            raise IndexError("rows out of range")
        out = np.empty((count,) + self.shape[1:], self.dtype)
        row = out.nbytes // max(count, 1)
        if out.nbytes:
            _check(_lib.wce_memcpy_dtoh(out.ctypes.data_as(c_void_p), c_void_p(self.addr + first * row), out.nbytes),
                   "wce_memcpy_dtoh")
        return out

    def free(self):
        if self.ptr is not None and self.ptr.value:
            _lib.wce_free(self.ptr)
            self.ptr = c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:  # pragma: no cover
            pass

    @property
    def addr(self) -> int:
        return self.ptr.value or 0


def _addr(x):
    if x is None:
        return None
    if isinstance(x, DeviceArray):
        return x.addr
    return int(x)


class Context:
    """wce_ctx: shared (frame-independent) state resident on one device."""

    def __init__(self, tx_pre=None, rx_pre=None, ow2=None, mode=MMSE_REF, device=0, empty=False, Rhh=None):
        lib = load()
        self.handle = c_void_p()
        self.device = device
        self.mode = MMSE_COV if Rhh is not None else mode
        if empty:
            _check(lib.wce_ctx_create_empty(byref(self.handle), device), "wce_ctx_create_empty")
            return
        tp, rp = _as_c128(tx_pre), _as_c128(rx_pre)
        if tp.shape != (NSC,) or rp.shape != (NSC,):
            raise ValueError("tx_pre / rx_pre must hold 53 subcarriers")
        if Rhh is not None:   # WCE_MMSE_COV: model channel covariance (53 x 53, time domain)
            R = _as_c128(Rhh)
            if R.shape != (NSC, NSC):
                raise ValueError("Rhh must be 53 x 53")
            _check(lib.wce_ctx_create_cov(byref(self.handle), device, tp.ctypes.data_as(c_void_p),
                                          rp.ctypes.data_as(c_void_p), R.ctypes.data_as(c_void_p), float(ow2)),
                   "wce_ctx_create_cov")
            return
        _check(lib.wce_ctx_create(byref(self.handle), device, tp.ctypes.data_as(c_void_p),
                                  rp.ctypes.data_as(c_void_p), float(ow2), mode), "wce_ctx_create")

    def set_fusion(self, on: bool):
        """A/B switch: LS family + equalization fused into the MMSE solve (default on)."""
        _check(_lib.wce_debug_set_fusion(self.handle, int(bool(on))), "wce_debug_set_fusion")

    def plan(self, frames: "Frames", outputs: "Outputs", mask: int) -> "Plan":
        """Capture one estimate call into a HIP graph (wce_plan_create)."""
        return Plan(self, frames, outputs, mask)

    def cov_info(self):
        """WCE_MMSE_COV: (rank r, low-rank path taken, lambda_max, lambda_min of the kept spectrum of C)."""
        r, lr = c_int(), c_int()
        lmax, lmin = c_double(), c_double()
        _check(load().wce_ctx_cov_info(self.handle, ctypes.byref(r), ctypes.byref(lr), ctypes.byref(lmax),
                                       ctypes.byref(lmin)), "cov_info")
        return r.value, bool(lr.value), lmax.value, lmin.value

    def set_modulus(self, x_ref):
        """WCE_MMSE_COV: the constant-modulus operator for frames with |x|^2 = |x_ref|^2 (None: off)."""
        if x_ref is None:
            _check(load().wce_ctx_set_modulus(self.handle, None), "wce_ctx_set_modulus")
            return
        x = _as_c128(x_ref)
        if x.shape != (NSC,):
            raise ValueError("x_ref must hold 53 subcarriers")
        _check(load().wce_ctx_set_modulus(self.handle, x.ctypes.data_as(c_void_p)), "wce_ctx_set_modulus")

    def set_cm(self, on: bool):
        """A/B switch of the constant-modulus path (default on once a pattern is set)."""
        _check(load().wce_debug_set_cm(self.handle, int(bool(on))), "wce_debug_set_cm")

    def set_cov_path(self, path: int):
        """A/B: 0 = the state's choice, 1 = dense Ryy solve, 2 = low-rank Gram path."""
        _check(load().wce_debug_set_cov_path(self.handle, path), "set_cov_path")

    def lr_kernel(self, units: int) -> str:
        """The low-rank kernel an estimate over `units` (frame, block) units runs ("" on the dense path)."""
        return load().wce_debug_lr_kernel(self.handle, int(units)).decode()

    def set_border_dot(self, on: bool):
        """A/B switch: rank-1 covariance via a second bordered row (default on)."""
        _check(_lib.wce_debug_set_border_dot(self.handle, int(bool(on))), "wce_debug_set_border_dot")

    def reserve(self, n_frames):
        """Pre-size the WCE_MMSE_FRAME_COV workspace (no allocation inside estimate)."""
        _check(_lib.wce_ctx_reserve(self.handle, n_frames), "wce_ctx_reserve")

    def close(self):
        if self.handle is not None and self.handle.value:
            _lib.wce_ctx_destroy(self.handle)
            self.handle = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    def state(self):
        ptr, nb = c_void_p(), c_size_t()
        _check(_lib.wce_ctx_state(self.handle, byref(ptr), byref(nb)), "wce_ctx_state")
        return ptr.value, nb.value

    def load_state(self, blob: np.ndarray):
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        _check(_lib.wce_ctx_load_state(self.handle, blob.ctypes.data_as(c_void_p), blob.nbytes),
               "wce_ctx_load_state")

    def mark_ready(self):
        _check(_lib.wce_ctx_mark_ready(self.handle), "wce_ctx_mark_ready")

    def shared(self):
        h = np.zeros(NSC, np.complex128)
        C = np.zeros((NSC, NSC), np.complex128)
        a, b = c_double(), c_double()
        _check(_lib.wce_ctx_get_shared(self.handle, h.ctypes.data_as(c_void_p), C.ctypes.data_as(c_void_p),
                                       byref(a), byref(b)), "wce_ctx_get_shared")
        return h, C, a.value, b.value

    # ---------------------------------------------------------------- batched
    @staticmethod
    def frames(tx, rx, n_frames, frame_stride=NBLK * NSC, block_stride=NSC, rx_pre=None, pre_stride=NSC,
               tx_pre=None, block=0, semantics=SEM_C) -> Frames:
        return Frames(_addr(tx), _addr(rx), _addr(rx_pre), _addr(tx_pre), frame_stride, block_stride, pre_stride,
                      n_frames, block, semantics)

    def nonfinite_scan(self, H, n_frames, stride=NSC, f32=False, bitmap=None, n_bad=None, stream=None):
        """wce_nonfinite_scan on a device output array.  With bitmap/n_bad
        None, allocates them, waits, and returns (bitmap as numpy uint32,
        number of non-finite frames); otherwise enqueues into the given
        device buffers and returns None."""
        own = bitmap is None
        if own:
            bitmap = DeviceArray(((n_frames + 31) // 32,), dtype=np.uint32)
            n_bad = DeviceArray((1,), dtype=np.uint64)
        _check(_lib.wce_nonfinite_scan(self.handle, _addr(H), stride, n_frames, OUT_LS_F32 if f32 else 0, _addr(bitmap),
                                       _addr(n_bad), stream), "wce_nonfinite_scan")
        if not own:
            return None
        if stream is not None:
            _check(_lib.wce_stream_synchronize(stream), "wce_stream_synchronize")
        return bitmap.numpy(), int(n_bad.numpy()[0])

    def estimate(self, frames: Frames, outputs: Outputs, mask: int, stream=None):
        _check(_lib.wce_estimate(self.handle, byref(frames), byref(outputs), mask, stream), "wce_estimate")

    def mmse_solve(self, frames: Frames, W, w_stride=NSC, stream=None):
        _check(_lib.wce_mmse_solve(self.handle, byref(frames), _addr(W), w_stride, stream), "wce_mmse_solve")

    def mmse_apply(self, W, H, n_frames, stride=NSC, stream=None):
        _check(_lib.wce_mmse_apply(self.handle, _addr(W), _addr(H), stride, n_frames, stream), "wce_mmse_apply")

    def synth(self, tx, rx, rx_pre, n_frames, first_frame=0, seed=0x80211, h_shared=None, amplitude=8.8753,
              ow2=9.6172e-08, frame_stride=NBLK * NSC, block_stride=NSC, pre_stride=NSC, stream=None):
        _check(_lib.wce_synth_frames(self.handle, _addr(tx), _addr(rx), _addr(rx_pre), frame_stride, block_stride,
                                     pre_stride, first_frame, n_frames, seed, _addr(h_shared), amplitude, ow2,
                                     stream), "wce_synth_frames")

    def front_end_blocks(self, samples, n_frames, n_blocks=NBLK, sym=None, packet_stride=None,
                         frame_stride=NBLK * NSC, block_stride=NSC, stream=None):
        """Time-domain packets (device) -> 53-bin OFDM symbols (WiFi_blocks_extraction.m)."""
        ps = packet_stride if packet_stride is not None else SAMPLES_PER_BLOCK * n_blocks
        _check(_lib.wce_front_end_blocks(self.handle, _addr(samples), ps, n_frames, n_blocks, _addr(sym),
                                         frame_stride, block_stride, stream), "wce_front_end_blocks")

    def front_end_preamble(self, lptot, n_frames, lptot_len, pre_fft, ow2=None, lptot_stride=None,
                           pre_stride=NSC, stream=None):
        """Long training fields (device) -> preamble FFT [53] and sigma^2 per frame (WiFi_RX.m:18-30)."""
        ls = lptot_stride if lptot_stride is not None else lptot_len
        _check(_lib.wce_front_end_preamble(self.handle, _addr(lptot), ls, lptot_len, n_frames, _addr(pre_fft),
                                           pre_stride, _addr(ow2), stream), "wce_front_end_preamble")

    def front_end_host(self, packets, lptot=None, n_blocks=NBLK):
        """Convenience: host packets [B][80 n_blocks] (+ lptot [B][L]) -> (sym [B][n_blocks][53],
        pre_fft [B][53] or None, ow2 [B] or None)."""
        packets = _as_c128(packets)
        B = packets.shape[0]
        dp = DeviceArray.from_numpy(packets)
        dsym = DeviceArray((B, n_blocks, NSC), zero=True)
        self.front_end_blocks(dp, B, n_blocks, dsym, packet_stride=packets.shape[1], frame_stride=n_blocks * NSC)
        pre = ow2 = None
        if lptot is not None:
            lptot = _as_c128(lptot)
            dl = DeviceArray.from_numpy(lptot)
            dpre = DeviceArray((B, NSC), zero=True)
            dow2 = DeviceArray((B,), np.float64, zero=True)
            self.front_end_preamble(dl, B, lptot.shape[1], dpre, dow2)
        synchronize()
        sym = dsym.numpy()
        if lptot is not None:
            pre, ow2 = dpre.numpy(), dow2.numpy()
        return sym, pre, ow2

    def estimate_host(self, tx, rx, rx_pre=None, mask=ALL, block=0, eq_source=PS_LINEAR, semantics=SEM_C,
                      tx_pre=None, ls_f32=False):
        """Convenience: host numpy frames [B][15][53] -> dict of host outputs."""
        tx, rx = _as_c128(tx), _as_c128(rx)
        B = tx.shape[0]
        if tx.shape != (B, NBLK, NSC) or rx.shape != tx.shape:
            raise ValueError("tx/rx must be [B][15][53] complex")
        dtx, drx = DeviceArray.from_numpy(tx), DeviceArray.from_numpy(rx)
        dpre = DeviceArray.from_numpy(_as_c128(rx_pre)) if rx_pre is not None else None
        names = [("lt_ls", LT_LS), ("ps_linear", PS_LINEAR), ("ps_cubic", PS_CUBIC), ("ps_sinc", PS_SINC),
                 ("ps_mmse", PS_MMSE)]
        lsdt = np.complex64 if ls_f32 else np.complex128
        outs = {n: DeviceArray((B, NSC), np.complex128 if n == "ps_mmse" else lsdt, zero=True)
                for n, bit in names if mask & bit}
        deq = DeviceArray((B, NBLK, NSC), lsdt, zero=True) if mask & EQUALIZE else None
        o = Outputs(*[(outs[n].addr if n in outs else None) for n, _ in names],
                    deq.addr if deq is not None else None, NSC, NBLK * NSC, NSC, eq_source,
                    OUT_LS_F32 if ls_f32 else 0)
        dtp = DeviceArray.from_numpy(_as_c128(tx_pre)) if tx_pre is not None else None
        fr = self.frames(dtx, drx, B, rx_pre=dpre, block=block, semantics=semantics, tx_pre=dtp)
        self.estimate(fr, o, mask)
        synchronize()
        res = {n: outs[n].numpy() for n in outs}
        if deq is not None:
            res["eq"] = deq.numpy()
        return res


class Plan:
    """wce_plan: a captured wce_estimate call, replayed with one graph launch.
    Keeps references to the frames/outputs structs (the buffers they point
    to must outlive the plan)."""

    def __init__(self, ctx, frames, outputs, mask):
        self.handle = c_void_p()
        self._keep = (ctx, frames, outputs)
        _check(_lib.wce_plan_create(byref(self.handle), ctx.handle, byref(frames), byref(outputs), mask),
               "wce_plan_create")

    def launch(self, stream=None):
        _check(_lib.wce_plan_launch(self.handle, stream), "wce_plan_launch")

    def close(self):
        if self.handle is not None and self.handle.value:
            _lib.wce_plan_destroy(self.handle)
            self.handle = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass


def state_blob(tx_pre, rx_pre, ow2, mode=MMSE_REF, Rhh=None) -> np.ndarray:
    """The shared state built on the host (no device): bytes to broadcast."""
    lib = load()
    n = lib.wce_state_size()
    blob = np.zeros(n, np.uint8)
    tp, rp = _as_c128(tx_pre), _as_c128(rx_pre)
    if Rhh is not None:
        R = _as_c128(Rhh)
        _check(lib.wce_state_build_cov(blob.ctypes.data_as(c_void_p), n, tp.ctypes.data_as(c_void_p),
                                       rp.ctypes.data_as(c_void_p), R.ctypes.data_as(c_void_p), float(ow2)),
               "wce_state_build_cov")
        return blob
    _check(lib.wce_state_build(blob.ctypes.data_as(c_void_p), n, tp.ctypes.data_as(c_void_p),
                               rp.ctypes.data_as(c_void_p), float(ow2), mode), "wce_state_build")
    return blob


def state_mode(blob: np.ndarray) -> int:
    """The MMSE mode of a valid state blob (wce_state_validate); raises if the bytes hold no state."""
    m = c_int()
    _check(load().wce_state_validate(blob.ctypes.data_as(c_void_p), blob.nbytes, byref(m)), "wce_state_validate")
    return m.value


def cov_factor(blob: np.ndarray):
    """A WCE_MMSE_COV state blob's low-rank factor: (U [53 x rank] with C = U U^H, rank, k0, lambda_max,
    lambda_min); k0 = -1 when the dense Ryy solve runs, else the Gram system's first block row."""
    U = np.zeros((NSC, 64), np.complex128)
    r, k0 = c_int(), c_int()
    lmax, lmin = c_double(), c_double()
    _check(load().wce_debug_cov_factor(blob.ctypes.data_as(c_void_p), blob.nbytes, U.ctypes.data_as(c_void_p),
                                       byref(r), byref(k0), byref(lmax), byref(lmin)), "wce_debug_cov_factor")
    return U[:, :r.value].copy(), r.value, k0.value, lmax.value, lmin.value


def ldc_to_complex(src, dst, n, stream=None):
    """wce_ldc_to_complex: n long double _Complex values (the reference's
    format, raw x87 bytes in device memory, e.g. DeviceArray of clongdouble)
    -> complex double in dst, rounded as C's (double) cast."""
    _check(load().wce_ldc_to_complex(_addr(src), _addr(dst), int(n), stream), "wce_ldc_to_complex")


def complex_to_ldc(src, dst, n, stream=None):
    """wce_complex_to_ldc: n complex double -> long double _Complex (exact)."""
    _check(load().wce_complex_to_ldc(_addr(src), _addr(dst), int(n), stream), "wce_complex_to_ldc")


def synchronize(stream=None):
    _check(load().wce_stream_synchronize(stream), "wce_stream_synchronize")


class Stream:
    def __init__(self):
        self.handle = c_void_p()
        _check(load().wce_stream_create(byref(self.handle)), "wce_stream_create")

    def synchronize(self):
        _check(_lib.wce_stream_synchronize(self.handle), "wce_stream_synchronize")

    def __del__(self):
        try:
            if self.handle.value:
                _lib.wce_stream_destroy(self.handle)
        except Exception:  # pragma: no cover
            pass


class Event:
    def __init__(self):
        self.handle = c_void_p()
        _check(load().wce_event_create(byref(self.handle)), "wce_event_create")

    def record(self, stream=None):
        s = stream.handle if isinstance(stream, Stream) else stream
        _check(_lib.wce_event_record(self.handle, s), "wce_event_record")

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _check(_lib.wce_event_elapsed_ms(byref(ms), self.handle, end.handle), "wce_event_elapsed_ms")
        return ms.value

    def __del__(self):
        try:
            if self.handle.value:
                _lib.wce_event_destroy(self.handle)
        except Exception:  # pragma: no cover
            pass


# ------------------------------------------------------------------------
# The reference's entry points (main.c:4-8): same names, same argument
# meaning, results written into H_EST (53 complex).  Arrays are numpy
# clongdouble (= long double _Complex) or anything convertible.
# ------------------------------------------------------------------------
def _ld(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.clongdouble))


def _call_compat(name, *arrays, out):
    lib = load()
    ins = [_ld(a) for a in arrays]
    if any(a.shape[0] < NSC for a in ins):
        raise ValueError("estimator inputs need 53 subcarriers")
    res = np.zeros(NSC, np.clongdouble)
    getattr(lib, name)(*[a.ctypes.data_as(c_void_p) for a in ins], res.ctypes.data_as(c_void_p))
    _check(lib.wce_compat_last_status(), name)
    if out is not None:
        out[:NSC] = res
    return res


def WiFi_channel_estimation_LT_LS(tx_pre, rx_pre, H_EST=None):
    """main.c:66-75 on the GPU."""
    return _call_compat("WiFi_channel_estimation_LT_LS", tx_pre, rx_pre, out=H_EST)


def WiFi_channel_estimation_PS_Linear(tx_symbols, rx_symbols, H_EST=None):
    """main.c:77-101 on the GPU."""
    return _call_compat("WiFi_channel_estimation_PS_Linear", tx_symbols, rx_symbols, out=H_EST)


def WiFi_channel_estimation_PS_Cubic(tx_symbols, rx_symbols, H_EST=None):
    """main.c:103-122 on the GPU."""
    return _call_compat("WiFi_channel_estimation_PS_Cubic", tx_symbols, rx_symbols, out=H_EST)


def WiFi_channel_estimation_PS_Sinc(tx_symbols, rx_symbols, H_EST=None):
    """main.c:124-146 on the GPU."""
    return _call_compat("WiFi_channel_estimation_PS_Sinc", tx_symbols, rx_symbols, out=H_EST)


def WiFi_channel_estimation_PS_MMSE(tx_symbols, rx_symbols, F, ow2, H_EST_LS, H_EST=None):
    """main.c:148-212 (REF-repaired) on the GPU.  F: 53x53."""
    lib = load()
    tx, rx, hls = _ld(tx_symbols), _ld(rx_symbols), _ld(H_EST_LS)
    Fm = np.ascontiguousarray(np.asarray(F, dtype=np.clongdouble).reshape(NSC, NSC))
    rows = (c_void_p * NSC)(*[Fm[i].ctypes.data for i in range(NSC)])
    res = np.zeros(NSC, np.clongdouble)
    lib.WiFi_channel_estimation_PS_MMSE(tx.ctypes.data_as(c_void_p), rx.ctypes.data_as(c_void_p),
                                        ctypes.cast(rows, c_void_p), float(ow2), hls.ctypes.data_as(c_void_p),
                                        res.ctypes.data_as(c_void_p))
    _check(lib.wce_compat_last_status(), "WiFi_channel_estimation_PS_MMSE")
    if H_EST is not None:
        H_EST[:NSC] = res
    return res
