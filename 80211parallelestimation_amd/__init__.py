"""MI355X-native 802.11 channel estimation (LT_LS, PS_Linear/Cubic/Sinc,
PS_MMSE, equalization) behind the reference's estimator API.

The package name starts with a digit, so import it with
``importlib.import_module("80211parallelestimation_amd")``.
"""
from .wce import (  # noqa: F401
    ALL, DC, EQUALIZE, FRAME_COV, LS_ALL, OUT_LS_F32, LT_LS, MMSE_COV, MMSE_REF, MMSE_TEXTBOOK, NBLK, NSC, PILOTS, PS_CUBIC, PS_LINEAR,
    PS_MMSE, PS_SINC, SEM_C, SEM_MATLAB, Context, DeviceArray, PinnedArray, Event, Frames, Outputs, Stream, WceError, device_count, load,
    state_blob, state_mode, cov_factor, synchronize, ldc_to_complex, complex_to_ldc, WiFi_channel_estimation_LT_LS, WiFi_channel_estimation_PS_Cubic,
    WiFi_channel_estimation_PS_Linear, WiFi_channel_estimation_PS_MMSE, WiFi_channel_estimation_PS_Sinc,
)

__version__ = "0.1.0"
