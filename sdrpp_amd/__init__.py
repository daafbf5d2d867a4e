"""sdrpp_amd: MI355X-native streaming-DSP hot path of SDR++ (qrp73/SDRPP).

The product is the C-ABI shared library ``sdrpp_amd/lib/libsdrgpu.so`` (HIP
kernels for gfx950, declared in ``include/sdrgpu.h``). This module is a thin
ctypes binding used by the tests and ``bench.py``; the drop-in C++ host classes
live in ``sdrpp_amd/dsp/``. There is no CPU fallback:
loading fails loudly if the library is missing.
"""
import ctypes
import os

__all__ = ["lib", "LIB_PATH", "check", "SdrGpuError"]

_HERE = os.path.dirname(os.path.abspath(__file__))
# SDRGPU_LIB_PATH: load another build of the same ABI (A/B timing of two builds on one box)
LIB_PATH = os.environ.get("SDRGPU_LIB_PATH") or os.path.join(_HERE, "lib", "libsdrgpu.so")

F32, C64 = 0, 1
WIN_RECTANGULAR, WIN_HAMMING, WIN_HANN, WIN_BLACKMAN, WIN_NUTTALL, WIN_BH4, WIN_BH7 = range(7)
CONV_U8, CONV_I16, CONV_I24, CONV_I32, CONV_F64, CONV_I8, CONV_F32 = range(7)


class SdrGpuError(RuntimeError):
    pass


def _load():
    # PyTorch wheels bundle their own libamdhip64.so.7 (same SONAME as /opt/rocm's). Load
    # torch first so libsdrgpu binds to the already-loaded runtime: one HIP/HSA runtime
    # per process, shared device pointers and streams with torch (bench, RCCL).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP extension is required; there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, i, d, ll, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_longlong, ctypes.c_void_p
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "sdrgpu_version": (i, []),
        "sdrgpu_last_error": (ctypes.c_char_p, []),
        "sdrgpu_device_count": (i, []),
        "sdrgpu_malloc": (i, [i, pp, ctypes.c_size_t]),
        "sdrgpu_free": (i, [vp]),
        "sdrgpu_memcpy_h2d": (i, [vp, vp, ctypes.c_size_t, vp]),
        "sdrgpu_memcpy_d2h": (i, [vp, vp, ctypes.c_size_t, vp]),
        "sdrgpu_stream_create": (i, [i, pp]),
        "sdrgpu_stream_destroy": (i, [vp]),
        "sdrgpu_stream_synchronize": (i, [vp]),
        "sdrgpu_host_register": (i, [vp, ctypes.c_size_t]),
        "sdrgpu_host_unregister": (i, [vp]),
        "sdrgpu_create_window": (i, [i, fp, i, i]),
        "sdrgpu_gen_reshape_params": (None, [d, i, d, ctypes.POINTER(i), ctypes.POINTER(i)]),
        "sdrgpu_taps_estimate_count": (i, [d, d]),
        "sdrgpu_taps_windowed_sinc": (i, [i, d, d, fp]),
        "sdrgpu_taps_low_pass": (i, [d, d, d, i, fp]),
        "sdrgpu_taps_high_pass": (i, [d, d, d, i, fp]),
        "sdrgpu_taps_band_pass_f": (i, [d, d, d, d, i, fp]),
        "sdrgpu_taps_band_pass_c": (i, [d, d, d, d, i, fp]),
        "sdrgpu_decim_plan": (i, [i, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(ctypes.POINTER(ctypes.c_float))]),
        "sdrgpu_fft_create": (i, [pp, i, i, i, i]),
        "sdrgpu_fft_set_window": (i, [vp, fp, i]),
        "sdrgpu_fft_set_window_type": (i, [vp, i, i]),
        "sdrgpu_fft_execute_dev": (i, [vp, vp, ll, i, vp, vp]),
        "sdrgpu_fft_execute_vfo_dev": (i, [vp, vp, i, vp, vp, vp, vp]),
        "sdrgpu_fft_execute_zoom_vfo_dev": (i, [vp, vp, i, vp, vp, i, vp, vp, vp]),
        "sdrgpu_fft_set_timing": (i, [vp, i]),
        "sdrgpu_fft_group_times": (i, [vp, fp, i]),
        "sdrgpu_fft_execute_zoom_dev": (i, [vp, vp, ll, i, vp, vp, i, vp]),
        "sdrgpu_fft_logmag": (i, [vp, vp, vp]),
        "sdrgpu_fft_size": (i, [vp]),
        "sdrgpu_fft_set_precision": (i, [vp, i]),
        "sdrgpu_fft_get_precision": (i, [vp]),
        "sdrgpu_fft_set_kernel": (i, [vp, i]),
        "sdrgpu_fft_set_tail_stream": (i, [vp, vp]),
        "sdrgpu_fft_destroy": (i, [vp]),
        "sdrgpu_xlator_create": (i, [pp, i, d]),
        "sdrgpu_xlator_set_offset": (i, [vp, d]),
        "sdrgpu_fir_create": (i, [pp, i, i, i, fp, i, i]),
        "sdrgpu_fir_set_taps": (i, [vp, fp, i]),
        "sdrgpu_fir_set_decimation": (i, [vp, i]),
        "sdrgpu_quadrature_create": (i, [pp, i, d]),
        "sdrgpu_quadrature_set_deviation": (i, [vp, d]),
        "sdrgpu_power_decimator_create": (i, [pp, i, i, i]),
        "sdrgpu_polyphase_resampler_create": (i, [pp, i, i, i, i, fp, i]),
        "sdrgpu_rational_resampler_create": (i, [pp, i, i, d, d]),
        "sdrgpu_rxvfo_create": (i, [pp, i, d, d, d, d]),
        "sdrgpu_rxvfo_set_offset": (i, [vp, d]),
        "sdrgpu_ddc_create": (i, [pp, i, d, fp, i, i]),
        "sdrgpu_gather_get_id": (i, [vp]),
        "sdrgpu_gather_create": (i, [pp, i, i, i, vp]),
        "sdrgpu_gather_rows": (i, [vp, vp, ll, vp, vp]),
        "sdrgpu_gather_set_timeout": (i, [vp, d]),
        "sdrgpu_gather_wait": (i, [vp, vp, d]),
        "sdrgpu_gather_destroy": (i, [vp]),
        "sdrgpu_ddc_fm_create": (i, [pp, i, d, fp, i, i, d]),
        "sdrgpu_fm_create": (i, [pp, i, d, d, i, i]),
        "sdrgpu_wfm_create": (i, [pp, i, d, d, i]),
        "sdrgpu_channelizer_create": (i, [pp, i, i, fp, i]),
        "sdrgpu_channelizer_set_dft": (i, [vp, i]),
        "sdrgpu_broadcast_fm_create": (i, [pp, i, d, d, i, i]),
        "sdrgpu_deemphasis_create": (i, [pp, i, i, d, d]),
        "sdrgpu_deemphasis_set": (i, [vp, d, d]),
        "sdrgpu_zoom_create": (i, [pp, i, d, d, d, i, i]),
        "sdrgpu_zoom_execute_dev": (i, [vp, vp, i, vp, vp]),
        "sdrgpu_zoom_destroy": (i, [vp]),
        "sdrgpu_compress_dev": (i, [i, i, vp, i, vp, vp, vp]),
        "sdrgpu_decompress_dev": (i, [i, vp, vp, i, vp, vp]),
        "sdrgpu_wav_encode_dev": (i, [i, i, vp, ll, vp, vp]),
        "sdrgpu_frontend_create": (i, [pp, i, d, i, i, i, d, i]),
        "sdrgpu_frontend_destroy": (i, [vp]),
        "sdrgpu_frontend_configure": (i, [vp, d, i, i]),
        "sdrgpu_frontend_set_invert_iq": (i, [vp, i]),
        "sdrgpu_frontend_set_fft": (i, [vp, i, d, i]),
        "sdrgpu_frontend_framing": (i, [vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(d)]),
        "sdrgpu_frontend_add_vfo": (i, [vp, ctypes.POINTER(i), d, d, d]),
        "sdrgpu_frontend_remove_vfo": (i, [vp, i]),
        "sdrgpu_frontend_set_vfo_offset": (i, [vp, i, d]),
        "sdrgpu_frontend_push": (i, [vp, vp, i, i]),
        "sdrgpu_frontend_push_dev": (i, [vp, vp, i, i, vp]),
        "sdrgpu_frontend_spectra_dev": (i, [vp, pp, ctypes.POINTER(i)]),
        "sdrgpu_frontend_read_spectra": (i, [vp, fp, i]),
        "sdrgpu_frontend_vfo_dev": (i, [vp, i, pp, ctypes.POINTER(i)]),
        "sdrgpu_frontend_read_vfo": (i, [vp, i, vp, i]),
        "sdrgpu_frontend_submit": (i, [vp, vp, i, i, i]),
        "sdrgpu_frontend_collect": (i, [vp, i, pp, pp, ctypes.POINTER(i)]),
        "sdrgpu_frontend_collected_vfo": (i, [vp, i, i, pp, ctypes.POINTER(i)]),
        "sdrgpu_frontend_release": (i, [vp, i]),
        "sdrgpu_host_alloc": (i, [pp, ctypes.c_size_t]),
        "sdrgpu_host_free": (i, [vp]),
        "sdrgpu_agc_create": (i, [pp, i, i, d, d, d, d, d, d]),
        "sdrgpu_agc_set_enabled": (i, [vp, i]),
        "sdrgpu_agc_set_gain": (i, [vp, ctypes.c_float]),
        "sdrgpu_agc_get_gain": (i, [vp, ctypes.POINTER(ctypes.c_float)]),
        "sdrgpu_dc_blocker_create": (i, [pp, i, i, d]),
        "sdrgpu_am_create": (i, [pp, i, i, d, d, d, d, d, i]),
        "sdrgpu_ssb_create": (i, [pp, i, i, d, d, i, d, d, i]),
        "sdrgpu_block_process": (i, [vp, vp, i, vp]),
        "sdrgpu_block_process_dev": (i, [vp, vp, i, vp, vp]),
        "sdrgpu_block_out_count": (i, [vp, i]),
        "sdrgpu_block_reset": (i, [vp]),
        "sdrgpu_block_destroy": (i, [vp]),
        "sdrgpu_convert_dev": (i, [i, i, vp, ll, vp, vp]),
        "sdrgpu_convert": (i, [i, i, vp, ll, vp]),
        "sdrgpu_convert_mono_dev": (i, [i, i, vp, ll, vp, vp]),
        "sdrgpu_broadcast_fm_set_rds": (i, [vp, i]),
        "sdrgpu_colormap_dev": (i, [i, vp, ll, ctypes.c_float, ctypes.c_float, vp, i, vp, vp]),
        "sdrgpu_fft_smooth_hold_dev": (i, [i, vp, i, i, i, ctypes.c_float, ctypes.c_float, vp, i, ctypes.c_float, vp, vp]),
        "sdrgpu_vfo_signal_info_dev": (i, [i, vp, i, i, d, d, d, vp, vp, vp]),
        "sdrgpu_broadcast_fm_rds_dev": (i, [vp, pp, ctypes.POINTER(i)]),
        "sdrgpu_broadcast_fm_read_rds": (i, [vp, vp, i]),
        "sdrgpu_convert_mono": (i, [i, i, vp, ll, vp]),
        "sdrgpu_wav_open": (i, [pp, ctypes.c_char_p]),
        "sdrgpu_wav_info": (i, [vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(d),
                                ctypes.POINTER(ll)]),
        "sdrgpu_wav_kind": (i, [vp]),
        "sdrgpu_wav_block_size": (i, [vp]),
        "sdrgpu_wav_read": (i, [vp, vp, i]),
        "sdrgpu_wav_seek": (i, [vp, ll]),
        "sdrgpu_wav_close": (i, [vp]),
    }
    alt = bool(os.environ.get("SDRGPU_LIB_PATH"))
    for name, (res, args) in sig.items():
        if alt and not hasattr(L, name):   # an older build under A/B timing: newer entry points absent
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()


def check(rc):
    """Raise SdrGpuError for a negative C-ABI status; return rc otherwise."""
    if rc is not None and rc < 0:
        raise SdrGpuError(f"sdrgpu error {rc}: {lib.sdrgpu_last_error().decode(errors='replace')}")
    return rc
