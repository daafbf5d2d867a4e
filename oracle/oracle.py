"""ctypes binding of the CPU restatement (oracle/libsdr_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the parity checker / CPU baseline. The product
(sdrpp_amd, libsdrgpu.so) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB_PATH: a host-built -march=native copy of the same source (bench.py's CPU baseline)
LIB_PATH = os.environ.get("ORACLE_LIB_PATH") or os.path.join(HERE, "libsdr_oracle.so")


def _load():
    if not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-C", HERE, "-s"])
    L = ctypes.CDLL(LIB_PATH)
    vp, i, d, l = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_long
    sig = {
        "orc_window_value": (d, [i, d, d]),
        "orc_create_window": (None, [i, vp, i, i]),
        "orc_gen_reshape_params": (None, [d, i, d, ctypes.POINTER(i), ctypes.POINTER(i)]),
        "orc_estimate_tap_count": (i, [d, d]),
        "orc_windowed_sinc": (i, [i, d, d, vp]),
        "orc_low_pass": (i, [d, d, d, i, vp]),
        "orc_high_pass": (i, [d, d, d, i, vp]),
        "orc_band_pass_f": (i, [d, d, d, d, i, vp]),
        "orc_band_pass_c": (i, [d, d, d, d, i, vp]),
        "orc_decim_plan": (i, [i, vp, vp, vp]),
        "orc_u8_to_f32": (None, [vp, vp, l]),
        "orc_i16_to_f32": (None, [vp, vp, l]),
        "orc_i24_to_f32": (None, [vp, vp, l]),
        "orc_i32_to_f32": (None, [vp, vp, l]),
        "orc_f64_to_f32": (None, [vp, vp, l]),
        "orc_i8_to_f32": (None, [vp, vp, l]),
        "orc_fft_c2c": (None, [vp, vp, i]),
        "orc_fft_c2c_f64": (None, [vp, vp, i]),
        "orc_power_spectrum_db": (None, [vp, vp, i]),
        "orc_fft_logmag": (None, [vp, i, i, vp, vp, vp]),
        "orc_fir_create": (vp, [i, i, vp, i, i, i]),
        "orc_fir_set_taps": (None, [vp, vp, i]),
        "orc_fir_reset": (None, [vp]),
        "orc_fir_process": (i, [vp, vp, i, vp]),
        "orc_fir_destroy": (None, [vp]),
        "orc_xlator_create": (vp, [d]),
        "orc_xlator_set_offset": (None, [vp, d]),
        "orc_xlator_reset": (None, [vp]),
        "orc_xlator_process": (i, [vp, vp, i, vp]),
        "orc_xlator_effective_omega": (d, [d]),
        "orc_xlator_destroy": (None, [vp]),
        "orc_quad_create": (vp, [d]),
        "orc_quad_reset": (None, [vp]),
        "orc_quad_process": (i, [vp, vp, i, vp]),
        "orc_quad_destroy": (None, [vp]),
        "orc_pdec_create": (vp, [i, i, i]),
        "orc_pdec_process": (i, [vp, vp, i, vp]),
        "orc_pdec_reset": (None, [vp]),
        "orc_pdec_destroy": (None, [vp]),
        "orc_poly_create": (vp, [i, i, i, vp, i, i]),
        "orc_poly_process": (i, [vp, vp, i, vp]),
        "orc_poly_reset": (None, [vp]),
        "orc_poly_destroy": (None, [vp]),
        "orc_rres_create": (vp, [i, d, d, i]),
        "orc_rres_process": (i, [vp, vp, i, vp]),
        "orc_rres_info": (i, [vp, vp, vp, vp, vp, vp]),
        "orc_rres_destroy": (None, [vp]),
        "orc_vfo_create": (vp, [d, d, d, d, i]),
        "orc_vfo_process": (i, [vp, vp, i, vp]),
        "orc_vfo_destroy": (None, [vp]),
        "orc_wfm_create": (vp, [d, d, i, i]),
        "orc_wfm_process": (i, [vp, vp, i, vp]),
        "orc_wfm_destroy": (None, [vp]),
        "orc_fm_create": (vp, [d, d, i, i, i]),
        "orc_fm_process": (i, [vp, vp, i, vp]),
        "orc_fm_destroy": (None, [vp]),
        "orc_agc_create": (vp, [i, d, d, d, d, d, d]),
        "orc_agc_set_enabled": (None, [vp, i]),
        "orc_agc_process": (i, [vp, vp, i, vp]),
        "orc_agc_destroy": (None, [vp]),
        "orc_agc_set_gain": (None, [vp, ctypes.c_float]),
        "orc_agc_get_gain": (ctypes.c_float, [vp]),
        "orc_dcb_create": (vp, [i, d]),
        "orc_dcb_process": (i, [vp, vp, i, vp]),
        "orc_dcb_destroy": (None, [vp]),
        "orc_am_create": (vp, [i, d, d, d, d, d, i]),
        "orc_am_process": (i, [vp, vp, i, vp]),
        "orc_am_destroy": (None, [vp]),
        "orc_ssb_create": (vp, [i, d, d, i, d, d]),
        "orc_ssb_process": (i, [vp, vp, i, vp]),
        "orc_ssb_destroy": (None, [vp]),
        "orc_compress": (i, [i, vp, i, vp]),
        "orc_decompress": (i, [vp, i, vp]),
        "orc_channelize": (i, [vp, l, vp, i, i, vp, i, vp]),
        "orc_wfms_create": (vp, [d, d, i, i, i]),
        "orc_wfms_process": (i, [vp, vp, i, vp]),
        "orc_wfms_destroy": (None, [vp]),
        "orc_deemp_create": (vp, [i, d, d]),
        "orc_deemp_process": (i, [vp, vp, i, vp]),
        "orc_deemp_destroy": (None, [vp]),
        "orc_zoom": (i, [vp, i, d, d, d, i, vp]),
        "orc_colormap": (None, [vp, ctypes.c_long, ctypes.c_float, ctypes.c_float, vp, i, vp]),
        "orc_fft_smooth_hold": (None, [vp, i, i, i, ctypes.c_float, ctypes.c_float, vp, i, ctypes.c_float, vp]),
        "orc_vfo_signal_info": (None, [vp, i, d, d, d, vp, vp]),
        "orc_ddcfm_create": (vp, [d, vp, i, i, d, i]),
        "orc_ddcfm_process": (i, [vp, vp, i, vp]),
        "orc_ddcfm_destroy": (None, [vp]),
        "orc_wav_encode": (i, [i, vp, i, vp]),
        "orc_chain_create": (vp, [d, i, d, i]),
        "orc_chain_process": (l, [vp, vp, l, vp, l, vp]),
        "orc_chain_destroy": (None, [vp]),
        "cf_chan_fir": (None, [vp, vp, i, i, i, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()
F32, C64 = 0, 1


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def create_window(wtype, size, centered=True):
    w = np.empty(size, dtype=np.float32)
    lib.orc_create_window(int(wtype), _p(w), int(size), int(centered))
    return w


def _taps(fn, *args):
    n = fn(*args, None)
    t = np.empty(n, dtype=np.float32)
    fn(*args, _p(t))
    return t


def windowed_sinc(count, omega, norm=1.0):
    """taps/windowed_sinc.h:9-35 with window::nuttall (float taps)."""
    out = np.empty(count, np.float32)
    lib.orc_windowed_sinc(int(count), float(omega), float(norm), _p(out))
    return out


def channelize(x, h, M, chans):
    """C4 definition: channel k = exact-NCO xlator(-k fs/M) -> DecimatingFIR(h, M), fp64.
    Returns complex128 [len(chans), ceil(len(x)/M)]."""
    x = np.ascontiguousarray(x, np.complex64)
    h = np.ascontiguousarray(h, np.float32)
    ch = np.ascontiguousarray(chans, np.int32)
    frames = (len(x) + M - 1) // M
    out = np.zeros((len(ch), frames), np.complex128)
    rc = lib.orc_channelize(_p(x), len(x), _p(h), len(h), int(M), _p(ch), len(ch), _p(out))
    assert rc == frames
    return out


def chan_branch_fir(x, h, frames, out=None):
    """CPU-baseline kernel (cpu_fast.c): the channelizer's branch FIRs u[f][m] = sum_q h[q][m] x[f+q][m]
    over x [frames + Q - 1][M] complex64 and h [Q][M] float32 -> u [frames][M] complex64."""
    Q, M = h.shape
    if out is None:
        out = np.empty((frames, M), np.complex64)
    lib.cf_chan_fir(_p(x), _p(h), int(M), int(Q), int(frames), _p(out))
    return out


def low_pass(cutoff, trans, fs, odd=False):
    return _taps(lib.orc_low_pass, float(cutoff), float(trans), float(fs), int(odd))


def high_pass(cutoff, trans, fs, odd=False):
    return _taps(lib.orc_high_pass, float(cutoff), float(trans), float(fs), int(odd))


def band_pass(start, stop, trans, fs, odd=False, complex_taps=False):
    if complex_taps:
        n = lib.orc_band_pass_c(float(start), float(stop), float(trans), float(fs), int(odd), None)
        t = np.empty(n, dtype=np.complex64)
        lib.orc_band_pass_c(float(start), float(stop), float(trans), float(fs), int(odd), _p(t))
        return t
    return _taps(lib.orc_band_pass_f, float(start), float(stop), float(trans), float(fs), int(odd))


def decim_plan(ratio):
    d = np.zeros(8, dtype=np.int32)
    n = np.zeros(8, dtype=np.int32)
    t = (ctypes.c_void_p * 8)()
    ns = lib.orc_decim_plan(int(ratio), _p(d), _p(n), ctypes.cast(t, ctypes.c_void_p))
    out = []
    for s in range(ns):
        arr = (ctypes.c_float * int(n[s])).from_address(t[s])
        out.append((int(d[s]), np.array(arr, dtype=np.float32)))
    return out


def gen_reshape_params(fs, size, rate):
    skip, nz = ctypes.c_int(), ctypes.c_int()
    lib.orc_gen_reshape_params(float(fs), int(size), float(rate), ctypes.byref(skip), ctypes.byref(nz))
    return skip.value, nz.value


def convert(kind, x):
    x = np.ascontiguousarray(x)
    fns = [lib.orc_u8_to_f32, lib.orc_i16_to_f32, lib.orc_i24_to_f32, lib.orc_i32_to_f32, lib.orc_f64_to_f32,
           lib.orc_i8_to_f32]
    n = x.size if kind != 2 else x.size // 3
    out = np.empty(n, dtype=np.float32)
    fns[kind](_p(x), _p(out), n)
    return out


def fft_logmag(x, nz, N, window):
    x = np.ascontiguousarray(x, dtype=np.complex64)
    w = np.ascontiguousarray(window, dtype=np.float32)
    work = np.empty(4 * N, dtype=np.float32)
    out = np.empty(N, dtype=np.float32)
    lib.orc_fft_logmag(_p(x), int(nz), int(N), _p(w), _p(work), _p(out))
    return out


def fft_truth_power(x, nz, N, window):
    """fp64 truth: |DFT(x*w)|^2 with the window product rounded to float as the reference does."""
    xw = (np.asarray(x[:nz], dtype=np.complex64) * np.asarray(window, dtype=np.float32)).astype(np.complex64)
    buf = np.zeros(N, dtype=np.complex128)
    buf[:nz] = xw
    X = np.fft.fft(buf)
    return X.real ** 2 + X.imag ** 2


class _Obj:
    _destroy = None

    def __init__(self, h, in_dt, out_dt, ratio_hint=1.0):
        self._h = h
        self.in_dt, self.out_dt = in_dt, out_dt
        self.ratio_hint = ratio_hint

    def process(self, x, fn):
        x = np.ascontiguousarray(x, dtype=self.in_dt)
        n = x.shape[0]
        cap = int(n * max(self.ratio_hint, 1.0)) + 64
        out = np.empty(cap, dtype=self.out_dt)
        m = fn(self._h, _p(x), n, _p(out))
        return out[:m]

    def __del__(self):
        try:
            if self._h and self._destroy:
                type(self)._destroy(self._h)
        except Exception:
            pass


class FIR(_Obj):
    _destroy = lib.orc_fir_destroy

    def __init__(self, taps, decim=1, complex_data=True, precise=True):
        t = np.ascontiguousarray(taps)
        ttype = C64 if np.iscomplexobj(t) else F32
        t = t.astype(np.complex64 if ttype == C64 else np.float32)
        dt = np.complex64 if complex_data else np.float32
        super().__init__(lib.orc_fir_create(C64 if complex_data else F32, ttype, _p(t), t.shape[0], int(decim),
                                            int(precise)), dt, dt)

    def process(self, x):
        return super().process(x, lib.orc_fir_process)

    def reset(self):
        lib.orc_fir_reset(self._h)

    def set_taps(self, taps):
        t = np.ascontiguousarray(taps)
        t = t.astype(np.complex64 if np.iscomplexobj(t) else np.float32)
        lib.orc_fir_set_taps(self._h, _p(t), t.shape[0])


class Xlator(_Obj):
    _destroy = lib.orc_xlator_destroy

    def __init__(self, offset_rad):
        super().__init__(lib.orc_xlator_create(float(offset_rad)), np.complex64, np.complex64)

    def process(self, x):
        return super().process(x, lib.orc_xlator_process)

    def set_offset(self, offset_rad):
        lib.orc_xlator_set_offset(self._h, float(offset_rad))


class Quadrature(_Obj):
    _destroy = lib.orc_quad_destroy

    def __init__(self, deviation_rad):
        super().__init__(lib.orc_quad_create(float(deviation_rad)), np.complex64, np.float32)

    def process(self, x):
        return super().process(x, lib.orc_quad_process)


class PowerDecimator(_Obj):
    _destroy = lib.orc_pdec_destroy

    def __init__(self, ratio, complex_data=True, precise=True):
        dt = np.complex64 if complex_data else np.float32
        super().__init__(lib.orc_pdec_create(C64 if complex_data else F32, int(ratio), int(precise)), dt, dt)

    def process(self, x):
        return super().process(x, lib.orc_pdec_process)


class PolyphaseResampler(_Obj):
    _destroy = lib.orc_poly_destroy

    def __init__(self, interp, decim, taps, complex_data=True, precise=True):
        t = np.ascontiguousarray(taps, dtype=np.float32)
        dt = np.complex64 if complex_data else np.float32
        super().__init__(lib.orc_poly_create(C64 if complex_data else F32, int(interp), int(decim), _p(t), t.shape[0],
                                             int(precise)), dt, dt, ratio_hint=interp / decim)

    def process(self, x):
        return super().process(x, lib.orc_poly_process)


class RationalResampler(_Obj):
    _destroy = lib.orc_rres_destroy

    def __init__(self, in_sr, out_sr, complex_data=True, precise=True):
        dt = np.complex64 if complex_data else np.float32
        super().__init__(lib.orc_rres_create(C64 if complex_data else F32, float(in_sr), float(out_sr), int(precise)),
                         dt, dt, ratio_hint=out_sr / in_sr)

    def process(self, x):
        return super().process(x, lib.orc_rres_process)

    def info(self):
        v = [ctypes.c_int() for _ in range(5)]
        lib.orc_rres_info(self._h, *[ctypes.byref(x) for x in v])
        return dict(zip(["mode", "predec", "interp", "decim", "ntaps"], [x.value for x in v]))


class RxVFO(_Obj):
    _destroy = lib.orc_vfo_destroy

    def __init__(self, in_sr, out_sr, bw, offset, precise=True):
        super().__init__(lib.orc_vfo_create(float(in_sr), float(out_sr), float(bw), float(offset), int(precise)),
                         np.complex64, np.complex64, ratio_hint=max(out_sr / in_sr, 1.0))

    def process(self, x):
        return super().process(x, lib.orc_vfo_process)


STEREO = np.dtype([("l", np.float32), ("r", np.float32)])


class BroadcastFM(_Obj):
    _destroy = lib.orc_wfm_destroy

    def __init__(self, deviation, samplerate, low_pass=True, precise=True):
        super().__init__(lib.orc_wfm_create(float(deviation), float(samplerate), int(low_pass), int(precise)),
                         np.complex64, STEREO)

    def process(self, x):
        return super().process(x, lib.orc_wfm_process)


class BroadcastFMStereo(_Obj):
    """demod/broadcast_fm.h with the stereo decoder (pilot BPF -> PLL -> L+R / L-R matrix)."""
    _destroy = lib.orc_wfms_destroy

    def __init__(self, deviation, samplerate, stereo=True, low_pass=True, precise=True):
        super().__init__(lib.orc_wfms_create(float(deviation), float(samplerate), int(stereo), int(low_pass), int(precise)),
                         np.complex64, STEREO)

    def process(self, x):
        return super().process(x, lib.orc_wfms_process)


class DDCFM(_Obj):
    """C3: FrequencyXlator -> DecimatingFIR<complex_t,float> -> Quadrature (precise=False: the
    VOLK-style fp32 CPU path used as the CPU baseline)."""
    _destroy = lib.orc_ddcfm_destroy

    def __init__(self, offset_rad, taps, decim, deviation_rad, precise=False):
        self._t = np.ascontiguousarray(taps, np.float32)
        super().__init__(lib.orc_ddcfm_create(float(offset_rad), _p(self._t), len(self._t), int(decim), float(deviation_rad),
                                              int(precise)), np.complex64, np.float32, 1.0 / decim)

    def process(self, x):
        return super().process(x, lib.orc_ddcfm_process)


class Deemphasis(_Obj):
    """filter/deephasis.h (stereo=True: stereo_t pairs)."""
    _destroy = lib.orc_deemp_destroy

    def __init__(self, tau, samplerate, stereo=False):
        dt = STEREO if stereo else np.float32
        super().__init__(lib.orc_deemp_create(2 if stereo else 1, float(tau), float(samplerate)), dt, dt)

    def process(self, x):
        return super().process(x, lib.orc_deemp_process)


def zoom(row, view_offset, view_bw, whole_bw, out_size):
    """gui/widgets/fft_scaler.h doZoom of one spectrum row."""
    row = np.ascontiguousarray(row, np.float32)
    out = np.empty(out_size, np.float32)
    lib.orc_zoom(_p(row), len(row), float(view_offset), float(view_bw), float(whole_bw), int(out_size), _p(out))
    return out


def colormap(x, wf_min, wf_max, pallet):
    """waterfall.cpp:903-910: dB -> pallet entries."""
    x = np.ascontiguousarray(x, np.float32)
    pallet = np.ascontiguousarray(pallet, np.uint32)
    out = np.empty(x.shape, np.uint32)
    lib.orc_colormap(_p(x), x.size, float(wf_min), float(wf_max), _p(pallet), len(pallet), _p(out))
    return out


def fft_smooth_hold(rows, smoothing, alpha, beta, smooth, hold_on, hold_speed, hold):
    """waterfall.cpp:918-925, 952-957 over consecutive rows; returns (rows, smooth, hold) updated."""
    rows = np.array(rows, np.float32, copy=True, order="C")
    smooth = np.array(smooth, np.float32, copy=True)
    hold = np.array(hold, np.float32, copy=True)
    lib.orc_fft_smooth_hold(_p(rows), rows.shape[0], rows.shape[1], int(smoothing), float(alpha), float(beta), _p(smooth),
                            int(hold_on), float(hold_speed), _p(hold))
    return rows, smooth, hold


def vfo_signal_info(line, whole_bw, center_offset, bandwidth):
    """WaterFall::calculateVFOSignalInfo (waterfall.cpp:563-601) -> (strength, snr)."""
    line = np.ascontiguousarray(line, np.float32)
    st, sn = ctypes.c_float(), ctypes.c_float()
    lib.orc_vfo_signal_info(_p(line), len(line), float(whole_bw), float(center_offset), float(bandwidth),
                            ctypes.byref(st), ctypes.byref(sn))
    return st.value, sn.value


def compress(pcm_type, x):
    """compression/sample_stream_compressor.h: bytes of one block."""
    x = np.ascontiguousarray(x, np.complex64)
    out = np.empty(8 + 8 * len(x), np.uint8)
    n = lib.orc_compress(int(pcm_type), _p(x), len(x), _p(out))
    return out[:n]


def wav_encode(kind, x):
    """utils/wav.cpp:296-336 recorder encoders: kind 0 u8, 1 i16, 2 i24, 3 i32, 4 f32 -> bytes."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    out = np.empty(4 * len(x) + 4, np.uint8)
    n = lib.orc_wav_encode(int(kind), _p(x), len(x), _p(out))
    return out[:n]


def decompress(buf):
    buf = np.ascontiguousarray(buf, np.uint8)
    out = np.empty(max(len(buf) // 2, 1), np.complex64)
    n = lib.orc_decompress(_p(buf), len(buf), _p(out))
    return out[:n]


class FM(_Obj):
    _destroy = lib.orc_fm_destroy

    def __init__(self, samplerate, bandwidth, low_pass=True, high_pass=False, precise=True):
        super().__init__(lib.orc_fm_create(float(samplerate), float(bandwidth), int(low_pass), int(high_pass),
                                           int(precise)), np.complex64, np.float32)

    def process(self, x):
        return super().process(x, lib.orc_fm_process)


class AGC(_Obj):
    _destroy = lib.orc_agc_destroy

    def __init__(self, complex_data, set_point, attack, decay, max_gain, max_out, init_gain=1.0):
        dt = np.complex64 if complex_data else np.float32
        super().__init__(lib.orc_agc_create(C64 if complex_data else F32, set_point, attack, decay, max_gain, max_out,
                                            init_gain), dt, dt)

    def process(self, x):
        return super().process(x, lib.orc_agc_process)

    def set_enabled(self, en):
        lib.orc_agc_set_enabled(self._h, int(bool(en)))

    def set_gain(self, g):
        lib.orc_agc_set_gain(self._h, float(g))

    def get_gain(self):
        return lib.orc_agc_get_gain(self._h)


class DCBlocker(_Obj):
    """correction/dc_blocker.h:54-60"""
    _destroy = lib.orc_dcb_destroy

    def __init__(self, rate, complex_data=False):
        dt = np.complex64 if complex_data else np.float32
        super().__init__(lib.orc_dcb_create(C64 if complex_data else F32, float(rate)), dt, dt)

    def process(self, x):
        return super().process(x, lib.orc_dcb_process)


class AM(_Obj):
    _destroy = lib.orc_am_destroy

    def __init__(self, agc_mode, bandwidth, attack, decay, dc_rate, samplerate, precise=True):
        super().__init__(lib.orc_am_create(int(agc_mode), bandwidth, attack, decay, dc_rate, samplerate, int(precise)),
                         np.complex64, np.float32)

    def process(self, x):
        return super().process(x, lib.orc_am_process)


class SSB(_Obj):
    _destroy = lib.orc_ssb_destroy

    def __init__(self, mode, bandwidth, samplerate, agc, attack, decay):
        super().__init__(lib.orc_ssb_create(int(mode), bandwidth, samplerate, int(agc), attack, decay),
                         np.complex64, np.float32)

    def process(self, x):
        return super().process(x, lib.orc_ssb_process)


class Chain(_Obj):
    """C5 per-stream chain (CPU baseline): 64k BH7 spectra + RxVFO + BroadcastFM mono."""
    _destroy = lib.orc_chain_destroy

    def __init__(self, fs, fft_size, vfo_offset, precise=False):
        super().__init__(lib.orc_chain_create(float(fs), int(fft_size), float(vfo_offset), int(precise)),
                         np.complex64, STEREO)
        self.N = fft_size

    def process(self, x, spectra=None):
        x = np.ascontiguousarray(x, dtype=np.complex64)
        audio = np.empty(x.shape[0] // 200 + 64, dtype=STEREO)
        sp = spectra if spectra is not None else np.empty((0, self.N), dtype=np.float32)
        m = lib.orc_chain_process(self._h, _p(x), x.shape[0], _p(sp) if sp.size else None, sp.shape[0], _p(audio))
        return audio[:m]
