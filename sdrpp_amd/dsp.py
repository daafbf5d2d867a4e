"""Python-side handles over the libsdrgpu C ABI, named after the reference blocks.

Each class mirrors one ``dsp::`` block of the reference (file:line in the C
header ``include/sdrgpu.h``): ``process(x)`` is the reference's
``process(count, in, out) -> outCount`` on host numpy buffers (synchronous,
staged through pinned memory), ``process_dev(in_ptr, count, out_ptr, stream)``
runs on device-resident buffers (torch tensors' ``data_ptr()``) on a caller
stream and returns the output count without synchronising.
"""
import ctypes

import numpy as np

from . import lib, check, F32, C64

_vp = ctypes.c_void_p


def _fptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _taps_arg(taps):
    t = np.ascontiguousarray(taps)
    if np.iscomplexobj(t):
        t = t.astype(np.complex64)
        return t, C64
    return t.astype(np.float32), F32


class Block:
    """Owns one sdrgpu_block handle."""

    def __init__(self, handle, in_dtype, out_dtype):
        self._h = handle
        self.in_dtype = in_dtype      # numpy dtype of one input element
        self.out_dtype = out_dtype

    def out_count(self, count):
        return check(lib.sdrgpu_block_out_count(self._h, int(count)))

    def process(self, x):
        x = np.ascontiguousarray(x, dtype=self.in_dtype)
        n = x.shape[0]
        out = np.empty(max(self.out_count(n), 1), dtype=self.out_dtype)
        m = check(lib.sdrgpu_block_process(self._h, _fptr(x), n, _fptr(out)))
        return out[:m]

    def process_dev(self, in_ptr, count, out_ptr, stream=None):
        return check(lib.sdrgpu_block_process_dev(self._h, _vp(in_ptr), int(count), _vp(out_ptr), _vp(stream or 0)))

    def reset(self):
        check(lib.sdrgpu_block_reset(self._h))

    def close(self):
        if self._h:
            lib.sdrgpu_block_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _make(fn, *args):
    h = ctypes.c_void_p()
    check(fn(ctypes.byref(h), *args))
    return h


STEREO = np.dtype([("l", np.float32), ("r", np.float32)])


class FrequencyXlator(Block):
    """dsp::channel::FrequencyXlator (channel/frequency_xlator.h:15-50); offset in rad/sample."""

    def __init__(self, offset_rad, device=0):
        super().__init__(_make(lib.sdrgpu_xlator_create, device, float(offset_rad)), np.complex64, np.complex64)

    def set_offset(self, offset_rad):
        check(lib.sdrgpu_xlator_set_offset(self._h, float(offset_rad)))


class FIR(Block):
    """dsp::filter::FIR<D,T> (filter/fir.h) / DecimatingFIR<D,T> (filter/decimating_fir.h)."""

    def __init__(self, taps, decim=1, complex_data=True, device=0):
        t, ttype = _taps_arg(taps)
        dtype = C64 if complex_data else F32
        self._taps = t
        h = _make(lib.sdrgpu_fir_create, device, dtype, ttype, _fptr(t), int(t.shape[0]), int(decim))
        npd = np.complex64 if complex_data else np.float32
        super().__init__(h, npd, npd)

    def set_taps(self, taps):
        t, _ = _taps_arg(taps)
        self._taps = t
        check(lib.sdrgpu_fir_set_taps(self._h, _fptr(t), int(t.shape[0])))

    def set_decimation(self, decim):
        check(lib.sdrgpu_fir_set_decimation(self._h, int(decim)))


def DecimatingFIR(taps, decim, complex_data=True, device=0):
    return FIR(taps, decim, complex_data, device)


class Quadrature(Block):
    """dsp::demod::Quadrature (demod/quadrature.h:41-56); deviation in rad/sample."""

    def __init__(self, deviation_rad, device=0):
        super().__init__(_make(lib.sdrgpu_quadrature_create, device, float(deviation_rad)), np.complex64, np.float32)


class PowerDecimator(Block):
    """dsp::multirate::PowerDecimator<T> (multirate/power_decimator.h)."""

    def __init__(self, ratio, complex_data=True, device=0):
        npd = np.complex64 if complex_data else np.float32
        super().__init__(_make(lib.sdrgpu_power_decimator_create, device, C64 if complex_data else F32, int(ratio)), npd, npd)


class PolyphaseResampler(Block):
    """dsp::multirate::PolyphaseResampler<T> (multirate/polyphase_resampler.h)."""

    def __init__(self, interp, decim, taps, complex_data=True, device=0):
        t = np.ascontiguousarray(taps, dtype=np.float32)
        npd = np.complex64 if complex_data else np.float32
        h = _make(lib.sdrgpu_polyphase_resampler_create, device, C64 if complex_data else F32, int(interp), int(decim),
                  _fptr(t), int(t.shape[0]))
        super().__init__(h, npd, npd)


class RationalResampler(Block):
    """dsp::multirate::RationalResampler<T> (multirate/rational_resampler.h)."""

    def __init__(self, in_sr, out_sr, complex_data=True, device=0):
        npd = np.complex64 if complex_data else np.float32
        h = _make(lib.sdrgpu_rational_resampler_create, device, C64 if complex_data else F32, float(in_sr), float(out_sr))
        super().__init__(h, npd, npd)


class RxVFO(Block):
    """dsp::channel::RxVFO (channel/rx_vfo.h)."""

    def __init__(self, in_sr, out_sr, bandwidth, offset, device=0):
        h = _make(lib.sdrgpu_rxvfo_create, device, float(in_sr), float(out_sr), float(bandwidth), float(offset))
        super().__init__(h, np.complex64, np.complex64)

    def set_offset(self, offset):
        check(lib.sdrgpu_rxvfo_set_offset(self._h, float(offset)))


class DDC(Block):
    """Fused FrequencyXlator -> DecimatingFIR<complex_t,float> (complex out): the FIR stage of DDCFM."""

    def __init__(self, offset_rad, taps, decim, device=0):
        t = np.ascontiguousarray(taps, dtype=np.float32)
        self._taps = t
        h = _make(lib.sdrgpu_ddc_create, device, float(offset_rad), _fptr(t), int(t.shape[0]), int(decim))
        super().__init__(h, np.complex64, np.complex64)


class DDCFM(Block):
    """Fused FrequencyXlator -> DecimatingFIR<complex_t,float> -> Quadrature (BASELINE config C3)."""

    def __init__(self, offset_rad, taps, decim, deviation_rad, device=0):
        t = np.ascontiguousarray(taps, dtype=np.float32)
        self._taps = t
        h = _make(lib.sdrgpu_ddc_fm_create, device, float(offset_rad), _fptr(t), int(t.shape[0]), int(decim),
                  float(deviation_rad))
        super().__init__(h, np.complex64, np.float32)


class FM(Block):
    """dsp::demod::FM<float> (demod/fm.h)."""

    def __init__(self, samplerate, bandwidth, low_pass=True, high_pass=False, device=0):
        h = _make(lib.sdrgpu_fm_create, device, float(samplerate), float(bandwidth), int(low_pass), int(high_pass))
        super().__init__(h, np.complex64, np.float32)


class BroadcastFM(Block):
    """dsp::demod::BroadcastFM (demod/broadcast_fm.h:144-215); stereo_t out. stereo=False is
    the mono path (the C5 bench chain); stereo=True adds the pilot PLL stereo decoder."""

    def __init__(self, deviation, samplerate, low_pass=True, device=0, stereo=False, rds=False):
        if stereo or rds:   # the RDS branch lives in the full BroadcastFM block (mono or stereo)
            h = _make(lib.sdrgpu_broadcast_fm_create, device, float(deviation), float(samplerate), int(stereo),
                      int(low_pass))
        else:
            h = _make(lib.sdrgpu_wfm_create, device, float(deviation), float(samplerate), int(low_pass))
        super().__init__(h, np.complex64, STEREO)
        if rds:
            self.set_rds(True)

    def set_rds(self, enabled):
        """setRDSOut (broadcast_fm.h:121-127)."""
        check(lib.sdrgpu_broadcast_fm_set_rds(self._h, int(bool(enabled))))

    def rds_output(self):
        """RDS baseband (complex64, 5 kS/s) produced by the last process() call."""
        n = ctypes.c_int()
        check(lib.sdrgpu_broadcast_fm_rds_dev(self._h, None, ctypes.byref(n)))
        out = np.empty(n.value, np.complex64)
        if n.value:
            check(lib.sdrgpu_broadcast_fm_read_rds(self._h, _fptr(out), n.value))
        return out


class FFTSpectrum:
    """IQFrontEnd's FFT path (signal_path/iq_frontend.cpp:230-249, 272-296)."""

    def __init__(self, fft_size, nz=None, window=6, device=0, precision="f32"):
        """precision "f64": the fp64-interior parity mode (sdrgpu_fft_set_precision(h, 1))."""
        self.N = int(fft_size)
        self.nz = int(nz if nz is not None else fft_size)
        self._h = _make(lib.sdrgpu_fft_create, device, self.N, self.nz, int(window))
        if precision != "f32":
            self.set_precision(precision)

    def set_precision(self, precision):
        check(lib.sdrgpu_fft_set_precision(self._h, {"f32": 0, "f64": 1}[precision]))

    def set_tail_stream(self, stream):
        """sdrgpu_fft_set_tail_stream: the fused VFO's later stages and the zoom fold of
        execute_zoom_vfo_dev on `stream` (a HIP stream handle, or 0 / None to turn it off)."""
        check(lib.sdrgpu_fft_set_tail_stream(self._h, stream or None))

    def set_kernel(self, mode):
        """64k transform form (sdrgpu_fft_set_kernel): "two-pass", "one-pass" or "auto" (per call size,
        the default). Returns the previous mode's name."""
        names = ("two-pass", "one-pass", "auto")
        return names[check(lib.sdrgpu_fft_set_kernel(self._h, names.index(mode)))]

    @property
    def precision(self):
        return ("f32", "f64")[check(lib.sdrgpu_fft_get_precision(self._h))]

    def set_window(self, w):
        w = np.ascontiguousarray(w, dtype=np.float32)
        check(lib.sdrgpu_fft_set_window(self._h, _fptr(w), int(w.shape[0])))
        self.nz = int(w.shape[0])

    def logmag(self, x):
        """Host drop-in: x = complex64[nz] -> float32[N] dB."""
        x = np.ascontiguousarray(x, dtype=np.complex64)
        assert x.shape[0] >= self.nz
        out = np.empty(self.N, dtype=np.float32)
        check(lib.sdrgpu_fft_logmag(self._h, _fptr(x), _fptr(out)))
        return out

    def execute_dev(self, in_ptr, frame_stride, frames, out_ptr, stream=None):
        return check(lib.sdrgpu_fft_execute_dev(self._h, _vp(in_ptr), int(frame_stride), int(frames), _vp(out_ptr),
                                                _vp(stream or 0)))

    def execute_zoom_dev(self, in_ptr, frame_stride, frames, out_ptr, zoom_ptr, zoom_size, stream=None):
        """dB rows + the waterfall's full-span zoom rows (frames x zoom_size; fused at 64k / 2048)."""
        return check(lib.sdrgpu_fft_execute_zoom_dev(self._h, _vp(in_ptr), int(frame_stride), int(frames), _vp(out_ptr),
                                                     _vp(zoom_ptr), int(zoom_size), _vp(stream or 0)))

    def execute_vfo_dev(self, in_ptr, frames, out_ptr, vfo, vfo_out_ptr, stream=None):
        """Spectra of `frames` back-to-back frames + one RxVFO over the same device batch (the VFO's
        first stage fused into the 64k spectrum's input pass); returns the VFO's output count."""
        return check(lib.sdrgpu_fft_execute_vfo_dev(self._h, _vp(in_ptr), int(frames), _vp(out_ptr), vfo._h,
                                                    _vp(vfo_out_ptr), _vp(stream or 0)))

    def execute_zoom_vfo_dev(self, in_ptr, frames, out_ptr, zoom_ptr, zoom_size, vfo, vfo_out_ptr, stream=None):
        """Spectra (+ zoom rows when zoom_ptr) + one RxVFO over `frames` back-to-back frames; the VFO's
        first stage runs inside the spectrum launches where the plan allows. Returns the VFO's output count."""
        return check(lib.sdrgpu_fft_execute_zoom_vfo_dev(self._h, _vp(in_ptr), int(frames), _vp(out_ptr), _vp(zoom_ptr or 0),
                                                         int(zoom_size), vfo._h, _vp(vfo_out_ptr), _vp(stream or 0)))

    def set_timing(self, on=True):
        check(lib.sdrgpu_fft_set_timing(self._h, int(bool(on))))

    def group_times(self, n=256):
        """ms of the spectrum launch group of the last n timed calls (waits for them)."""
        ms = np.zeros(n, dtype=np.float32)
        k = check(lib.sdrgpu_fft_group_times(self._h, _fptr(ms), int(n)))
        return ms[:k]

    def close(self):
        if self._h:
            lib.sdrgpu_fft_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def convert(kind, x, device=0):
    """file_source / rtl_sdr / hackrf ingest converters on the GPU (host buffers)."""
    x = np.ascontiguousarray(x)
    n = x.size if kind != 2 else x.size // 3
    out = np.empty(n, dtype=np.float32)
    check(lib.sdrgpu_convert(device, int(kind), _fptr(x), n, _fptr(out)))
    return out


def convert_mono(kind, x, device=0):
    """One-channel file_source ingest (main.cpp:294-430): n samples -> complex64 with I = Q."""
    x = np.ascontiguousarray(x)
    n = x.size if kind != 2 else x.size // 3
    out = np.empty(n, dtype=np.complex64)
    check(lib.sdrgpu_convert_mono(device, int(kind), _fptr(x), n, _fptr(out)))
    return out


_CONV_BYTES = (1, 2, 3, 4, 8, 1, 4)
_CONV_VIEW = (np.uint8, np.int16, np.uint8, np.int32, np.float64, np.int8, np.float32)   # (i24: packed bytes)


class WavFile:
    """file_source's WavReader (C++ in libsdrgpu: sdrgpu_wav_*, wavreader.h:34-226) with the
    worker's framing: ``read()`` returns the next raw block of block_size frames (fs / 200), as
    bytes, and ``samples(block)`` converts it on the GPU to complex64 exactly as worker_1ch /
    worker_2ch do (main.cpp:294-560)."""

    def __init__(self, path, device=0):
        self._h = _make(lib.sdrgpu_wav_open, str(path).encode())
        f, c, b, sr, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_double(), ctypes.c_longlong()
        check(lib.sdrgpu_wav_info(self._h, ctypes.byref(f), ctypes.byref(c), ctypes.byref(b), ctypes.byref(sr),
                                  ctypes.byref(n)))
        self.format, self.channels, self.bits = f.value, c.value, b.value
        self.sample_rate, self.sample_count = sr.value, n.value
        self.device = device
        self.kind = check(lib.sdrgpu_wav_kind(self._h))
        self.block_size = check(lib.sdrgpu_wav_block_size(self._h))
        self.frame_bytes = self.channels * _CONV_BYTES[self.kind]

    def read(self, max_frames=None):
        n = self.block_size if max_frames is None else int(max_frames)
        buf = np.empty(n * self.frame_bytes, np.uint8)
        got = check(lib.sdrgpu_wav_read(self._h, _fptr(buf), n))
        return buf[:got * self.frame_bytes]

    def samples(self, raw):
        if raw.size == 0:
            return np.empty(0, np.complex64)
        typed = raw.view(_CONV_VIEW[self.kind])
        if self.channels == 1:
            return convert_mono(self.kind, typed, self.device)
        return convert(self.kind, typed, self.device).view(np.complex64)

    def blocks(self):
        while True:
            raw = self.read()
            if raw.size == 0:
                return
            yield raw

    def seek(self, frame):
        check(lib.sdrgpu_wav_seek(self._h, int(frame)))

    def close(self):
        if self._h:
            lib.sdrgpu_wav_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- host-side design functions (no GPU) ----------------------------------
def create_window(wtype, size, centered=True):
    w = np.empty(size, dtype=np.float32)
    check(lib.sdrgpu_create_window(int(wtype), _fptr(w), int(size), int(centered)))
    return w


def _taps(fn, *args):
    n = check(fn(*args, None))
    t = np.empty(n, dtype=np.float32)
    fn(*args, _fptr(t))
    return t


def windowed_sinc(count, omega, norm=1.0):
    """taps::windowedSinc<float>(count, omega, window::nuttall, norm) (taps/windowed_sinc.h:9)."""
    out = np.empty(int(count), np.float32)
    check(lib.sdrgpu_taps_windowed_sinc(int(count), float(omega), float(norm), _fptr(out)))
    return out


class PolyphaseChannelizer(Block):
    """M-channel critically sampled polyphase channelizer (BASELINE C4): channel k of frame m is
    FrequencyXlator(-k fs/M) -> DecimatingFIR(taps, M) with an exact NCO. ``process`` returns
    complex64 [frames * M] laid out out[m * M + k]. ``dft="gemm"`` (M = 1024) computes each
    frame's DFT as two complex 32x32 matrix products on the f32 matrix cores instead of the LDS
    FFT (sdrgpu_channelizer_set_dft)."""

    def __init__(self, channels, taps, device=0, dft="fft"):
        t = np.ascontiguousarray(taps, np.float32)
        self._taps = t
        self.channels = int(channels)
        h = _make(lib.sdrgpu_channelizer_create, device, int(channels), _fptr(t), int(t.shape[0]))
        super().__init__(h, np.complex64, np.complex64)
        if dft not in ("fft", "gemm"):
            raise ValueError(f"dft must be 'fft' or 'gemm', not {dft!r}")
        check(lib.sdrgpu_channelizer_set_dft(self._h, 1 if dft == "gemm" else 0))


class AGC(Block):
    """dsp::loop::AGC<T> (loop/agc.h); complex_data selects T = complex_t (else float)."""

    def __init__(self, set_point, attack, decay, max_gain, max_output_amp, init_gain=1.0, complex_data=False, device=0):
        dt = C64 if complex_data else F32
        h = _make(lib.sdrgpu_agc_create, device, dt, float(set_point), float(attack), float(decay), float(max_gain),
                  float(max_output_amp), float(init_gain))
        npd = np.complex64 if complex_data else np.float32
        super().__init__(h, npd, npd)

    def set_enabled(self, enabled):
        check(lib.sdrgpu_agc_set_enabled(self._h, int(bool(enabled))))

    def set_gain(self, gain):
        check(lib.sdrgpu_agc_set_gain(self._h, float(gain)))

    def get_gain(self):
        g = ctypes.c_float()
        check(lib.sdrgpu_agc_get_gain(self._h, ctypes.byref(g)))
        return g.value


class DCBlocker(Block):
    """dsp::correction::DCBlocker<T> (correction/dc_blocker.h); rate in 1/sample."""

    def __init__(self, rate, complex_data=False, device=0):
        dt = C64 if complex_data else F32
        npd = np.complex64 if complex_data else np.float32
        super().__init__(_make(lib.sdrgpu_dc_blocker_create, device, dt, float(rate)), npd, npd)


class AM(Block):
    """dsp::demod::AM<T> (demod/am.h); agc_mode 0 OFF, 1 CARRIER, 2 AUDIO."""

    def __init__(self, agc_mode, bandwidth, attack, decay, dc_rate, samplerate, stereo=False, device=0):
        h = _make(lib.sdrgpu_am_create, device, int(agc_mode), float(bandwidth), float(attack), float(decay),
                  float(dc_rate), float(samplerate), int(bool(stereo)))
        super().__init__(h, np.complex64, STEREO if stereo else np.float32)


class SSB(Block):
    """dsp::demod::SSB<T> (demod/ssb.h); mode 0 USB, 1 LSB, 2 DSB."""

    def __init__(self, mode, bandwidth, samplerate, agc_enabled, attack, decay, stereo=False, device=0):
        h = _make(lib.sdrgpu_ssb_create, device, int(mode), float(bandwidth), float(samplerate), int(bool(agc_enabled)),
                  float(attack), float(decay), int(bool(stereo)))
        super().__init__(h, np.complex64, STEREO if stereo else np.float32)


class IQFrontEnd:
    """Device IQ front end (signal_path/iq_frontend.cpp; include/sdrgpu.h sdrgpu_frontend_*):
    ingest conversion -> [decimation] -> [DC block] -> [IQ inversion] -> VFOs + spectrum rows.
    ``push(block, kind=-1)`` takes a host block (complex64, or raw interleaved samples of a
    SDRGPU_CONV_* kind) and returns the dB rows completed by it; ``vfo_output(id)`` is that
    VFO's output for the block."""

    def __init__(self, sample_rate, decim=1, dc_blocking=False, fft_size=65536, fft_rate=15.0, window=6, device=0):
        self._h = _make(lib.sdrgpu_frontend_create, device, float(sample_rate), int(decim), int(bool(dc_blocking)),
                        int(fft_size), float(fft_rate), int(window))
        self.fft_size = int(fft_size)

    def framing(self):
        nz, skip, sr = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        check(lib.sdrgpu_frontend_framing(self._h, ctypes.byref(nz), ctypes.byref(skip), ctypes.byref(sr)))
        return nz.value, skip.value, sr.value

    def configure(self, sample_rate, decim=1, dc_blocking=False):
        check(lib.sdrgpu_frontend_configure(self._h, float(sample_rate), int(decim), int(bool(dc_blocking))))

    def set_invert_iq(self, enabled):
        check(lib.sdrgpu_frontend_set_invert_iq(self._h, int(bool(enabled))))

    def set_fft(self, fft_size, fft_rate, window=6):
        check(lib.sdrgpu_frontend_set_fft(self._h, int(fft_size), float(fft_rate), int(window)))
        self.fft_size = int(fft_size)

    def add_vfo(self, out_sr, bandwidth, offset):
        i = ctypes.c_int()
        check(lib.sdrgpu_frontend_add_vfo(self._h, ctypes.byref(i), float(out_sr), float(bandwidth), float(offset)))
        return i.value

    def remove_vfo(self, vid):
        check(lib.sdrgpu_frontend_remove_vfo(self._h, int(vid)))

    def set_vfo_offset(self, vid, offset):
        check(lib.sdrgpu_frontend_set_vfo_offset(self._h, int(vid), float(offset)))

    def push(self, block, kind=-1):
        a = np.ascontiguousarray(block)
        count = a.shape[0] if kind < 0 else a.size // 2
        nf = check(lib.sdrgpu_frontend_push(self._h, _fptr(a), int(count), int(kind)))
        rows = np.empty((nf, self.fft_size), np.float32)
        if nf:
            check(lib.sdrgpu_frontend_read_spectra(self._h, _fptr(rows), nf))
        return rows

    def push_dev(self, ptr, count, kind=-1, stream=None):
        return check(lib.sdrgpu_frontend_push_dev(self._h, _vp(ptr), int(count), int(kind), _vp(stream or 0)))

    # pipelined host call style (the C++ drop-in's worker): submit returns a ticket at once; collect
    # waits for it and copies its results out of the pinned result slot; at most two in flight
    def submit(self, block, kind=-1, want_iq=False, ptr=None, count=None):
        """Host block (numpy array, or `ptr`/`count` of host memory) -> ticket."""
        if ptr is None:
            a = np.ascontiguousarray(block)
            ptr, count = a.ctypes.data, (a.shape[0] if kind < 0 else a.size // 2)
        return check(lib.sdrgpu_frontend_submit(self._h, _vp(ptr), int(count), int(kind), 1 if want_iq else 0))

    def collect(self, ticket, vfos=(), copy=True):
        """(rows [nrows, N] float32, {vid: complex64 output}, iq complex64 or None) of a ticket; the
        ticket is released afterwards. copy=False only waits and releases (timing)."""
        rows_p, iq_p, niq = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int()
        nf = check(lib.sdrgpu_frontend_collect(self._h, int(ticket), ctypes.byref(rows_p), ctypes.byref(iq_p),
                                               ctypes.byref(niq)))
        rows, outs, iq = None, {}, None
        if copy:
            rows = np.empty((nf, self.fft_size), np.float32)
            if nf:
                ctypes.memmove(rows.ctypes.data, rows_p.value, rows.nbytes)
            for vid in vfos:
                p, n = ctypes.c_void_p(), ctypes.c_int()
                check(lib.sdrgpu_frontend_collected_vfo(self._h, int(ticket), int(vid), ctypes.byref(p), ctypes.byref(n)))
                o = np.empty(n.value, np.complex64)
                if n.value:
                    ctypes.memmove(o.ctypes.data, p.value, o.nbytes)
                outs[vid] = o
            if niq.value:
                iq = np.empty(niq.value, np.complex64)
                ctypes.memmove(iq.ctypes.data, iq_p.value, iq.nbytes)
        check(lib.sdrgpu_frontend_release(self._h, int(ticket)))
        return rows, outs, iq

    def vfo_dev(self, vid):
        """(device pointer, count) of the VFO's output for the last push."""
        ptr, n = ctypes.c_void_p(), ctypes.c_int()
        check(lib.sdrgpu_frontend_vfo_dev(self._h, int(vid), ctypes.byref(ptr), ctypes.byref(n)))
        return ptr.value, n.value

    def vfo_output(self, vid):
        n = ctypes.c_int()
        check(lib.sdrgpu_frontend_vfo_dev(self._h, int(vid), None, ctypes.byref(n)))
        out = np.empty(n.value, np.complex64)
        if n.value:
            check(lib.sdrgpu_frontend_read_vfo(self._h, int(vid), _fptr(out), n.value))
        return out

    def close(self):
        if self._h:
            lib.sdrgpu_frontend_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Deemphasis(Block):
    """dsp::filter::Deemphasis<T> (filter/deephasis.h); stereo=True for stereo_t."""

    def __init__(self, tau, samplerate, stereo=False, device=0):
        h = _make(lib.sdrgpu_deemphasis_create, device, C64 if stereo else F32, float(tau), float(samplerate))
        super().__init__(h, STEREO if stereo else np.float32, STEREO if stereo else np.float32)


def gather_id():
    """Rank 0: a new RCCL communicator id (bytes) for SpectraGather."""
    buf = ctypes.create_string_buffer(128)
    check(lib.sdrgpu_gather_get_id(buf))
    return buf.raw


class SpectraGather:
    """Rank-0 gather of spectrum rows over RCCL (sdrgpu_gather_*): one rank per GPU / IQ stream."""

    def __init__(self, rank, world, comm_id, device=0, timeout=None):
        """device < 0: the calling thread's current HIP device. Every wait on the peers (this
        constructor, gather_dev, wait) has a deadline: `timeout` s, else SDRGPU_GATHER_TIMEOUT_S
        (default 120); on expiry the communicator is aborted and SdrGpuError names the rank."""
        assert len(comm_id) == 128
        self.rank, self.world = rank, world
        self._id = ctypes.create_string_buffer(bytes(comm_id), 128)
        self._h = _make(lib.sdrgpu_gather_create, int(device), int(rank), int(world), self._id)
        if timeout is not None:
            check(lib.sdrgpu_gather_set_timeout(self._h, float(timeout)))

    def gather_dev(self, rows_ptr, count, out_ptr, stream=None):
        """count device floats -> rank 0's out (world x count); asynchronous on `stream`."""
        check(lib.sdrgpu_gather_rows(self._h, _vp(rows_ptr), int(count), _vp(out_ptr or 0), _vp(stream or 0)))

    def wait(self, stream=None, timeout=0.0):
        """Wait for the gathers enqueued on `stream` against the deadline (timeout <= 0: the
        handle's); raises SdrGpuError (communicator aborted) when a peer never completes its part."""
        check(lib.sdrgpu_gather_wait(self._h, _vp(stream or 0), float(timeout)))

    def close(self):
        if self._h:
            lib.sdrgpu_gather_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Zoom:
    """fft_scaler::doZoom on device dB rows (gui/widgets/fft_scaler.h)."""

    def __init__(self, view_offset, view_bw, whole_bw, fft_size, out_size, device=0):
        self._h = _make(lib.sdrgpu_zoom_create, device, float(view_offset), float(view_bw), float(whole_bw), int(fft_size),
                        int(out_size))
        self.out_size = int(out_size)

    def execute_dev(self, rows_ptr, nrows, out_ptr, stream=None):
        return check(lib.sdrgpu_zoom_execute_dev(self._h, _vp(rows_ptr), int(nrows), _vp(out_ptr), _vp(stream or 0)))

    def __del__(self):
        try:
            if self._h:
                lib.sdrgpu_zoom_destroy(self._h)
        except Exception:
            pass


def low_pass(cutoff, trans, fs, odd=False):
    return _taps(lib.sdrgpu_taps_low_pass, float(cutoff), float(trans), float(fs), int(odd))


def high_pass(cutoff, trans, fs, odd=False):
    return _taps(lib.sdrgpu_taps_high_pass, float(cutoff), float(trans), float(fs), int(odd))


def band_pass(start, stop, trans, fs, odd=False, complex_taps=False):
    if complex_taps:
        n = check(lib.sdrgpu_taps_band_pass_c(float(start), float(stop), float(trans), float(fs), int(odd), None))
        t = np.empty(n, dtype=np.complex64)
        lib.sdrgpu_taps_band_pass_c(float(start), float(stop), float(trans), float(fs), int(odd), _fptr(t))
        return t
    return _taps(lib.sdrgpu_taps_band_pass_f, float(start), float(stop), float(trans), float(fs), int(odd))


def gen_reshape_params(fs, size, rate):
    skip, nz = ctypes.c_int(), ctypes.c_int()
    lib.sdrgpu_gen_reshape_params(float(fs), int(size), float(rate), ctypes.byref(skip), ctypes.byref(nz))
    return skip.value, nz.value


def decim_plan(ratio):
    d = (ctypes.c_int * 8)()
    n = (ctypes.c_int * 8)()
    t = (ctypes.POINTER(ctypes.c_float) * 8)()
    ns = check(lib.sdrgpu_decim_plan(int(ratio), d, n, t))
    return [(d[i], np.ctypeslib.as_array(t[i], shape=(n[i],)).copy()) for i in range(ns)]
