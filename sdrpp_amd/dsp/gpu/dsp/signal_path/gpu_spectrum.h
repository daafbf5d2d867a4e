// GPU spectrum path for IQFrontEnd (core/src/signal_path/iq_frontend.{h,cpp}).
// Replaces the FFTW/VOLK members (fftWindowBuf, fftInBuf/OutBuf, fftwPlan) and the body of
// IQFrontEnd::handler (iq_frontend.cpp:230-249) / updateFFTSize (:272-296):
//   update(N, nz, windowType)  -- createWindow(nz, centred) on the host, upload, plan
//   handler(data, count)       -- window * FFT * 10log10|X|^2 into the acquired buffer
// The acquire -> compute -> release order and the NULL-buffer case are kept: when
// acquireFFTBuffer returns NULL the spectrum is computed but not written, and release is
// still called. See INTEGRATION.md for the patch.
#pragma once
#include <cstdio>
#include <sdrgpu.h>
#include "../sdrgpu_handle.h"

namespace dsp::gpu {
class Spectrum {
public:
    Spectrum() = default;
    Spectrum(const Spectrum&) = delete;
    Spectrum& operator=(const Spectrum&) = delete;
    ~Spectrum() { if (_h) sdrgpu_fft_destroy(_h); }

    // IQFrontEnd::updateFFTSize: size = _fftSize, nz = _nzFFTSize, windowType = _fftWindow
    bool update(int size, int nz, int windowType) {
        if (_h && sdrgpu_fft_size(_h) == size) {
            return ok(sdrgpu_fft_set_window_type(_h, windowType, nz), "fft_set_window_type");
        }
        if (_h) sdrgpu_fft_destroy(_h);
        _h = nullptr;
        if (_dev < 0) _dev = device();   // placement (sdrgpu_handle.h), kept across size changes
        return ok(sdrgpu_fft_create(&_h, _dev, size, nz, windowType), "fft_create");
    }
    // IQFrontEnd::handler body: `data` holds nz samples (Reshaper keep = nz)
    template <class Acquire, class Release>
    void handler(const void* data, int count, Acquire acquire, Release release) {
        float* buf = acquire();
        if (_h) ok(sdrgpu_fft_logmag(_h, data, buf), "fft_logmag");
        release();
        (void)count;
    }
    sdrgpu_fft* raw() { return _h; }
    int getDevice() const { return _dev; }

private:
    sdrgpu_fft* _h = nullptr;
    int _dev = -1;
};
}  // namespace dsp::gpu
