// GPU-backed dsp::demod::FM<T> -- drop-in for core/src/dsp/demod/fm.h (T = float or stereo_t):
// quadrature(bw/2) -> optional low/high/band-pass exactly as updateFilter (fm.h:117-133).
#pragma once
#include <type_traits>
#include <vector>
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/demod/fm.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include "quadrature.h"
#include "../filter/fir.h"
#if __has_include("../taps/low_pass.h")
#include "../taps/low_pass.h"
#endif
#if __has_include("../taps/high_pass.h")
#include "../taps/high_pass.h"
#endif
#if __has_include("../taps/band_pass.h")
#include "../taps/band_pass.h"
#endif
#if __has_include("../convert/mono_to_stereo.h")
#include "../convert/mono_to_stereo.h"
#endif

namespace dsp::demod {
template <class T>
class FM : public dsp::Processor<dsp::complex_t, T> {
    using base_type = dsp::Processor<dsp::complex_t, T>;
public:
    FM() {}
    FM(dsp::stream<dsp::complex_t>* in, double samplerate, double bandwidth, bool lowPass) { init(in, samplerate, bandwidth, lowPass, false); }
    void init(dsp::stream<dsp::complex_t>* in, double samplerate, double bandwidth, bool lowPass, bool highPass) {
        _samplerate = samplerate;
        _bandwidth = bandwidth;
        _lowPass = lowPass;
        _highPass = highPass;
        rebuild();
        base_type::init(in);
    }
    void setSamplerate(double samplerate) { set(samplerate, _bandwidth, _lowPass, _highPass); }
    void setBandwidth(double bandwidth) { if (bandwidth != _bandwidth) set(_samplerate, bandwidth, _lowPass, _highPass); }
    void setLowPass(bool lowPass) { set(_samplerate, _bandwidth, lowPass, _highPass); }
    void setHighPass(bool highPass) { set(_samplerate, _bandwidth, _lowPass, highPass); }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "fm_reset");
        base_type::tempStart();
    }
    inline int process(int count, dsp::complex_t* in, T* out) {
        if constexpr (std::is_same_v<T, float>) {
            return _h.process(in, count, out, "fm");
        } else {
            if ((int)_mono.size() < count) _mono.resize(count);
            int n = _h.process(in, count, _mono.data(), "fm");
            for (int i = 0; i < n; i++) out[i] = {_mono[i], _mono[i]};   // MonoToStereo
            return n;
        }
    }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        return count;
    }

private:
    void set(double sr, double bw, bool lp, bool hp) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _samplerate = sr; _bandwidth = bw; _lowPass = lp; _highPass = hp;
        rebuild();
        base_type::tempStart();
    }
    void rebuild() {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_fm_create(&h, _h.bind(gpu::device()), _samplerate, _bandwidth, _lowPass, _highPass), "fm_create");
        _h.reset(h);
    }
    double _samplerate = 0, _bandwidth = 0;
    bool _lowPass = false, _highPass = false;
    std::vector<float> _mono;
    gpu::Handle _h;
};
}  // namespace dsp::demod
