// GPU-backed dsp::filter::Deemphasis<T> -- drop-in for core/src/dsp/filter/deephasis.h
// (T = float or stereo_t). The one-pole recurrence out[i] = alpha*in[i] + (1-alpha)*out[i-1]
// (:58-77) runs as a serial device kernel, bit-identical to the reference arithmetic; alpha is
// formed exactly as updateAlpha() (:91-94) does, on the host.
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"

namespace dsp::filter {
template <class T>
class Deemphasis : public Processor<T, T> {
    using base_type = Processor<T, T>;
    static_assert(std::is_same_v<T, float> || std::is_same_v<T, stereo_t>, "Deemphasis<T>: T = float or stereo_t");
public:
    Deemphasis() {}
    Deemphasis(stream<T>* in, double tau, double samplerate) { init(in, tau, samplerate); }
    void init(stream<T>* in, double tau, double samplerate) {
        _tau = tau;
        _samplerate = samplerate;
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_deemphasis_create(&h, _h.bind(gpu::device()), std::is_same_v<T, float> ? SDRGPU_F32 : SDRGPU_C64, tau, samplerate),
                "deemphasis_create");
        _h.reset(h);
        base_type::init(in);
    }
    void setTau(double tau) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        _tau = tau;
        gpu::ok(sdrgpu_deemphasis_set(_h.h, _tau, _samplerate), "deemphasis_set");
    }
    void setSamplerate(double samplerate) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        _samplerate = samplerate;
        gpu::ok(sdrgpu_deemphasis_set(_h.h, _tau, _samplerate), "deemphasis_set");
    }
    void reset() {   // lastOut = 0 (:45-56)
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "deemphasis_reset");
        base_type::tempStart();
    }
    int process(int count, const T* in, T* out) { return _h.process(in, count, out, "deemphasis"); }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        return count;
    }

protected:
    double _tau = 0.0, _samplerate = 0.0;
    gpu::Handle _h;
};
}  // namespace dsp::filter
