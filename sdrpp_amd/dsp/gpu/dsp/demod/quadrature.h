// GPU-backed dsp::demod::Quadrature -- drop-in for core/src/dsp/demod/quadrature.h.
// out[i] = arg(x[i] * conj(x[i-1])) / deviation; the previous sample is carried on the
// device (0 after init/reset; the reference leaves it uninitialised until reset()).
#pragma once
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/demod/quadrature.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#if __has_include("../math/fast_atan2.h")
#include "../math/fast_atan2.h"
#endif
#if __has_include("../math/hz_to_rads.h")
#include "../math/hz_to_rads.h"
#endif
#if __has_include("../math/normalize_phase.h")
#include "../math/normalize_phase.h"
#endif

namespace dsp::demod {
class Quadrature : public Processor<complex_t, float> {
    using base_type = Processor<complex_t, float>;
public:
    Quadrature() {}
    Quadrature(stream<complex_t>* in, double deviation) { init(in, deviation); }
    Quadrature(stream<complex_t>* in, double deviation, double samplerate) { init(in, deviation, samplerate); }
    virtual void init(stream<complex_t>* in, double deviation) {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_quadrature_create(&h, _h.bind(gpu::device()), deviation), "quadrature_create");
        _h.reset(h);
        base_type::init(in);
    }
    virtual void init(stream<complex_t>* in, double deviation, double samplerate) {
        init(in, 2.0 * 3.14159265358979323846 * (deviation / samplerate));
    }
    void setDeviation(double deviation) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        gpu::ok(sdrgpu_quadrature_set_deviation(_h.h, deviation), "quadrature_set_deviation");
    }
    void setDeviation(double deviation, double samplerate) {
        setDeviation(2.0 * 3.14159265358979323846 * (deviation / samplerate));
    }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        gpu::ok(sdrgpu_block_reset(_h.h), "quadrature_reset");
    }
    inline int process(int count, const complex_t* in, float* out) { return _h.process(in, count, out, "quadrature"); }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        return count;
    }

protected:
    gpu::Handle _h;
};
}  // namespace dsp::demod
