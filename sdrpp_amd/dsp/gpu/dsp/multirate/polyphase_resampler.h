// GPU-backed dsp::multirate::PolyphaseResampler<T> -- drop-in for
// core/src/dsp/multirate/polyphase_resampler.h (bank of polyphase_bank.h:15-47; outputs
// computed in closed form from the carried (offset, phase)).
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../taps/tap.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/multirate/polyphase_resampler.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#if __has_include("polyphase_bank.h")
#include "polyphase_bank.h"
#endif

namespace dsp::multirate {
template <class T>
class PolyphaseResampler : public Processor<T, T> {
    using base_type = Processor<T, T>;
public:
    PolyphaseResampler() {}
    PolyphaseResampler(stream<T>* in, int interp, int decim, tap<float> taps) { init(in, interp, decim, taps); }
    void init(stream<T>* in, int interp, int decim, tap<float> taps) {
        build(interp, decim, taps);
        base_type::init(in);
    }
    void setRatio(int interp, int decim, tap<float>& taps) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        build(interp, decim, taps);   // setRatio resets history, phase and offset (polyphase_resampler.h:41-59)
        base_type::tempStart();
    }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "polyphase_reset");
        base_type::tempStart();
    }
    inline int process(int count, const T* in, T* out) { return _h.process(in, count, out, "polyphase"); }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0) return -1;
        if (n && !base_type::out.swap(n)) return -1;
        return n;
    }

protected:
    void build(int interp, int decim, tap<float>& taps) {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_polyphase_resampler_create(&h, _h.bind(gpu::device()), std::is_same_v<T, float> ? SDRGPU_F32 : SDRGPU_C64,
                                                  interp, decim, taps.taps, (int)taps.size), "polyphase_create");
        _h.reset(h);
    }
    gpu::Handle _h;
};
}  // namespace dsp::multirate
