// GPU-backed dsp::multirate::RationalResampler<T> -- drop-in for
// core/src/dsp/multirate/rational_resampler.h: power-of-two pre-decimation + polyphase
// interp/decim planned exactly like reconfigure() (rational_resampler.h:121-167).
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/multirate/rational_resampler.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include <vector>
#include <numeric>
#include "../filter/decimating_fir.h"
#if __has_include("../taps/from_array.h")
#include "../taps/from_array.h"
#endif
#include "polyphase_resampler.h"
#include "power_decimator.h"
#if __has_include("../taps/low_pass.h")
#include "../taps/low_pass.h"
#endif
#if __has_include("../window/nuttall.h")
#include "../window/nuttall.h"
#endif
#if __has_include("utils/flog.h")
#include "utils/flog.h"
#endif

namespace dsp::multirate {
template <class T>
class RationalResampler : public Processor<T, T> {
    using base_type = Processor<T, T>;
public:
    RationalResampler() {}
    RationalResampler(stream<T>* in, double inSamplerate, double outSamplerate) { init(in, inSamplerate, outSamplerate); }
    void init(stream<T>* in, double inSamplerate, double outSamplerate) {
        _inSamplerate = inSamplerate;
        _outSamplerate = outSamplerate;
        reconfigure();
        base_type::init(in);
    }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "rational_reset");
        base_type::tempStart();
    }
    void setInSamplerate(double inSamplerate) { setRates(inSamplerate, _outSamplerate); }
    void setOutSamplerate(double outSamplerate) { setRates(_inSamplerate, outSamplerate); }
    void setRates(double inSamplerate, double outSamplerate) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _inSamplerate = inSamplerate;
        _outSamplerate = outSamplerate;
        reconfigure();
        base_type::tempStart();
    }
    inline int process(int count, const T* in, T* out) { return _h.process(in, count, out, "rational_resampler"); }
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
    void reconfigure() {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_rational_resampler_create(&h, _h.bind(gpu::device()), std::is_same_v<T, float> ? SDRGPU_F32 : SDRGPU_C64,
                                                 _inSamplerate, _outSamplerate), "rational_create");
        _h.reset(h);
    }
    double _inSamplerate = 0, _outSamplerate = 0;
    gpu::Handle _h;
};
}  // namespace dsp::multirate
