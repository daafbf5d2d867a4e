// GPU-backed dsp::multirate::PowerDecimator<T> -- drop-in for core/src/dsp/multirate/power_decimator.h.
// Cascade of the reference's 13 fixed decimation plans (ratio 2..8192) run as device FIR stages.
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/multirate/power_decimator.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include "../filter/decimating_fir.h"
#if __has_include("../taps/from_array.h")
#include "../taps/from_array.h"
#endif
#if __has_include("decim/plans.h")
#include "decim/plans.h"
#endif

namespace dsp::multirate {
template <class T>
class PowerDecimator : public Processor<T, T> {
    using base_type = Processor<T, T>;
public:
    PowerDecimator() {}
    PowerDecimator(stream<T>* in, unsigned int ratio) { init(in, ratio); }
    void init(stream<T>* in, unsigned int ratio) {
        _ratio = ratio;
        build();
        base_type::init(in);
    }
    static inline unsigned int getMaxRatio() { return 1 << 13; }
    void setRatio(unsigned int ratio) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _ratio = ratio;
        build();
        base_type::tempStart();
    }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "power_decimator_reset");
        base_type::tempStart();
    }
    inline int process(int count, const T* in, T* out) { return _h.process(in, count, out, "power_decimator"); }
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
    void build() {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_power_decimator_create(&h, _h.bind(gpu::device()), std::is_same_v<T, float> ? SDRGPU_F32 : SDRGPU_C64,
                                              (int)_ratio), "power_decimator_create");
        _h.reset(h);
    }
    unsigned int _ratio = 1;
    gpu::Handle _h;
};
}  // namespace dsp::multirate
