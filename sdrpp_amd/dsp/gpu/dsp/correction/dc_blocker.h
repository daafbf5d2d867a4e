// GPU-backed dsp::correction::DCBlocker<T> -- drop-in for core/src/dsp/correction/dc_blocker.h
// (T = float, complex_t or stereo_t: per-component recurrence, bit-identical to :54-60).
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"

namespace dsp::correction {
template <class T>
class DCBlocker : public Processor<T, T> {
    using base_type = Processor<T, T>;
public:
    DCBlocker() {}
    DCBlocker(stream<T>* in, double rate) { init(in, rate); }
    DCBlocker(stream<T>* in, double rate, double samplerate) { init(in, rate, samplerate); }
    void init(stream<T>* in, double rate) {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_dc_blocker_create(&h, _h.bind(gpu::device()), std::is_same_v<T, float> ? SDRGPU_F32 : SDRGPU_C64, rate), "dc_blocker_create");
        _h.reset(h);
        base_type::init(in);
    }
    void init(stream<T>* in, double rate, double samplerate) { init(in, rate / samplerate); }
    void setRate(double rate) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_dc_blocker_set_rate(_h.h, rate), "dc_blocker_set_rate"); }
    void setRate(double rate, double samplerate) { setRate(rate / samplerate); }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "dc_blocker_reset");
        base_type::tempStart();
    }
    int process(int count, T* in, T* out) { return _h.process(in, count, out, "dc_blocker"); }
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
}  // namespace dsp::correction
