// GPU-backed dsp::loop::AGC<T> -- drop-in for core/src/dsp/loop/agc.h (T = float or complex_t).
// The recurrence runs on the device bit-identically to agc.h:88-147 (sdrpp_amd/csrc/loops.hip);
// setters keep the running amplitude and gain, setGain is applied at the next process().
#pragma once
#include <cmath>
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"

namespace dsp::loop {
template <class T>
class AGC : public Processor<T, T> {
    using base_type = Processor<T, T>;
    static_assert(std::is_same_v<T, float> || std::is_same_v<T, complex_t>, "AGC<T>: T = float or complex_t");
public:
    AGC() {}
    void init(stream<T>* in, double setPoint, double attack, double decay, double maxGain, double maxOutputAmp, double initGain = 1.0) {
        _setPoint = setPoint; _attack = attack; _decay = decay; _maxGain = maxGain; _maxOutputAmp = maxOutputAmp; _initGain = initGain;
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_agc_create(&h, _h.bind(gpu::device()), std::is_same_v<T, complex_t> ? SDRGPU_C64 : SDRGPU_F32, setPoint, attack,
                                  decay, maxGain, maxOutputAmp, initGain), "agc_create");
        _h.reset(h);
        base_type::init(in);
    }
    float getGain() {
        float g = 0.0f;
        gpu::ok(sdrgpu_agc_get_gain(_h.h, &g), "agc_get_gain");
        return g;
    }
    void setGain(float gain) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_agc_set_gain(_h.h, gain), "agc_set_gain"); }
    void setEnabled(bool enabled) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_agc_set_enabled(_h.h, enabled), "agc_set_enabled"); }
    void setSetPoint(double v) { _setPoint = v; params(); }
    void setAttack(double v) { _attack = v; params(); }
    void setDecay(double v) { _decay = v; params(); }
    void setMaxGain(double v) { _maxGain = v; params(); }
    void setMaxOutputAmp(double v) { _maxOutputAmp = v; params(); }
    void setInitialGain(double v) { _initGain = v; params(); }
    void reset() { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_block_reset(_h.h), "agc_reset"); }
    inline int process(int count, T* in, T* out) { return _h.process(in, count, out, "agc"); }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        return count;
    }

protected:
    void params() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        gpu::ok(sdrgpu_agc_set_params(_h.h, _setPoint, _attack, _decay, _maxGain, _maxOutputAmp, _initGain), "agc_set_params");
    }
    double _setPoint = 1, _attack = 0, _decay = 0, _maxGain = 1, _maxOutputAmp = 1, _initGain = 1;
    gpu::Handle _h;
};
}  // namespace dsp::loop
