// GPU-backed dsp::demod::SSB<T> -- drop-in for core/src/dsp/demod/ssb.h (T = float or stereo_t):
// xlate by getTranslation() -> real part -> AGC (ssb.h:90-105) on the device. setMode /
// setBandwidth / setSamplerate rebuild the chain (the AGC gain is carried over).
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/demod/ssb.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include "../channel/frequency_xlator.h"
#if __has_include("../convert/complex_to_real.h")
#include "../convert/complex_to_real.h"
#endif
#include "../loop/agc.h"
#if __has_include("../convert/mono_to_stereo.h")
#include "../convert/mono_to_stereo.h"
#endif

namespace dsp::demod {
template <class T>
class SSB : public Processor<complex_t, T> {
    using base_type = Processor<complex_t, T>;
    static_assert(std::is_same_v<T, float> || std::is_same_v<T, stereo_t>, "SSB<T>: T = float or stereo_t");
public:
    enum Mode { USB, LSB, DSB };
    SSB() {}
    void init(stream<complex_t>* in, Mode mode, double bandwidth, double samplerate, bool agcEnabled, double agcAttack, double agcDecay) {
        _mode = mode; _bandwidth = bandwidth; _samplerate = samplerate; _agcEnabled = agcEnabled; _attack = agcAttack; _decay = agcDecay;
        rebuild();
        base_type::init(in);
    }
    void setMode(Mode mode) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); _mode = mode; keepGainRebuild(); }
    void setBandwidth(double bandwidth) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); _bandwidth = bandwidth; keepGainRebuild(); }
    void setSamplerate(double samplerate) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); _samplerate = samplerate; keepGainRebuild(); }
    void setAGCEnabled(bool enabled) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); _agcEnabled = enabled; gpu::ok(sdrgpu_demod_agc_set_enabled(_h.h, 0, enabled), "ssb_set_agc_enabled"); }
    void setAGCGain(float gain) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_demod_agc_set_gain(_h.h, 0, gain), "ssb_set_agc_gain"); }
    float getAGCGain() { float g = 0.0f; gpu::ok(sdrgpu_demod_agc_get_gain(_h.h, 0, &g), "ssb_get_agc_gain"); return g; }
    void setAGCAttack(double attack) { _attack = attack; ad(); }
    void setAGCDecay(double decay) { _decay = decay; ad(); }
    int process(int count, const complex_t* in, T* out) { return _h.process(in, count, out, "ssb"); }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        return count;
    }

protected:
    void ad() { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_demod_agc_set_attack_decay(_h.h, _attack, _decay), "ssb_set_attack_decay"); }
    void keepGainRebuild() {
        base_type::tempStop();
        float g = getAGCGain();
        rebuild();
        setAGCGain(g);
        base_type::tempStart();
    }
    void rebuild() {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_ssb_create(&h, _h.bind(gpu::device()), (int)_mode, _bandwidth, _samplerate, _agcEnabled, _attack, _decay,
                                  std::is_same_v<T, stereo_t>), "ssb_create");
        _h.reset(h);
    }
    Mode _mode = USB;
    double _bandwidth = 0, _samplerate = 0, _attack = 0, _decay = 0;
    bool _agcEnabled = false;
    gpu::Handle _h;
};
}  // namespace dsp::demod
