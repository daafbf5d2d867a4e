// GPU-backed dsp::demod::AM<T> -- drop-in for core/src/dsp/demod/am.h (T = float or stereo_t):
// [carrier AGC] -> |x| -> DC block -> [audio AGC] -> low-pass, all on the device (am.h:114-142).
// setBandwidth / setAGCMode rebuild the device chain (the AGC gain is carried over like
// am.h:63-71); setAGCGain / setAGCAttack / setAGCDecay / setDCBlockRate keep the state.
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/demod/am.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include "../loop/agc.h"
#include "../correction/dc_blocker.h"
#if __has_include("../convert/mono_to_stereo.h")
#include "../convert/mono_to_stereo.h"
#endif
#include "../filter/fir.h"
#if __has_include("../taps/low_pass.h")
#include "../taps/low_pass.h"
#endif

namespace dsp::demod {
template <class T>
class AM : public Processor<dsp::complex_t, T> {
    using base_type = Processor<dsp::complex_t, T>;
    static_assert(std::is_same_v<T, float> || std::is_same_v<T, stereo_t>, "AM<T>: T = float or stereo_t");
public:
    enum AGCMode { OFF, CARRIER, AUDIO };
    AM() {}
    void init(stream<complex_t>* in, AGCMode agcMode, double bandwidth, double agcAttack, double agcDecay, double dcBlockRate, double samplerate) {
        _agcMode = agcMode; _bandwidth = bandwidth; _attack = agcAttack; _decay = agcDecay; _dcRate = dcBlockRate; _samplerate = samplerate;
        rebuild();
        base_type::init(in);
    }
    void setBandwidth(double bandwidth) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        if (bandwidth == _bandwidth) return;
        _bandwidth = bandwidth;
        float g = getAGCGain();
        rebuild();
        setAGCGain(g);
    }
    void setAGCMode(AGCMode agcMode) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        float g = getAGCGain();
        _agcMode = agcMode;
        rebuild();
        setAGCGain(g);
    }
    void setAGCGain(float gain) {   // the audio AGC (am.h:72-76); absent in CARRIER mode
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        if (_agcMode != CARRIER) gpu::ok(sdrgpu_demod_agc_set_gain(_h.h, 1, gain), "am_set_agc_gain");
    }
    float getAGCGain() {
        float g = 0.0f;
        gpu::ok(sdrgpu_demod_agc_get_gain(_h.h, _agcMode == CARRIER ? 0 : 1, &g), "am_get_agc_gain");
        return g;
    }
    void setAGCAttack(double attack) { _attack = attack; ad(); }
    void setAGCDecay(double decay) { _decay = decay; ad(); }
    void setDCBlockRate(double rate) { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); _dcRate = rate; gpu::ok(sdrgpu_dc_blocker_set_rate(_h.h, rate), "am_set_dc_rate"); }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "am_reset");
        base_type::tempStart();
    }
    int process(int count, complex_t* in, T* out) { return _h.process(in, count, out, "am"); }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        return count;
    }

protected:
    void ad() { std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx); gpu::ok(sdrgpu_demod_agc_set_attack_decay(_h.h, _attack, _decay), "am_set_attack_decay"); }
    void rebuild() {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_am_create(&h, _h.bind(gpu::device()), (int)_agcMode, _bandwidth, _attack, _decay, _dcRate, _samplerate,
                                 std::is_same_v<T, stereo_t>), "am_create");
        _h.reset(h);
    }
    AGCMode _agcMode = OFF;
    double _bandwidth = 0, _attack = 0, _decay = 0, _dcRate = 0, _samplerate = 0;
    gpu::Handle _h;
};
}  // namespace dsp::demod
