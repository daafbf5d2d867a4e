// GPU-backed dsp::channel::FrequencyXlator -- drop-in for core/src/dsp/channel/frequency_xlator.h.
// Same class, constructors, setters and process(count, in, out); the rotation runs on the GPU
// (sdrgpu_xlator_*, NCO at the float-quantised phase increment, phase carried across calls).
#pragma once
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/channel/frequency_xlator.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#if __has_include("../math/hz_to_rads.h")
#include "../math/hz_to_rads.h"
#endif

namespace dsp::channel {
class FrequencyXlator : public Processor<complex_t, complex_t> {
    using base_type = Processor<complex_t, complex_t>;
public:
    FrequencyXlator() {}
    FrequencyXlator(stream<complex_t>* in, double offset) { init(in, offset); }
    FrequencyXlator(stream<complex_t>* in, double offset, double samplerate) { init(in, offset, samplerate); }

    void init(stream<complex_t>* in, double offset) {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_xlator_create(&h, _h.bind(gpu::device()), offset), "xlator_create");
        _h.reset(h);
        base_type::init(in);
    }
    void init(stream<complex_t>* in, double offset, double samplerate) { init(in, 2.0 * 3.14159265358979323846 * (offset / samplerate)); }
    void setOffset(double offset) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        gpu::ok(sdrgpu_xlator_set_offset(_h.h, offset), "xlator_set_offset");
    }
    void setOffset(double offset, double samplerate) { setOffset(2.0 * 3.14159265358979323846 * (offset / samplerate)); }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "xlator_reset");
        base_type::tempStart();
    }
    inline int process(int count, const complex_t* in, complex_t* out) { return _h.process(in, count, out, "xlator"); }
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
}  // namespace dsp::channel
