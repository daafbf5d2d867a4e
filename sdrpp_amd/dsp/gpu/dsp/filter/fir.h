// GPU-backed dsp::filter::FIR<D,T> -- drop-in for core/src/dsp/filter/fir.h.
// D in {float, complex_t, stereo_t}, T in {float, complex_t}; correlation order (no tap
// reversal), history kept on the device across calls, setTaps keeps it aligned (fir.h:31-52).
// The taps are copied to the device on init/setTaps (the caller keeps ownership, like the
// reference's borrowed tap<T>).
#pragma once
#include <type_traits>
#include "../processor.h"
#include "../taps/tap.h"
#include "../sdrgpu_handle.h"

namespace dsp::filter {
template <class D, class T>
class FIR : public Processor<D, D> {
    using base_type = Processor<D, D>;
public:
    FIR() {}
    FIR(stream<D>* in, tap<T>& taps) { init(in, taps); }

    virtual void init(stream<D>* in, tap<T>& taps) { init(in, taps, 1); }

    virtual void setTaps(tap<T>& taps) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _taps = taps;
        gpu::ok(sdrgpu_fir_set_taps(_h.h, (const float*)taps.taps, (int)taps.size), "fir_set_taps");
        base_type::tempStart();
    }
    virtual void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "fir_reset");
        base_type::tempStart();
    }
    inline int process(int count, const D* in, D* out) { return _h.process(in, count, out, "fir"); }
    virtual int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0) return -1;
        if (n && !base_type::out.swap(n)) return -1;
        return n;
    }

protected:
    static constexpr int dtype() { return std::is_same_v<D, float> ? SDRGPU_F32 : SDRGPU_C64; }
    static constexpr int ttype() { return std::is_same_v<T, float> ? SDRGPU_F32 : SDRGPU_C64; }
    void init(stream<D>* in, tap<T>& taps, int decim) {
        _taps = taps;
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_fir_create(&h, _h.bind(gpu::device()), dtype(), ttype(), (const float*)taps.taps, (int)taps.size, decim),
                "fir_create");
        _h.reset(h);
        base_type::init(in);
    }
    tap<T> _taps;
    gpu::Handle _h;
};
}  // namespace dsp::filter
