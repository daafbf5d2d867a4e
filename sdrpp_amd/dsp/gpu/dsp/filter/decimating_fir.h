// GPU-backed dsp::filter::DecimatingFIR<D,T> -- drop-in for core/src/dsp/filter/decimating_fir.h.
// Outputs only at offset, offset+D, ...; the decimation phase is carried across calls and
// reset by setTaps/setDecimation/reset exactly as decimating_fir.h:19-43.
#pragma once
#include "fir.h"

namespace dsp::filter {
template <class D, class T>
class DecimatingFIR : public FIR<D, T> {
    using base_type = FIR<D, T>;
public:
    DecimatingFIR() {}
    DecimatingFIR(stream<D>* in, tap<T>& taps, int decimation) { init(in, taps, decimation); }
    void init(stream<D>* in, tap<T>& taps, int decimation) {
        _decimation = decimation;
        base_type::init(in, taps, decimation);
    }
    void setDecimation(int decimation) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _decimation = decimation;
        gpu::ok(sdrgpu_fir_set_decimation(base_type::_h.h, decimation), "fir_set_decimation");
        base_type::tempStart();
    }

protected:
    int _decimation = 1;
};
}  // namespace dsp::filter
