// GPU-backed dsp::channel::RxVFO -- drop-in for core/src/dsp/channel/rx_vfo.h:
// xlator(-offset) fused into the first full-rate decimation stage, then the remaining
// plan stages / polyphase resampler and the bw/2 low-pass (when bw != outSr).
#pragma once
#include "../processor.h"
#include "../sdrgpu_handle.h"

namespace dsp::channel {
class RxVFO : public Processor<complex_t, complex_t> {
    using base_type = Processor<complex_t, complex_t>;
public:
    RxVFO() {}
    RxVFO(stream<complex_t>* in, double inSamplerate, double outSamplerate, double bandwidth, double offset) {
        init(in, inSamplerate, outSamplerate, bandwidth, offset);
    }
    void init(stream<complex_t>* in, double inSamplerate, double outSamplerate, double bandwidth, double offset) {
        _inSamplerate = inSamplerate;
        _outSamplerate = outSamplerate;
        _bandwidth = bandwidth;
        _offset = offset;
        rebuild();
        base_type::init(in);
    }
    void setInSamplerate(double inSamplerate) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _inSamplerate = inSamplerate;
        rebuild();
        base_type::tempStart();
    }
    void setOutSamplerate(double outSamplerate, double bandwidth) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _outSamplerate = outSamplerate;
        _bandwidth = bandwidth;
        rebuild();
        base_type::tempStart();
    }
    void setBandwidth(double bandwidth) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _bandwidth = bandwidth;
        rebuild();
        base_type::tempStart();
    }
    // keeps the running NCO phase (frequency_xlator.h:25-29); latched at the next process()
    void setOffset(double offset) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        _offset = offset;
        gpu::ok(sdrgpu_rxvfo_set_offset(_h.h, offset), "rxvfo_set_offset");
    }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "rxvfo_reset");
        base_type::tempStart();
    }
    // GPU placement (sdrgpu_handle.h): this VFO's device; setDevice moves it (state restarts)
    int getDevice() const { return _h.dev; }
    void setDevice(int device) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _h.dev = device;
        rebuild();
        base_type::tempStart();
    }
    inline int process(int count, const complex_t* in, complex_t* out) { return _h.process(in, count, out, "rxvfo"); }
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
    void rebuild() {
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_rxvfo_create(&h, _h.bind(gpu::stream_device()), _inSamplerate, _outSamplerate, _bandwidth, _offset), "rxvfo_create");
        _h.reset(h);
    }
    double _inSamplerate = 0, _outSamplerate = 0, _bandwidth = 0, _offset = 0;
    gpu::Handle _h;
};
}  // namespace dsp::channel
