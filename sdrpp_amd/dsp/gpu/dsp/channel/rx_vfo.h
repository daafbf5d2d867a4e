// GPU-backed dsp::channel::RxVFO -- drop-in for core/src/dsp/channel/rx_vfo.h:
// xlator(-offset) fused into the first full-rate decimation stage, then the remaining
// plan stages / polyphase resampler and the bw/2 low-pass (when bw != outSr).
#pragma once
#include <mutex>
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/channel/rx_vfo.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include "frequency_xlator.h"
#include "../multirate/rational_resampler.h"

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
        pause();
        _inSamplerate = inSamplerate;
        rebuild();
        resume();
    }
    void setOutSamplerate(double outSamplerate, double bandwidth) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        pause();
        _outSamplerate = outSamplerate;
        _bandwidth = bandwidth;
        rebuild();
        resume();
    }
    void setBandwidth(double bandwidth) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        pause();
        _bandwidth = bandwidth;
        rebuild();
        resume();
    }
    // keeps the running NCO phase (frequency_xlator.h:25-29); latched at the next process()
    void setOffset(double offset) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        _offset = offset;
        if (_fe) {
            std::lock_guard<std::mutex> fl(*_feMtx);
            gpu::ok(sdrgpu_frontend_set_vfo_offset(_fe, _feId, offset), "frontend_set_vfo_offset");
            return;
        }
        gpu::ok(sdrgpu_rxvfo_set_offset(_h.h, offset), "rxvfo_set_offset");
    }
    // ---- attached to a device front end (the IQFrontEnd drop-in, signal_path/iq_frontend.h):
    // the front end runs this VFO on the block it already holds on the device and writes `out`
    // (this block's own worker does nothing); the setters re-plan it there, under the front
    // end's lock. `in` is an idle placeholder input (the block API needs one).
    void attach(stream<complex_t>* in, sdrgpu_frontend* fe, int id, std::mutex* feMtx, block* feWorker, double inSamplerate,
                double outSamplerate, double bandwidth, double offset) {
        _fe = fe;
        _feId = id;
        _feMtx = feMtx;
        _feWorker = feWorker;
        _inSamplerate = inSamplerate;
        _outSamplerate = outSamplerate;
        _bandwidth = bandwidth;
        _offset = offset;
        base_type::init(in);
    }
    int frontEndId() const { return _feId; }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        pause();
        if (_fe) rebuild();
        else gpu::ok(sdrgpu_block_reset(_h.h), "rxvfo_reset");
        resume();
    }
    // GPU placement (sdrgpu_handle.h): this VFO's device; setDevice moves it (state restarts)
    int getDevice() const { return _h.dev; }
    void setDevice(int device) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        pause();
        _h.dev = device;
        rebuild();
        resume();
    }
    inline int process(int count, const complex_t* in, complex_t* out) { return _h.process(in, count, out, "rxvfo"); }
    int run() override {
        if (_fe) return -1;   // attached: the front end's worker produces `out`
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf);
        base_type::_in->flush();
        if (n < 0) return -1;
        if (n && !base_type::out.swap(n)) return -1;
        return n;
    }

protected:
    // Park the producer of `out` around a re-plan. Standalone, that is this block's own worker
    // (block.h tempStop). Attached, the front end's worker writes `out`: it is parked instead, and
    // this block's own streams are left alone -- stopping `out`'s writer here would make the
    // front end's next swap() fail and end its worker for good.
    void pause() {
        if (_fe && _feWorker) _feWorker->tempStop();
        else if (!_fe) base_type::tempStop();
    }
    void resume() {
        if (_fe && _feWorker) _feWorker->tempStart();
        else if (!_fe) base_type::tempStart();
    }
    void rebuild() {
        if (_fe) {   // attached: the front end's VFO is re-planned (its filter state restarts)
            std::lock_guard<std::mutex> fl(*_feMtx);
            gpu::ok(sdrgpu_frontend_remove_vfo(_fe, _feId), "frontend_remove_vfo");
            int id = -1;
            gpu::ok(sdrgpu_frontend_add_vfo(_fe, &id, _outSamplerate, _bandwidth, _offset), "frontend_add_vfo");
            _feId = id;
            return;
        }
        sdrgpu_block* h = nullptr;
        gpu::ok(sdrgpu_rxvfo_create(&h, _h.bind(gpu::stream_device()), _inSamplerate, _outSamplerate, _bandwidth, _offset), "rxvfo_create");
        _h.reset(h);
    }
    double _inSamplerate = 0, _outSamplerate = 0, _bandwidth = 0, _offset = 0;
    gpu::Handle _h;
    sdrgpu_frontend* _fe = nullptr;   // attached mode
    int _feId = -1;
    std::mutex* _feMtx = nullptr;
    block* _feWorker = nullptr;   // attached: the front end's worker (writes `out`)
};
}  // namespace dsp::channel
