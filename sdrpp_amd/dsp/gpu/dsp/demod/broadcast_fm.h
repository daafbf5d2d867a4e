// GPU-backed dsp::demod::BroadcastFM -- drop-in for core/src/dsp/demod/broadcast_fm.h:
//  stereo: quadrature -> pilot band-pass -> PLL -> L+R / L-R matrix -> audio low-pass
//          (broadcast_fm.h:144-191, sdrgpu_broadcast_fm_create);
//  mono:   quadrature -> 15 kHz low-pass -> LRToStereo (:193-211, sdrgpu_wfm_create);
//  RDS:    MPX -> FrequencyXlator(-57 kHz) -> RationalResampler(fs -> 5 kHz) into rdsOut
//          (:164-171, 193-203; sdrgpu_broadcast_fm_set_rds / _read_rds).
// As in the reference, the constructor does not pass rdsOut on to init() (:23): use init() or
// setRDSOut() to enable the RDS branch.
#pragma once
#include "../processor.h"
#include "../sdrgpu_handle.h"
// the reference header's own includes (core/src/dsp/demod/broadcast_fm.h): callers such as
// decoder_modules/radio/src/demodulators/*.h rely on them transitively. Headers that exist
// only in the SDR++ tree are guarded, so the block-API mirror build skips them.
#include "quadrature.h"
#if __has_include("../taps/low_pass.h")
#include "../taps/low_pass.h"
#endif
#if __has_include("../taps/band_pass.h")
#include "../taps/band_pass.h"
#endif
#include "../filter/fir.h"
#if __has_include("../loop/pll.h")
#include "../loop/pll.h"
#endif
#if __has_include("../convert/l_r_to_stereo.h")
#include "../convert/l_r_to_stereo.h"
#endif
#if __has_include("../convert/real_to_complex.h")
#include "../convert/real_to_complex.h"
#endif
#if __has_include("../convert/complex_to_real.h")
#include "../convert/complex_to_real.h"
#endif
#if __has_include("../math/conjugate.h")
#include "../math/conjugate.h"
#endif
#if __has_include("../math/delay.h")
#include "../math/delay.h"
#endif
#if __has_include("../math/multiply.h")
#include "../math/multiply.h"
#endif
#if __has_include("../math/add.h")
#include "../math/add.h"
#endif
#if __has_include("../math/subtract.h")
#include "../math/subtract.h"
#endif
#include "../multirate/rational_resampler.h"

namespace dsp::demod {
class BroadcastFM : public Processor<complex_t, stereo_t> {
    using base_type = Processor<complex_t, stereo_t>;
public:
    BroadcastFM() {}
    BroadcastFM(stream<complex_t>* in, double deviation, double samplerate, bool stereo = true, bool lowPass = true,
                bool rdsOut = false) {
        init(in, deviation, samplerate, stereo, lowPass);   // (reference: rdsOut is dropped here)
    }
    virtual void init(stream<complex_t>* in, double deviation, double samplerate, bool stereo = true, bool lowPass = true,
                      bool rdsOut = false) {
        _deviation = deviation;
        _samplerate = samplerate;
        _stereo = stereo;
        _lowPass = lowPass;
        _rdsOut = rdsOut;
        rebuild();
        base_type::init(in);
    }
    void setDeviation(double deviation) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        _deviation = deviation;
        rebuild();
    }
    void setSamplerate(double samplerate) { set(samplerate, _stereo, _lowPass, _rdsOut); }
    void setStereo(bool stereo) { set(_samplerate, stereo, _lowPass, _rdsOut); }
    void setLowPass(bool lowPass) { set(_samplerate, _stereo, lowPass, _rdsOut); }
    void setRDSOut(bool rdsOut) { set(_samplerate, _stereo, _lowPass, rdsOut); }
    void reset() {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        gpu::ok(sdrgpu_block_reset(_h.h), "wfm_reset");
        base_type::tempStart();
    }
    inline int process(int count, complex_t* in, stereo_t* out, int& rdsOutCount, complex_t* rdsout = nullptr) {
        rdsOutCount = 0;
        const int n = _h.process(in, count, out, "wfm");
        if (n >= 0 && _rdsOut && rdsout) {
            const int r = sdrgpu_broadcast_fm_read_rds(_h.h, rdsout, STREAM_BUFFER_SIZE);
            if (!gpu::ok(r, "broadcast_fm_read_rds")) return -1;
            rdsOutCount = r;
        }
        return n;
    }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        int rds = 0;
        int n = process(count, base_type::_in->readBuf, base_type::out.writeBuf, rds, rdsOut.writeBuf);
        base_type::_in->flush();
        if (n < 0 || !base_type::out.swap(count)) return -1;
        if (rds && _rdsOut && !rdsOut.swap(rds)) return -1;
        return count;
    }
    stream<complex_t> rdsOut;

protected:
    void set(double sr, bool stereo, bool lp, bool rds) {
        std::lock_guard<std::recursive_mutex> lck(base_type::ctrlMtx);
        base_type::tempStop();
        _samplerate = sr; _stereo = stereo; _lowPass = lp; _rdsOut = rds;
        rebuild();
        base_type::tempStart();
    }
    void rebuild() {
        sdrgpu_block* h = nullptr;
        if (_stereo || _rdsOut) {
            gpu::ok(sdrgpu_broadcast_fm_create(&h, _h.bind(gpu::device()), _deviation, _samplerate, _stereo, _lowPass), "broadcast_fm_create");
            if (h && _rdsOut) gpu::ok(sdrgpu_broadcast_fm_set_rds(h, 1), "broadcast_fm_set_rds");
        } else {
            gpu::ok(sdrgpu_wfm_create(&h, _h.bind(gpu::device()), _deviation, _samplerate, _lowPass), "wfm_create");
        }
        _h.reset(h);
    }
    double _deviation = 0, _samplerate = 0;
    bool _stereo = false, _lowPass = true, _rdsOut = false;
    gpu::Handle _h;
};
}  // namespace dsp::demod
