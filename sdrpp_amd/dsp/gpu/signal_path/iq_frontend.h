// GPU-backed IQFrontEnd -- drop-in for core/src/signal_path/iq_frontend.{h,cpp}: the same class
// name and public interface (init, setSampleRate, setDecimation, setInvertIQ, setDCBlocking,
// bindIQStream, addVFO / removeVFO, setFFTSize / Rate / Window, start / stop, ...), header-only.
//
// The whole data path runs in libsdrgpu's device front end (sdrgpu_frontend_*, include/sdrgpu.h):
// one H2D per input block, then on the device the preprocessing (PowerDecimator, DCBlocker,
// Conjugate), the reshaper's keep / skip framing (genReshapeParams, iq_frontend.h:56-60),
// window * FFT * log-power (iq_frontend.cpp:230-249), and every VFO reading the block in place
// (addVFO, :122-142) -- instead of the SampleFrameBuffer -> Splitter -> Reshaper memcpy fan-out.
// One worker thread (a dsp::block) moves each block of the input stream to the device and hands
// back, in order:
//   * each dB row through acquire / releaseFFTBuffer (a NULL buffer skips the copy but release
//     is still called, as in handler);
//   * each VFO's output into that VFO's `out` stream (the VFO is an RxVFO attached to the front
//     end: its own worker is idle, its setters re-plan it on the device);
//   * the preprocessed IQ into every bound stream (bindIQStream: the recorder, IQ exporters).
// Buffering (SampleFrameBuffer) is not needed: blocks are consumed as they come, losslessly.
// Inside the SDR++ tree (core.h present) it keeps the reference's couplings:
// core::setInputSampleRate on a rate change and gui::waterfall.setRawFFTSize on an FFT change.
#pragma once
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>
#include <sdrgpu.h>
#include "../dsp/block.h"
#include "../dsp/stream.h"
#include "../dsp/window/window.h"
#include "../dsp/channel/rx_vfo.h"
#if __has_include("../core.h")
#include "../core.h"
#include "../gui/gui.h"
#include <utils/flog.h>
#define SDRGPU_FE_INPUT_SAMPLERATE(sr) core::setInputSampleRate(sr)
#define SDRGPU_FE_RAW_FFT_SIZE(n) gui::waterfall.setRawFFTSize(n)
#define SDRGPU_FE_ERROR(...) flog::error(__VA_ARGS__)
#else
#define SDRGPU_FE_INPUT_SAMPLERATE(sr) ((void)(sr))
#define SDRGPU_FE_RAW_FFT_SIZE(n) ((void)(n))
#define SDRGPU_FE_ERROR(...) (std::fprintf(stderr, "[IQFrontEnd] " __VA_ARGS__), std::fprintf(stderr, "\n"))
#endif

class IQFrontEnd {
public:
    ~IQFrontEnd() {
        if (!_init) return;
        stop();
        for (auto& [name, v] : vfos) {
            v.vfo->stop();
            delete v.vfo;
            delete v.in;
        }
        vfos.clear();
        if (_fe) sdrgpu_frontend_destroy(_fe);
    }

    void init(dsp::stream<dsp::complex_t>* in, double sampleRate, bool buffering, int decimRatio, bool dcBlocking,
              int fftSize, double fftRate, dsp::window::windowType fftWindow, float* (*acquireFFTBuffer)(void* ctx),
              void (*releaseFFTBuffer)(void* ctx), void* fftCtx) {
        _sampleRate = sampleRate;
        _decimRatio = decimRatio;
        _dcBlocking = dcBlocking;
        _fftSize = fftSize;
        _fftRate = fftRate;
        _fftWindow = fftWindow;
        _acquireFFTBuffer = acquireFFTBuffer;
        _releaseFFTBuffer = releaseFFTBuffer;
        _fftCtx = fftCtx;
        (void)buffering;
        dsp::gpu::ok(sdrgpu_frontend_create(&_fe, dsp::gpu::device(), sampleRate, decimRatio, dcBlocking, fftSize, fftRate,
                                            (int)fftWindow),
                     "frontend_create");
        refreshFraming();
        _worker.fe = this;
        _worker.setInput(in);
        _init = true;
    }

    // IQFrontEnd::updateFFTSize (iq_frontend.cpp:272-296): window + plan for the current framing
    void updateFFTSize() {
        std::lock_guard<std::mutex> l(_mtx);
        dsp::gpu::ok(sdrgpu_frontend_set_fft(_fe, _fftSize, _fftRate, (int)_fftWindow), "frontend_set_fft");
        refreshFraming();
    }

    void setInput(dsp::stream<dsp::complex_t>* in) { _worker.setInput(in); }
    void setSampleRate(double sampleRate) {
        _worker.tempStop();
        {
            std::lock_guard<std::mutex> l(_mtx);
            _sampleRate = sampleRate;
            dsp::gpu::ok(sdrgpu_frontend_configure(_fe, _sampleRate, _decimRatio, _dcBlocking), "frontend_configure");
            refreshFraming();
        }
        for (auto& [name, v] : vfos) v.vfo->setInSamplerate(effectiveSr);   // re-planned at the new rate
        SDRGPU_FE_INPUT_SAMPLERATE(_sampleRate);
        _worker.tempStart();
    }
    inline double getSampleRate() { return _sampleRate / _decimRatio; }

    void setBuffering(bool enabled) { (void)enabled; }   // blocks are consumed losslessly
    void setDecimation(int ratio) {
        _decimRatio = ratio;
        setSampleRate(_sampleRate);
    }
    void setInvertIQ(bool enabled) {
        std::lock_guard<std::mutex> l(_mtx);
        dsp::gpu::ok(sdrgpu_frontend_set_invert_iq(_fe, enabled), "frontend_set_invert_iq");
    }
    void setDCBlocking(bool enabled) {
        _worker.tempStop();
        {
            std::lock_guard<std::mutex> l(_mtx);
            _dcBlocking = enabled;
            dsp::gpu::ok(sdrgpu_frontend_configure(_fe, _sampleRate, _decimRatio, _dcBlocking), "frontend_configure");
        }
        _worker.tempStart();
    }

    void bindIQStream(dsp::stream<dsp::complex_t>* stream) {
        _worker.tempStop();
        _worker.bind(stream);
        _worker.tempStart();
    }
    void unbindIQStream(dsp::stream<dsp::complex_t>* stream) {
        _worker.tempStop();
        _worker.unbind(stream);
        _worker.tempStart();
    }

    dsp::channel::RxVFO* addVFO(std::string name, double sampleRate, double bandwidth, double offset) {
        if (vfos.find(name) != vfos.end()) {
            SDRGPU_FE_ERROR("[IQFrontEnd] Tried to add VFO with existing name.");
            return NULL;
        }
        _worker.tempStop();
        int id = -1;
        {
            std::lock_guard<std::mutex> l(_mtx);
            if (!dsp::gpu::ok(sdrgpu_frontend_add_vfo(_fe, &id, sampleRate, bandwidth, offset), "frontend_add_vfo")) {
                _worker.tempStart();
                return NULL;
            }
        }
        auto* in = new dsp::stream<dsp::complex_t>;
        auto* vfo = new dsp::channel::RxVFO();
        vfo->attach(in, _fe, id, &_mtx, effectiveSr, sampleRate, bandwidth, offset);
        vfos[name] = {vfo, in};
        _worker.addOutput(&vfo->out);
        _worker.tempStart();
        vfo->start();
        return vfo;
    }
    void removeVFO(std::string name) {
        auto it = vfos.find(name);
        if (it == vfos.end()) {
            SDRGPU_FE_ERROR("[IQFrontEnd] Tried to remove a VFO that doesn't exist.");
            return;
        }
        _worker.tempStop();
        auto v = it->second;
        vfos.erase(it);
        _worker.removeOutput(&v.vfo->out);
        {
            std::lock_guard<std::mutex> l(_mtx);
            dsp::gpu::ok(sdrgpu_frontend_remove_vfo(_fe, v.vfo->frontEndId()), "frontend_remove_vfo");
        }
        _worker.tempStart();
        v.vfo->stop();
        delete v.vfo;
        delete v.in;
    }

    void setFFTSize(int size) {
        _worker.tempStop();
        _fftSize = size;
        updateFFTSize();
        SDRGPU_FE_RAW_FFT_SIZE(_fftSize);
        _worker.tempStart();
    }
    void setFFTRate(double rate) {
        _worker.tempStop();
        _fftRate = rate;
        updateFFTSize();
        _worker.tempStart();
    }
    void setFFTWindow(dsp::window::windowType fftWindow) {
        _worker.tempStop();
        _fftWindow = fftWindow;
        updateFFTSize();
        _worker.tempStart();
    }

    void flushInputBuffer() {}   // no input buffer to flush
    void start() { _worker.start(); }
    void stop() { _worker.stop(); }
    double getEffectiveSamplerate() { return effectiveSr; }

    // (not in the reference) the device front end under this object, for sdrgpu_frontend_* calls
    sdrgpu_frontend* device_frontend() { return _fe; }

protected:
    struct Vfo {
        dsp::channel::RxVFO* vfo;
        dsp::stream<dsp::complex_t>* in;   // idle placeholder input of the attached VFO
    };

    // the worker: one input block per run()
    class Worker : public dsp::block {
    public:
        IQFrontEnd* fe = nullptr;
        void setInput(dsp::stream<dsp::complex_t>* in) {
            std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
            tempStop();
            if (_in) unregisterInput(_in);
            _in = in;
            registerInput(_in);
            _block_init = true;
            tempStart();
        }
        void addOutput(dsp::stream<dsp::complex_t>* s) { registerOutput(s); }
        void removeOutput(dsp::stream<dsp::complex_t>* s) { unregisterOutput(s); }
        void bind(dsp::stream<dsp::complex_t>* s) {
            bound.push_back(s);
            registerOutput(s);
        }
        void unbind(dsp::stream<dsp::complex_t>* s) {
            bound.erase(std::remove(bound.begin(), bound.end(), s), bound.end());
            unregisterOutput(s);
        }
        int run() override { return fe->iteration(_in, bound); }
        dsp::stream<dsp::complex_t>* _in = nullptr;
        std::vector<dsp::stream<dsp::complex_t>*> bound;
    };

    // one block: push it to the device, then hand back rows, VFO outputs and preprocessed IQ
    int iteration(dsp::stream<dsp::complex_t>* in, const std::vector<dsp::stream<dsp::complex_t>*>& bound) {
        const int count = in->read();
        if (count < 0) return -1;
        int nf = 0, niq = 0;
        std::vector<std::pair<dsp::channel::RxVFO*, int>> outs;
        {
            std::lock_guard<std::mutex> l(_mtx);
            nf = sdrgpu_frontend_push(_fe, in->readBuf, count, -1);
            in->flush();
            if (!dsp::gpu::ok(nf, "frontend_push")) return -1;
            if (nf > 0) {
                _rows.resize((size_t)nf * _fftSize);
                sdrgpu_frontend_read_spectra(_fe, _rows.data(), nf);
            }
            for (auto& [name, v] : vfos) {
                const int n = sdrgpu_frontend_read_vfo(_fe, v.vfo->frontEndId(), v.vfo->out.writeBuf, STREAM_BUFFER_SIZE);
                if (!dsp::gpu::ok(n, "frontend_read_vfo")) return -1;
                outs.emplace_back(v.vfo, n);
            }
            if (!bound.empty()) niq = sdrgpu_frontend_read_iq(_fe, bound[0]->writeBuf, STREAM_BUFFER_SIZE);
        }
        for (int r = 0; r < nf; r++) {   // IQFrontEnd::handler's acquire -> write -> release per row
            float* buf = _acquireFFTBuffer(_fftCtx);
            if (buf) std::memcpy(buf, _rows.data() + (size_t)r * _fftSize, sizeof(float) * _fftSize);
            _releaseFFTBuffer(_fftCtx);
        }
        for (auto& [vfo, n] : outs)
            if (n > 0 && !vfo->out.swap(n)) return -1;
        for (size_t k = 0; k < bound.size() && niq > 0; k++) {
            if (k > 0) std::memcpy(bound[k]->writeBuf, bound[0]->writeBuf, sizeof(dsp::complex_t) * niq);
            if (!bound[k]->swap(niq)) return -1;
        }
        return count;
    }

    void refreshFraming() {
        int nz = 0, skip = 0;
        sdrgpu_frontend_framing(_fe, &nz, &skip, &effectiveSr);
        _nzFFTSize = nz;
    }

    sdrgpu_frontend* _fe = nullptr;
    std::mutex _mtx;   // one thread at a time on the device front end (worker vs setters)
    Worker _worker;
    std::map<std::string, Vfo> vfos;
    std::vector<float> _rows;

    double _sampleRate = 0;
    int _decimRatio = 1;
    bool _dcBlocking = false;
    int _fftSize = 0;
    double _fftRate = 0;
    dsp::window::windowType _fftWindow = dsp::window::BLACKMAN_HARRIS7;
    float* (*_acquireFFTBuffer)(void* ctx) = nullptr;
    void (*_releaseFFTBuffer)(void* ctx) = nullptr;
    void* _fftCtx = nullptr;
    int _nzFFTSize = 0;
    double effectiveSr = 0;
    bool _init = false;
};
