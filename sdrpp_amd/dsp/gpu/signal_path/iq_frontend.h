// GPU-backed IQFrontEnd -- drop-in for core/src/signal_path/iq_frontend.{h,cpp}: the same class
// name and public interface (init, setSampleRate, setBuffering, setDecimation, setInvertIQ,
// setDCBlocking, bindIQStream, addVFO / removeVFO, setFFTSize / Rate / Window, flushInputBuffer,
// start / stop, ...), header-only.
//
// The whole data path runs in libsdrgpu's device front end (sdrgpu_frontend_*, include/sdrgpu.h):
// one H2D per input block, then on the device the preprocessing (PowerDecimator, DCBlocker,
// Conjugate), the reshaper's keep / skip framing (genReshapeParams, iq_frontend.h:56-60),
// window * FFT * log-power (iq_frontend.cpp:230-249), and every VFO reading the block in place
// (addVFO, :122-142) -- instead of the SampleFrameBuffer -> Splitter -> Reshaper memcpy fan-out.
//
// Two threads, as the reference's SampleFrameBuffer has (buffer/frame_buffer.h:52-94):
//   * the input buffer (InputRing, "dspBuf:loop") copies each block of the input stream into a
//     slot of a 32-slot ring of pinned host buffers. With buffering on (the reference's default,
//     gui/main_window.cpp:89) it never blocks the source: when every slot is taken, the oldest
//     queued block is dropped (the reference overwrites slots, frame_buffer.h:64-71; its ring
//     then also looks empty for a whole lap, which drops 32 blocks at once -- here exactly the
//     oldest one goes). With buffering off (bypass) the source waits for a free slot;
//   * the device worker (Worker, a dsp::block) takes queued slots and submits them to the device
//     front end without waiting (sdrgpu_frontend_submit: the slot is DMA'd straight to the GPU);
//     while blocks are queued it submits block k + 1 before it collects block k, so the H2D of one
//     block overlaps the kernels and read-back of the previous one and the host hand-off of the
//     results. The results of a block go out, in order:
//       - each dB row through acquire / releaseFFTBuffer (a NULL buffer skips the copy but release
//         is still called, as in handler);
//       - each VFO's output into that VFO's `out` stream (the VFO is an RxVFO attached to the
//         front end: its own worker is idle, its setters re-plan it on the device and pause this
//         worker instead of stopping the VFO's own streams);
//       - the preprocessed IQ into every bound stream (bindIQStream: the recorder, IQ exporters).
// Inside the SDR++ tree (core.h present) it keeps the reference's couplings:
// core::setInputSampleRate on a rate change and gui::waterfall.setRawFFTSize on an FFT change.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>
#include <sdrgpu.h>
#include "../dsp/block.h"
#include "../dsp/stream.h"
#include "../dsp/window/window.h"
#include "../dsp/channel/rx_vfo.h"
// the reference header's own includes (core/src/signal_path/iq_frontend.h:2-12): callers rely on
// them transitively (the radio module's WFM takes dsp::sink::Handler and dsp::buffer::Reshaper
// through signal_path.h). Headers that exist only in the SDR++ tree are guarded.
#if __has_include("../dsp/buffer/frame_buffer.h")
#include "../dsp/buffer/frame_buffer.h"
#endif
#if __has_include("../dsp/buffer/reshaper.h")
#include "../dsp/buffer/reshaper.h"
#endif
#if __has_include("../dsp/multirate/power_decimator.h")
#include "../dsp/multirate/power_decimator.h"
#endif
#if __has_include("../dsp/correction/dc_blocker.h")
#include "../dsp/correction/dc_blocker.h"
#endif
#if __has_include("../dsp/chain.h")
#include "../dsp/chain.h"
#endif
#if __has_include("../dsp/routing/splitter.h")
#include "../dsp/routing/splitter.h"
#endif
#if __has_include("../dsp/sink/handler_sink.h")
#include "../dsp/sink/handler_sink.h"
#endif
#if __has_include("../dsp/math/conjugate.h")
#include "../dsp/math/conjugate.h"
#endif
#if __has_include(<fftw3.h>)
#include <fftw3.h>
#endif
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
    static constexpr int RING_SLOTS = 32;   // TEST_BUFFER_SIZE (frame_buffer.h:3)

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
        dsp::gpu::ok(sdrgpu_frontend_create(&_fe, dsp::gpu::device(), sampleRate, decimRatio, dcBlocking, fftSize, fftRate,
                                            (int)fftWindow),
                     "frontend_create");
        refreshFraming();
        _ring.lossy = buffering;
        _inBuf.ring = &_ring;
        _inBuf.setInput(in);
        _worker.fe = this;
        _worker.ring = &_ring;
        _worker.init();
        _init = true;
    }

    // IQFrontEnd::updateFFTSize (iq_frontend.cpp:272-296): window + plan for the current framing
    void updateFFTSize() {
        std::lock_guard<std::mutex> l(_mtx);
        dsp::gpu::ok(sdrgpu_frontend_set_fft(_fe, _fftSize, _fftRate, (int)_fftWindow), "frontend_set_fft");
        refreshFraming();
    }

    void setInput(dsp::stream<dsp::complex_t>* in) { _inBuf.setInput(in); }
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

    // SampleFrameBuffer bypass = !enabled (iq_frontend.cpp:27-28)
    void setBuffering(bool enabled) { _ring.setLossy(enabled); }
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
        vfo->attach(in, _fe, id, &_mtx, &_worker, effectiveSr, sampleRate, bandwidth, offset);
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

    // SampleFrameBuffer::flush (frame_buffer.h:46-49): drop every queued block
    void flushInputBuffer() { _ring.flush(); }
    void start() {
        _worker.start();
        _inBuf.start();
    }
    void stop() {
        _inBuf.stop();
        _worker.stop();
    }
    double getEffectiveSamplerate() { return effectiveSr; }

    // (not in the reference) the device front end under this object, for sdrgpu_frontend_* calls
    sdrgpu_frontend* device_frontend() { return _fe; }
    // (not in the reference) input blocks dropped by the lossy ring since init
    long long droppedBlocks() { return _ring.droppedCount(); }
    // (not in the reference; test hook, call with the worker stopped) every input-ring slot is
    // exactly once free, queued or held by the worker's block in flight
    bool ringSlotsConsistent() { return _ring.consistent(_worker.pendingSlot >= 0 ? 1 : 0); }

protected:
    struct Vfo {
        dsp::channel::RxVFO* vfo;
        dsp::stream<dsp::complex_t>* in;   // idle placeholder input of the attached VFO
    };

    // 32 pinned block slots: free -> queued (FIFO) -> in flight on the device -> free
    class InputRing {
    public:
        bool lossy = true;
        ~InputRing() {
            for (auto& s : slots)
                if (s.buf) sdrgpu_host_free(s.buf);
        }
        void setLossy(bool l) {
            std::lock_guard<std::mutex> lk(mtx);
            lossy = l;
            cv.notify_all();
        }
        // writer (input thread): one block; false when stopped
        bool push(const dsp::complex_t* data, int count) {
            std::unique_lock<std::mutex> lk(mtx);
            int idx = -1;
            for (;;) {
                if (wstop) return false;
                if (!freeList.empty()) {
                    idx = freeList.back();
                    freeList.pop_back();
                    break;
                }
                if (lossy && !queue.empty()) {   // drop the oldest queued block
                    idx = queue.front();
                    queue.pop_front();
                    dropped++;
                    break;
                }
                cv.wait(lk);   // bypass (or every slot in flight): wait for the device worker
            }
            Slot& s = slots[idx];
            if (s.cap < count) {
                if (s.buf) sdrgpu_host_free(s.buf);
                s.buf = nullptr;
                s.cap = 0;
                void* p = nullptr;
                const int cap = std::max(count, 1 << 16);
                if (!dsp::gpu::ok(sdrgpu_host_alloc(&p, sizeof(dsp::complex_t) * (size_t)cap), "host_alloc")) {
                    freeList.push_back(idx);
                    return false;
                }
                s.buf = (dsp::complex_t*)p;
                s.cap = cap;
            }
            // the copy runs under the lock: flush() / the worker never see a half-written slot
            std::memcpy(s.buf, data, sizeof(dsp::complex_t) * (size_t)count);
            s.count = count;
            queue.push_back(idx);
            cv.notify_all();
            return true;
        }
        // device worker: next queued slot (wait = block until one arrives); -1 when stopped / none
        int pop(bool wait) {
            std::unique_lock<std::mutex> lk(mtx);
            if (wait) cv.wait(lk, [this] { return !queue.empty() || rstop; });
            if (rstop || queue.empty()) return -1;
            const int idx = queue.front();
            queue.pop_front();
            return idx;
        }
        bool empty() {
            std::lock_guard<std::mutex> lk(mtx);
            return queue.empty();
        }
        // false (and no change) when idx is out of range, already free or still queued
        bool release(int idx) {
            std::lock_guard<std::mutex> lk(mtx);
            if (idx < 0 || idx >= RING_SLOTS) return false;
            if (std::find(freeList.begin(), freeList.end(), idx) != freeList.end()) return false;
            if (std::find(queue.begin(), queue.end(), idx) != queue.end()) return false;
            freeList.push_back(idx);
            cv.notify_all();
            return true;
        }
        // every slot index exactly once over free + queued + the n in flight (test hook)
        bool consistent(int inFlight) {
            std::lock_guard<std::mutex> lk(mtx);
            std::vector<int> seen(RING_SLOTS, 0);
            for (int i : freeList) seen[i]++;
            for (int i : queue) seen[i]++;
            int missing = 0;
            for (int c : seen) {
                if (c > 1) return false;
                missing += c == 0;
            }
            return missing == inFlight;
        }
        void flush() {
            std::lock_guard<std::mutex> lk(mtx);
            for (int i : queue) freeList.push_back(i);
            queue.clear();
            cv.notify_all();
        }
        void stopWriter(bool v) {
            std::lock_guard<std::mutex> lk(mtx);
            wstop = v;
            cv.notify_all();
        }
        void stopReader(bool v) {
            std::lock_guard<std::mutex> lk(mtx);
            rstop = v;
            cv.notify_all();
        }
        long long droppedCount() {
            std::lock_guard<std::mutex> lk(mtx);
            return dropped;
        }
        const dsp::complex_t* data(int idx) const { return slots[idx].buf; }
        int count(int idx) const { return slots[idx].count; }

    private:
        struct Slot {
            dsp::complex_t* buf = nullptr;
            int cap = 0, count = 0;
        };
        Slot slots[RING_SLOTS];
        std::vector<int> freeList = [] {
            std::vector<int> v;
            for (int i = RING_SLOTS - 1; i >= 0; i--) v.push_back(i);
            return v;
        }();
        std::deque<int> queue;
        std::mutex mtx;
        std::condition_variable cv;
        bool wstop = false, rstop = false;
        long long dropped = 0;
    };

    // input stream -> ring (SampleFrameBuffer::run, frame_buffer.h:52-75)
    class InputBuffer : public dsp::block {
    public:
        InputRing* ring = nullptr;
        void setInput(dsp::stream<dsp::complex_t>* in) {
            std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
            tempStop();
            if (_in) unregisterInput(_in);
            _in = in;
            registerInput(_in);
            _block_init = true;
            tempStart();
        }
        int run() override {
            const int count = _in->read();
            if (count < 0) return -1;
            const bool ok = ring->push(_in->readBuf, count);
            _in->flush();
            return ok ? count : -1;
        }

    protected:
        void doStop() override {
            ring->stopWriter(true);
            dsp::block::doStop();
            ring->stopWriter(false);
        }
        dsp::stream<dsp::complex_t>* _in = nullptr;
    };

    // ring -> device front end -> rows / VFO outputs / bound IQ streams
    class Worker : public dsp::block {
    public:
        IQFrontEnd* fe = nullptr;
        InputRing* ring = nullptr;
        void init() { _block_init = true; }
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
        int run() override { return fe->iteration(*this); }
        std::vector<dsp::stream<dsp::complex_t>*> bound;
        // the block submitted but not yet handed on (ticket, ring slot)
        int pendingTicket = -1, pendingSlot = -1;

    protected:
        void doStop() override {
            ring->stopReader(true);
            dsp::block::doStop();
            ring->stopReader(false);
            fe->dropPending(*this);   // a block in flight when the worker parks is dropped
        }
    };

    // one worker step: submit the next block, hand on the previous one's results
    int iteration(Worker& w) {
        // nothing queued: hand on the block in flight first (no extra latency when keeping up)
        if (w.pendingTicket >= 0 && _ring.empty()) {
            // deliver() releases the ticket and the slot whatever it returns: clear them first,
            // or a stop landing in an output swap would drop them a second time (doStop)
            const int t = w.pendingTicket, s = w.pendingSlot;
            w.pendingTicket = w.pendingSlot = -1;
            if (!deliver(w, t, s)) return -1;
        }
        const int slot = _ring.pop(true);
        if (slot < 0) return -1;
        int ticket;
        {
            std::lock_guard<std::mutex> l(_mtx);
            ticket = sdrgpu_frontend_submit(_fe, _ring.data(slot), _ring.count(slot), -1, w.bound.empty() ? 0 : SDRGPU_FE_IQ);
        }
        if (!dsp::gpu::ok(ticket, "frontend_submit")) {
            releaseSlot(slot);
            return -1;
        }
        if (w.pendingTicket >= 0) {
            const int t = w.pendingTicket, s = w.pendingSlot;
            w.pendingTicket = w.pendingSlot = -1;
            if (!deliver(w, t, s)) {
                dropTicket(ticket, slot);
                return -1;
            }
        }
        w.pendingTicket = ticket;
        w.pendingSlot = slot;
        return _ring.count(slot);
    }

    // collect a block's results and hand them on; false when an output stream was stopped
    bool deliver(Worker& w, int ticket, int slot) {
        const float* rows = nullptr;
        const void* iq = nullptr;
        int niq = 0, nf;
        std::vector<std::pair<dsp::channel::RxVFO*, std::pair<const void*, int>>> outs;
        {
            std::lock_guard<std::mutex> l(_mtx);
            nf = sdrgpu_frontend_collect(_fe, ticket, &rows, &iq, &niq);
            for (auto& [name, v] : vfos) {
                const void* p = nullptr;
                int n = 0;
                if (sdrgpu_frontend_collected_vfo(_fe, ticket, v.vfo->frontEndId(), &p, &n) >= 0) outs.push_back({v.vfo, {p, n}});
            }
        }
        releaseSlot(slot);   // the block's H2D is done
        bool ok = dsp::gpu::ok(nf, "frontend_collect");
        // a stream buffer holds STREAM_BUFFER_SIZE samples (stream.h): an interpolating VFO's
        // output past that fails the delivery instead of writing past writeBuf
        for (auto& [vfo, pn] : outs)
            if (pn.second > STREAM_BUFFER_SIZE) ok = dsp::gpu::ok(SDRGPU_EARG, "VFO output exceeds STREAM_BUFFER_SIZE");
        if (niq > STREAM_BUFFER_SIZE) ok = dsp::gpu::ok(SDRGPU_EARG, "IQ block exceeds STREAM_BUFFER_SIZE");
        for (int r = 0; ok && r < nf; r++) {   // IQFrontEnd::handler's acquire -> write -> release per row
            float* buf = _acquireFFTBuffer(_fftCtx);
            if (buf) std::memcpy(buf, rows + (size_t)r * _fftSize, sizeof(float) * _fftSize);
            _releaseFFTBuffer(_fftCtx);
        }
        for (auto& [vfo, pn] : outs) {
            if (!ok || pn.second <= 0) continue;
            std::memcpy(vfo->out.writeBuf, pn.first, sizeof(dsp::complex_t) * (size_t)pn.second);
            ok = vfo->out.swap(pn.second);
        }
        for (size_t k = 0; ok && k < w.bound.size() && niq > 0; k++) {
            std::memcpy(w.bound[k]->writeBuf, iq, sizeof(dsp::complex_t) * (size_t)niq);
            ok = w.bound[k]->swap(niq);
        }
        std::lock_guard<std::mutex> l(_mtx);
        sdrgpu_frontend_release(_fe, ticket);
        return ok;
    }

    void releaseSlot(int slot) {
        if (!_ring.release(slot)) SDRGPU_FE_ERROR("input ring slot released twice");
    }
    void dropTicket(int ticket, int slot) {
        {
            std::lock_guard<std::mutex> l(_mtx);
            sdrgpu_frontend_collect(_fe, ticket, nullptr, nullptr, nullptr);
            sdrgpu_frontend_release(_fe, ticket);
        }
        releaseSlot(slot);
    }
    void dropPending(Worker& w) {
        if (w.pendingTicket < 0) return;
        dropTicket(w.pendingTicket, w.pendingSlot);
        w.pendingTicket = w.pendingSlot = -1;
    }

    void refreshFraming() {
        int nz = 0, skip = 0;
        sdrgpu_frontend_framing(_fe, &nz, &skip, &effectiveSr);
        _nzFFTSize = nz;
    }

    sdrgpu_frontend* _fe = nullptr;
    std::mutex _mtx;   // one thread at a time on the device front end (worker vs setters)
    InputRing _ring;
    InputBuffer _inBuf;
    Worker _worker;
    std::map<std::string, Vfo> vfos;

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
