// C++ drop-in test of the GPU-backed IQFrontEnd (sdrpp_amd/dsp/gpu/signal_path/iq_frontend.h)
// inside the threaded stream model: a source thread writes blocks into the input stream (as a
// source module does, fs / 200 samples per block); the front end's worker hands back dB rows
// through acquire / releaseFFTBuffer, VFO outputs through the RxVFO's `out` stream (read by a
// consumer thread, as the radio module's demodulator would), and the IQ through a bound stream.
// Everything is checked against the same blocks pushed straight into a second device front end
// through the C ABI (same kernels: bit-exact), against the oracle (every delivered dB row vs the
// oracle's window * FFT * log-power of its reshaper frame, the VFO output vs the oracle's RxVFO),
// and the bound stream against the input. A second run checks the lossy input buffer
// (buffering = true, frame_buffer.h:64-71: a slow consumer makes the front end drop input blocks
// instead of blocking the source) and re-planning an attached VFO while the front end runs.
// Built and run by tests/test_cpp_dropin.py.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "signal_path/iq_frontend.h"
#include "sdr_oracle.h"

static int failures = 0;
#define CHECK(c, ...) do { if (!(c)) { std::printf("FAIL %s:%d ", __FILE__, __LINE__); std::printf(__VA_ARGS__); std::printf("\n"); failures++; } } while (0)

struct RowSink {
    std::vector<float> buf, rows;
    int n = 0, nullEvery = 0, acquired = 0, released = 0;
};
static float* acquire(void* ctx) {
    auto* s = (RowSink*)ctx;
    s->acquired++;
    if (s->nullEvery && s->acquired % s->nullEvery == 0) return nullptr;   // a consumer without a buffer
    return s->buf.data();
}
static void release(void* ctx) {
    auto* s = (RowSink*)ctx;
    s->released++;
    if (!(s->nullEvery && s->acquired % s->nullEvery == 0)) s->rows.insert(s->rows.end(), s->buf.begin(), s->buf.end());
    s->n++;
}

template <class T>
static void drain(dsp::stream<T>* s, std::vector<T>* out, int expect) {
    while ((int)out->size() < expect) {
        const int n = s->read();
        if (n < 0) return;
        out->insert(out->end(), s->readBuf, s->readBuf + n);
        s->flush();
    }
}

int main() {
    const double fs = 2.4e6;
    const int N = 65536, blk = 12000, nblk = 40;   // fs / 200 per block, 0.2 s
    std::mt19937 gen(0xACE1);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<dsp::complex_t> x((size_t)blk * nblk);
    for (size_t i = 0; i < x.size(); i++) {
        const double t = (double)i / fs;
        x[i] = {(float)(0.3 * std::cos(2 * M_PI * 150e3 * t)) + 1e-3f * U(gen), (float)(0.3 * std::sin(2 * M_PI * 150e3 * t)) + 1e-3f * U(gen)};
    }

    RowSink sink;
    sink.buf.resize(N);
    sink.nullEvery = 3;   // every third acquire returns NULL: computed, not written, released anyway
    dsp::stream<dsp::complex_t> in, iq;
    IQFrontEnd fe;
    fe.init(&in, fs, false, 1, false, N, 15.0, dsp::window::BLACKMAN_HARRIS7, acquire, release, &sink);
    CHECK(std::fabs(fe.getEffectiveSamplerate() - fs) < 1e-6, "effective rate %f", fe.getEffectiveSamplerate());
    dsp::channel::RxVFO* vfo = fe.addVFO("radio", 48000, 12500, 150e3);
    CHECK(vfo != nullptr, "addVFO");
    CHECK(fe.addVFO("radio", 48000, 12500, 0) == nullptr, "duplicate VFO name accepted");
    fe.bindIQStream(&iq);
    fe.start();

    // the reference path of the same blocks: a second device front end through the C ABI
    sdrgpu_frontend* ref = nullptr;
    CHECK(sdrgpu_frontend_create(&ref, 0, fs, 1, 0, N, 15.0, 6) == 0, "ref create");
    int rid = -1;
    CHECK(sdrgpu_frontend_add_vfo(ref, &rid, 48000, 12500, 150e3) == 0, "ref add_vfo");
    std::vector<float> refRows;
    std::vector<dsp::complex_t> refVfo;
    for (int b = 0; b < nblk; b++) {
        const int nf = sdrgpu_frontend_push(ref, x.data() + (size_t)b * blk, blk, -1);
        std::vector<float> r((size_t)std::max(nf, 0) * N);
        if (nf > 0) sdrgpu_frontend_read_spectra(ref, r.data(), nf);
        refRows.insert(refRows.end(), r.begin(), r.end());
        std::vector<dsp::complex_t> v(blk);
        const int n = sdrgpu_frontend_read_vfo(ref, rid, v.data(), blk);
        refVfo.insert(refVfo.end(), v.begin(), v.begin() + std::max(n, 0));
    }
    const int nRows = (int)(refRows.size() / N), nVfo = (int)refVfo.size();

    // consumers (the demodulator behind the VFO, the recorder behind the bound stream)
    std::vector<dsp::complex_t> gotVfo, gotIq;
    std::thread tv(drain<dsp::complex_t>, &vfo->out, &gotVfo, nVfo);
    std::thread ti(drain<dsp::complex_t>, &iq, &gotIq, blk * nblk);
    // the source module: one block per swap
    for (int b = 0; b < nblk; b++) {
        std::memcpy(in.writeBuf, x.data() + (size_t)b * blk, sizeof(dsp::complex_t) * blk);
        if (!in.swap(blk)) break;
    }
    tv.join();
    ti.join();
    for (int k = 0; k < 200 && sink.n < nRows; k++) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    fe.stop();

    CHECK(sink.n == nRows && sink.acquired == nRows && sink.released == nRows, "rows %d acquired %d released %d, expected %d",
          sink.n, sink.acquired, sink.released, nRows);
    int r = 0;
    for (int k = 0; k < nRows; k++) {
        if ((k + 1) % sink.nullEvery == 0) continue;
        if ((size_t)(r + 1) * N > sink.rows.size()) break;
        CHECK(std::memcmp(sink.rows.data() + (size_t)r * N, refRows.data() + (size_t)k * N, sizeof(float) * N) == 0,
              "dB row %d differs from the C-ABI front end", k);
        r++;
    }
    CHECK((int)gotVfo.size() == nVfo && nVfo > 0, "VFO samples %zu, expected %d", gotVfo.size(), nVfo);
    if ((int)gotVfo.size() == nVfo)
        CHECK(std::memcmp(gotVfo.data(), refVfo.data(), sizeof(dsp::complex_t) * nVfo) == 0, "VFO output differs");
    CHECK(gotIq.size() == x.size() && std::memcmp(gotIq.data(), x.data(), sizeof(dsp::complex_t) * x.size()) == 0,
          "bound IQ stream differs from the input (%zu samples)", gotIq.size());

    // setters on the attached VFO re-plan it on the device; removeVFO detaches it
    vfo->setOffset(-200e3);
    vfo->setBandwidth(25000);
    fe.removeVFO("radio");
    fe.setFFTSize(8192);
    CHECK(fe.getEffectiveSamplerate() > 0, "after setFFTSize");
    sdrgpu_frontend_destroy(ref);

    // ---- against the oracle: rows (reshaper framing: frame j at j * (nz + skip)) and the VFO
    {
        int skip = 0, nz = 0;
        orc_gen_reshape_params(fs, N, 15.0, &skip, &nz);
        std::vector<float> win(nz), work(4 * (size_t)N), ref(N);
        orc_create_window(6, win.data(), nz, 1);
        double worst = 0;
        int rr = 0;
        for (int k = 0; k < nRows; k++) {
            if ((k + 1) % sink.nullEvery == 0) continue;
            if ((size_t)(rr + 1) * N > sink.rows.size()) break;
            orc_fft_logmag((const float*)(x.data() + (size_t)k * (nz + skip)), nz, N, win.data(), work.data(), ref.data());
            const float* got = sink.rows.data() + (size_t)rr * N;
            const float peak = *std::max_element(ref.begin(), ref.end());
            for (int i = 0; i < N; i++)
                if (ref[i] > peak - 60) worst = std::max(worst, (double)std::fabs(got[i] - ref[i]));
            rr++;
        }
        CHECK(rr > 0 && worst < 1e-3, "dB rows vs oracle: max |err| %g dB over %d rows (bins within 60 dB of peak)", worst, rr);
        orc_vfo* ov = orc_vfo_create(fs, 48000, 12500, 150e3, 1);
        std::vector<float> ob(2 * (size_t)blk);
        std::vector<dsp::complex_t> want;
        for (int b = 0; b < nblk; b++) {
            const int m = orc_vfo_process(ov, (const float*)(x.data() + (size_t)b * blk), blk, ob.data());
            for (int i = 0; i < m; i++) want.push_back({ob[2 * i], ob[2 * i + 1]});
        }
        orc_vfo_destroy(ov);
        double verr = 0;
        for (size_t i = 0; i < std::min(want.size(), gotVfo.size()); i++)
            verr = std::max(verr, (double)std::max(std::fabs(want[i].re - gotVfo[i].re), std::fabs(want[i].im - gotVfo[i].im)));
        CHECK(want.size() == gotVfo.size() && verr < 5e-5, "VFO vs oracle RxVFO: %zu vs %zu samples, max |err| %g",
              gotVfo.size(), want.size(), verr);
    }
    std::printf("rows %d (every %d-th acquire NULL), VFO %d samples, IQ %zu samples\n", nRows, sink.nullEvery, nVfo, gotIq.size());

    // ---- lossy input buffer + live re-planning of an attached VFO
    {
        RowSink s2;
        s2.buf.resize(N);
        dsp::stream<dsp::complex_t> in2;
        IQFrontEnd fe2;
        fe2.init(&in2, fs, true, 1, false, N, 15.0, dsp::window::BLACKMAN_HARRIS7, acquire, release, &s2);
        dsp::channel::RxVFO* v2 = fe2.addVFO("slow", 48000, 12500, 150e3);
        fe2.start();
        std::atomic<long long> got{0};
        std::atomic<bool> quit{false};
        std::thread slow([&] {   // a demodulator that takes 3 ms per block (the source delivers one per 0.05 ms)
            while (!quit) {
                const int n = v2->out.read();
                if (n < 0) return;
                got += n;
                v2->out.flush();
                std::this_thread::sleep_for(std::chrono::milliseconds(3));
            }
        });
        const int nb2 = 300;
        const auto t0 = std::chrono::steady_clock::now();
        long long atSet = -1;
        int rowsAtSet = -1;
        for (int b = 0; b < nb2; b++) {
            std::memcpy(in2.writeBuf, x.data() + (size_t)(b % nblk) * blk, sizeof(dsp::complex_t) * blk);
            if (!in2.swap(blk)) break;
            if (b == nb2 / 2) {   // SDR++ re-plans VFOs while the radio runs (bandwidth slider)
                v2->setBandwidth(25000);
                v2->setOffset(-100e3);
                atSet = got.load();
                rowsAtSet = s2.n;
            }
        }
        const double srcMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::this_thread::sleep_for(std::chrono::milliseconds(400));
        const long long dropped = fe2.droppedBlocks();
        const long long gotEnd = got.load();
        const int rowsEnd = s2.n;
        quit = true;
        fe2.stop();
        v2->out.stopReader();
        slow.join();
        CHECK(dropped > 0, "lossy buffer dropped no block behind a slow consumer");
        CHECK(atSet >= 0 && gotEnd > atSet, "VFO output stopped after setBandwidth (%lld -> %lld samples)", atSet, gotEnd);
        CHECK(rowsAtSet >= 0 && rowsEnd > rowsAtSet, "rows stopped after setBandwidth (%d -> %d)", rowsAtSet, rowsEnd);
        std::printf("lossy run: %d source blocks in %.1f ms, %lld dropped, VFO %lld -> %lld samples, rows %d -> %d\n", nb2,
                    srcMs, dropped, atSet, gotEnd, rowsAtSet, rowsEnd);
    }
    // ---- a setter parks the worker while it is blocked in a VFO out.swap with the ring empty
    // (the delivered block's ticket and ring slot were dropped a second time)
    {
        RowSink s3;
        s3.buf.resize(N);
        dsp::stream<dsp::complex_t> in3;
        IQFrontEnd fe3;
        fe3.init(&in3, fs, false, 1, false, N, 15.0, dsp::window::BLACKMAN_HARRIS7, acquire, release, &s3);
        dsp::channel::RxVFO* v3 = fe3.addVFO("stalled", 48000, 12500, 150e3);   // nobody reads v3->out
        fe3.start();
        for (int round = 0; round < 4; round++) {
            for (int b = 0; b < 3; b++) {   // the second delivery blocks in out.swap: the reader never flushes
                std::memcpy(in3.writeBuf, x.data() + (size_t)b * blk, sizeof(dsp::complex_t) * blk);
                if (!in3.swap(blk)) break;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(50));   // worker now waits in swap, ring empty
            v3->setBandwidth(round % 2 ? 25000 : 12500);   // pause: tempStop -> stopWriter(out) -> swap false
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
            fe3.stop();   // and again from stop() itself
            CHECK(fe3.ringSlotsConsistent(), "round %d: an input-ring slot is free / queued twice or lost", round);
            fe3.start();
        }
        fe3.stop();
        CHECK(fe3.ringSlotsConsistent(), "after the stalled-consumer rounds: ring slots inconsistent");
        std::printf("stalled-consumer run: ring slots consistent after 4 parks in out.swap\n");
    }
    std::printf(failures ? "FAILED (%d)\n" : "ALL OK\n", failures);
    return failures ? 1 : 0;
}
