// C++ drop-in test of the GPU-backed IQFrontEnd (sdrpp_amd/dsp/gpu/signal_path/iq_frontend.h)
// inside the threaded stream model: a source thread writes blocks into the input stream (as a
// source module does, fs / 200 samples per block); the front end's worker hands back dB rows
// through acquire / releaseFFTBuffer, VFO outputs through the RxVFO's `out` stream (read by a
// consumer thread, as the radio module's demodulator would), and the IQ through a bound stream.
// Everything is checked against the same blocks pushed straight into a second device front end
// through the C ABI (same kernels: bit-exact), and the bound stream against the input.
// Built and run by tests/test_cpp_dropin.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "signal_path/iq_frontend.h"

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
    std::printf("rows %d (every %d-th acquire NULL), VFO %d samples, IQ %zu samples\n", nRows, sink.nullEvery, nVfo, gotIq.size());
    std::printf(failures ? "FAILED (%d)\n" : "ALL OK\n", failures);
    return failures ? 1 : 0;
}
