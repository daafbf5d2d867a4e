// C++ drop-in test: the GPU-backed dsp:: blocks run inside the reference's threaded
// stream/block model (runtime mirror) and match the CPU restatement (oracle) sample for
// sample within the stated tolerances. Built and run by tests/test_cpp_dropin.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include <dsp/stream.h>
#include <dsp/sink/handler_sink.h>
#include "dsp/channel/rx_vfo.h"
#include "dsp/demod/broadcast_fm.h"
#include "dsp/demod/quadrature.h"
#include "dsp/filter/decimating_fir.h"
#include "dsp/signal_path/gpu_spectrum.h"
#include "dsp/correction/dc_blocker.h"
#include "dsp/demod/am.h"
#include "dsp/demod/ssb.h"
#include "dsp/loop/agc.h"
#include "dsp/filter/deephasis.h"
#include "sdr_oracle.h"

static int failures = 0;
#define CHECK(c, ...) do { if (!(c)) { std::printf("FAIL %s:%d ", __FILE__, __LINE__); std::printf(__VA_ARGS__); std::printf("\n"); failures++; } } while (0)

// feeds `blocks` of IQ into a stream from a writer thread (SpeedTester-style)
struct Feeder {
    dsp::stream<dsp::complex_t> out;
};

int main() {
    std::mt19937 gen(0xACE1);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    const int blk = 307200, nblk = 6;
    std::vector<dsp::complex_t> x((size_t)blk * nblk);
    for (auto& v : x) v = {U(gen), U(gen)};

    // 1. threaded pipeline: stream -> RxVFO(61.44M -> 240k) -> BroadcastFM mono -> collector
    {
        dsp::stream<dsp::complex_t> src;
        dsp::channel::RxVFO vfo(&src, 61.44e6, 240000, 200000, 2.5e6);
        dsp::demod::BroadcastFM wfm(&vfo.out, 100000, 240000, false, true, false);
        std::vector<dsp::stereo_t> got;
        dsp::sink::Handler<dsp::stereo_t> sink(&wfm.out, [](dsp::stereo_t* d, int n, void* ctx) {
            auto* g = (std::vector<dsp::stereo_t>*)ctx;
            g->insert(g->end(), d, d + n);
        }, &got);
        vfo.start(); wfm.start(); sink.start();
        for (int b = 0; b < nblk; b++) {
            std::memcpy(src.writeBuf, x.data() + (size_t)b * blk, sizeof(dsp::complex_t) * blk);
            CHECK(src.swap(blk), "swap");
        }
        // wait for the last batch to drain
        for (int i = 0; i < 200 && (int)got.size() < nblk * blk / 256; i++) std::this_thread::sleep_for(std::chrono::milliseconds(10));
        sink.stop(); wfm.stop(); vfo.stop();

        orc_vfo* ov = orc_vfo_create(61.44e6, 240000, 200000, 2.5e6, 1);
        orc_wfm* ow = orc_wfm_create(100000, 240000, 1, 1);
        std::vector<float> ifb(2 * blk), aud(2 * blk);
        std::vector<float> want;
        for (int b = 0; b < nblk; b++) {
            int m = orc_vfo_process(ov, (const float*)(x.data() + (size_t)b * blk), blk, ifb.data());
            orc_wfm_process(ow, ifb.data(), m, aud.data());
            want.insert(want.end(), aud.begin(), aud.begin() + 2 * m);
        }
        CHECK(got.size() * 2 == want.size(), "pipeline output count %zu vs %zu", got.size() * 2, want.size());
        double err = 0;
        for (size_t i = 0; i < got.size() && 2 * i + 1 < want.size(); i++) {
            err = std::fmax(err, std::fabs(got[i].l - want[2 * i]));
            CHECK(got[i].l == got[i].r, "mono l != r at %zu", i);
            if (failures > 5) break;
        }
        CHECK(err < 1e-3, "pipeline audio max err %g", err);
        std::printf("pipeline RxVFO->WFM: %zu stereo samples, max err %.3g\n", got.size(), err);
        orc_vfo_destroy(ov); orc_wfm_destroy(ow);
    }

    // 2. direct process() calls (the reference's synchronous call style)
    {
        std::vector<float> taps(256);
        int n = sdrgpu_taps_low_pass(3.0e6, 912000.0, 61.44e6, 0, taps.data());
        CHECK(n == 256, "tap count %d", n);
        dsp::tap<float> t{taps.data(), (unsigned)n};
        dsp::stream<dsp::complex_t> dummy;
        dsp::filter::DecimatingFIR<dsp::complex_t, float> fir(&dummy, t, 8);
        orc_fir* of = orc_fir_create(1, 0, taps.data(), n, 8, 1);
        std::vector<dsp::complex_t> y(blk);
        std::vector<float> yo(2 * blk);
        double err = 0;
        for (int b = 0; b < 3; b++) {
            int m = fir.process(blk, x.data() + (size_t)b * blk, y.data());
            int mo = orc_fir_process(of, (const float*)(x.data() + (size_t)b * blk), blk, yo.data());
            CHECK(m == mo, "decim fir count %d vs %d", m, mo);
            for (int i = 0; i < m; i++) err = std::fmax(err, std::fmax(std::fabs(y[i].re - yo[2 * i]), std::fabs(y[i].im - yo[2 * i + 1])));
        }
        CHECK(err < 1e-5, "decim fir err %g", err);
        std::printf("DecimatingFIR<complex_t,float> 256/8: max err %.3g\n", err);
        orc_fir_destroy(of);
    }

    // 3. spectrum handler with acquire/release (including the NULL-buffer case)
    {
        dsp::gpu::Spectrum sp;
        CHECK(sp.update(65536, 65536, 6), "spectrum update");
        std::vector<float> row(65536), work(4 * 65536), ref(65536), win(65536);
        int acquired = 0, released = 0;
        sp.handler(x.data(), 65536, [&]() { acquired++; return row.data(); }, [&]() { released++; });
        sp.handler(x.data(), 65536, [&]() { acquired++; return (float*)nullptr; }, [&]() { released++; });
        CHECK(acquired == 2 && released == 2, "acquire/release %d/%d", acquired, released);
        orc_create_window(6, win.data(), 65536, 1);
        orc_fft_logmag((const float*)x.data(), 65536, 65536, win.data(), work.data(), ref.data());
        double err = 0, peak = -1e30;
        for (float v : ref) peak = std::fmax(peak, v);
        for (int k = 0; k < 65536; k++) if (ref[k] > peak - 60) err = std::fmax(err, std::fabs(row[k] - ref[k]));
        CHECK(err < 2e-3, "spectrum err %g dB", err);
        std::printf("Spectrum 64k BH7 via handler: max |dB err| within 60 dB of peak %.3g\n", err);
    }
    // 4. AM<stereo_t> / SSB<float> / AGC<float> / DCBlocker<float> on 48 kS/s IF (am.h, ssb.h)
    {
        const int n = 48000;
        std::vector<dsp::complex_t> ifx(n);
        for (int i = 0; i < n; i++) {
            double t = i / 48000.0, env = 1.0 + 0.5 * std::sin(2 * M_PI * 600 * t);
            ifx[i] = {(float)(0.05 * env * std::cos(2 * M_PI * 400 * t)), (float)(0.05 * env * std::sin(2 * M_PI * 400 * t))};
        }
        dsp::stream<dsp::complex_t> dummy;
        dsp::demod::AM<dsp::stereo_t> am;
        am.init(&dummy, dsp::demod::AM<dsp::stereo_t>::AUDIO, 10000, 50.0 / 48000, 5.0 / 48000, 10.0 / 48000, 48000);
        std::vector<dsp::stereo_t> st(n);
        std::vector<float> ref(n);
        orc_am* oa = orc_am_create(2, 10000, 50.0 / 48000, 5.0 / 48000, 10.0 / 48000, 48000, 1);
        int m = am.process(n / 2, ifx.data(), st.data());
        m += am.process(n - n / 2, ifx.data() + n / 2, st.data() + n / 2);
        orc_am_process(oa, (const float*)ifx.data(), n / 2, ref.data());
        orc_am_process(oa, (const float*)(ifx.data() + n / 2), n - n / 2, ref.data() + n / 2);
        double err = 0, pk = 0;
        for (int i = 0; i < m; i++) { err = std::fmax(err, std::fabs(st[i].l - ref[i])); pk = std::fmax(pk, std::fabs(ref[i])); CHECK(st[i].l == st[i].r, "am l!=r"); if (failures > 5) break; }
        CHECK(m == n && err <= 2e-5 * std::fmax(pk, 1.0), "AM<stereo_t> n %d err %g (peak %g)", m, err, pk);
        std::printf("AM<stereo_t> AUDIO AGC: max err %.3g (peak %.3g), gain %.4g\n", err, pk, am.getAGCGain());
        orc_am_destroy(oa);

        dsp::demod::SSB<float> ssb;
        ssb.init(&dummy, dsp::demod::SSB<float>::USB, 2800, 48000, true, 50.0 / 48000, 5.0 / 48000);
        std::vector<float> so(n), sr(n);
        orc_ssb* os = orc_ssb_create(0, 2800, 48000, 1, 50.0 / 48000, 5.0 / 48000);
        int k = ssb.process(n, ifx.data(), so.data());
        orc_ssb_process(os, (const float*)ifx.data(), n, sr.data());
        err = 0; pk = 0;
        for (int i = 0; i < k; i++) { err = std::fmax(err, std::fabs(so[i] - sr[i])); pk = std::fmax(pk, std::fabs(sr[i])); }
        CHECK(k == n && err <= 1e-5 * std::fmax(pk, 1e-30) + 1e-6, "SSB<float> err %g (peak %g)", err, pk);
        std::printf("SSB<float> USB: max err %.3g (peak %.3g)\n", err, pk);
        orc_ssb_destroy(os);

        dsp::stream<float> fdummy;
        dsp::loop::AGC<float> agc;
        agc.init(&fdummy, 1.0, 0.01, 0.001, 10e6, 10.0, INFINITY);
        dsp::correction::DCBlocker<float> dcb(&fdummy, 10.0, 48000.0);
        std::vector<float> a(n), b(n), c(n), d(n);
        for (int i = 0; i < n; i++) a[i] = 0.3f + 0.2f * (float)std::sin(0.01 * i) * (i % 5000 < 2500 ? 1.0f : 0.01f);
        dcb.process(n, a.data(), b.data());
        agc.process(n, b.data(), c.data());
        orc_dcb* od = orc_dcb_create(0, 10.0 / 48000.0);
        orc_agc* og = orc_agc_create(0, 1.0, 0.01, 0.001, 10e6, 10.0, INFINITY);
        orc_dcb_process(od, a.data(), n, d.data());
        orc_agc_process(og, d.data(), n, d.data());
        CHECK(std::memcmp(c.data(), d.data(), sizeof(float) * n) == 0, "DCBlocker->AGC not bit-exact");
        std::printf("DCBlocker<float> -> AGC<float>: bit-exact %s\n", std::memcmp(c.data(), d.data(), sizeof(float) * n) == 0 ? "yes" : "NO");
        orc_dcb_destroy(od); orc_agc_destroy(og);

        // BroadcastFM with the RDS branch (init(..., rdsOut = true)): 5 kS/s complex baseband per block
        {
            dsp::demod::BroadcastFM bfm;
            bfm.init(&dummy, 100000, 240000, true, true, true);
            std::vector<dsp::stereo_t> aud(n);
            std::vector<dsp::complex_t> rds(n);
            int rdsCount = -1;
            const int a1 = bfm.process(n, ifx.data(), aud.data(), rdsCount, rds.data());
            double e = 0;
            for (int i = 0; i < rdsCount; i++) e += (double)rds[i].re * rds[i].re + (double)rds[i].im * rds[i].im;
            CHECK(a1 == n && std::abs(rdsCount - (int)((long long)n * 5000 / 240000)) <= 2 && e > 0, "BroadcastFM RDS: audio %d rds %d", a1, rdsCount);
            std::printf("BroadcastFM stereo + RDS: %d audio, %d RDS samples\n", a1, rdsCount);
        }

        // Deemphasis<float> over two blocks vs the reference recurrence (filter/deephasis.h:58-65, 91-94)
        dsp::filter::Deemphasis<float> de(&fdummy, 50e-6, 48000.0);
        std::vector<float> e(n), g(n);
        de.process(n / 3, c.data(), e.data());
        de.process(n - n / 3, c.data() + n / 3, e.data() + n / 3);
        const double tau = 50e-6, fsr = 48000.0;
        const float dt = 1.0f / fsr;
        const float alpha = dt / (tau + dt);
        float last = 0;
        for (int i = 0; i < n; i++) { g[i] = (alpha * c[i]) + ((1 - alpha) * last); last = g[i]; }
        CHECK(std::memcmp(e.data(), g.data(), sizeof(float) * n) == 0, "Deemphasis not bit-exact");
        std::printf("Deemphasis<float>: bit-exact %s\n", std::memcmp(e.data(), g.data(), sizeof(float) * n) == 0 ? "yes" : "NO");
    }
    // device placement (sdrgpu_handle.h): a DeviceScope pins the blocks built in it; without one,
    // SDRGPU_PLACEMENT=spread deals the RxVFOs round-robin over the visible GPUs; the device is
    // kept across re-plans; setDevice moves a VFO and it still matches a fresh one
    {
        const int ndev = sdrgpu_device_count();
        {
            dsp::gpu::DeviceScope on(ndev - 1);
            dsp::stream<dsp::complex_t> in;
            dsp::channel::RxVFO v(&in, 61.44e6, 240000, 200000, 2.5e6);
            CHECK(v.getDevice() == ndev - 1, "scope placement: %d", v.getDevice());
            v.setBandwidth(150000);
            CHECK(v.getDevice() == ndev - 1, "device kept across a re-plan: %d", v.getDevice());
        }
        setenv("SDRGPU_PLACEMENT", "spread", 1);
        std::vector<int> seen;
        for (int k = 0; k < 2 * ndev; k++) {
            dsp::stream<dsp::complex_t> in;
            dsp::channel::RxVFO v(&in, 61.44e6, 240000, 200000, 2.5e6);
            seen.push_back(v.getDevice());
        }
        unsetenv("SDRGPU_PLACEMENT");
        for (int k = 0; k < 2 * ndev; k++) CHECK(seen[k] == (seen[0] + k) % ndev,
                                                 "spread placement: VFO %d on %d", k, seen[k]);
        dsp::stream<dsp::complex_t> in;
        dsp::channel::RxVFO a(&in, 61.44e6, 240000, 200000, 2.5e6), b(&in, 61.44e6, 240000, 200000, 2.5e6);
        a.setDevice(ndev - 1);
        std::vector<dsp::complex_t> ya(blk / 256 + 8), yb(blk / 256 + 8);
        const int ma = a.process(blk, x.data(), ya.data()), mb = b.process(blk, x.data(), yb.data());
        CHECK(ma == mb && ma > 0, "moved VFO output count %d vs %d", ma, mb);
        float d = 0.f;
        for (int i = 0; i < ma && i < mb; i++) d = std::fmax(d, std::fabs(ya[i].re - yb[i].re) + std::fabs(ya[i].im - yb[i].im));
        CHECK(d <= 1e-5f, "moved VFO output differs by %g", d);
        std::printf("placement: %d device(s), spread ->", ndev);
        for (int v : seen) std::printf(" %d", v);
        std::printf("\n");
    }

    std::printf(failures ? "FAILED (%d)\n" : "ALL OK\n", failures);
    return failures ? 1 : 0;
}
