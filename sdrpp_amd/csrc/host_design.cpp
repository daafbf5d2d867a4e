// Host-side design code of libsdrgpu: windows, FIR taps, decimation plans, NCO
// phase bookkeeping. Setup-time only (the reference also computes these on the
// host). Compiled with -ffp-contract=off and no fast-math so every expression
// rounds exactly as the reference source's does (bit-exact tables).
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <cstdlib>
#include "sdrgpu_internal.h"
#include "decim_plans_data.h"

namespace sdrgpu {

static const double DB_M_PI = 3.14159265358979323846;   // dsp/math/constants.h:3

static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
const char* last_error() { return g_err; }

// dsp/window/cosine.h:7-16 -- evaluated in double in the reference's order
static double cosine_sum(double n, double N, const double* coefs, int k) {
    double win = 0.0, sign = 1.0;
    for (int i = 0; i < k; i++) {
        win += sign * coefs[i] * std::cos((double)i * 2.0 * DB_M_PI * n / N);
        sign = -sign;
    }
    return win;
}

static const double C_HAMMING[] = {0.53836, 0.46164};                         // window/hamming.h
static const double C_HANN[] = {0.5, 0.5};                                    // window/hann.h
static const double C_BLACKMAN[] = {0.42, 0.5, 0.08};                         // window/blackman.h
static const double C_NUTTALL[] = {0.355768, 0.487396, 0.144232, 0.012604};   // window/nuttall.h
static const double C_BH4[] = {0.35875, 0.48829, 0.14128, 0.01168};           // window/blackman_harris4.h
static const double C_BH7[] = {0.27105140069342, 0.43329793923448, 0.21812299954311,  // window/blackman_harris7.h
                               0.06592544638803, 0.01081174209837, 0.00077658482522, 0.00001388721735};

double window_value(int type, double n, double N) {
    switch (type) {
    case SDRGPU_WIN_RECTANGULAR: return 1.0;
    case SDRGPU_WIN_HAMMING: return cosine_sum(n, N, C_HAMMING, 2);
    case SDRGPU_WIN_HANN: return cosine_sum(n, N, C_HANN, 2);
    case SDRGPU_WIN_BLACKMAN: return cosine_sum(n, N, C_BLACKMAN, 3);
    case SDRGPU_WIN_NUTTALL: return cosine_sum(n, N, C_NUTTALL, 4);
    case SDRGPU_WIN_BLACKMAN_HARRIS4: return cosine_sum(n, N, C_BH4, 4);
    case SDRGPU_WIN_BLACKMAN_HARRIS7: return cosine_sum(n, N, C_BH7, 7);
    default: return NAN;
    }
}
static double nuttall(double n, double N) { return cosine_sum(n, N, C_NUTTALL, 4); }

// dsp::window::createWindow (window/window.h:38-64): unity coherent gain; the
// centred form flips the sign of even samples (spectrum shifted by N/2). The
// reference writes buffer[size] for odd centred sizes; this stops at size-1.
int create_window(int type, float* buffer, int size, int centered) {
    if (!buffer || size <= 0 || type < 0 || type > SDRGPU_WIN_BLACKMAN_HARRIS7) {
        set_error("create_window: bad argument (type %d, size %d)", type, size);
        return SDRGPU_EARG;
    }
    for (int i = 0; i < size; i++) buffer[i] = (float)window_value(type, i, size);
    double wscale = 0.0f;
    for (int i = 0; i < size; i++) wscale += buffer[i];
    wscale = 1.0 / wscale;
    if (!centered) {
        for (int i = 0; i < size; i++) buffer[i] = (float)(buffer[i] * wscale);
    } else {
        for (int i = 0; i < size; i += 2) {
            buffer[i] = (float)(buffer[i] * -wscale);
            if (i + 1 < size) buffer[i + 1] = (float)(buffer[i + 1] * wscale);
        }
    }
    return SDRGPU_OK;
}

double hz_to_rads(double f, double fs) { return 2.0 * DB_M_PI * (f / fs); }   // math/hz_to_rads.h
static double sinc(double x) { return (x == 0.0) ? 1.0 : (std::sin(x) / x); } // math/sinc.h
static int estimate_tap_count(double tw, double fs) { return (int)(3.8 * fs / tw); }  // taps/estimate_tap_count.h

// taps/windowed_sinc.h:9-35 with the nuttall window; `win` multiplies the
// window term exactly like the lambdas of high_pass.h / band_pass.h
template <typename W>
static void windowed_sinc(int count, double omega, float* out, W win, double norm = 1.0) {
    double half = (double)count / 2.0;
    double corr = norm * omega / DB_M_PI;
    for (int i = 0; i < count; i++) {
        double t = (double)i - half + 0.5;
        out[i] = (float)(sinc(t * omega) * win(t - half, (double)count) * corr);
    }
}

int taps_windowed_sinc(int count, double omega, double norm, float* out) {   // windowed_sinc.h:9-35, window::nuttall
    if (count < 1) { set_error("windowed_sinc: count %d < 1", count); return SDRGPU_EARG; }
    if (out) windowed_sinc(count, omega, out, [](double n, double N) { return nuttall(n, N); }, norm);
    return count;
}

int taps_low_pass(double cutoff, double tw, double fs, int odd, float* out) {   // taps/low_pass.h:7-11
    if (!(tw > 0) || !(fs > 0)) { set_error("low_pass: bad transition/samplerate"); return SDRGPU_EARG; }
    int count = estimate_tap_count(tw, fs);
    if (odd && !(count % 2)) count++;
    if (out) windowed_sinc(count, hz_to_rads(cutoff, fs), out, [](double n, double N) { return nuttall(n, N); });
    return count;
}

int taps_high_pass(double cutoff, double tw, double fs, int odd, float* out) {  // taps/high_pass.h:7-14
    if (!(tw > 0) || !(fs > 0)) { set_error("high_pass: bad transition/samplerate"); return SDRGPU_EARG; }
    int count = estimate_tap_count(tw, fs);
    if (odd && !(count % 2)) count++;
    if (out)
        windowed_sinc(count, hz_to_rads((fs / 2.0) - cutoff, fs), out, [](double n, double N) {
            return nuttall(n, N) * (((int)std::round(n) % 2) ? -1.0f : 1.0f);
        });
    return count;
}

int taps_band_pass_f(double start, double stop, double tw, double fs, int odd, float* out) {  // taps/band_pass.h:11-27
    if (!(stop > start) || !(tw > 0) || !(fs > 0)) { set_error("band_pass: bad band"); return SDRGPU_EARG; }
    float offsetOmega = (float)hz_to_rads((start + stop) / 2.0, fs);
    int count = estimate_tap_count(tw, fs);
    if (odd && !(count % 2)) count++;
    if (out)
        windowed_sinc(count, hz_to_rads((stop - start) / 2.0, fs), out, [=](double n, double N) {
            return 2.0f * std::cos(offsetOmega * (float)n) * nuttall(n, N);
        });
    return count;
}

// complex taps: complex_t{sinc,0} * phasor(-offsetOmega*n)*nuttall * corr, all in complex_t float ops
int taps_band_pass_c(double start, double stop, double tw, double fs, int odd, float* out) {
    if (!(stop > start) || !(tw > 0) || !(fs > 0)) { set_error("band_pass: bad band"); return SDRGPU_EARG; }
    float offsetOmega = (float)hz_to_rads((start + stop) / 2.0, fs);
    int count = estimate_tap_count(tw, fs);
    if (odd && !(count % 2)) count++;
    if (!out) return count;
    double omega = hz_to_rads((stop - start) / 2.0, fs);
    double half = (double)count / 2.0, corr = omega / DB_M_PI;
    for (int i = 0; i < count; i++) {
        double t = (double)i - half + 0.5;
        double n = t - half;
        float ph = -offsetOmega * (float)n;
        float nut = (float)nuttall(n, count);
        float wre = std::cos(ph) * nut, wim = std::sin(ph) * nut;
        float s = (float)sinc(t * omega);
        float pre = s * wre - 0.0f * wim;
        float pim = 0.0f * wre + s * wim;
        out[2 * i] = pre * (float)corr;
        out[2 * i + 1] = pim * (float)corr;
    }
    return count;
}

int decim_plan(int ratio, int* decims, int* ntaps, const float** taps) {        // multirate/decim/plans.h
    int id = -1;
    for (int p = 0; p < SDRGPU_DECIM_PLAN_COUNT; p++)
        if ((2 << p) == ratio) id = p;
    if (id < 0) { set_error("decim_plan: ratio %d is not a power of two in 2..8192", ratio); return SDRGPU_EARG; }
    const sdrgpu_decim_plan_t& pl = sdrgpu_decim_plans[id];
    for (unsigned s = 0; s < pl.stage_count; s++) {
        const sdrgpu_decim_stage_t& st = sdrgpu_decim_stages[pl.first_stage + s];
        if (decims) decims[s] = (int)st.decim;
        if (ntaps) ntaps[s] = (int)st.ntaps;
        if (taps) taps[s] = &sdrgpu_decim_pool[st.offset];
    }
    return (int)pl.stage_count;
}

// FrequencyXlator quantises phaseDelta = (cos w, sin w) to float
// (channel/frequency_xlator.h:17,28); the rotator therefore turns by
// arg(float phasor) per sample. The device NCO uses exactly that rate.
double xlator_effective_omega(double offsetRad) {
    float c = (float)std::cos(offsetRad), s = (float)std::sin(offsetRad);
    return std::atan2((double)s, (double)c);
}

void PhaseAcc::advance(double w, long long n) {
    static const double TWO_PI_HI = 6.283185307179586;
    static const double TWO_PI_LO = 2.4492935982947064e-16;
    double dn = (double)n;
    double p = w * dn;
    double pe = std::fma(w, dn, -p);          // exact product error
    double s = hi + p;                        // two-sum
    double bp = s - hi;
    double se = (hi - (s - bp)) + (p - bp);
    double l = lo + pe + se;
    double k = std::rint((s + l) / TWO_PI_HI);
    s = std::fma(-k, TWO_PI_HI, s);
    l = std::fma(-k, TWO_PI_LO, l);
    hi = s + l;
    lo = l - (hi - s);
}

}  // namespace sdrgpu
