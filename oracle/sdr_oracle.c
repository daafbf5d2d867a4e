/*
 * sdr_oracle.c -- CPU restatement of SDR++'s streaming-DSP hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline). See sdr_oracle.h.
 * Built with -ffp-contract=off and no fast-math so that every setup-time
 * quantity (windows, taps, converters) is evaluated in the reference's own
 * operation order and rounds exactly as the reference source does.
 */
#include "sdr_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#include "../sdrpp_amd/csrc/decim_plans_data.h" /* data: reference plan tap tables */

#define DB_M_PI 3.14159265358979323846          /* math/constants.h:3 */
#define FL_M_PI 3.1415926535f                   /* math/constants.h:4 */

/* ------------------------------------------------------------------ window */
/* window/cosine.h:7-16: sum_i (-1)^i a_i cos(i*2*pi*n/N), evaluated in double */
static double cosine_win(double n, double N, const double* c, int k) {
    double win = 0.0, sign = 1.0;
    for (int i = 0; i < k; i++) {
        win += sign * c[i] * cos((double)i * 2.0 * DB_M_PI * n / N);
        sign = -sign;
    }
    return win;
}
static const double W_HAMMING[] = {0.53836, 0.46164};                               /* hamming.h */
static const double W_HANN[] = {0.5, 0.5};                                          /* hann.h */
static const double W_BLACKMAN[] = {0.42, 0.5, 0.08};                               /* blackman.h */
static const double W_NUTTALL[] = {0.355768, 0.487396, 0.144232, 0.012604};         /* nuttall.h */
static const double W_BH4[] = {0.35875, 0.48829, 0.14128, 0.01168};                 /* blackman_harris4.h */
static const double W_BH7[] = {0.27105140069342, 0.43329793923448, 0.21812299954311, /* blackman_harris7.h:22-30 */
                               0.06592544638803, 0.01081174209837, 0.00077658482522,
                               0.00001388721735};

static double nuttall(double n, double N) { return cosine_win(n, N, W_NUTTALL, 4); }

double orc_window_value(int type, double n, double N) {
    switch (type) {
    case ORC_WIN_RECTANGULAR: return 1.0;
    case ORC_WIN_HAMMING: return cosine_win(n, N, W_HAMMING, 2);
    case ORC_WIN_HANN: return cosine_win(n, N, W_HANN, 2);
    case ORC_WIN_BLACKMAN: return cosine_win(n, N, W_BLACKMAN, 3);
    case ORC_WIN_NUTTALL: return cosine_win(n, N, W_NUTTALL, 4);
    case ORC_WIN_BLACKMAN_HARRIS4: return cosine_win(n, N, W_BH4, 4);
    case ORC_WIN_BLACKMAN_HARRIS7: return cosine_win(n, N, W_BH7, 7);
    }
    return 0.0;
}

/* window/window.h:38-64. Quirk: the reference writes buffer[size] for odd
 * centred sizes (one past the end); the restatement stops at size-1. */
void orc_create_window(int type, float* buffer, int size, int centered) {
    for (int i = 0; i < size; i++) buffer[i] = (float)orc_window_value(type, i, size);
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
}

/* signal_path/iq_frontend.h:56-60 */
void orc_gen_reshape_params(double sampleRate, int size, double rate, int* skip, int* nz) {
    int fftInterval = (int)round(sampleRate / rate);
    *nz = fftInterval < size ? fftInterval : size;
    *skip = fftInterval - *nz;
}

/* -------------------------------------------------------------------- taps */
static double sinc(double x) { return (x == 0.0) ? 1.0 : (sin(x) / x); }        /* math/sinc.h */
static double hz_to_rads(double f, double fs) { return 2.0 * DB_M_PI * (f / fs); } /* math/hz_to_rads.h */

int orc_estimate_tap_count(double transWidth, double samplerate) {             /* taps/estimate_tap_count.h:4-6 */
    return (int)(3.8 * samplerate / transWidth);
}

/* taps/windowed_sinc.h:9-35 (float taps, nuttall window) */
int orc_windowed_sinc(int count, double omega, double norm, float* out) {
    if (!out) return count;
    double half = (double)count / 2.0;
    double corr = norm * omega / DB_M_PI;
    for (int i = 0; i < count; i++) {
        double t = (double)i - half + 0.5;
        out[i] = (float)(sinc(t * omega) * nuttall(t - half, count) * corr);
    }
    return count;
}

int orc_low_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out) { /* taps/low_pass.h:7-11 */
    int count = orc_estimate_tap_count(transWidth, sampleRate);
    if (odd && !(count % 2)) count++;
    return orc_windowed_sinc(count, hz_to_rads(cutoff, sampleRate), 1.0, out);
}

int orc_high_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out) { /* taps/high_pass.h:7-14 */
    int count = orc_estimate_tap_count(transWidth, sampleRate);
    if (odd && !(count % 2)) count++;
    if (!out) return count;
    double omega = hz_to_rads((sampleRate / 2.0) - cutoff, sampleRate);
    double half = (double)count / 2.0, corr = omega / DB_M_PI;
    for (int i = 0; i < count; i++) {
        double t = (double)i - half + 0.5;
        double n = t - half;
        double w = nuttall(n, count) * ((((int)round(n)) % 2) ? -1.0f : 1.0f);
        out[i] = (float)(sinc(t * omega) * w * corr);
    }
    return count;
}

int orc_band_pass_f(double start, double stop, double transWidth, double sampleRate, int odd, float* out) { /* taps/band_pass.h:11-27 */
    float offsetOmega = (float)hz_to_rads((start + stop) / 2.0, sampleRate);
    int count = orc_estimate_tap_count(transWidth, sampleRate);
    if (odd && !(count % 2)) count++;
    if (!out) return count;
    double omega = hz_to_rads((stop - start) / 2.0, sampleRate);
    double half = (double)count / 2.0, corr = omega / DB_M_PI;
    for (int i = 0; i < count; i++) {
        double t = (double)i - half + 0.5;
        double n = t - half;
        double w = 2.0f * cosf(offsetOmega * (float)n) * nuttall(n, count);
        out[i] = (float)(sinc(t * omega) * w * corr);
    }
    return count;
}

int orc_band_pass_c(double start, double stop, double transWidth, double sampleRate, int odd, float* out) {
    float offsetOmega = (float)hz_to_rads((start + stop) / 2.0, sampleRate);
    int count = orc_estimate_tap_count(transWidth, sampleRate);
    if (odd && !(count % 2)) count++;
    if (!out) return count;
    double omega = hz_to_rads((stop - start) / 2.0, sampleRate);
    double half = (double)count / 2.0, corr = omega / DB_M_PI;
    for (int i = 0; i < count; i++) {
        double t = (double)i - half + 0.5;
        double n = t - half;
        /* window: math::phasor(-offsetOmega*(float)n) * nuttall(n,N)  (complex_t * double) */
        float ph = -offsetOmega * (float)n;
        float nut = (float)nuttall(n, count);
        float wre = cosf(ph) * nut, wim = sinf(ph) * nut;
        /* cplx = {(float)sinc, 0}; cplx * window (complex_t product) * corr (complex_t * double) */
        float s = (float)sinc(t * omega);
        float pre = s * wre - 0.0f * wim;
        float pim = 0.0f * wre + s * wim;
        out[2 * i] = pre * (float)corr;
        out[2 * i + 1] = pim * (float)corr;
    }
    return count;
}

/* multirate/decim/plans.h: ratio 2..8192 */
int orc_decim_plan(int ratio, int* decims, int* ntaps, const float** taps) {
    int id = -1;
    for (int p = 0; p < SDRGPU_DECIM_PLAN_COUNT; p++) if ((2 << p) == ratio) id = p;
    if (id < 0) return 0;
    const sdrgpu_decim_plan_t* pl = &sdrgpu_decim_plans[id];
    for (unsigned s = 0; s < pl->stage_count; s++) {
        const sdrgpu_decim_stage_t* st = &sdrgpu_decim_stages[pl->first_stage + s];
        if (decims) decims[s] = (int)st->decim;
        if (ntaps) ntaps[s] = (int)st->ntaps;
        if (taps) taps[s] = &sdrgpu_decim_pool[st->offset];
    }
    return (int)pl->stage_count;
}

/* -------------------------------------------------------------- converters */
void orc_u8_to_f32(const uint8_t* in, float* out, long n) {   /* file_source main.cpp:489 */
    for (long i = 0; i < n; i++) out[i] = (in[i] - 128 + 0.5f) / (128.0f - 0.5f);
}
void orc_i16_to_f32(const int16_t* in, float* out, long n) {  /* main.cpp:506 */
    for (long i = 0; i < n; i++) out[i] = (in[i] + 0.5f) / (32768.0f - 0.5f);
}
void orc_i24_to_f32(const uint8_t* in, float* out, long n) {  /* main.cpp:522-525 */
    for (long i = 0; i < n; i++) {
        const uint8_t* p = in + 3 * i;
        int32_t v = (int32_t)((uint32_t)(p[0] | (p[1] << 8) | (p[2] << 16)) << 8) >> 8;
        out[i] = (v + 0.5f) / (8388608.0f - 0.5f);
    }
}
void orc_i32_to_f32(const int32_t* in, float* out, long n) {  /* main.cpp:542 */
    for (long i = 0; i < n; i++) out[i] = (float)((in[i] + 0.5) / (2147483648.0 - 0.5));
}
void orc_f64_to_f32(const double* in, float* out, long n) {   /* main.cpp:475 volk_64f_convert_32f */
    for (long i = 0; i < n; i++) out[i] = (float)in[i];
}
void orc_i8_to_f32(const int8_t* in, float* out, long n) {    /* hackrf main.cpp:386 volk_8i_s32f_convert_32f(.,.,128) */
    const float iScalar = 1.0 / 128.0f;
    for (long i = 0; i < n; i++) out[i] = ((float)in[i]) * iScalar;
}

/* --------------------------------------------------------------------- FFT */
/* Forward (e^{-i}) unnormalised DFT, radix-2 Stockham autosort (the restated
 * fftwf_plan_dft_1d(N, FFTW_FORWARD) of iq_frontend.cpp:292). N = 2^k. */
#define FFT_BODY(T, COS, SIN)                                                   \
    int n = N, s = 1;                                                           \
    T* x = work0; T* y = work1;                                                 \
    while (n > 1) {                                                             \
        int m = n / 2;                                                          \
        double th = 2.0 * DB_M_PI / n;                                          \
        for (int p = 0; p < m; p++) {                                           \
            T wr = (T)COS(p * th), wi = (T)-SIN(p * th);                        \
            for (int q = 0; q < s; q++) {                                       \
                T ar = x[2 * (q + s * p)], ai = x[2 * (q + s * p) + 1];         \
                T br = x[2 * (q + s * (p + m))], bi = x[2 * (q + s * (p + m)) + 1]; \
                y[2 * (q + s * 2 * p)] = ar + br;                               \
                y[2 * (q + s * 2 * p) + 1] = ai + bi;                           \
                T dr = ar - br, di = ai - bi;                                   \
                y[2 * (q + s * (2 * p + 1))] = dr * wr - di * wi;               \
                y[2 * (q + s * (2 * p + 1)) + 1] = dr * wi + di * wr;           \
            }                                                                   \
        }                                                                       \
        n = m; s *= 2;                                                          \
        T* t = x; x = y; y = t;                                                 \
    }

void orc_fft_c2c(const float* in, float* out, int N) {
    float* work0 = (float*)malloc(sizeof(float) * 2 * N);
    float* work1 = (float*)malloc(sizeof(float) * 2 * N);
    memcpy(work0, in, sizeof(float) * 2 * N);
    FFT_BODY(float, cos, sin)
    memcpy(out, x, sizeof(float) * 2 * N);
    free(work0); free(work1);
}

void orc_fft_c2c_f64(const double* in, double* out, int N) {
    double* work0 = (double*)malloc(sizeof(double) * 2 * N);
    double* work1 = (double*)malloc(sizeof(double) * 2 * N);
    memcpy(work0, in, sizeof(double) * 2 * N);
    FFT_BODY(double, cos, sin)
    memcpy(out, x, sizeof(double) * 2 * N);
    free(work0); free(work1);
}

/* volk_32fc_s32f_power_spectrum_32f(out, X, 1.0, N) at iq_frontend.cpp:244:
 * dB = 10*log10(re^2 + im^2) with normalisation factor 1. */
void orc_power_spectrum_db(const float* X, float* out, int N) {
    for (int k = 0; k < N; k++) {
        float re = X[2 * k], im = X[2 * k + 1];
        out[k] = 10.0f * log10f(re * re + im * im);
    }
}

/* IQFrontEnd::handler (iq_frontend.cpp:230-249) + the zero tail of updateFFTSize (:295).
 * work: 4*N floats scratch. */
void orc_fft_logmag(const float* in, int nz, int N, const float* window, float* work, float* out_db) {
    float* fin = work;
    float* fout = work + 2 * N;
    for (int n = 0; n < nz; n++) {                 /* volk_32fc_32f_multiply_32fc (:234) */
        fin[2 * n] = in[2 * n] * window[n];
        fin[2 * n + 1] = in[2 * n + 1] * window[n];
    }
    for (int n = nz; n < N; n++) fin[2 * n] = fin[2 * n + 1] = 0.0f;
    orc_fft_c2c(fin, fout, N);                     /* fftwf_execute (:237) */
    orc_power_spectrum_db(fout, out_db, N);        /* (:244) */
}

/* -------------------------------------------------------------- dot products */
/* volk_32fc_32f_dot_prod_32fc / volk_32f_x2_dot_prod_32f / volk_32fc_x2_dot_prod_32fc
 * as used by filter/fir.h:69-75. Correlation order: x[i+j]*h[j], no reversal. */
static void dot_cf(const float* x, const float* h, int n, float* o, int precise) {
    if (precise) {
        double re = 0, im = 0;
        for (int j = 0; j < n; j++) { re += (double)x[2 * j] * h[j]; im += (double)x[2 * j + 1] * h[j]; }
        o[0] = (float)re; o[1] = (float)im;
    } else {
        float a[8] = {0}, b[8] = {0};
        int j = 0;
        for (; j + 4 <= n; j += 4)
            for (int k = 0; k < 4; k++) { a[2 * k] += x[2 * (j + k)] * h[j + k]; a[2 * k + 1] += x[2 * (j + k) + 1] * h[j + k]; }
        for (; j < n; j++) { b[0] += x[2 * j] * h[j]; b[1] += x[2 * j + 1] * h[j]; }
        o[0] = ((a[0] + a[2]) + (a[4] + a[6])) + b[0];
        o[1] = ((a[1] + a[3]) + (a[5] + a[7])) + b[1];
    }
}
static void dot_ff(const float* x, const float* h, int n, float* o, int precise) {
    if (precise) {
        double s = 0;
        for (int j = 0; j < n; j++) s += (double)x[j] * h[j];
        o[0] = (float)s;
    } else {
        float a[8] = {0}, b = 0;
        int j = 0;
        for (; j + 8 <= n; j += 8) for (int k = 0; k < 8; k++) a[k] += x[j + k] * h[j + k];
        for (; j < n; j++) b += x[j] * h[j];
        o[0] = (((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]))) + b;
    }
}
/* CPU-baseline dot products (precise = 0), VOLK-class: 16-float vector multiply-adds (GCC vector
 * extensions, lowered to AVX2 / AVX-512 by -march=native) with two accumulators, like
 * volk_32fc_32f_dot_prod_32fc's SIMD kernels. Complex data x real taps runs as a float dot of
 * length 2n against taps duplicated per (re, im) pair, hh[2j] = hh[2j + 1] = h[j]. */
typedef float v16f __attribute__((vector_size(64)));
static inline v16f ld16(const float* p) { v16f v; memcpy(&v, p, sizeof(v)); return v; }
static float dot_vec(const float* x, const float* h, int m, float* odd) {
    v16f a0 = {0}, a1 = {0};
    int k = 0;
    for (; k + 32 <= m; k += 32) {
        a0 += ld16(x + k) * ld16(h + k);
        a1 += ld16(x + k + 16) * ld16(h + k + 16);
    }
    for (; k + 16 <= m; k += 16) a0 += ld16(x + k) * ld16(h + k);
    v16f a = a0 + a1;
    float e = 0, o = 0;
    for (int i = 0; i < 16; i += 2) { e += a[i]; o += a[i + 1]; }
    for (; k < m; k++) { if (k & 1) o += x[k] * h[k]; else e += x[k] * h[k]; }
    if (odd) { *odd = o; return e; }
    return e + o;
}
static void dot_cf_vec(const float* x, const float* hh, int n, float* o) { o[0] = dot_vec(x, hh, 2 * n, o + 1); }
static void dot_ff_vec(const float* x, const float* h, int n, float* o) { o[0] = dot_vec(x, h, n, NULL); }
static float* dup_taps(const float* h, int n) {
    float* hh = (float*)malloc(sizeof(float) * 2 * (size_t)(n > 0 ? n : 1));
    for (int j = 0; j < n; j++) hh[2 * j] = hh[2 * j + 1] = h[j];
    return hh;
}

static void dot_cc(const float* x, const float* h, int n, float* o, int precise) {
    if (precise) {
        double re = 0, im = 0;
        for (int j = 0; j < n; j++) {
            double xr = x[2 * j], xi = x[2 * j + 1], hr = h[2 * j], hi = h[2 * j + 1];
            re += xr * hr - xi * hi; im += xr * hi + xi * hr;
        }
        o[0] = (float)re; o[1] = (float)im;
    } else {
        float re = 0, im = 0;
        for (int j = 0; j < n; j++) {
            float xr = x[2 * j], xi = x[2 * j + 1], hr = h[2 * j], hi = h[2 * j + 1];
            re += xr * hr - xi * hi; im += xr * hi + xi * hr;
        }
        o[0] = re; o[1] = im;
    }
}

/* ------------------------------------------------------ FIR / DecimatingFIR */
/* filter/fir.h:62-83 and filter/decimating_fir.h:45-68 */
/* CPU-baseline kernels (cpu_fast.c) */
void cf_rotate(const float* in, float* out, int count, float* pr, float* pi, float dr, float di, int* cnt);
int  cf_fir_cf_decim(const float* x, const float* hh, int m16, int offset, int D, int count, float* out);
void cf_quad(const float* in, int count, float* out, float* dre, float* dim, float inv);

struct orc_fir {
    int dtype, ttype, ntaps, decim, offset, precise, cap;
    float* taps;
    float* hh;    /* taps duplicated per (re, im) pair (CPU-baseline complex x real dot) */
    float* hh16;  /* hh zero-padded to m16 floats (cf_fir_cf_decim) */
    int m16;
    float* buf;   /* [ntaps-1 history | input | 16 floats of zero slack], elements of dtype */
};

static int esz(int dtype) { return dtype == ORC_C64 ? 2 : 1; }

orc_fir* orc_fir_create(int dtype, int ttype, const float* taps, int ntaps, int decim, int precise) {
    orc_fir* f = (orc_fir*)calloc(1, sizeof(orc_fir));
    f->dtype = dtype; f->ttype = ttype; f->decim = decim < 1 ? 1 : decim; f->precise = precise;
    f->cap = 0; f->buf = NULL; f->taps = NULL; f->ntaps = 0;
    orc_fir_set_taps(f, taps, ntaps);
    return f;
}

void orc_fir_set_taps(orc_fir* f, const float* taps, int ntaps) {
    /* FIR::setTaps (fir.h:31-52): keep the history aligned to the newest sample */
    int e = esz(f->dtype), old = f->ntaps;
    float* nb = (float*)calloc((size_t)(ntaps > 1 ? ntaps - 1 : 1) * e, sizeof(float));
    if (old > 0) {
        int keep = (old - 1 < ntaps - 1) ? old - 1 : ntaps - 1;
        memcpy(nb + (size_t)(ntaps - 1 - keep) * e, f->buf + (size_t)(old - 1 - keep) * e, sizeof(float) * keep * e);
    }
    free(f->buf); f->buf = nb; f->cap = 0;
    free(f->taps);
    f->taps = (float*)malloc(sizeof(float) * ntaps * esz(f->ttype));
    memcpy(f->taps, taps, sizeof(float) * ntaps * esz(f->ttype));
    free(f->hh);
    f->hh = (f->ttype == ORC_F32) ? dup_taps(taps, ntaps) : NULL;
    free(f->hh16);
    f->hh16 = NULL;
    f->m16 = (2 * ntaps + 15) / 16 * 16;
    if (f->ttype == ORC_F32) {
        f->hh16 = (float*)calloc((size_t)f->m16, sizeof(float));
        memcpy(f->hh16, f->hh, sizeof(float) * 2 * (size_t)ntaps);
    }
    f->ntaps = ntaps;
    f->offset = 0;   /* DecimatingFIR::setTaps (decimating_fir.h:19-26) */
}

void orc_fir_reset(orc_fir* f) {
    memset(f->buf, 0, sizeof(float) * (f->ntaps - 1) * esz(f->dtype));
    f->offset = 0;
}

int orc_fir_process(orc_fir* f, const float* in, int count, float* out) {
    int e = esz(f->dtype), h = f->ntaps - 1;
    if (f->cap < count) {
        float* nb = (float*)malloc(sizeof(float) * ((size_t)(h + count) * e + 16));
        memcpy(nb, f->buf, sizeof(float) * h * e);
        free(f->buf); f->buf = nb; f->cap = count;
    }
    memcpy(f->buf + (size_t)h * e, in, sizeof(float) * (size_t)count * e);
    int outCount = 0;
    if (!f->precise && f->dtype == ORC_C64 && f->ttype == ORC_F32) {   /* CPU baseline (cpu_fast.c) */
        memset(f->buf + (size_t)(h + count) * e, 0, sizeof(float) * 16);
        outCount = cf_fir_cf_decim(f->buf, f->hh16, f->m16, f->offset, f->decim, count, out);
        f->offset += outCount * f->decim - count;
        memmove(f->buf, f->buf + (size_t)count * e, sizeof(float) * h * e);
        return outCount;
    }
    for (; f->offset < count; f->offset += f->decim) {
        const float* x = f->buf + (size_t)f->offset * e;
        float* o = out + (size_t)outCount * e;
        if (f->dtype == ORC_F32) {
            if (f->precise) dot_ff(x, f->taps, f->ntaps, o, 1); else dot_ff_vec(x, f->taps, f->ntaps, o);
        } else if (f->ttype == ORC_F32) {
            if (f->precise) dot_cf(x, f->taps, f->ntaps, o, 1); else dot_cf_vec(x, f->hh, f->ntaps, o);
        } else {
            dot_cc(x, f->taps, f->ntaps, o, f->precise);
        }
        outCount++;
    }
    f->offset -= count;
    memmove(f->buf, f->buf + (size_t)count * e, sizeof(float) * h * e);
    return outCount;
}

void orc_fir_destroy(orc_fir* f) { if (!f) return; free(f->buf); free(f->taps); free(f->hh); free(f->hh16); free(f); }

/* ------------------------------------------------------------------ xlator */
/* channel/frequency_xlator.h:15-50. phaseDelta = lv_cmake(cos(w), sin(w)) is
 * quantised to float; the rotator advances phase by that float phasor each
 * sample (VOLK rotator, renormalised). The restatement evaluates the ideal of
 * that recurrence, phase_n = exp(i*n*w') with w' = arg(float phaseDelta),
 * in long double, then rounds the product to float. */
struct orc_xlator { double w; long double origin; long long n; int fast; float pr, pi, dr, di; int cnt; };

double orc_xlator_effective_omega(double offset_rad) {
    float c = (float)cos(offset_rad), s = (float)sin(offset_rad);
    return atan2((double)s, (double)c);
}
orc_xlator* orc_xlator_create(double offset_rad) {
    orc_xlator* x = (orc_xlator*)calloc(1, sizeof(orc_xlator));
    x->w = orc_xlator_effective_omega(offset_rad);
    x->pr = 1.0f; x->dr = (float)cos(offset_rad); x->di = (float)sin(offset_rad);
    return x;
}
/* CPU-baseline variant: the VOLK rotator recurrence itself (float phasor, phase *= delta,
 * renormalised every 512 samples like volk_32fc_s32fc_x2_rotator2_32fc_generic). */
orc_xlator* orc_xlator_create_fast(double offset_rad) {
    orc_xlator* x = orc_xlator_create(offset_rad);
    x->fast = 1;
    return x;
}
/* setOffset (frequency_xlator.h:25-29) changes the increment and keeps the
 * running phasor: fold the accumulated phase into the origin. */
void orc_xlator_set_offset(orc_xlator* x, double offset_rad) {
    const long double twopi = 2.0L * (long double)DB_M_PI;
    x->origin = fmodl(x->origin + (long double)x->w * (long double)x->n, twopi);
    x->n = 0;
    x->w = orc_xlator_effective_omega(offset_rad);
}
void orc_xlator_reset(orc_xlator* x) { x->n = 0; x->origin = 0; }   /* reset(): phase = 1+0j */
int orc_xlator_process(orc_xlator* x, const float* in, int count, float* out) {
    if (x->fast) {   /* CPU baseline: the rotator on 8 lanes per vector (cpu_fast.c) */
        cf_rotate(in, out, count, &x->pr, &x->pi, x->dr, x->di, &x->cnt);
        return count;
    }
    const long double twopi = 2.0L * (long double)DB_M_PI;
    for (int i = 0; i < count; i++) {
        long double a = fmodl(x->origin + (long double)x->w * (long double)(x->n + i), twopi);
        double c = (double)cosl(a), s = (double)sinl(a);
        double re = in[2 * i], im = in[2 * i + 1];
        out[2 * i] = (float)(re * c - im * s);
        out[2 * i + 1] = (float)(re * s + im * c);
    }
    x->n += count;
    return count;
}
void orc_xlator_destroy(orc_xlator* x) { free(x); }

/* -------------------------------------------------------------- quadrature */
/* demod/quadrature.h:41-56 (USE_QUAD_FM_DEMOD=1): out = arg(y*conj(d)) / dev.
 * _din is uninitialised until reset(); the restatement uses 0. */
struct orc_quad { float inv; float dre, dim; int fast; };
orc_quad* orc_quad_create(double deviation_rad) {
    orc_quad* q = (orc_quad*)calloc(1, sizeof(orc_quad));
    q->inv = (float)(1.0 / deviation_rad);
    return q;
}
void orc_quad_reset(orc_quad* q) { q->dre = 0.0f; q->dim = 0.0f; }
int orc_quad_process(orc_quad* q, const float* in, int count, float* out) {
    if (q->fast) {   /* CPU baseline: 16 outputs per vector, polynomial atan (cpu_fast.c) */
        cf_quad(in, count, out, &q->dre, &q->dim, q->inv);
        return count;
    }
    for (int i = 0; i < count; i++) {
        float yr = in[2 * i], yi = in[2 * i + 1];
        float br = q->dre, bi = -q->dim;                 /* _din.conj() */
        float re = (yr * br) - (yi * bi);                /* complex_t::operator* (types.h:23-25) */
        float im = (yi * br) + (yr * bi);
        out[i] = atan2f(im, re) * q->inv;
        q->dre = yr; q->dim = yi;
    }
    return count;
}
void orc_quad_destroy(orc_quad* q) { free(q); }

/* --------------------------------------------------------- PowerDecimator */
/* multirate/power_decimator.h:51-108 */
struct orc_pdec { int dtype, ratio, nst; orc_fir* st[8]; float* tmp; int tcap; };
orc_pdec* orc_pdec_create(int dtype, int ratio, int precise) {
    orc_pdec* p = (orc_pdec*)calloc(1, sizeof(orc_pdec));
    p->dtype = dtype; p->ratio = ratio;
    if (ratio > 1) {
        int d[8], n[8]; const float* t[8];
        p->nst = orc_decim_plan(ratio, d, n, t);
        for (int s = 0; s < p->nst; s++) p->st[s] = orc_fir_create(dtype, ORC_F32, t[s], n[s], d[s], precise);
    }
    return p;
}
int orc_pdec_process(orc_pdec* p, const float* in, int count, float* out) {
    int e = esz(p->dtype);
    if (p->ratio == 1) { memmove(out, in, sizeof(float) * (size_t)count * e); return count; }
    const float* data = in;
    for (int s = 0; s < p->nst; s++) { count = orc_fir_process(p->st[s], data, count, out); data = out; }
    return count;
}
void orc_pdec_reset(orc_pdec* p) { for (int s = 0; s < p->nst; s++) orc_fir_reset(p->st[s]); }
void orc_pdec_destroy(orc_pdec* p) { if (!p) return; for (int s = 0; s < p->nst; s++) orc_fir_destroy(p->st[s]); free(p->tmp); free(p); }

/* ----------------------------------------------------- PolyphaseResampler */
/* multirate/polyphase_bank.h:15-47 + polyphase_resampler.h:69-99 */
struct orc_poly {
    int dtype, interp, decim, tpp, phase, offset, precise, cap;
    float* bank;  /* [interp][tpp] */
    float* hh;    /* bank duplicated per (re, im) pair (CPU-baseline complex dot) */
    float* buf;
};
orc_poly* orc_poly_create(int dtype, int interp, int decim, const float* taps, int ntaps, int precise) {
    orc_poly* p = (orc_poly*)calloc(1, sizeof(orc_poly));
    p->dtype = dtype; p->interp = interp; p->decim = decim; p->precise = precise;
    p->tpp = (ntaps + interp - 1) / interp;
    p->bank = (float*)calloc((size_t)interp * p->tpp, sizeof(float));
    int tot = interp * p->tpp;
    for (int i = 0; i < tot; i++)
        p->bank[(size_t)((interp - 1) - (i % interp)) * p->tpp + i / interp] = (i < ntaps) ? taps[i] : 0.0f;
    p->hh = dup_taps(p->bank, tot);
    p->buf = (float*)calloc((size_t)(p->tpp > 1 ? p->tpp - 1 : 1) * esz(dtype), sizeof(float));
    return p;
}
void orc_poly_reset(orc_poly* p) {
    memset(p->buf, 0, sizeof(float) * (p->tpp - 1) * esz(p->dtype));
    p->phase = 0; p->offset = 0;
}
int orc_poly_process(orc_poly* p, const float* in, int count, float* out) {
    int e = esz(p->dtype), h = p->tpp - 1;
    if (p->cap < count) {
        float* nb = (float*)malloc(sizeof(float) * (size_t)(h + count) * e);
        memcpy(nb, p->buf, sizeof(float) * h * e);
        free(p->buf); p->buf = nb; p->cap = count;
    }
    memcpy(p->buf + (size_t)h * e, in, sizeof(float) * (size_t)count * e);
    int outCount = 0;
    while (p->offset < count) {
        const float* x = p->buf + (size_t)p->offset * e;
        const float* ph = p->bank + (size_t)p->phase * p->tpp;
        if (p->precise) {
            if (p->dtype == ORC_F32) dot_ff(x, ph, p->tpp, out + outCount, 1);
            else dot_cf(x, ph, p->tpp, out + 2 * outCount, 1);
        } else if (p->dtype == ORC_F32) {
            dot_ff_vec(x, ph, p->tpp, out + outCount);
        } else {
            dot_cf_vec(x, p->hh + 2 * (size_t)p->phase * p->tpp, p->tpp, out + 2 * outCount);
        }
        outCount++;
        p->phase += p->decim;
        p->offset += p->phase / p->interp;
        p->phase = p->phase % p->interp;
    }
    p->offset -= count;
    memmove(p->buf, p->buf + (size_t)count * e, sizeof(float) * h * e);
    return outCount;
}
void orc_poly_destroy(orc_poly* p) { if (!p) return; free(p->bank); free(p->hh); free(p->buf); free(p); }

/* ------------------------------------------------------ RationalResampler */
/* multirate/rational_resampler.h:83-167 */
enum { RR_BOTH = 0, RR_DECIM_ONLY, RR_RESAMP_ONLY, RR_NONE };
struct orc_rres { int dtype, mode, predec, interp, decim, ntaps; orc_pdec* pd; orc_poly* pp; };
static int gcd_i(int a, int b) { while (b) { int t = a % b; a = b; b = t; } return a < 0 ? -a : a; }
orc_rres* orc_rres_create(int dtype, double inSr, double outSr, int precise) {
    orc_rres* r = (orc_rres*)calloc(1, sizeof(orc_rres));
    r->dtype = dtype;
    const int maxRatio = 1 << SDRGPU_DECIM_PLAN_COUNT;
    int predecPower = (int)floor(log2(inSr / outSr));
    if (predecPower > maxRatio) predecPower = maxRatio;
    int predecRatio = (predecPower >= 31 || predecPower < 0) ? maxRatio : (1 << predecPower);
    if (predecRatio > maxRatio) predecRatio = maxRatio;
    double intSr = inSr;
    int useDecim = (inSr > outSr && predecPower > 0);
    if (useDecim) { intSr = inSr / (double)predecRatio; r->pd = orc_pdec_create(dtype, predecRatio, precise); }
    r->predec = useDecim ? predecRatio : 1;
    int IntSR = (int)round(intSr), OutSR = (int)round(outSr);
    int g = gcd_i(IntSR, OutSR);
    int interp = OutSR / g, decim = IntSR / g;
    r->interp = interp; r->decim = decim;
    if (interp == decim) { r->mode = useDecim ? RR_DECIM_ONLY : RR_NONE; return r; }
    double tapSr = intSr * (double)interp;
    double tapBw = (inSr < outSr ? inSr : outSr) / 2.0;
    double tapTw = tapBw * 0.1;
    int n = orc_low_pass(tapBw, tapTw, tapSr, 0, NULL);
    float* t = (float*)malloc(sizeof(float) * n);
    orc_low_pass(tapBw, tapTw, tapSr, 0, t);
    for (int i = 0; i < n; i++) t[i] *= (float)interp;
    r->pp = orc_poly_create(dtype, interp, decim, t, n, precise);
    r->ntaps = n;
    free(t);
    r->mode = useDecim ? RR_BOTH : RR_RESAMP_ONLY;
    return r;
}
int orc_rres_info(orc_rres* r, int* mode, int* predec, int* interp, int* decim, int* ntaps) {
    if (mode) *mode = r->mode;
    if (predec) *predec = r->predec;
    if (interp) *interp = r->interp;
    if (decim) *decim = r->decim;
    if (ntaps) *ntaps = r->ntaps;
    return 0;
}
int orc_rres_process(orc_rres* r, const float* in, int count, float* out) {
    switch (r->mode) {
    case RR_BOTH: count = orc_pdec_process(r->pd, in, count, out); return orc_poly_process(r->pp, out, count, out);
    case RR_DECIM_ONLY: return orc_pdec_process(r->pd, in, count, out);
    case RR_RESAMP_ONLY: return orc_poly_process(r->pp, in, count, out);
    default: memmove(out, in, sizeof(float) * (size_t)count * esz(r->dtype)); return count;
    }
}
void orc_rres_destroy(orc_rres* r) { if (!r) return; orc_pdec_destroy(r->pd); orc_poly_destroy(r->pp); free(r); }

/* ------------------------------------------------------------------ RxVFO */
/* channel/rx_vfo.h:24-121 */
struct orc_vfo { orc_xlator* x; orc_rres* rr; orc_fir* lpf; int filterNeeded; float* tmp; int cap; };
orc_vfo* orc_vfo_create(double inSr, double outSr, double bw, double offset, int precise) {
    orc_vfo* v = (orc_vfo*)calloc(1, sizeof(orc_vfo));
    v->x = precise ? orc_xlator_create(hz_to_rads(-offset, inSr)) : orc_xlator_create_fast(hz_to_rads(-offset, inSr));
    v->rr = orc_rres_create(ORC_C64, inSr, outSr, precise);
    v->filterNeeded = (bw != outSr);
    double fw = bw / 2.0;
    int n = orc_low_pass(fw, fw * 0.1, outSr, 0, NULL);
    float* t = (float*)malloc(sizeof(float) * n);
    orc_low_pass(fw, fw * 0.1, outSr, 0, t);
    v->lpf = orc_fir_create(ORC_C64, ORC_F32, t, n, 1, precise);
    free(t);
    return v;
}
int orc_vfo_process(orc_vfo* v, const float* in, int count, float* out) {
    if (!v->lpf->precise) {   /* CPU baseline: L2-sized sub-blocks (same stream, state carried) */
        const int sub = 32768;
        if (v->cap < (count < sub ? count : sub)) { free(v->tmp); v->cap = count < sub ? count : sub; v->tmp = (float*)malloc(sizeof(float) * 2 * (size_t)v->cap); }
        int total = 0;
        for (int i = 0; i < count; i += sub) {
            const int c = count - i < sub ? count - i : sub;
            orc_xlator_process(v->x, in + 2 * (size_t)i, c, v->tmp);
            int m = orc_rres_process(v->rr, v->tmp, c, v->tmp);
            if (v->filterNeeded) orc_fir_process(v->lpf, v->tmp, m, v->tmp);
            memcpy(out + 2 * (size_t)total, v->tmp, sizeof(float) * 2 * (size_t)m);
            total += m;
        }
        return total;
    }
    orc_xlator_process(v->x, in, count, out);
    count = orc_rres_process(v->rr, out, count, out);
    if (v->filterNeeded) orc_fir_process(v->lpf, out, count, out);
    return count;
}
void orc_vfo_destroy(orc_vfo* v) { if (!v) return; orc_xlator_destroy(v->x); orc_rres_destroy(v->rr); orc_fir_destroy(v->lpf); free(v->tmp); free(v); }

/* ------------------------------------------------------- BroadcastFM mono */
/* demod/broadcast_fm.h:18-49 (init), :144-215 (process, _stereo == false, no RDS) */
struct orc_wfm { orc_quad* q; orc_fir* al; int lowPass; float* tmp; int cap; };
orc_wfm* orc_wfm_create(double deviation, double samplerate, int lowPass, int precise) {
    orc_wfm* w = (orc_wfm*)calloc(1, sizeof(orc_wfm));
    w->q = orc_quad_create(hz_to_rads(deviation, samplerate));
    w->q->fast = !precise;
    int n = orc_low_pass(15000.0, 4000.0, samplerate, 0, NULL);
    float* t = (float*)malloc(sizeof(float) * n);
    orc_low_pass(15000.0, 4000.0, samplerate, 0, t);
    w->al = orc_fir_create(ORC_F32, ORC_F32, t, n, 1, precise);
    free(t);
    w->lowPass = lowPass;
    return w;
}
int orc_wfm_process(orc_wfm* w, const float* in, int count, float* out) {
    if (w->cap < count) { free(w->tmp); w->tmp = (float*)malloc(sizeof(float) * count); w->cap = count; }
    orc_quad_process(w->q, in, count, w->tmp);
    if (w->lowPass) orc_fir_process(w->al, w->tmp, count, w->tmp);
    for (int i = 0; i < count; i++) { out[2 * i] = w->tmp[i]; out[2 * i + 1] = w->tmp[i]; } /* LRToStereo */
    return count;
}
void orc_wfm_destroy(orc_wfm* w) { if (!w) return; orc_quad_destroy(w->q); orc_fir_destroy(w->al); free(w->tmp); free(w); }

/* ----------------------------------------------------- BroadcastFM stereo */
/* demod/broadcast_fm.h:34-60 (init), :144-191 (process, _stereo == true, no RDS);
 * loop/pll.h:13-72, loop/phase_control_loop.h:17-89, math/normalize_phase.h,
 * math/phasor.h, math/delay.h. All PLL state and coefficients are float (T = float). */
struct orc_pll { float alpha, beta, phase, freq, minPhase, maxPhase, phaseDelta, minFreq, maxFreq, initPhase, initFreq; };
static void orc_pll_init(struct orc_pll* p, double bandwidth, double initPhase, double initFreq, double minFreq, double maxFreq) {
    /* PhaseControlLoop<float>::criticallyDamped (phase_control_loop.h:31-36), T = float */
    float bw = (float)bandwidth;
    float df = (float)(sqrt(2.0) / 2.0);
    float denominator = (float)((1.0 + 2.0 * (double)df * (double)bw) + (double)(bw * bw));
    p->alpha = ((float)4 * df * bw) / denominator;
    p->beta = ((float)4 * bw * bw) / denominator;
    p->initPhase = (float)initPhase;
    p->initFreq = (float)initFreq;
    p->phase = p->initPhase;
    p->minPhase = -FL_M_PI; p->maxPhase = FL_M_PI;
    p->phaseDelta = p->maxPhase - p->minPhase;
    p->freq = p->initFreq;
    p->minFreq = (float)minFreq; p->maxFreq = (float)maxFreq;
}
static void orc_pll_process(struct orc_pll* p, const float* in, int count, float* out) {
    for (int i = 0; i < count; i++) {
        out[2 * i] = cosf(p->phase);                                   /* math::phasor */
        out[2 * i + 1] = sinf(p->phase);
        float diff = atan2f(in[2 * i + 1], in[2 * i]) - p->phase;      /* in[i].phase() - phase */
        if (diff > FL_M_PI) diff -= 2.0f * FL_M_PI;                    /* normalizePhase */
        else if (diff <= -FL_M_PI) diff += 2.0f * FL_M_PI;
        p->freq += p->beta * diff;                                     /* advance */
        if (p->freq > p->maxFreq) p->freq = p->maxFreq;
        else if (p->freq < p->minFreq) p->freq = p->minFreq;
        p->phase += p->freq + (p->alpha * diff);
        while (p->phase > p->maxPhase) p->phase -= p->phaseDelta;
        while (p->phase < p->minPhase) p->phase += p->phaseDelta;
    }
}

struct orc_wfms {
    orc_quad* q; orc_fir *pilot, *al, *ar; struct orc_pll pll;
    int stereo, lowPass, delay;
    float *mpx, *cplx, *pf, *vco, *lmr, *l, *r, *dlpr, *dlmr; int cap;
};
orc_wfms* orc_wfms_create(double deviation, double samplerate, int stereo, int lowPass, int precise) {
    orc_wfms* w = (orc_wfms*)calloc(1, sizeof(orc_wfms));
    w->q = orc_quad_create(hz_to_rads(deviation, samplerate));
    int np = orc_band_pass_c(18750.0, 19250.0, 3000.0, samplerate, 1, NULL);
    float* pt = (float*)malloc(sizeof(float) * 2 * np);
    orc_band_pass_c(18750.0, 19250.0, 3000.0, samplerate, 1, pt);
    w->pilot = orc_fir_create(ORC_C64, ORC_C64, pt, np, 1, precise);
    free(pt);
    orc_pll_init(&w->pll, 25000.0 / samplerate, 0.0, hz_to_rads(19000.0, samplerate), hz_to_rads(18750.0, samplerate),
                 hz_to_rads(19250.0, samplerate));
    w->delay = ((np - 1) / 2) + 1;
    int n = orc_low_pass(15000.0, 4000.0, samplerate, 0, NULL);
    float* t = (float*)malloc(sizeof(float) * n);
    orc_low_pass(15000.0, 4000.0, samplerate, 0, t);
    w->al = orc_fir_create(ORC_F32, ORC_F32, t, n, 1, precise);
    w->ar = orc_fir_create(ORC_F32, ORC_F32, t, n, 1, precise);
    free(t);
    w->stereo = stereo; w->lowPass = lowPass;
    w->dlpr = (float*)calloc(w->delay, sizeof(float));            /* Delay<float> state */
    w->dlmr = (float*)calloc(2 * w->delay, sizeof(float));        /* Delay<complex_t> state */
    return w;
}
static void orc_delay(float* state, int delay, int e, const float* in, int count, float* out) {
    /* math/delay.h:39-50: out = [state || in][0:count], state = last `delay` of [state || in] */
    float* buf = (float*)malloc(sizeof(float) * e * (delay + count));
    memcpy(buf, state, sizeof(float) * e * delay);
    memcpy(buf + e * delay, in, sizeof(float) * e * count);
    memcpy(out, buf, sizeof(float) * e * count);
    memcpy(state, buf + e * count, sizeof(float) * e * delay);
    free(buf);
}
int orc_wfms_process(orc_wfms* w, const float* in, int count, float* out) {
    if (w->cap < count) {
        free(w->mpx); free(w->cplx); free(w->pf); free(w->vco); free(w->lmr); free(w->l); free(w->r);
        w->mpx = (float*)malloc(sizeof(float) * count); w->cplx = (float*)malloc(sizeof(float) * 2 * count);
        w->pf = (float*)malloc(sizeof(float) * 2 * count); w->vco = (float*)malloc(sizeof(float) * 2 * count);
        w->lmr = (float*)malloc(sizeof(float) * 2 * count); w->l = (float*)malloc(sizeof(float) * count);
        w->r = (float*)malloc(sizeof(float) * count);
        w->cap = count;
    }
    orc_quad_process(w->q, in, count, w->mpx);
    if (!w->stereo) {
        if (w->lowPass) orc_fir_process(w->al, w->mpx, count, w->mpx);
        for (int i = 0; i < count; i++) { out[2 * i] = w->mpx[i]; out[2 * i + 1] = w->mpx[i]; }
        return count;
    }
    for (int i = 0; i < count; i++) { w->cplx[2 * i] = w->mpx[i]; w->cplx[2 * i + 1] = 0.0f; }   /* RealToComplex */
    orc_fir_process(w->pilot, w->cplx, count, w->pf);
    orc_pll_process(&w->pll, w->pf, count, w->vco);
    orc_delay(w->dlpr, w->delay, 1, w->mpx, count, w->mpx);          /* lprDelay (in place) */
    orc_delay(w->dlmr, w->delay, 2, w->cplx, count, w->lmr);         /* lmrDelay */
    for (int i = 0; i < count; i++) {
        float vr = w->vco[2 * i], vi = -w->vco[2 * i + 1];            /* Conjugate */
        for (int k = 0; k < 2; k++) {                                  /* Multiply<complex_t> twice */
            float ar = w->lmr[2 * i], ai = w->lmr[2 * i + 1];
            w->lmr[2 * i] = (ar * vr) - (ai * vi);
            w->lmr[2 * i + 1] = (ai * vr) + (ar * vi);
        }
        float lmr = w->lmr[2 * i] * 2.0f;                              /* ComplexToReal, x2 */
        w->l[i] = w->mpx[i] + lmr;                                     /* Add */
        w->r[i] = w->mpx[i] - lmr;                                     /* Subtract */
    }
    if (w->lowPass) {
        orc_fir_process(w->al, w->l, count, w->l);
        orc_fir_process(w->ar, w->r, count, w->r);
    }
    for (int i = 0; i < count; i++) { out[2 * i] = w->l[i]; out[2 * i + 1] = w->r[i]; }   /* LRToStereo */
    return count;
}
void orc_wfms_destroy(orc_wfms* w) {
    if (!w) return;
    orc_quad_destroy(w->q); orc_fir_destroy(w->pilot); orc_fir_destroy(w->al); orc_fir_destroy(w->ar);
    free(w->mpx); free(w->cplx); free(w->pf); free(w->vco); free(w->lmr); free(w->l); free(w->r);
    free(w->dlpr); free(w->dlmr); free(w);
}

/* --------------------------------------------------------------- FM (NFM) */
/* demod/fm.h:25-96 (T = float) */
struct orc_fm { orc_quad* q; orc_fir* fir; int filtering; };
orc_fm* orc_fm_create(double samplerate, double bandwidth, int lowPass, int highPass, int precise) {
    orc_fm* f = (orc_fm*)calloc(1, sizeof(orc_fm));
    f->q = orc_quad_create(hz_to_rads(bandwidth / 2.0, samplerate));
    f->filtering = lowPass || highPass;
    int n; float* t;
    if (lowPass && highPass) {
        n = orc_band_pass_f(300.0, bandwidth / 2.0, 100.0, samplerate, 0, NULL);
        t = (float*)malloc(sizeof(float) * n); orc_band_pass_f(300.0, bandwidth / 2.0, 100.0, samplerate, 0, t);
    } else if (highPass) {
        n = orc_high_pass(300.0, 100.0, samplerate, 0, NULL);
        t = (float*)malloc(sizeof(float) * n); orc_high_pass(300.0, 100.0, samplerate, 0, t);
    } else if (lowPass) {
        n = orc_low_pass(bandwidth / 2.0, (bandwidth / 2.0) * 0.1, samplerate, 0, NULL);
        t = (float*)malloc(sizeof(float) * n); orc_low_pass(bandwidth / 2.0, (bandwidth / 2.0) * 0.1, samplerate, 0, t);
    } else {
        n = 1; t = (float*)malloc(sizeof(float)); t[0] = 1.0f;
    }
    f->fir = orc_fir_create(ORC_F32, ORC_F32, t, n, 1, precise);
    free(t);
    return f;
}
int orc_fm_process(orc_fm* f, const float* in, int count, float* out) {
    orc_quad_process(f->q, in, count, out);
    if (f->filtering) orc_fir_process(f->fir, out, count, out);
    return count;
}
void orc_fm_destroy(orc_fm* f) { if (!f) return; orc_quad_destroy(f->q); orc_fir_destroy(f->fir); free(f); }

/* --------------------------------------------------------------------- AGC */
/* loop/agc.h:13-147 */
struct orc_agc {
    int dtype, enabled;
    float setPoint, attack, invAttack, decay, invDecay, maxGain, maxOutputAmp, initGain, gain, amp;
};
orc_agc* orc_agc_create(int dtype, double setPoint, double attack, double decay, double maxGain, double maxOutputAmp, double initGain) {
    orc_agc* a = (orc_agc*)calloc(1, sizeof(orc_agc));
    a->dtype = dtype;
    a->setPoint = (float)setPoint; a->attack = (float)attack; a->invAttack = 1.0f - a->attack;
    a->decay = (float)decay; a->invDecay = 1.0f - a->decay;
    a->maxGain = (float)maxGain; a->maxOutputAmp = (float)maxOutputAmp; a->initGain = (float)initGain;
    a->amp = a->setPoint / a->initGain;
    a->gain = a->initGain < a->maxGain ? a->initGain : a->maxGain;
    a->enabled = 1;
    return a;
}
void orc_agc_set_enabled(orc_agc* a, int en) { a->enabled = en; }
void orc_agc_set_gain(orc_agc* a, float g) { a->gain = g; }   /* agc.h:31-35 */
float orc_agc_get_gain(orc_agc* a) { return a->gain; }
static float amp_of(const float* x, int dtype, int i) {
    if (dtype == ORC_C64) { float re = x[2 * i], im = x[2 * i + 1]; return sqrtf((re * re) + (im * im)); }
    return fabsf(x[i]);
}
static float fminf_std(float a, float b) { return (b < a) ? b : a; }   /* std::min<float> */
int orc_agc_process(orc_agc* a, const float* in, int count, float* out) {
    int e = esz(a->dtype);
    for (int i = 0; i < count; i++) {
        float inAmp = amp_of(in, a->dtype, i);
        float g;
        if (a->enabled) {
            if (inAmp != 0.0f) {
                a->amp = (inAmp > a->amp) ? ((a->amp * a->invAttack) + (inAmp * a->attack))
                                          : ((a->amp * a->invDecay) + (inAmp * a->decay));
                a->gain = fminf_std(a->setPoint / a->amp, a->maxGain);
            } else {
                a->gain = 1.0f;
            }
            if (inAmp * a->gain > a->maxOutputAmp) {
                float maxAmp = 0;
                for (int j = i; j < count; j++) { float v = amp_of(in, a->dtype, j); if (v > maxAmp) maxAmp = v; }
                a->amp = maxAmp;
                a->gain = fminf_std(a->setPoint / a->amp, a->maxGain);
            }
            g = a->gain;
        } else {
            float gainAmp = inAmp * a->gain;
            g = (gainAmp > a->maxOutputAmp) ? (a->maxOutputAmp / inAmp) : a->gain;
        }
        for (int k = 0; k < e; k++) out[e * i + k] = in[e * i + k] * g;
    }
    return count;
}
void orc_agc_destroy(orc_agc* a) { free(a); }

/* -------------------------------------------------------------- DCBlocker */
/* correction/dc_blocker.h:54-60 */
struct orc_dcb { int dtype; float rate; float off[2]; };
orc_dcb* orc_dcb_create(int dtype, double rate) {
    orc_dcb* d = (orc_dcb*)calloc(1, sizeof(orc_dcb));
    d->dtype = dtype; d->rate = (float)rate;
    return d;
}
int orc_dcb_process(orc_dcb* d, const float* in, int count, float* out) {
    int e = esz(d->dtype);
    for (int i = 0; i < count; i++)
        for (int k = 0; k < e; k++) {
            out[e * i + k] = in[e * i + k] - d->off[k];
            d->off[k] += out[e * i + k] * d->rate;
        }
    return count;
}
void orc_dcb_destroy(orc_dcb* d) { free(d); }

/* ------------------------------------------------------------------- AM */
/* demod/am.h:18-142 (T = float) */
enum { AM_AGC_OFF = 0, AM_AGC_CARRIER, AM_AGC_AUDIO };
struct orc_am { int mode; orc_agc *carrier, *audio; orc_dcb* dcb; orc_fir* lpf; float* tmp; int cap; };
orc_am* orc_am_create(int agcMode, double bandwidth, double agcAttack, double agcDecay, double dcBlockRate, double samplerate, int precise) {
    orc_am* a = (orc_am*)calloc(1, sizeof(orc_am));
    a->mode = agcMode;
    a->carrier = orc_agc_create(ORC_C64, 1.0, agcAttack, agcDecay, 10e6, 10.0, INFINITY);
    a->audio = orc_agc_create(ORC_F32, 1.0, agcAttack, agcDecay, 10e6, 10.0, INFINITY);
    a->dcb = orc_dcb_create(ORC_F32, dcBlockRate);
    int n = orc_low_pass(bandwidth / 2.0, (bandwidth / 2.0) * 0.1, samplerate, 0, NULL);
    float* t = (float*)malloc(sizeof(float) * n);
    orc_low_pass(bandwidth / 2.0, (bandwidth / 2.0) * 0.1, samplerate, 0, t);
    a->lpf = orc_fir_create(ORC_F32, ORC_F32, t, n, 1, precise);
    free(t);
    orc_agc_set_enabled(a->carrier, 1);
    orc_agc_set_enabled(a->audio, agcMode == AM_AGC_AUDIO);
    return a;
}
int orc_am_process(orc_am* a, const float* in, int count, float* out) {
    if (a->mode == AM_AGC_CARRIER) {
        if (a->cap < count) { free(a->tmp); a->tmp = (float*)malloc(sizeof(float) * 2 * count); a->cap = count; }
        orc_agc_process(a->carrier, in, count, a->tmp);
        in = a->tmp;
    }
    for (int i = 0; i < count; i++) { float re = in[2 * i], im = in[2 * i + 1]; out[i] = sqrtf((re * re) + (im * im)); }
    orc_dcb_process(a->dcb, out, count, out);
    if (a->mode != AM_AGC_CARRIER) orc_agc_process(a->audio, out, count, out);
    orc_fir_process(a->lpf, out, count, out);
    return count;
}
void orc_am_destroy(orc_am* a) {
    if (!a) return;
    orc_agc_destroy(a->carrier); orc_agc_destroy(a->audio); orc_dcb_destroy(a->dcb); orc_fir_destroy(a->lpf); free(a->tmp); free(a);
}

/* ------------------------------------------------------------------- SSB */
/* demod/ssb.h:27-105 (T = float) */
struct orc_ssb { orc_xlator* x; orc_agc* agc; float* tmp; int cap; };
orc_ssb* orc_ssb_create(int mode, double bandwidth, double samplerate, int agcEnabled, double agcAttack, double agcDecay) {
    orc_ssb* s = (orc_ssb*)calloc(1, sizeof(orc_ssb));
    double tr = mode == 0 ? bandwidth / 2.0 : (mode == 1 ? -bandwidth / 2.0 : 0.0);
    s->x = orc_xlator_create(hz_to_rads(tr, samplerate));
    s->agc = orc_agc_create(ORC_F32, 1.0, agcAttack, agcDecay, 10e6, 10.0, INFINITY);
    orc_agc_set_enabled(s->agc, agcEnabled);
    return s;
}
int orc_ssb_process(orc_ssb* s, const float* in, int count, float* out) {
    if (s->cap < count) { free(s->tmp); s->tmp = (float*)malloc(sizeof(float) * 2 * count); s->cap = count; }
    orc_xlator_process(s->x, in, count, s->tmp);
    for (int i = 0; i < count; i++) out[i] = s->tmp[2 * i];           /* ComplexToReal */
    orc_agc_process(s->agc, out, count, out);
    return count;
}
void orc_ssb_destroy(orc_ssb* s) { if (!s) return; orc_xlator_destroy(s->x); orc_agc_destroy(s->agc); free(s->tmp); free(s); }

/* ----------------------------------------------------------- compression */
/* compression/sample_stream_compressor.h:26-60: 8-byte header
 * {u16 compressionType=0, u16 sampleType, f32 scaler}; scaler = the SIGNED max
 * (volk_32f_index_max_32u, first index on ties). VOLK generic convert kernels:
 * 8i/16i: r = x*scalar, clamp to the integer range, rintf. */
int orc_compress(int pcmType, const float* in, int count, uint8_t* out) {
    uint16_t ct = 0, st = (uint16_t)pcmType;
    memcpy(out, &ct, 2); memcpy(out + 2, &st, 2);
    if (pcmType == 2) {
        float z = 0; memcpy(out + 4, &z, 4);
        memcpy(out + 8, in, sizeof(float) * 2 * (size_t)count);
        return 8 + count * 8;
    }
    int n = count * 2; unsigned idx = 0; float mv = in[0];
    for (int i = 1; i < n; i++) if (in[i] > mv) { mv = in[i]; idx = i; }
    memcpy(out + 4, &mv, 4);
    if (pcmType == 0) {
        float sc = 128.0f / mv; int8_t* o = (int8_t*)(out + 8);
        for (int i = 0; i < n; i++) { float r = in[i] * sc; if (r > 127.0f) r = 127.0f; else if (r < -128.0f) r = -128.0f; o[i] = (int8_t)rintf(r); }
        return 8 + n;
    }
    if (pcmType == 1) {
        float sc = 32768.0f / mv;
        for (int i = 0; i < n; i++) {
            float r = in[i] * sc; if (r > 32767.0f) r = 32767.0f; else if (r < -32768.0f) r = -32768.0f;
            int16_t v = (int16_t)rintf(r); memcpy(out + 8 + 2 * i, &v, 2);
        }
        return 8 + 2 * n;
    }
    (void)idx;
    return count;
}
/* compression/sample_stream_decompressor.h:13-33 */
int orc_decompress(const uint8_t* in, int nbytes, float* out) {
    uint16_t st; float scaler; memcpy(&st, in + 2, 2); memcpy(&scaler, in + 4, 4);
    if (st == 2) { memcpy(out, in + 8, nbytes - 8); return (nbytes - 8) / 8; }
    if (st == 1) {
        int oc = (nbytes - 8) / 4; float sc = 32768.0f / scaler;
        for (int i = 0; i < oc * 2; i++) { int16_t v; memcpy(&v, in + 8 + 2 * i, 2); out[i] = ((float)v) / sc; }
        return oc;
    }
    if (st == 0) {
        int oc = (nbytes - 8) / 2; float sc = 128.0f / scaler; const float isc = 1.0 / sc;
        for (int i = 0; i < oc * 2; i++) out[i] = ((float)((const int8_t*)(in + 8))[i]) * isc;
        return oc;
    }
    return 0;
}

/* ------------------------------------------------------------ C5 chain */
struct orc_chain { int N; float* window; float* work; float* db; orc_vfo* vfo; orc_wfm* wfm; float* vbuf; long vcap; };
orc_chain* orc_chain_create(double fs, int fftSize, double vfoOffset, int precise) {
    orc_chain* c = (orc_chain*)calloc(1, sizeof(orc_chain));
    c->N = fftSize;
    c->window = (float*)malloc(sizeof(float) * fftSize);
    orc_create_window(ORC_WIN_BLACKMAN_HARRIS7, c->window, fftSize, 1);
    c->work = (float*)malloc(sizeof(float) * 4 * fftSize);
    c->db = (float*)malloc(sizeof(float) * fftSize);
    c->vfo = orc_vfo_create(fs, 240000.0, 200000.0, vfoOffset, precise);
    c->wfm = orc_wfm_create(100000.0, 240000.0, 1, precise);
    return c;
}
long orc_chain_process(orc_chain* c, const float* in, long count, float* spectra, long maxFrames, float* audio) {
    long frames = count / c->N;
    for (long f = 0; f < frames; f++) {
        float* dst = (spectra && f < maxFrames) ? spectra + (size_t)f * c->N : c->db;
        orc_fft_logmag(in + 2 * (size_t)f * c->N, c->N, c->N, c->window, c->work, dst);
    }
    if (c->vcap < count) { free(c->vbuf); c->vbuf = (float*)malloc(sizeof(float) * 2 * count); c->vcap = count; }
    long total = 0;
    for (long off = 0; off < count; off += 1000000) {   /* STREAM_BUFFER_SIZE blocks */
        int n = (int)((count - off) < 1000000 ? (count - off) : 1000000);
        int m = orc_vfo_process(c->vfo, in + 2 * off, n, c->vbuf);
        orc_wfm_process(c->wfm, c->vbuf, m, audio + 2 * total);
        total += m;
    }
    return total;
}
void orc_chain_destroy(orc_chain* c) {
    if (!c) return;
    free(c->window); free(c->work); free(c->db); orc_vfo_destroy(c->vfo); orc_wfm_destroy(c->wfm); free(c->vbuf); free(c);
}

/* ---------------------------------------------------------------- C4 channelizer
 * Definition restated from its parts: xlator (frequency_xlator.h:43-50) with the exact
 * angle -2 pi k n / M (reduced as the integer k n mod M, so no phase drift), then the
 * decimating FIR (decimating_fir.h:45-68): buf = [ntaps-1 zeros || x],
 * y[m] = sum_j h[j] buf[m M + j]. Accumulated in double. */
int orc_channelize(const float* in, long count, const float* h, int ntaps, int M, const int* chans, int nchan,
                   double* out) {
    if (M < 1 || ntaps < 1 || count < 0) return -1;
    const long frames = (count + M - 1) / M;
    const long H = ntaps - 1;
    double* cs = (double*)malloc(sizeof(double) * 2 * M);
    for (int c = 0; c < nchan; c++) {
        const long k = chans[c];
        for (int i = 0; i < M; i++) {            /* e^{-2 pi i t / M}, t = (k n) mod M */
            const double a = -2.0 * DB_M_PI * (double)i / (double)M;
            cs[2 * i] = cos(a);
            cs[2 * i + 1] = sin(a);
        }
        for (long m = 0; m < frames; m++) {
            double ar = 0.0, ai = 0.0;
            for (int j = 0; j < ntaps; j++) {
                const long n = m * M + j - H;     /* absolute input index of buf[m M + j] */
                if (n < 0 || n >= count) continue;
                const long t = (long)(((k % M) * (n % M)) % M);
                const double xr = in[2 * n], xi = in[2 * n + 1];
                const double pr = cs[2 * t], pi = cs[2 * t + 1];
                const double zr = xr * pr - xi * pi, zi = xr * pi + xi * pr;
                ar += (double)h[j] * zr;
                ai += (double)h[j] * zi;
            }
            out[2 * ((long)c * frames + m)] = ar;
            out[2 * ((long)c * frames + m) + 1] = ai;
        }
    }
    free(cs);
    return (int)frames;
}

/* ------------------------------------------------------------ Deemphasis */
/* filter/deephasis.h:14-93 (T = float or stereo_t: `ch` interleaved channels) */
struct orc_deemp { float alpha; float last[2]; int ch; };
orc_deemp* orc_deemp_create(int channels, double tau, double samplerate) {
    orc_deemp* d = (orc_deemp*)calloc(1, sizeof(orc_deemp));
    float dt = (float)(1.0f / samplerate);              /* float dt = 1.0f / _samplerate */
    d->alpha = (float)((double)dt / (tau + (double)dt)); /* alpha = dt / (_tau + dt) */
    d->ch = channels;
    return d;
}
int orc_deemp_process(orc_deemp* d, const float* in, int count, float* out) {
    const float beta = 1 - d->alpha;
    for (int i = 0; i < count; i++)
        for (int c = 0; c < d->ch; c++) {
            float y = (d->alpha * in[i * d->ch + c]) + (beta * d->last[c]);
            out[i * d->ch + c] = y;
            d->last[c] = y;
        }
    return count;
}
void orc_deemp_destroy(orc_deemp* d) { free(d); }

/* ------------------------------------------------------ fft_scaler::doZoom */
/* gui/widgets/fft_scaler.h:27-64 */
int orc_zoom(const float* data, int fftSize, double viewOffset, double viewBandwidth, double wholeBandwidth,
             int outSize, float* out) {
    const double offsetRatio = viewOffset / (wholeBandwidth / 2.0);
    double width = (viewBandwidth / wholeBandwidth) * fftSize;
    double offset = (((double)fftSize / 2.0) * (offsetRatio + 1)) - (width / 2);
    if (offset < 0) offset = 0;
    if (width > fftSize - offset) width = fftSize - offset;
    const double factor = width / outSize;
    double f0 = offset;
    if (factor <= 1.0) {
        for (int i = 0; i < outSize; i++) {
            double f1 = f0 + factor;
            int i0 = (int)roundf((float)f0);
            *out++ = data[i0];
            f0 = f1;
        }
    } else {
        int i0 = (int)roundf((float)f0);
        for (int i = 0; i < outSize; i++) {
            double f1 = f0 + factor;
            int i1 = (int)roundf((float)f1);
            float maxVal = data[i0];
            for (int j = i0 + 1; j < i1; j++) maxVal = (maxVal < data[j]) ? data[j] : maxVal;   /* std::max */
            *out++ = maxVal;
            f0 = f1;
            i0 = i1;
        }
    }
    return outSize;
}

/* ------------------------------------------- WaterFall::pushFFT consumers */
/* colormap of zoomed rows into the waterfall framebuffer (gui/widgets/waterfall.cpp:903-910) */
void orc_colormap(const float* in, long n, float wfMin, float wfMax, const unsigned* pallet, int res, unsigned* out) {
    const float dataRange = wfMax - wfMin;
    for (long j = 0; j < n; j++) {
        float v = in[j];
        v = v < wfMin ? wfMin : (wfMax < v ? wfMax : v);   /* std::clamp<float> */
        const float pixel = (v - wfMin) / dataRange;
        const int id = (int)(pixel * (res - 1));
        out[j] = pallet[id];
    }
}

/* FFT smoothing then FFT hold on consecutive zoomed rows (waterfall.cpp:918-925, 952-957):
 * row <- smooth = row*alpha + smooth*beta (three volk roundings); hold[i] = max(row[i], hold[i]-speed), i >= 1 */
void orc_fft_smooth_hold(float* rows, int nrows, int width, int smoothing, float alpha, float beta, float* smooth,
                         int holdOn, float holdSpeed, float* hold) {
    for (int r = 0; r < nrows; r++) {
        float* latest = rows + (long)r * width;
        if (smoothing) {
            for (int i = 0; i < width; i++) {
                const float a = latest[i] * alpha;
                const float b = smooth[i] * beta;
                smooth[i] = b + a;
                latest[i] = smooth[i];
            }
        }
        if (holdOn) {
            for (int i = 1; i < width; i++) {
                const float h = hold[i] - holdSpeed;
                hold[i] = (latest[i] < h) ? h : latest[i];   /* std::max<float>(latest, hold - speed) */
            }
        }
    }
}

/* WaterFall::calculateVFOSignalInfo (waterfall.cpp:563-601) on one raw dB row. The reference's max
 * loop runs to i <= vfoMaxOffset, which reads one past the row when vfoMaxOffset == fftSize; here that
 * bin is skipped (a conscious fix: it cannot change the result of a correct read). */
void orc_vfo_signal_info(const float* line, int fftSize, double wholeBandwidth, double centerOffset, double bandwidth,
                         float* strength, float* snr) {
    const double minSide = centerOffset - bandwidth, minF = centerOffset - (bandwidth / 2.0);
    const double maxF = centerOffset + (bandwidth / 2.0), maxSide = centerOffset + bandwidth;
#define OFS(f) ({ double v_ = (((f) / (wholeBandwidth / 2.0)) * (double)(fftSize / 2)) + (fftSize / 2); int i_ = (int)v_; \
                  i_ < 0 ? 0 : (i_ > fftSize ? fftSize : i_); })
    const int a0 = OFS(minSide), a1 = OFS(minF), b0 = OFS(maxF), b1 = OFS(maxSide);
#undef OFS
    double avg = 0;
    int cnt = 0;
    for (int i = a0; i < a1; i++) { avg += line[i]; cnt++; }
    for (int i = b0 + 1; i < b1; i++) { avg += line[i]; cnt++; }
    avg /= (double)cnt;
    float mx = -INFINITY;
    for (int i = a1; i <= b0 && i < fftSize; i++) if (line[i] > mx) mx = line[i];
    *strength = mx;
    *snr = mx - avg;
}

/* ----------------------------------------------------- C3 chain (CPU baseline) */
/* FrequencyXlator -> DecimatingFIR<complex_t, float> -> Quadrature, one block at a time
 * (the three reference blocks back to back; precise = 0: VOLK-style fp32 rotator and dots) */
struct orc_ddcfm { orc_xlator* x; orc_fir* f; orc_quad* q; float *a, *b; int cap; };
orc_ddcfm* orc_ddcfm_create(double offsetRad, const float* taps, int ntaps, int decim, double deviationRad, int precise) {
    orc_ddcfm* d = (orc_ddcfm*)calloc(1, sizeof(orc_ddcfm));
    d->x = precise ? orc_xlator_create(offsetRad) : orc_xlator_create_fast(offsetRad);
    d->f = orc_fir_create(ORC_C64, ORC_F32, taps, ntaps, decim, precise);
    d->q = orc_quad_create(deviationRad);
    d->q->fast = !precise;
    return d;
}
int orc_ddcfm_process(orc_ddcfm* d, const float* in, int count, float* out) {
    /* the CPU baseline (precise = 0) runs the chain in L2-sized sub-blocks so the intermediates
     * stay in cache (the result is the same stream: every stage carries its state) */
    const int sub = d->f->precise ? count : 16384;
    const int cap = count < sub ? count : sub;
    if (d->cap < cap) { free(d->a); free(d->b); d->a = (float*)malloc(sizeof(float) * 2 * cap); d->b = (float*)malloc(sizeof(float) * 2 * cap); d->cap = cap; }
    int total = 0;
    for (int i = 0; i < count; i += sub) {
        const int c = count - i < sub ? count - i : sub;
        orc_xlator_process(d->x, in + 2 * (size_t)i, c, d->a);
        int m = orc_fir_process(d->f, d->a, c, d->b);
        total += orc_quad_process(d->q, d->b, m, out + total);
    }
    return total;
}
void orc_ddcfm_destroy(orc_ddcfm* d) {
    if (!d) return;
    orc_xlator_destroy(d->x); orc_fir_destroy(d->f); orc_quad_destroy(d->q); free(d->a); free(d->b); free(d);
}

/* ------------------------------------------------------ recorder encoders */
/* utils/wav.cpp:296-336 (WAV writer): kind 0 u8, 1 i16, 2 i24 (packed LE), 3 i32, 4 f32.
 * n = sample values; returns bytes written. */
static float orc_clampf(float v) { return (v < -1.0f) ? -1.0f : (1.0f < v) ? 1.0f : v; }   /* std::clamp */
int orc_wav_encode(int kind, const float* in, int n, uint8_t* out) {
    for (int i = 0; i < n; i++) {
        const float c = orc_clampf(in[i]);
        switch (kind) {
        case 0: out[i] = (uint8_t)lroundf(c * (128.0f - 0.5f) - 0.5f + 128); break;
        case 1: { int16_t v = (int16_t)lroundf(c * (32768.0f - 0.5f) - 0.5f); memcpy(out + 2 * i, &v, 2); } break;
        case 2: {
            int32_t v = (int32_t)lroundf(c * (8388608.0f - 0.5f) - 0.5f);
            out[3 * i] = (uint8_t)v; out[3 * i + 1] = (uint8_t)(v >> 8); out[3 * i + 2] = (uint8_t)(v >> 16);
        } break;
        case 3: { int32_t v = (int32_t)lroundf((float)((double)c * (2147483648.0 - 0.5) - 0.5)); memcpy(out + 4 * i, &v, 4); } break;
        default: memcpy(out + 4 * i, &in[i], 4); break;
        }
    }
    static const int sz[] = {1, 2, 3, 4, 4};
    return n * sz[kind < 0 || kind > 4 ? 4 : kind];
}
