/* CPU-baseline kernels of the oracle (TEST INFRASTRUCTURE: they run only on the precise = 0
 * paths, which bench.py's cpu_baseline leg times; the parity checker uses the precise paths).
 *
 * The reference's CPU path calls VOLK per output (filter/decimating_fir.h:45-68: one
 * volk_32fc_32f_dot_prod_32fc per output, a horizontal reduction each time), the VOLK rotator
 * per block (channel/frequency_xlator.h:43-50) and atan2f per sample (demod/quadrature.h:41-56).
 * These are the same computations written the fastest way this restatement knows for one
 * AVX-512 core, so that every GPU / CPU ratio is taken against a CPU that is not held back by
 * per-output overheads:
 *   - cf_rotate: the rotator on 8 complex lanes per 512-bit vector (lane i carries
 *     phase * delta^i, the vector advances by delta^8), renormalised every 512 samples like
 *     volk_32fc_s32fc_x2_rotator2_32fc;
 *   - cf_fir_cf_decim: complex data x real taps, EIGHT outputs per pass over the taps (one tap
 *     vector load feeds eight FMAs), the eight 16-lane accumulators reduced together by a
 *     3-round shuffle transpose into one vector of 8 complex outputs (no per-output horizontal
 *     reduction);
 *   - cf_quad: arg(y conj(y_prev)) on 16 outputs per vector with a degree-17 odd polynomial
 *     atan (|error| <= 2e-8 rad, Abramowitz & Stegun 4.4.49) -- VOLK's atan2 kernels are
 *     polynomial too.
 * GCC vector extensions; -march=native lowers them to AVX-512 on the GPU box's EPYC 9575F. */
#include <math.h>
#include <string.h>
#include "sdr_oracle.h"

typedef float v16f __attribute__((vector_size(64)));
typedef int v16i __attribute__((vector_size(64)));

static inline v16f ld(const float* p) { v16f v; memcpy(&v, p, sizeof(v)); return v; }
static inline void st(float* p, v16f v) { memcpy(p, &v, sizeof(v)); }
static inline v16f splat(float a) { return (v16f){a, a, a, a, a, a, a, a, a, a, a, a, a, a, a, a}; }
static inline v16f swap_pairs(v16f v) { return __builtin_shuffle(v, (v16i){1, 0, 3, 2, 5, 4, 7, 6, 9, 8, 11, 10, 13, 12, 15, 14}); }
static inline v16f dup_even(v16f v) { return __builtin_shuffle(v, (v16i){0, 0, 2, 2, 4, 4, 6, 6, 8, 8, 10, 10, 12, 12, 14, 14}); }
static inline v16f dup_odd(v16f v) { return __builtin_shuffle(v, (v16i){1, 1, 3, 3, 5, 5, 7, 7, 9, 9, 11, 11, 13, 13, 15, 15}); }
static const v16f SIGN_ALT = {-1, 1, -1, 1, -1, 1, -1, 1, -1, 1, -1, 1, -1, 1, -1, 1};
/* interleaved complex product v * w (8 complex lanes) */
static inline v16f cmul_il(v16f v, v16f w) { return v * dup_even(w) + swap_pairs(v) * (dup_odd(w) * SIGN_ALT); }

/* ---------------------------------------------------------------- rotator */
void cf_rotate(const float* in, float* out, int count, float* pr, float* pi, float dr, float di, int* cnt) {
    /* lane phasors p * d^i, i < 8, and the vector step d^8 */
    float lr[8], li[8];
    float cr = *pr, ci = *pi, er = 1.0f, ei = 0.0f;   /* c = p d^i, e = d^i */
    for (int i = 0; i < 8; i++) {
        lr[i] = cr; li[i] = ci;
        float nr = cr * dr - ci * di, ni = cr * di + ci * dr;
        cr = nr; ci = ni;
        nr = er * dr - ei * di; ni = er * di + ei * dr;
        er = nr; ei = ni;
    }
    v16f P, D8;
    for (int i = 0; i < 8; i++) { P[2 * i] = lr[i]; P[2 * i + 1] = li[i]; D8[2 * i] = er; D8[2 * i + 1] = ei; }
    int i = 0, c = *cnt;
    for (; i + 8 <= count; i += 8) {
        st(out + 2 * i, cmul_il(ld(in + 2 * i), P));
        P = cmul_il(P, D8);
        c += 8;
        if (c >= 512) {   /* renormalise every lane to unit magnitude */
            v16f m2 = P * P;
            m2 = m2 + swap_pairs(m2);
            for (int k = 0; k < 16; k++) P[k] /= sqrtf(m2[k]);
            c = 0;
        }
    }
    float qr = P[0], qi = P[1];
    for (; i < count; i++) {   /* tail: scalar rotator from lane 0's phase */
        float re = in[2 * i], im = in[2 * i + 1];
        out[2 * i] = re * qr - im * qi;
        out[2 * i + 1] = re * qi + im * qr;
        float nr = qr * dr - qi * di, ni = qr * di + qi * dr;
        qr = nr; qi = ni;
        c++;
    }
    *pr = qr; *pi = qi; *cnt = c;
}

/* ------------------------------------------------- decimating FIR, c64 x f32 */
/* y[k] = sum_j x[o_k + j] h[j], o_k = offset + k D, over the interleaved buffer x; hh = taps
 * duplicated per (re, im), zero-padded to a multiple of 16 floats (m16); x readable for m16 floats
 * past every o_k. Returns the number of outputs (o_k < count). */
static inline v16f red_half(v16f a, v16f b, v16i lo, v16i hi) { return __builtin_shuffle(a, b, lo) + __builtin_shuffle(a, b, hi); }
int cf_fir_cf_decim(const float* x, const float* hh, int m16, int offset, int D, int count, float* out) {
    const v16i L1 = {0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18, 19, 20, 21, 22, 23};
    const v16i H1 = {8, 9, 10, 11, 12, 13, 14, 15, 24, 25, 26, 27, 28, 29, 30, 31};
    const v16i L2 = {0, 1, 2, 3, 8, 9, 10, 11, 16, 17, 18, 19, 24, 25, 26, 27};
    const v16i H2 = {4, 5, 6, 7, 12, 13, 14, 15, 20, 21, 22, 23, 28, 29, 30, 31};
    const v16i L3 = {0, 1, 4, 5, 8, 9, 12, 13, 16, 17, 20, 21, 24, 25, 28, 29};
    const v16i H3 = {2, 3, 6, 7, 10, 11, 14, 15, 18, 19, 22, 23, 26, 27, 30, 31};
    int n = 0, o = offset;
    if (D == 8) {
        /* one complex output step = 16 floats = one vector: output i's data at tap step k is
         * output 0's at step k + 16 i, so a register window of 8 data vectors slides one vector per
         * step -- two loads (taps, newest data) per eight FMAs */
        for (; o + 7 * D < count; o += 8 * D, n += 8) {
            const float* x0 = x + 2 * (size_t)o;
            v16f a0 = splat(0), a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;
            v16f w0 = ld(x0), w1 = ld(x0 + 16), w2 = ld(x0 + 32), w3 = ld(x0 + 48), w4 = ld(x0 + 64), w5 = ld(x0 + 80),
                 w6 = ld(x0 + 96), w7;
            /* two accumulator sets (even / odd tap steps): 16 independent FMA chains */
            v16f b0 = a0, b1 = a0, b2 = a0, b3 = a0, b4 = a0, b5 = a0, b6 = a0, b7 = a0;
            int k = 0;
            for (; k + 32 <= m16; k += 32) {
                w7 = ld(x0 + k + 112);
                v16f h = ld(hh + k);
                a0 += w0 * h; a1 += w1 * h; a2 += w2 * h; a3 += w3 * h;
                a4 += w4 * h; a5 += w5 * h; a6 += w6 * h; a7 += w7 * h;
                w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5; w5 = w6; w6 = w7;
                w7 = ld(x0 + k + 128);
                h = ld(hh + k + 16);
                b0 += w0 * h; b1 += w1 * h; b2 += w2 * h; b3 += w3 * h;
                b4 += w4 * h; b5 += w5 * h; b6 += w6 * h; b7 += w7 * h;
                w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5; w5 = w6; w6 = w7;
            }
            for (; k < m16; k += 16) {
                w7 = ld(x0 + k + 112);
                const v16f h = ld(hh + k);
                a0 += w0 * h; a1 += w1 * h; a2 += w2 * h; a3 += w3 * h;
                a4 += w4 * h; a5 += w5 * h; a6 += w6 * h; a7 += w7 * h;
                w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5; w5 = w6; w6 = w7;
            }
            a0 += b0; a1 += b1; a2 += b2; a3 += b3; a4 += b4; a5 += b5; a6 += b6; a7 += b7;
            const v16f b01 = red_half(a0, a1, L1, H1), b23 = red_half(a2, a3, L1, H1);
            const v16f b45 = red_half(a4, a5, L1, H1), b67 = red_half(a6, a7, L1, H1);
            const v16f c0 = red_half(b01, b23, L2, H2), c1 = red_half(b45, b67, L2, H2);
            st(out + 2 * (size_t)n, red_half(c0, c1, L3, H3));
        }
    }
    for (; o + 7 * D < count; o += 8 * D, n += 8) {
        const float* x0 = x + 2 * (size_t)o;
        const size_t s = 2 * (size_t)D;
        v16f a0 = splat(0), a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;
        for (int k = 0; k < m16; k += 16) {
            const v16f h = ld(hh + k);
            a0 += ld(x0 + k) * h;
            a1 += ld(x0 + s + k) * h;
            a2 += ld(x0 + 2 * s + k) * h;
            a3 += ld(x0 + 3 * s + k) * h;
            a4 += ld(x0 + 4 * s + k) * h;
            a5 += ld(x0 + 5 * s + k) * h;
            a6 += ld(x0 + 6 * s + k) * h;
            a7 += ld(x0 + 7 * s + k) * h;
        }
        const v16f b01 = red_half(a0, a1, L1, H1), b23 = red_half(a2, a3, L1, H1);
        const v16f b45 = red_half(a4, a5, L1, H1), b67 = red_half(a6, a7, L1, H1);
        const v16f c0 = red_half(b01, b23, L2, H2), c1 = red_half(b45, b67, L2, H2);
        st(out + 2 * (size_t)n, red_half(c0, c1, L3, H3));
    }
    for (; o < count; o += D, n++) {   /* tail outputs one at a time */
        const float* xo = x + 2 * (size_t)o;
        v16f a = splat(0);
        for (int k = 0; k < m16; k += 16) a += ld(xo + k) * ld(hh + k);
        float re = 0, im = 0;
        for (int l = 0; l < 16; l += 2) { re += a[l]; im += a[l + 1]; }
        out[2 * (size_t)n] = re;
        out[2 * (size_t)n + 1] = im;
    }
    return n;
}

/* ----------------------------------------------------------- quadrature */
static inline v16f blendv(v16i m, v16f a, v16f b) {   /* m ? a : b */
    v16i r = (m & (v16i)a) | (~m & (v16i)b);
    return (v16f)r;
}
static inline v16f vabs(v16f a) { return (v16f)(((v16i)a & (v16i)splat(-0.0f)) ^ (v16i)a); }
static inline v16f atan2_v(v16f y, v16f x) {
    const v16f ax = vabs(x), ay = vabs(y);
    const v16i swp = ay > ax;
    const v16f mn = blendv(swp, ax, ay), mx = blendv(swp, ay, ax);
    const v16f a = mn / blendv(mx == splat(0), splat(1), mx);
    const v16f s = a * a;
    v16f p = splat(0.0028662257f);
    p = p * s + splat(-0.0161657367f);
    p = p * s + splat(0.0429096138f);
    p = p * s + splat(-0.0752896400f);
    p = p * s + splat(0.1065626393f);
    p = p * s + splat(-0.1420889944f);
    p = p * s + splat(0.1999355085f);
    p = p * s + splat(-0.3333314528f);
    v16f r = a + a * s * p;
    r = blendv(swp, splat(1.57079632679489662f) - r, r);
    r = blendv(x < splat(0), splat(3.14159265358979324f) - r, r);
    return (v16f)(((v16i)r & ~(v16i)splat(-0.0f)) | ((v16i)y & (v16i)splat(-0.0f)));   /* sign of y */
}
void cf_quad(const float* in, int count, float* out, float* dre, float* dim, float inv) {
    const v16i EV = {0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30};
    const v16i OD = {1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 21, 23, 25, 27, 29, 31};
    int i = 0;
    float pr = *dre, pim = *dim;
    if (count >= 17) {
        /* output 0 from the carried sample, then 16 at a time with y[i - 1] loaded shifted */
        for (; i < 1; i++) {
            float yr = in[0], yi = in[1];
            float re = yr * pr + yi * pim, im = yi * pr - yr * pim;
            out[0] = atan2f(im, re) * inv;
        }
        for (; i + 16 <= count; i += 16) {
            const v16f a = ld(in + 2 * i), b = ld(in + 2 * i + 16);
            const v16f c = ld(in + 2 * i - 2), d = ld(in + 2 * i + 14);
            const v16f yr = __builtin_shuffle(a, b, EV), yi = __builtin_shuffle(a, b, OD);
            const v16f br = __builtin_shuffle(c, d, EV), bi = __builtin_shuffle(c, d, OD);
            const v16f re = yr * br + yi * bi, im = yi * br - yr * bi;   /* y * conj(prev) */
            st(out + i, atan2_v(im, re) * splat(inv));
        }
        pr = in[2 * (i - 1)]; pim = in[2 * (i - 1) + 1];
    }
    for (; i < count; i++) {
        float yr = in[2 * i], yi = in[2 * i + 1];
        float re = yr * pr + yi * pim, im = yi * pr - yr * pim;
        out[i] = atan2f(im, re) * inv;
        pr = yr; pim = yi;
    }
    *dre = pr; *dim = pim;
}

/* ------------------------------------------------ C4 channelizer branch FIRs */
/* The polyphase channelizer's branch filters (the GPU's algorithm, SURVEY 8d C4: bank layout
 * polyphase_bank.h:32, 16 taps per branch): u[f][m] = sum_q h[q][m] x[f + q][m] for f < frames,
 * m < M; x = frames + Q - 1 rows of M complex samples (interleaved), h = Q rows of M real taps.
 * Eight complex outputs per vector; the Q tap rows and the Q input rows of one output row stay in
 * L2 (Q x 8 KB each at M = 1024). The caller FFTs each row u[f]. */
void cf_chan_fir(const float* x, const float* h, int M, int Q, int frames, float* u) {
    const size_t row = 2 * (size_t)M;
    for (int f = 0; f < frames; f++) {
        float* uo = u + (size_t)f * row;
        int m = 0;
        for (; m + 8 <= M; m += 8) {
            v16f acc = splat(0);
            for (int q = 0; q < Q; q++) {
                const float* hq = h + (size_t)q * M + m;
                const v16f hv = {hq[0], hq[0], hq[1], hq[1], hq[2], hq[2], hq[3], hq[3],
                                 hq[4], hq[4], hq[5], hq[5], hq[6], hq[6], hq[7], hq[7]};
                acc += ld(x + (size_t)(f + q) * row + 2 * (size_t)m) * hv;
            }
            st(uo + 2 * (size_t)m, acc);
        }
        for (; m < M; m++) {
            float re = 0, im = 0;
            for (int q = 0; q < Q; q++) {
                const float* xq = x + (size_t)(f + q) * row + 2 * (size_t)m;
                re += xq[0] * h[(size_t)q * M + m];
                im += xq[1] * h[(size_t)q * M + m];
            }
            uo[2 * (size_t)m] = re;
            uo[2 * (size_t)m + 1] = im;
        }
    }
}
