// fp64-interior spectrum: the opt-in parity mode of the spectrum hot path
// (IQFrontEnd::handler, signal_path/iq_frontend.cpp:230-249; sdrgpu_fft_set_precision(h, 1)).
//
// The reference's arithmetic up to the FFT input is kept exactly: the window product is the fp32
// volk_32fc_32f_multiply_32fc (re * w, im * w, each rounded to fp32). From there every operation is
// fp64: butterflies, stage twiddles (host cos/sin tables), the four-step twiddle W_N^(n2 k1) (two
// 1024-entry fp64 tables, W_N^(1024 h) x W_N^l, one complex fp64 product), |X|^2 and 10 log10.
// The dB row is then the fp64 value rounded once to fp32: the correctly rounded dB of the exact DFT
// of the float-windowed frame up to the fp64 error (~1e-15 relative), i.e. within the north_star's
// 1 ulp on every bin (tests/test_gpu_parity.py::test_spectrum_f64_*).
//
// CDNA4 layout: gfx950 has no packed fp64, so the butterflies issue
// at the non-packed VALU rate; the intermediate of the four-step split is double2 (16 B per element),
// so the two-pass transform moves 8 + 16 + 16 + 4 = 44 B per sample instead of 28. Structure:
//   * N <= 4096: fft64_single_kernel, S frames per workgroup, all stages in LDS;
//   * N  > 4096: N = N1 x N2 (N1 >= N2, both <= 1024). Pass A: S consecutive columns of one frame
//     (S x 8-B row segments of the input), column FFTs of length N1, x W_N^(n2 k1) on the store
//     (S x 16-B row segments of the intermediate). Pass B: S consecutive rows k1, row FFTs of length
//     N2, dB stored at k1 + N1 k2 (S consecutive floats). Frames go in chunks of 128 MB of
//     intermediate, so it stays in the Infinity Cache between the passes.
//   * In LDS: Stockham autosort, radix 16 (radix 2/4/8 for the last stage), one pad element per 16.
#include <algorithm>
#include <cmath>
#include <vector>
#include "sdrgpu_internal.h"

namespace sdrgpu {
namespace {

__device__ __forceinline__ double2 zadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 zsub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 znegi(double2 a) { return make_double2(a.y, -a.x); }   // a * (-i)

__device__ __forceinline__ void zdft4(double2& x0, double2& x1, double2& x2, double2& x3) {
    const double2 a0 = zadd(x0, x2), a1 = zsub(x0, x2), a2 = zadd(x1, x3), d = znegi(zsub(x1, x3));
    x0 = zadd(a0, a2);
    x2 = zsub(a0, a2);
    x1 = zadd(a1, d);
    x3 = zsub(a1, d);
}

// forward DFT of R values in registers (e^{-i}), R in {2, 4, 8, 16}
template <int R>
__device__ __forceinline__ void zdft(double2* v) {
    if constexpr (R == 2) {
        const double2 a = v[0], b = v[1];
        v[0] = zadd(a, b);
        v[1] = zsub(a, b);
    } else if constexpr (R == 4) {
        zdft4(v[0], v[1], v[2], v[3]);
    } else if constexpr (R == 8) {
        const double R2 = 0.70710678118654752440;
        double2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6], o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
        zdft4(e0, e1, e2, e3);
        zdft4(o0, o1, o2, o3);
        o1 = make_double2(R2 * (o1.x + o1.y), R2 * (o1.y - o1.x));    // x W8^1
        o2 = znegi(o2);                                                // x W8^2
        o3 = make_double2(R2 * (o3.y - o3.x), -R2 * (o3.x + o3.y));   // x W8^3
        v[0] = zadd(e0, o0); v[4] = zsub(e0, o0);
        v[1] = zadd(e1, o1); v[5] = zsub(e1, o1);
        v[2] = zadd(e2, o2); v[6] = zsub(e2, o2);
        v[3] = zadd(e3, o3); v[7] = zsub(e3, o3);
    } else {   // 16 = 4 x 4: X[k1 + 4 k2] = sum_n2 W4^(n2 k2) W16^(n2 k1) DFT4_n1(x[4 n1 + n2])
        const double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173, R2 = 0.70710678118654752440;
        double2 y[4][4];
#pragma unroll
        for (int n2 = 0; n2 < 4; n2++) {
            y[n2][0] = v[n2]; y[n2][1] = v[4 + n2]; y[n2][2] = v[8 + n2]; y[n2][3] = v[12 + n2];
            zdft4(y[n2][0], y[n2][1], y[n2][2], y[n2][3]);
        }
        y[1][1] = zmul(y[1][1], make_double2(C1, -S1));
        y[1][2] = zmul(y[1][2], make_double2(R2, -R2));
        y[1][3] = zmul(y[1][3], make_double2(S1, -C1));
        y[2][1] = zmul(y[2][1], make_double2(R2, -R2));
        y[2][2] = znegi(y[2][2]);
        y[2][3] = zmul(y[2][3], make_double2(-R2, -R2));
        y[3][1] = zmul(y[3][1], make_double2(S1, -C1));
        y[3][2] = zmul(y[3][2], make_double2(-R2, -R2));
        y[3][3] = zmul(y[3][3], make_double2(-C1, S1));
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++) {
            double2 a = y[0][k1], b = y[1][k1], c = y[2][k1], d = y[3][k1];
            zdft4(a, b, c, d);
            v[k1] = a; v[k1 + 4] = b; v[k1 + 8] = c; v[k1 + 12] = d;
        }
    }
}

__device__ __forceinline__ int zpad(int i) { return i + (i >> 4); }
template <int L> struct ZLds { static constexpr int LS = L + L / 16 + 1; };

// One Stockham radix-R stage of S sequences of length L in LDS (sequence s at lds + s * LS), by
// S * L / 16 threads: thread (s, t) owns butterflies j = t + b * T (T = L / 16, b < 16 / R). With
// LAST the outputs go to st(s, k, value) instead of back to LDS. SF: s is the fastest thread
// coordinate (consecutive lanes = consecutive sequences), else t is.
template <int L, int S, int R, int NS, bool LAST, bool SF, class Store>
__device__ __forceinline__ void zstage(double2* lds, const double2* __restrict__ twL, Store&& st) {
    constexpr int T = L / 16, BPT = 16 / R, LS = ZLds<L>::LS;
    const int tid = threadIdx.x;
    const int s = SF ? tid % S : tid / T, t = SF ? tid / S : tid % T;
    double2* seq = lds + s * LS;
    double2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T;
#pragma unroll
        for (int r = 0; r < R; r++) v[b][r] = seq[zpad(j + r * (L / R))];
        if constexpr (NS > 1) {
            const int jm = j % NS;
#pragma unroll
            for (int r = 1; r < R; r++) v[b][r] = zmul(v[b][r], twL[r * jm * (L / (NS * R))]);
        }
        zdft<R>(v[b]);
    }
    if constexpr (LAST) {
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = t + b * T;
            const int idxD = (j / NS) * NS * R + (j % NS);
#pragma unroll
            for (int r = 0; r < R; r++) st(s, idxD + r * NS, v[b][r]);
        }
    } else {
        __syncthreads();
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = t + b * T;
            const int idxD = (j / NS) * NS * R + (j % NS);
#pragma unroll
            for (int r = 0; r < R; r++) seq[zpad(idxD + r * NS)] = v[b][r];
        }
        __syncthreads();
    }
}

// the whole length-L FFT of the S sequences in LDS (natural order in, caller's barrier done);
// outputs through st(s, k, X_k)
template <int L, int S, bool SF, class Store>
__device__ __forceinline__ void zfft(double2* lds, const double2* __restrict__ twL, Store&& st) {
    auto none = [](int, int, double2) {};
    if constexpr (L == 64) {
        zstage<L, S, 16, 1, false, SF>(lds, twL, none);
        zstage<L, S, 4, 16, true, SF>(lds, twL, st);
    } else if constexpr (L == 128) {
        zstage<L, S, 16, 1, false, SF>(lds, twL, none);
        zstage<L, S, 8, 16, true, SF>(lds, twL, st);
    } else if constexpr (L == 256) {
        zstage<L, S, 16, 1, false, SF>(lds, twL, none);
        zstage<L, S, 16, 16, true, SF>(lds, twL, st);
    } else {
        zstage<L, S, 16, 1, false, SF>(lds, twL, none);
        zstage<L, S, 16, 16, false, SF>(lds, twL, none);
        if constexpr (L == 512) zstage<L, S, 2, 256, true, SF>(lds, twL, st);
        else if constexpr (L == 1024) zstage<L, S, 4, 256, true, SF>(lds, twL, st);
        else if constexpr (L == 2048) zstage<L, S, 8, 256, true, SF>(lds, twL, st);
        else zstage<L, S, 16, 256, true, SF>(lds, twL, st);
    }
}

// K3 in fp64: 10 log10 |X|^2, rounded once (p = 0 -> -inf, as log10f). 10 log10 p = (10 / ln 10) (e ln 2
// + ln c_k + ln(1 + u)) with p = m 2^e, m in [1/2, 1), c_k the centre of m's 1/256-wide interval k (a
// 128-entry fp64 table of ln c_k and 1 / c_k, L1-resident) and u = m / c_k - 1 (one fma, |u| <= 2^-8):
// ln(1 + u) by six terms of its series (remainder below u^7 / 7 ~ 1e-17), so the result carries a few fp64
// ulps (~1e-15 relative), far inside one fp32 ulp of the dB value. Round 6: the table replaces a ten-term
// atanh series behind an fp64 division (the pass-B kernel's largest cost); SDRGPU_F64_LIBLOG: A/B builds.
#ifndef SDRGPU_F64_LIBLOG
#define SDRGPU_F64_LIBLOG 0
#endif
constexpr int kLnTab = 128;
__device__ __forceinline__ float zdb(double2 X, const double2* __restrict__ lnt) {
    const double p = X.x * X.x + X.y * X.y;
#if SDRGPU_F64_LIBLOG
    return (float)(10.0 * log10(p));
#else
    if (!(p > 0.0) || !(p < 1.0e308)) return (float)(10.0 * log10(p));   // (0, inf, nan: the libm path)
    int e;
    const double m = frexp(p, &e);   // [0.5, 1)
    const int k = min((int)((m - 0.5) * 256.0), kLnTab - 1);
    const double2 t = lnt[k];         // (ln c_k, 1 / c_k)
    const double u = fma(m, t.y, -1.0);
    double P = -1.0 / 6.0;
    P = fma(P, u, 1.0 / 5.0);
    P = fma(P, u, -1.0 / 4.0);
    P = fma(P, u, 1.0 / 3.0);
    P = fma(P, u, -1.0 / 2.0);
    const double l1u = fma(u * u, P, u);   // u + u^2 (-1/2 + u / 3 - ...)
    const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double ln = fma((double)e, LN2_HI, fma((double)e, LN2_LO, t.x + l1u));
    return (float)(4.34294481903251827651 * ln);
#endif
}

// K1: the reference's fp32 window product, then exact promotion
__device__ __forceinline__ double2 windowed(float2 x, float w) {
    return make_double2((double)(x.x * w), (double)(x.y * w));
}

// ---- N <= 4096: S frames per workgroup --------------------------------------------------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft64_single_kernel(const float2* __restrict__ in, long long stride, int frames,
                                                                  const float* __restrict__ win, int nz,
                                                                  const double2* __restrict__ twL, float* __restrict__ out,
                                                                  const double2* __restrict__ lnt) {
    extern __shared__ __attribute__((aligned(16))) double2 zlds[];
    constexpr int LS = ZLds<L>::LS, NT = S * L / 16;
    const long long f0 = (long long)blockIdx.x * S;
    for (int e = threadIdx.x; e < S * L; e += NT) {   // frame-contiguous loads
        const int s = e / L, n = e % L;
        const long long f = f0 + s;
        double2 v = make_double2(0.0, 0.0);
        if (f < frames && n < nz) v = windowed(in[f * stride + n], win[n]);
        zlds[s * LS + zpad(n)] = v;
    }
    __syncthreads();
    zfft<L, S, false>(zlds, twL, [&](int s, int k, double2 X) {
        const long long f = f0 + s;
        if (f < frames) out[f * L + k] = zdb(X, lnt);
    });
}

// ---- pass A: S columns of one frame ---------------------------------------------------------------
// frame viewed as N1 x N2 (x[n1 N2 + n2]); column FFT over n1 -> k1; x W_N^(n2 k1) on the store.
// (The output order of zstage's last stage is relied on by the twiddle recurrence below. Round 6, measured: a persistent form with the next tile's loads in flight spilled at two workgroups
// per CU and ran at half the speed of this one-tile kernel, r7i.)
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft64_passA_kernel(const float2* __restrict__ in, long long stride, int frames,
                                                                 const float* __restrict__ win, int nz, int N2, int logN,
                                                                 const double2* __restrict__ twL, const double2* __restrict__ thi,
                                                                 const double2* __restrict__ tlo, double2* __restrict__ scratch) {
    extern __shared__ __attribute__((aligned(16))) double2 zlds[];
    constexpr int LS = ZLds<L>::LS, NT = S * L / 16;
    const int nb = N2 / S;
    const int b = blockIdx.x % nb;
    const long long f = blockIdx.x / nb;
    if (f >= frames) return;
    const float2* x = in + f * stride;
    const int c0 = b * S;
    // column fastest: S x 8-B row segments. Each thread's 16 elements are loaded in one batch (all
    // in flight), then written to LDS: as a loop the loads waited one by one (vmcnt(0) per element;
    // round 6: 82 -> 57 us per 128 64k frames, r7f)
    static_assert(S * L == 16 * NT, "16 elements per thread");
    float2 xv[16];
    float wv[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = threadIdx.x + k * NT;
        const int n = (e / S) * N2 + c0 + e % S;
        const int nc = n < nz ? n : 0;   // (zero padding: an in-bounds load, selected away)
        xv[k] = x[nc];
        wv[k] = win[nc];
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = threadIdx.x + k * NT;
        const int c = e % S, n1 = e / S;
        const int n = n1 * N2 + c0 + c;
        zlds[c * LS + zpad(n1)] = n < nz ? windowed(xv[k], wv[k]) : make_double2(0.0, 0.0);
    }
    __syncthreads();
    const int N = 1 << logN;
    double2* sc = scratch + (f << logN);
    // The last stage (radix R, NS = L / R, BPT = 16 / R butterflies per thread) hands this thread its outputs
    // k1 = t + (L / 16) b + NS r in order b = 0.., r = 0..R-1: W_N^(n2 k1) by an fp64 recurrence from three
    // table products, W_N^(n2 t), W_N^(n2 L / 16) (next b), W_N^(n2 NS) (next r), one fp64 product per output
    // (at most ~20 in a chain: a few fp64 ulps) instead of two dependent table loads (r7g: 57 -> 47 us per
    // 128 64k frames)
    constexpr int RL = L == 64 ? 4 : L == 128 ? 8 : L == 256 ? 16 : L == 512 ? 2 : L == 1024 ? 4 : L == 2048 ? 8 : 16;
    constexpr int NSL = L / RL;
    auto twn = [&](long long e) {
        const int m = (int)(e & (N - 1));   // exact argument mod N
        return zmul(thi[m >> 10], tlo[m & 1023]);
    };
    double2 cb = make_double2(1.0, 0.0), w = cb, sb = cb, sr = cb;
    int idx = 0;
    zfft<L, S, true>(zlds, twL, [&](int c, int k1, double2 X) {
        const int n2 = c0 + c;
        if (idx == 0) {
            cb = twn((long long)n2 * k1);
            sb = twn((long long)n2 * (L / 16));
            sr = twn((long long)n2 * NSL);
            w = cb;
        } else if (idx % RL == 0) {
            cb = zmul(cb, sb);
            w = cb;
        } else {
            w = zmul(w, sr);
        }
        idx++;
        sc[(long long)k1 * N2 + n2] = zmul(X, w);
    });
}

// ---- pass B: S rows k1 of one frame ----------------------------------------------------------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft64_passB_kernel(const double2* __restrict__ scratch, int frames, int N1, int logN,
                                                                 const double2* __restrict__ twL, float* __restrict__ out,
                                                                 const double2* __restrict__ lnt) {
    extern __shared__ __attribute__((aligned(16))) double2 zlds[];
    constexpr int LS = ZLds<L>::LS, NT = S * L / 16;
    const int nb = N1 / S;
    const int b = blockIdx.x % nb;
    const long long f = blockIdx.x / nb;
    if (f >= frames) return;
    const int r0 = b * S;
    const double2* sc = scratch + (f << logN) + (long long)r0 * L;
    static_assert(S * L == 16 * NT, "16 elements per thread");
    double2 rv[16];   // S contiguous rows, each thread's 16 elements loaded in one batch
#pragma unroll
    for (int k = 0; k < 16; k++) rv[k] = sc[threadIdx.x + k * NT];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = threadIdx.x + k * NT;
        zlds[(e / L) * LS + zpad(e % L)] = rv[k];
    }
    __syncthreads();
    float* o = out + (f << logN);
    zfft<L, S, true>(zlds, twL, [&](int s, int k2, double2 X) { o[r0 + s + (long long)N1 * k2] = zdb(X, lnt); });
}

template <typename K>
int zset_lds(K kernel, size_t bytes) {
    SDRGPU_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    return SDRGPU_OK;
}

// columns / rows per workgroup for a length-L transform (LDS: S x LS x 16 B <= 140 KB)
constexpr int zS(int L) { return L <= 256 ? 16 : L <= 1024 ? 8 : L == 2048 ? 2 : 1; }
#ifndef SDRGPU_F64_SA256
#define SDRGPU_F64_SA256 16   // (A/B builds) pass-A columns per workgroup at N1 = 256
#endif
constexpr int zSA(int L) { return L == 256 ? SDRGPU_F64_SA256 : zS(L); }
#ifndef SDRGPU_F64_SB256
#define SDRGPU_F64_SB256 16   // (A/B builds) pass-B rows per workgroup at N2 = 256 (32: 128-B dB segments, 1 workgroup per CU: slower, r7h)
#endif
constexpr int zSB(int L) { return L == 256 ? SDRGPU_F64_SB256 : zS(L); }

template <int L>
int launch_single64(const double2* tw, const float2* in, long long stride, int frames, const float* win, int nz, float* out,
                    const double2* lnt, hipStream_t s) {
    constexpr int S = zS(L);
    auto k = fft64_single_kernel<L, S>;
    const size_t lds = sizeof(double2) * S * ZLds<L>::LS;
    SDRGPU_CHECK(zset_lds(k, lds));
    hipLaunchKernelGGL(k, dim3((frames + S - 1) / S), dim3(S * L / 16), lds, s, in, stride, frames, win, nz, tw, out, lnt);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int L>
int launch_passA64(const double2* tw, const float2* in, long long stride, int frames, const float* win, int nz, int N2, int logN,
                   const double2* thi, const double2* tlo, double2* scratch, hipStream_t s) {
    constexpr int S = zSA(L);
    if (N2 % S) { set_error("fft64: N2 %d not a multiple of %d", N2, S); return SDRGPU_ESTATE; }
    auto k = fft64_passA_kernel<L, S>;
    const size_t lds = sizeof(double2) * S * ZLds<L>::LS;
    SDRGPU_CHECK(zset_lds(k, lds));
    hipLaunchKernelGGL(k, dim3((N2 / S) * frames), dim3(S * L / 16), lds, s, in, stride, frames, win, nz, N2, logN, tw, thi, tlo,
                       scratch);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int L>
int launch_passB64(const double2* tw, const double2* scratch, int frames, int N1, int logN, float* out, const double2* lnt,
                   hipStream_t s) {
    constexpr int S = zSB(L);
    if (N1 % S) { set_error("fft64: N1 %d not a multiple of %d", N1, S); return SDRGPU_ESTATE; }
    auto k = fft64_passB_kernel<L, S>;
    const size_t lds = sizeof(double2) * S * ZLds<L>::LS;
    SDRGPU_CHECK(zset_lds(k, lds));
    hipLaunchKernelGGL(k, dim3((N1 / S) * frames), dim3(S * L / 16), lds, s, scratch, frames, N1, logN, tw, out, lnt);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

// W_L^m = exp(-2 pi i m / L), m < count, fp64 (m * step taken mod L exactly)
int upload_zt(DevBuf& b, long long L, int count, long long step) {
    std::vector<double2> t(count);
    for (int m = 0; m < count; m++) {
        const double a = -2.0 * M_PI * (double)((m * step) % L) / (double)L;
        t[m] = make_double2(std::cos(a), std::sin(a));
    }
    SDRGPU_CHECK(b.ensure(sizeof(double2) * count));
    SDRGPU_HIP(hipMemcpy(b.p, t.data(), sizeof(double2) * count, hipMemcpyHostToDevice));
    return SDRGPU_OK;
}

}  // namespace

struct Fft64Plan {
    int N = 0, logN = 0, N1 = 0, N2 = 0, chunkFrames = 1;
    DevBuf tw1, tw2, thi, tlo, scratch;
    DevBuf lnt;   // zdb's (ln c_k, 1 / c_k), k < kLnTab
};

int fft64_create(Fft64Plan** out, int N) {
    *out = nullptr;
    int logN = 0;
    while ((1 << logN) < N) logN++;
    if (N < 64 || N > (1 << 20) || (1 << logN) != N) { set_error("fft64: size %d", N); return SDRGPU_EARG; }
    auto* p = new Fft64Plan();
    p->N = N;
    p->logN = logN;
    int rc;
    {
        std::vector<double2> t(kLnTab);
        for (int k = 0; k < kLnTab; k++) {
            const double c = 0.5 + (k + 0.5) / 256.0;
            t[k] = make_double2(std::log(c), 1.0 / c);
        }
        rc = p->lnt.ensure(sizeof(double2) * kLnTab);
        if (rc >= 0 && hipMemcpy(p->lnt.p, t.data(), sizeof(double2) * kLnTab, hipMemcpyHostToDevice) != hipSuccess) {
            set_error("fft64: table upload failed");
            rc = SDRGPU_EHIP;
        }
    }
    if (rc < 0) {
    } else if (N <= 4096) {
        rc = upload_zt(p->tw1, N, N, 1);
    } else {
        p->N1 = 1 << ((logN + 1) / 2);
        p->N2 = N / p->N1;
        rc = upload_zt(p->tw1, p->N1, p->N1, 1);
        if (rc >= 0) rc = upload_zt(p->tw2, p->N2, p->N2, 1);
        const int nhi = std::max(1, N >> 10);
        if (rc >= 0) rc = upload_zt(p->thi, N, nhi, 1024);   // W_N^(1024 h)
        if (rc >= 0) rc = upload_zt(p->tlo, N, 1024, 1);     // W_N^l
        p->chunkFrames = std::max(1, (int)((128LL << 20) / ((long long)N * 16)));
    }
    if (rc < 0) {
        delete p;
        return rc;
    }
    *out = p;
    return SDRGPU_OK;
}

void fft64_destroy(Fft64Plan* p) { delete p; }

int fft64_execute(Fft64Plan* p, const float2* in, long long stride, int frames, const float* win, int nz, float* out,
                  hipStream_t s) {
    const double2* lt = p->lnt.as<double2>();
    if (p->N1 == 0) {
        const double2* tw = p->tw1.as<double2>();
        switch (p->N) {
        case 64: SDRGPU_CHECK(launch_single64<64>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        case 128: SDRGPU_CHECK(launch_single64<128>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        case 256: SDRGPU_CHECK(launch_single64<256>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        case 512: SDRGPU_CHECK(launch_single64<512>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        case 1024: SDRGPU_CHECK(launch_single64<1024>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        case 2048: SDRGPU_CHECK(launch_single64<2048>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        case 4096: SDRGPU_CHECK(launch_single64<4096>(tw, in, stride, frames, win, nz, out, lt, s)); return frames;
        }
        set_error("fft64: size %d", p->N);
        return SDRGPU_EARG;
    }
    SDRGPU_CHECK(p->scratch.ensure((size_t)std::min(p->chunkFrames, frames) * p->N * sizeof(double2)));
    double2* sc = p->scratch.as<double2>();
    const double2 *t1 = p->tw1.as<double2>(), *t2 = p->tw2.as<double2>(), *th = p->thi.as<double2>(), *tl = p->tlo.as<double2>();
    for (int f0 = 0; f0 < frames; f0 += p->chunkFrames) {
        const int nf = std::min(p->chunkFrames, frames - f0);
        const float2* x = in + (long long)f0 * stride;
        float* o = out + (long long)f0 * p->N;
        switch (p->N1) {
        case 128: SDRGPU_CHECK(launch_passA64<128>(t1, x, stride, nf, win, nz, p->N2, p->logN, th, tl, sc, s)); break;
        case 256: SDRGPU_CHECK(launch_passA64<256>(t1, x, stride, nf, win, nz, p->N2, p->logN, th, tl, sc, s)); break;
        case 512: SDRGPU_CHECK(launch_passA64<512>(t1, x, stride, nf, win, nz, p->N2, p->logN, th, tl, sc, s)); break;
        case 1024: SDRGPU_CHECK(launch_passA64<1024>(t1, x, stride, nf, win, nz, p->N2, p->logN, th, tl, sc, s)); break;
        default: set_error("fft64: N1 %d", p->N1); return SDRGPU_EARG;
        }
        switch (p->N2) {
        case 64: SDRGPU_CHECK(launch_passB64<64>(t2, sc, nf, p->N1, p->logN, o, lt, s)); break;
        case 128: SDRGPU_CHECK(launch_passB64<128>(t2, sc, nf, p->N1, p->logN, o, lt, s)); break;
        case 256: SDRGPU_CHECK(launch_passB64<256>(t2, sc, nf, p->N1, p->logN, o, lt, s)); break;
        case 512: SDRGPU_CHECK(launch_passB64<512>(t2, sc, nf, p->N1, p->logN, o, lt, s)); break;
        case 1024: SDRGPU_CHECK(launch_passB64<1024>(t2, sc, nf, p->N1, p->logN, o, lt, s)); break;
        default: set_error("fft64: N2 %d", p->N2); return SDRGPU_EARG;
        }
    }
    return frames;
}

}  // namespace sdrgpu
