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
#include "fir_rows.h"   // static_for

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
// + ln m) with p = m 2^e, m in [sqrt(1/2), sqrt(2)); ln m = 2 atanh(s) = 2 s (1 + s^2/3 + ... + s^20/21),
// s = (m - 1) / (m + 1), |s| <= 0.1716, so the series' remainder is below 3e-17 and the result carries
// a few fp64 ulps (~1e-15 relative), far inside one fp32 ulp of the dB value; about half the VALU of
// the device libm's log10, which was the pass-B kernel's largest cost (SDRGPU_F64_LIBLOG: A/B builds)
#ifndef SDRGPU_F64_LIBLOG
#define SDRGPU_F64_LIBLOG 0
#endif
__device__ __forceinline__ float zdb(double2 X) {
    const double p = X.x * X.x + X.y * X.y;
#if SDRGPU_F64_LIBLOG
    return (float)(10.0 * log10(p));
#else
    if (!(p > 0.0) || !(p < 1.0e308)) return (float)(10.0 * log10(p));   // (0, inf, nan: the libm path)
    int e;
    double m = frexp(p, &e);   // [0.5, 1)
    if (m < 0.70710678118654752440) {
        m *= 2.0;
        e -= 1;
    }
    const double s = (m - 1.0) / (m + 1.0), t = s * s;
    double P = 1.0 / 21.0;
    P = fma(P, t, 1.0 / 19.0);
    P = fma(P, t, 1.0 / 17.0);
    P = fma(P, t, 1.0 / 15.0);
    P = fma(P, t, 1.0 / 13.0);
    P = fma(P, t, 1.0 / 11.0);
    P = fma(P, t, 1.0 / 9.0);
    P = fma(P, t, 1.0 / 7.0);
    P = fma(P, t, 1.0 / 5.0);
    P = fma(P, t, 1.0 / 3.0);
    const double lnm = 2.0 * s + (2.0 * s * t) * P;   // 2 s (1 + t P)
    const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double ln = fma((double)e, LN2_HI, fma((double)e, LN2_LO, lnm));
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
                                                                  const double2* __restrict__ twL, float* __restrict__ out) {
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
        if (f < frames) out[f * L + k] = zdb(X);
    });
}

// ---- pass A: S columns of one frame ---------------------------------------------------------------
// frame viewed as N1 x N2 (x[n1 N2 + n2]); column FFT over n1 -> k1; x W_N^(n2 k1) on the store
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
    for (int e = threadIdx.x; e < S * L; e += NT) {   // column fastest: S x 8-B row segments
        const int c = e % S, n1 = e / S;
        const int n = n1 * N2 + c0 + c;
        double2 v = make_double2(0.0, 0.0);
        if (n < nz) v = windowed(x[n], win[n]);
        zlds[c * LS + zpad(n1)] = v;
    }
    __syncthreads();
    const int N = 1 << logN;
    double2* sc = scratch + (f << logN);
    zfft<L, S, true>(zlds, twL, [&](int c, int k1, double2 X) {
        const int n2 = c0 + c;
        const int m = (int)(((long long)n2 * k1) & (N - 1));   // W_N^(n2 k1), exact argument mod N
        sc[(long long)k1 * N2 + n2] = zmul(X, zmul(thi[m >> 10], tlo[m & 1023]));
    });
}

// ---- pass B: S rows k1 of one frame ----------------------------------------------------------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft64_passB_kernel(const double2* __restrict__ scratch, int frames, int N1, int logN,
                                                                 const double2* __restrict__ twL, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double2 zlds[];
    constexpr int LS = ZLds<L>::LS, NT = S * L / 16;
    const int nb = N1 / S;
    const int b = blockIdx.x % nb;
    const long long f = blockIdx.x / nb;
    if (f >= frames) return;
    const int r0 = b * S;
    const double2* sc = scratch + (f << logN) + (long long)r0 * L;
    for (int e = threadIdx.x; e < S * L; e += NT) zlds[(e / L) * LS + zpad(e % L)] = sc[e];   // S contiguous rows
    __syncthreads();
    float* o = out + (f << logN);
    zfft<L, S, true>(zlds, twL, [&](int s, int k2, double2 X) { o[r0 + s + (long long)N1 * k2] = zdb(X); });
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

template <int L>
int launch_single64(const double2* tw, const float2* in, long long stride, int frames, const float* win, int nz, float* out,
                    hipStream_t s) {
    constexpr int S = zS(L);
    auto k = fft64_single_kernel<L, S>;
    const size_t lds = sizeof(double2) * S * ZLds<L>::LS;
    SDRGPU_CHECK(zset_lds(k, lds));
    hipLaunchKernelGGL(k, dim3((frames + S - 1) / S), dim3(S * L / 16), lds, s, in, stride, frames, win, nz, tw, out);
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
int launch_passB64(const double2* tw, const double2* scratch, int frames, int N1, int logN, float* out, hipStream_t s) {
    constexpr int S = zS(L);
    if (N1 % S) { set_error("fft64: N1 %d not a multiple of %d", N1, S); return SDRGPU_ESTATE; }
    auto k = fft64_passB_kernel<L, S>;
    const size_t lds = sizeof(double2) * S * ZLds<L>::LS;
    SDRGPU_CHECK(zset_lds(k, lds));
    hipLaunchKernelGGL(k, dim3((N1 / S) * frames), dim3(S * L / 16), lds, s, scratch, frames, N1, logN, tw, out);
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

// ---- N = 65536 in one pass (round 6) ---------------------------------------------------------------
// No double2 intermediate: one radix-8 decimation-in-frequency step splits the frame into eight 8,192-
// point transforms, X[8 m + r] = sum_{n < M} W_M^(n m) y_r[n], y_r[n] = W_N^(n r) sum_{j < 8} W_8^(j r)
// v[n + M j], M = 8192, v = the fp32 window product promoted exactly. An 8k fp64 image (128 KB) fits the
// LDS. Workgroup (f, p) computes r0 = 2 p and r0 + 1, so a frame's four workgroups (one XCD) each read the
// frame (its first reader from HBM, the others mostly from that XCD's L2) and the dB rows of the pair
// leave as 8-byte bin pairs. The 8k transform is M = 16 x 32 x 16 (cf. fft.hip's fft_1p_kernel):
//   stage 1 (registers): thread t holds y_r[t + 512 i], i < 16; W_128^(r i), a radix-16 DFT over i, and
//     W_N^(t (8 k2 + r)) (fp64 recurrence from table values) give A[t][k2];
//   stage 2 (LDS): per (k2, t0), t = t0 + 32 t1: radix 16 over t1 -> q1, twiddle W_512^(t0 q1);
//   stage 3 (LDS): per (k2, q1): radix 32 over t0 -> q2 on a lane pair (each lane a radix 16 of its
//     parity, one DPP swap): Y[k2 + 16 q1 + 256 q2], dB, store.
// Whole aligned frames stream into LDS by LDS-DMA through 3 ring slots of one row set (samples
// [512 i, 512 i + 512) of the eight eighths: x 8 x 4 KiB, w 8 x 2 KiB; 48 pieces, 6 per wave); other
// frames (zero padding, odd strides) through range-checked register loads.
namespace z1p {
constexpr int M = 8192;
constexpr int RS = 513;                    // stage-1 image [k2][t] row stride (double2)
constexpr int SLOT = 49152;                // ring slot (bytes)
constexpr int NSLOT = 3;
constexpr int IMG = NSLOT * SLOT;          // bytes (>= 16 x 513 x 16, 8192 x 16)
constexpr int TW = IMG;                    // bytes: W_512^(t0 q1) at [q1][t0], q1 < 16, t0 < 32
constexpr int W128 = TW + 512 * 16;        // bytes: W_128^(r i) at [h][i], r = r0 + h, i < 16
constexpr int LDS_BYTES = W128 + 32 * 16;
constexpr int TAB = 4096 + 512 + 128;      // device table: W_N^m (m < 4096), [q1][t0] W_512^(t0 q1), [r][i] W_128^(r i)
static_assert(16 * RS * 16 <= IMG && M * 16 <= IMG && LDS_BYTES <= 160 * 1024, "z1p LDS");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t zrsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// the double of the partner lane (lane ^ 1), as two DPP moves (quad_perm [1,0,3,2])
__device__ __forceinline__ double zswap1(double v) {
    const long long u = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp((int)u, (int)u, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(u >> 32), (int)(u >> 32), 0xB1, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// radix 32 on a lane pair: in a[m] = x[2 m + e], out a[k] = X[k + 16 e]
__device__ __forceinline__ void zpair_dft32(double2 (&a)[16], int e) {
    zdft<16>(a);
    const double sg = e ? -1.0 : 1.0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
        const double c = cos(-2.0 * M_PI * k / 32.0), sn = sin(-2.0 * M_PI * k / 32.0);   // (constant-folded)
        a[k] = zmul(a[k], make_double2(e ? c : 1.0, e ? sn : 0.0));
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const double px = zswap1(a[k].x), py = zswap1(a[k].y);
        a[k] = make_double2(fma(sg, a[k].x, px), fma(sg, a[k].y, py));
    }
}

template <bool PAD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1))) void fft64_1p_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz,
    const double2* __restrict__ tab, float* __restrict__ out) {
    using z1p::M;
    using z1p::RS;
    extern __shared__ __attribute__((aligned(16))) double2 zlds[];
    const int b = blockIdx.x, k = b >> 3;
    const int f = 8 * (k >> 2) + (b & 7), p = k & 3, r0 = 2 * p;   // transforms r0, r0 + 1 of frame f
    if (f >= frames) return;
    auto tid = [] {
        int u = threadIdx.x;
        asm volatile("" : "+v"(u));
        return u;
    };
    char* const lb = reinterpret_cast<char*>(zlds);
    {
        const int t = threadIdx.x;
        reinterpret_cast<double2*>(lb + z1p::TW)[t] = tab[4096 + t];
        if (t < 32) reinterpret_cast<double2*>(lb + z1p::W128)[t] = tab[4096 + 512 + 16 * (r0 + (t >> 4)) + (t & 15)];
    }
    // y_r0, y_r0+1 from the eight eighths: Y_r = E_r + W_8^r O_r, E / O the 4-point DFTs of the even /
    // odd eighths at r mod 4 (r0 mod 4 in {0, 2}, r0 + 1 mod 4 in {1, 3}: signs sg0, sg1)
    const double sg0 = (p & 1) ? -1.0 : 1.0, sg1 = (p & 1) ? 1.0 : -1.0;
    const double R2 = 0.70710678118654752440;
    const double2 w80 = p == 0 ? make_double2(1.0, 0.0) : p == 1 ? make_double2(0.0, -1.0) : p == 2 ? make_double2(-1.0, 0.0)
                                                                                                   : make_double2(0.0, 1.0);
    const double2 w81 = p == 0 ? make_double2(R2, -R2) : p == 1 ? make_double2(-R2, -R2) : p == 2 ? make_double2(-R2, R2)
                                                                                                 : make_double2(R2, R2);
    auto combine = [&](const double2 (&v)[8], double2& ya, double2& yb) {
        const double2 a0 = zadd(v[0], v[4]), b0 = zsub(v[0], v[4]), c0 = zadd(v[2], v[6]), d0 = zsub(v[2], v[6]);
        const double2 a1 = zadd(v[1], v[5]), b1 = zsub(v[1], v[5]), c1 = zadd(v[3], v[7]), d1 = zsub(v[3], v[7]);
        const double2 E0 = make_double2(fma(sg0, c0.x, a0.x), fma(sg0, c0.y, a0.y));
        const double2 O0 = make_double2(fma(sg0, c1.x, a1.x), fma(sg0, c1.y, a1.y));
        const double2 E1 = make_double2(fma(-sg1, d0.y, b0.x), fma(sg1, d0.x, b0.y));   // b -+ i d
        const double2 O1 = make_double2(fma(-sg1, d1.y, b1.x), fma(sg1, d1.x, b1.y));
        ya = zadd(E0, zmul(O0, w80));
        yb = zadd(E1, zmul(O1, w81));
    };
    double2 za[16], zb[16];
    if constexpr (PAD) {
        const __amdgpu_buffer_rsrc_t rw = zrsrc(win, (unsigned)nz * 4u);
        const __amdgpu_buffer_rsrc_t rx = zrsrc(in + (long long)f * frameStride, (unsigned)nz * 8u);
        float2 xv[2][8];
        float wv[2][8];
        auto issue = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const int t = tid();
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int n = t + 512 * i + M * j;
                xv[i & 1][j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, n * 8, 0, 0));
                wv[i & 1][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, n * 4, 0, 0));
            }
        };
        issue(std::integral_constant<int, 0>{});
        issue(std::integral_constant<int, 1>{});
        static_for<0, 16>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            double2 v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = windowed(xv[i & 1][j], wv[i & 1][j]);
            if constexpr (i + 2 < 16) issue(std::integral_constant<int, i + 2>{});
            combine(v, za[i], zb[i]);
        });
    } else {
        constexpr int S = z1p::NSLOT, SLOT = z1p::SLOT;
        typedef __attribute__((address_space(3))) char lchar;
        const unsigned ldsBase = (unsigned)(size_t)(lchar*)zlds;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const char* gb[6];
        unsigned rstep[6], loff[6];
        const float2* xf = in + (long long)f * frameStride;
#pragma unroll
        for (int e = 0; e < 6; e++) {
            const int m = 6 * wave + e;
            const int jx = m >> 2, cx = m & 3, jw = (m - 32) >> 1, cw = (m - 32) & 1;
            gb[e] = m < 32 ? reinterpret_cast<const char*>(xf + M * jx + 128 * cx)
                           : reinterpret_cast<const char*>(win + M * jw + 256 * cw);
            rstep[e] = m < 32 ? 512u * 8u : 512u * 4u;
            loff[e] = m < 32 ? (unsigned)(4096 * jx + 1024 * cx) : (unsigned)(32768 + 2048 * jw + 1024 * cw);
        }
        auto dma = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const unsigned lane16 = (unsigned)(tid() & 63) * 16u;
#pragma unroll
            for (int e = 0; e < 6; e++) {
                const char* src = gb[e] + lane16;
                gb[e] += rstep[e];
                asm volatile("" : "+s"(gb[e]));
                const unsigned dst = __builtin_amdgcn_readfirstlane(ldsBase + (unsigned)((i % S) * SLOT) + loff[e]);
                unsigned keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
            }
        };
        static_for<0, S - 1>(dma);
        static_for<0, 16>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int younger = (S - 2 < 15 - i) ? S - 2 : 15 - i;   // row sets issued after i, in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * younger) : "memory");
            __builtin_amdgcn_s_barrier();   // every wave's pieces landed; every read of slot i - 1 done
            asm volatile("" ::: "memory");
            if constexpr (i + S - 1 < 16) dma(std::integral_constant<int, i + S - 1>{});
            const int t = tid();
            const char* slot = lb + (i % S) * SLOT;
            double2 v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float2 xx = *reinterpret_cast<const float2*>(slot + 4096 * j + 8 * t);
                const float ww = *reinterpret_cast<const float*>(slot + 32768 + 2048 * j + 4 * t);
                v[j] = windowed(xx, ww);
            }
            combine(v, za[i], zb[i]);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    const __amdgpu_buffer_rsrc_t ro = zrsrc(out + ((long long)f << 16), 65536u * 4u);
    float dA[16];   // transform r0's dB values, paired with r0 + 1's in 8-byte stores
    auto transform = [&](auto hc, double2 (&z)[16]) {
        constexpr int h = decltype(hc)::value;
        const int r = r0 + h;
        __syncthreads();   // (h = 0: the tables staged, the ring's reads done; h = 1: r0's stage-3 reads done)
        {   // stage-1 finish
            const int t = tid();
            const double2* w128 = reinterpret_cast<const double2*>(lb + z1p::W128) + 16 * h;
#pragma unroll
            for (int i = 1; i < 16; i++) z[i] = zmul(z[i], w128[i]);
            zdft<16>(z);
            const double2 st = tab[8 * t];
            double2 ce = tab[t * r], co = zmul(ce, st);
            const double2 st2 = zmul(st, st);
            double2* col = zlds + t;
#pragma unroll
            for (int k2 = 0; k2 < 16; k2 += 2) {
                col[k2 * RS] = zmul(z[k2], ce);
                col[(k2 + 1) * RS] = zmul(z[k2 + 1], co);
                if (k2 < 14) {
                    ce = zmul(ce, st2);
                    co = zmul(co, st2);
                }
            }
        }
        __syncthreads();
        {   // stage 2: item (k2, t0) = (u & 15, u >> 4)
            const int u = tid();
            const int k2 = u & 15, t0 = u >> 4;
            double2 a[16];
            const double2* src = zlds + k2 * RS + t0;
#pragma unroll
            for (int t1 = 0; t1 < 16; t1++) a[t1] = src[32 * t1];
            zdft<16>(a);
            const double2* tw = reinterpret_cast<const double2*>(lb + z1p::TW) + t0;
#pragma unroll
            for (int q1 = 1; q1 < 16; q1++) a[q1] = zmul(a[q1], tw[32 * q1]);
            __syncthreads();
            double2* dst = zlds + t0 * 16 + k2;
#pragma unroll
            for (int q1 = 0; q1 < 16; q1++) dst[q1 * 32 * 16] = a[q1];
        }
        __syncthreads();
        {   // stage 3: item (k2, q1), lane pair e: outputs q2 = kk + 16 e
            const int u = tid();
            const int e = u & 1, k2 = (u >> 1) & 15, q1 = u >> 5;
            double2 c[16];
            const double2* src = zlds + (q1 * 32 + e) * 16 + k2;
#pragma unroll
            for (int m = 0; m < 16; m++) c[m] = src[32 * m];
            zpair_dft32(c, e);
            if constexpr (h == 0) {
#pragma unroll
                for (int kk = 0; kk < 16; kk++) dA[kk] = zdb(c[kk]);
            } else {
                const unsigned vo = (unsigned)(8 * (k2 + 16 * q1 + 4096 * e) + r0) * 4u;
#pragma unroll
                for (int kk = 0; kk < 16; kk++) {
                    const float dv = zdb(c[kk]);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned,
                                                                             make_float2(dA[kk], dv)),
                                                          ro, vo, kk * 8192, 0);
                }
            }
        }
    };
    transform(std::integral_constant<int, 0>{}, za);
    transform(std::integral_constant<int, 1>{}, zb);
}

}  // namespace

struct Fft64Plan {
    int N = 0, logN = 0, N1 = 0, N2 = 0, chunkFrames = 1;
    DevBuf tw1, tw2, thi, tlo, scratch;
    DevBuf tab1p;   // N = 65536: fft64_1p_kernel's table (z1p::TAB)
    int onepass = 1;   // N = 65536: the one-pass kernel (SDRGPU_F64_1P=0: the two passes, A/B)
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
    if (N <= 4096) {
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
        if (rc >= 0 && N == 65536) {
            std::vector<double2> t(z1p::TAB);
            auto w = [&](long long m) {
                const double a = -2.0 * M_PI * (double)(m % N) / (double)N;
                return make_double2(std::cos(a), std::sin(a));
            };
            for (int m = 0; m < 4096; m++) t[m] = w(m);
            for (int q1 = 0; q1 < 16; q1++)
                for (int t0 = 0; t0 < 32; t0++) t[4096 + 32 * q1 + t0] = w(128LL * t0 * q1);   // W_512^(t0 q1)
            for (int r = 0; r < 8; r++)
                for (int i = 0; i < 16; i++) t[4096 + 512 + 16 * r + i] = w(512LL * r * i);     // W_128^(r i)
            rc = p->tab1p.ensure(sizeof(double2) * t.size());
            if (rc >= 0 && hipMemcpy(p->tab1p.p, t.data(), sizeof(double2) * t.size(), hipMemcpyHostToDevice) != hipSuccess) {
                set_error("fft64: table upload failed");
                rc = SDRGPU_EHIP;
            }
            if (const char* e = tuning_env("SDRGPU_F64_1P")) p->onepass = atoi(e);
        }
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
    if (p->N1 == 0) {
        const double2* tw = p->tw1.as<double2>();
        switch (p->N) {
        case 64: SDRGPU_CHECK(launch_single64<64>(tw, in, stride, frames, win, nz, out, s)); return frames;
        case 128: SDRGPU_CHECK(launch_single64<128>(tw, in, stride, frames, win, nz, out, s)); return frames;
        case 256: SDRGPU_CHECK(launch_single64<256>(tw, in, stride, frames, win, nz, out, s)); return frames;
        case 512: SDRGPU_CHECK(launch_single64<512>(tw, in, stride, frames, win, nz, out, s)); return frames;
        case 1024: SDRGPU_CHECK(launch_single64<1024>(tw, in, stride, frames, win, nz, out, s)); return frames;
        case 2048: SDRGPU_CHECK(launch_single64<2048>(tw, in, stride, frames, win, nz, out, s)); return frames;
        case 4096: SDRGPU_CHECK(launch_single64<4096>(tw, in, stride, frames, win, nz, out, s)); return frames;
        }
        set_error("fft64: size %d", p->N);
        return SDRGPU_EARG;
    }
    if (p->N == 65536 && p->onepass && p->tab1p.p) {
        const bool pad = nz < 65536 || (stride & 1) || ((uintptr_t)in & 15);
        auto k = pad ? fft64_1p_kernel<true> : fft64_1p_kernel<false>;
        SDRGPU_CHECK(zset_lds(k, z1p::LDS_BYTES));
        hipLaunchKernelGGL(k, dim3(32 * ((frames + 7) / 8)), dim3(512), z1p::LDS_BYTES, s, in, stride, frames, win, nz,
                           p->tab1p.as<double2>(), out);
        SDRGPU_HIP(hipGetLastError());
        return frames;
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
        case 64: SDRGPU_CHECK(launch_passB64<64>(t2, sc, nf, p->N1, p->logN, o, s)); break;
        case 128: SDRGPU_CHECK(launch_passB64<128>(t2, sc, nf, p->N1, p->logN, o, s)); break;
        case 256: SDRGPU_CHECK(launch_passB64<256>(t2, sc, nf, p->N1, p->logN, o, s)); break;
        case 512: SDRGPU_CHECK(launch_passB64<512>(t2, sc, nf, p->N1, p->logN, o, s)); break;
        case 1024: SDRGPU_CHECK(launch_passB64<1024>(t2, sc, nf, p->N1, p->logN, o, s)); break;
        default: set_error("fft64: N2 %d", p->N2); return SDRGPU_EARG;
        }
    }
    return frames;
}

}  // namespace sdrgpu
