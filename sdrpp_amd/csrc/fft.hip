// Spectrum hot path: window * FFT(N) * 10*log10(|X|^2), replacing
// IQFrontEnd::handler (signal_path/iq_frontend.cpp:230-249): K1 volk window
// multiply, K2 fftwf_execute (forward, unnormalised), K3 power spectrum.
//
// CDNA4 design (DESIGN.md "Spectrum kernels"):
//  * N <= 4096: one pass, S frames per workgroup entirely in LDS.
//  * N  > 4096: four-step N = N1 x N2 (N1, N2 <= 1024). Pass A = N2 column FFTs of
//    length N1 (window + zero-pad fused into the load, W_N^(n2 k1) twiddle fused into
//    the store); pass B = N1 row FFTs of length N2 with |X|^2 -> dB fused into a
//    transposing store. The intermediate is streamed in frame chunks sized to stay
//    resident in the 256 MB Infinity Cache between the passes.
//  * In-LDS FFT: Stockham autosort, radix-16 butterflies in registers (radix 2/4/8
//    for the last stage), one pad element per 16 so strided writes avoid bank
//    conflicts, twiddles from an fp64-generated table.
#include <cmath>
#include <cstring>
#include <algorithm>
#include "sdrgpu_internal.h"

namespace sdrgpu {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }   // a * (-i)

// ---- small forward DFTs in registers (e^{-i}) ------------------------------
__device__ __forceinline__ void dft2(float2* v) {
    float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}
__device__ __forceinline__ void dft4(float2& x0, float2& x1, float2& x2, float2& x3) {
    float2 a0 = cadd(x0, x2), a1 = csub(x0, x2), a2 = cadd(x1, x3), a3 = mul_negi(csub(x1, x3));
    x0 = cadd(a0, a2);
    x2 = csub(a0, a2);
    x1 = cadd(a1, a3);
    x3 = csub(a1, a3);
}
__device__ __forceinline__ void dft4v(float2* v) { dft4(v[0], v[1], v[2], v[3]); }

__device__ __forceinline__ void dft8(float2* v) {
    const float R2 = 0.70710678118654752440f;
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    o1 = make_float2(R2 * (o1.x + o1.y), R2 * (o1.y - o1.x));   // * W8^1 = (1-i)/sqrt2
    o2 = mul_negi(o2);                                           // * W8^2 = -i
    o3 = make_float2(R2 * (o3.y - o3.x), -R2 * (o3.x + o3.y));   // * W8^3 = (-1-i)/sqrt2
    v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
    v[1] = cadd(e1, o1); v[5] = csub(e1, o1);
    v[2] = cadd(e2, o2); v[6] = csub(e2, o2);
    v[3] = cadd(e3, o3); v[7] = csub(e3, o3);
}

// 16-point DFT as 4 x 4: X[k1 + 4 k2] = sum_n2 W4^(n2 k2) W16^(n2 k1) DFT4_n1(x[4 n1 + n2])
__device__ __forceinline__ void dft16(float2* v) {
    const float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
    float2 y[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) {
        y[n2][0] = v[n2]; y[n2][1] = v[4 + n2]; y[n2][2] = v[8 + n2]; y[n2][3] = v[12 + n2];
        dft4(y[n2][0], y[n2][1], y[n2][2], y[n2][3]);
    }
    // twiddles W16^(n2 k1) = exp(-2 pi i n2 k1 / 16)
    y[1][1] = cmul(y[1][1], make_float2(C1, -S1));
    y[1][2] = cmul(y[1][2], make_float2(R2, -R2));
    y[1][3] = cmul(y[1][3], make_float2(S1, -C1));
    y[2][1] = cmul(y[2][1], make_float2(R2, -R2));
    y[2][2] = mul_negi(y[2][2]);
    y[2][3] = cmul(y[2][3], make_float2(-R2, -R2));
    y[3][1] = cmul(y[3][1], make_float2(S1, -C1));
    y[3][2] = cmul(y[3][2], make_float2(-R2, -R2));
    y[3][3] = cmul(y[3][3], make_float2(-C1, S1));
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        float2 a = y[0][k1], b = y[1][k1], c = y[2][k1], d = y[3][k1];
        dft4(a, b, c, d);
        v[k1] = a; v[k1 + 4] = b; v[k1 + 8] = c; v[k1 + 12] = d;
    }
}

template <int R> __device__ __forceinline__ void dft(float2* v);
template <> __device__ __forceinline__ void dft<2>(float2* v) { dft2(v); }
template <> __device__ __forceinline__ void dft<4>(float2* v) { dft4v(v); }
template <> __device__ __forceinline__ void dft<8>(float2* v) { dft8(v); }
template <> __device__ __forceinline__ void dft<16>(float2* v) { dft16(v); }

__device__ __forceinline__ int pad16(int i) { return i + (i >> 4); }
template <int L> struct Lds { static constexpr int LS = L + L / 16 + 1; };   // sequence stride (odd)

// One Stockham radix-R stage over S sequences of length L held in LDS.
// Thread (s, t) owns butterflies j = t + b*T, T = L/16, b < 16/R.
template <int L, int S, int R, int NS>
__device__ __forceinline__ void stockham_stage(float2* lds, const float2* __restrict__ tw, int tid) {
    constexpr int T = L / 16;
    constexpr int BPT = 16 / R;
    constexpr int LS = Lds<L>::LS;
    const int s = tid / T, t = tid % T;
    float2* seq = lds + s * LS;
    float2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T;
#pragma unroll
        for (int r = 0; r < R; r++) v[b][r] = seq[pad16(j + r * (L / R))];
        if (NS > 1) {
            const int jm = j % NS;
#pragma unroll
            for (int r = 1; r < R; r++) v[b][r] = cmul(v[b][r], tw[r * jm * (L / (NS * R))]);
        }
        dft<R>(v[b]);
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T;
        const int idxD = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; r++) seq[pad16(idxD + r * NS)] = v[b][r];
    }
    __syncthreads();
}

// Full in-LDS FFT of S sequences of length L (L = 16^a * r).
template <int L, int S>
__device__ __forceinline__ void fft_lds(float2* lds, const float2* __restrict__ tw, int tid) {
    static_assert(L >= 64 && L <= 4096, "fft length");
    if constexpr (L == 64) {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 4, 16>(lds, tw, tid);
    } else if constexpr (L == 128) {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 8, 16>(lds, tw, tid);
    } else if constexpr (L == 256) {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 16, 16>(lds, tw, tid);
    } else if constexpr (L == 512) {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 16, 16>(lds, tw, tid);
        stockham_stage<L, S, 2, 256>(lds, tw, tid);
    } else if constexpr (L == 1024) {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 16, 16>(lds, tw, tid);
        stockham_stage<L, S, 4, 256>(lds, tw, tid);
    } else if constexpr (L == 2048) {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 16, 16>(lds, tw, tid);
        stockham_stage<L, S, 8, 256>(lds, tw, tid);
    } else {
        stockham_stage<L, S, 16, 1>(lds, tw, tid); stockham_stage<L, S, 16, 16>(lds, tw, tid);
        stockham_stage<L, S, 16, 256>(lds, tw, tid);
    }
}

__device__ __forceinline__ float db_of(float2 X) {
    // volk_32fc_s32f_power_spectrum_32f(out, X, 1.0, N): 10*log10(re^2 + im^2)
    return 10.0f * log10f(X.x * X.x + X.y * X.y);
}

// ---- single pass (N <= 4096): S frames per workgroup -------------------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft_single_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz,
    const float2* __restrict__ tw, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int NT = S * L / 16;
    constexpr int LS = Lds<L>::LS;
    const int tid = threadIdx.x;
    const int f0 = blockIdx.x * S;
    for (int e = tid; e < S * L; e += NT) {
        const int s = e / L, n = e % L;
        const int f = f0 + s;
        float2 v = make_float2(0.f, 0.f);
        if (f < frames && n < nz) {
            const float2 x = in[(long long)f * frameStride + n];
            const float w = win[n];
            v = make_float2(x.x * w, x.y * w);
        }
        lds[s * LS + pad16(n)] = v;
    }
    __syncthreads();
    fft_lds<L, S>(lds, tw, tid);
    for (int e = tid; e < S * L; e += NT) {
        const int s = e / L, k = e % L;
        const int f = f0 + s;
        if (f < frames) out[(long long)f * L + k] = db_of(lds[s * LS + pad16(k)]);
    }
}

// ---- pass A: S columns x N1 rows per workgroup ---------------------------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft_passA_kernel(
    const float2* __restrict__ in, long long frameStride, const float* __restrict__ win, int nz, int N2, int logN,
    const float2* __restrict__ tw, float2* __restrict__ scratch) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int NT = S * L / 16;
    constexpr int LS = Lds<L>::LS;
    const int tid = threadIdx.x;
    const int c0 = blockIdx.x * S;
    const long long f = blockIdx.y;
    const float2* x = in + f * frameStride;
    for (int e = tid; e < S * L; e += NT) {
        const int c = e % S, n1 = e / S;
        const int n = n1 * N2 + c0 + c;
        float2 v = make_float2(0.f, 0.f);
        if (n < nz) {
            const float2 xv = x[n];
            const float w = win[n];
            v = make_float2(xv.x * w, xv.y * w);
        }
        lds[c * LS + pad16(n1)] = v;
    }
    __syncthreads();
    fft_lds<L, S>(lds, tw, tid);
    const long long N = 1LL << logN;
    float2* dst = scratch + f * N;
    const float inv = 2.0f / (float)N;
    for (int e = tid; e < S * L; e += NT) {
        const int c = e % S, k1 = e / S;
        const int n2 = c0 + c;
        const int m = n2 * k1;                  // < N: exact twiddle index
        float sn, cs;
        sincospif(-(float)m * inv, &sn, &cs);   // W_N^(n2 k1)
        dst[(long long)k1 * N2 + n2] = cmul(lds[c * LS + pad16(k1)], make_float2(cs, sn));
    }
}

// ---- pass B: S rows of length N2 per workgroup, dB out, transposed store ------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft_passB_kernel(
    const float2* __restrict__ scratch, int N1, int logN, const float2* __restrict__ tw, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int NT = S * L / 16;
    constexpr int LS = Lds<L>::LS;
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * S;
    const long long f = blockIdx.y;
    const long long N = 1LL << logN;
    const float2* src = scratch + f * N + (long long)r0 * L;
    for (int e = tid; e < S * L; e += NT) {
        const int kk = e / L, n2 = e % L;
        lds[kk * LS + pad16(n2)] = src[e];
    }
    __syncthreads();
    fft_lds<L, S>(lds, tw, tid);
    float* dst = out + f * N;
    for (int e = tid; e < S * L; e += NT) {
        const int kk = e % S, k2 = e / S;
        dst[(long long)(r0 + kk) + (long long)N1 * k2] = db_of(lds[kk * LS + pad16(k2)]);
    }
}

// ---------------------------------------------------------------- host side
struct FftPlan {
    int device = 0, N = 0, logN = 0, nz = 0;
    int N1 = 0, N2 = 0;               // two-pass split (N1 * N2 = N); N1 = 0 -> single pass
    DevBuf win, tw1, tw2, scratch;
    int chunkFrames = 1;
    hipStream_t own = nullptr;
    PinnedBuf pin_in, pin_out;
    DevBuf dev_in, dev_out;
};

static int make_twiddles(DevBuf& b, int L) {
    std::vector<float2> t(L);
    for (int m = 0; m < L; m++) {
        double a = -2.0 * M_PI * (double)m / (double)L;
        t[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    SDRGPU_CHECK(b.ensure(sizeof(float2) * L));
    SDRGPU_HIP(hipMemcpy(b.p, t.data(), sizeof(float2) * L, hipMemcpyHostToDevice));
    return SDRGPU_OK;
}

template <typename K>
static int set_lds(K kernel, size_t bytes) {
    SDRGPU_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    return SDRGPU_OK;
}

template <int L, int S>
static int launch_single(const FftPlan& p, const float2* in, long long stride, int frames, float* out, hipStream_t s) {
    auto k = fft_single_kernel<L, S>;
    size_t lds = sizeof(float2) * S * Lds<L>::LS;
    SDRGPU_CHECK(set_lds(k, lds));
    dim3 grid((frames + S - 1) / S);
    hipLaunchKernelGGL(k, grid, dim3(S * L / 16), lds, s, in, stride, frames, p.win.as<float>(), p.nz,
                       p.tw1.as<float2>(), out);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int L, int S>
static int launch_passA(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    auto k = fft_passA_kernel<L, S>;
    size_t lds = sizeof(float2) * S * Lds<L>::LS;
    SDRGPU_CHECK(set_lds(k, lds));
    dim3 grid(p.N2 / S, frames);
    hipLaunchKernelGGL(k, grid, dim3(S * L / 16), lds, s, in, stride, p.win.as<float>(), p.nz, p.N2, p.logN,
                       p.tw1.as<float2>(), p.scratch.as<float2>());
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int L, int S>
static int launch_passB(const FftPlan& p, int frames, float* out, hipStream_t s) {
    auto k = fft_passB_kernel<L, S>;
    size_t lds = sizeof(float2) * S * Lds<L>::LS;
    SDRGPU_CHECK(set_lds(k, lds));
    dim3 grid(p.N1 / S, frames);
    hipLaunchKernelGGL(k, grid, dim3(S * L / 16), lds, s, p.scratch.as<float2>(), p.N1, p.logN,
                       p.tw2.as<float2>(), out);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

static int dispatch_single(const FftPlan& p, const float2* in, long long stride, int frames, float* out, hipStream_t s) {
    switch (p.N) {
    case 64: return launch_single<64, 16>(p, in, stride, frames, out, s);
    case 128: return launch_single<128, 16>(p, in, stride, frames, out, s);
    case 256: return launch_single<256, 16>(p, in, stride, frames, out, s);
    case 512: return launch_single<512, 8>(p, in, stride, frames, out, s);
    case 1024: return launch_single<1024, 4>(p, in, stride, frames, out, s);
    case 2048: return launch_single<2048, 2>(p, in, stride, frames, out, s);
    case 4096: return launch_single<4096, 1>(p, in, stride, frames, out, s);
    }
    set_error("fft: unsupported size %d", p.N);
    return SDRGPU_EARG;
}

// pass-A column FFT length N1 with 16 columns per workgroup (128-B row segments)
static int dispatch_passA(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    switch (p.N1) {
    case 64: return launch_passA<64, 16>(p, in, stride, frames, s);
    case 128: return launch_passA<128, 16>(p, in, stride, frames, s);
    case 256: return launch_passA<256, 16>(p, in, stride, frames, s);
    case 512: return launch_passA<512, 16>(p, in, stride, frames, s);
    case 1024: return launch_passA<1024, 16>(p, in, stride, frames, s);
    }
    set_error("fft: unsupported N1 %d", p.N1);
    return SDRGPU_EARG;
}

static int dispatch_passB(const FftPlan& p, int frames, float* out, hipStream_t s) {
    switch (p.N2) {
    case 64: return launch_passB<64, 32>(p, frames, out, s);
    case 128: return launch_passB<128, 32>(p, frames, out, s);
    case 256: return launch_passB<256, 32>(p, frames, out, s);
    case 512: return launch_passB<512, 16>(p, frames, out, s);
    case 1024: return launch_passB<1024, 16>(p, frames, out, s);
    }
    set_error("fft: unsupported N2 %d", p.N2);
    return SDRGPU_EARG;
}

}  // namespace sdrgpu

using namespace sdrgpu;

struct sdrgpu_fft {
    FftPlan p;
};

static int fft_upload_window(sdrgpu_fft* h, const float* window, int nz) {
    if (nz <= 0 || nz > h->p.N) { set_error("fft: nz %d out of range (N %d)", nz, h->p.N); return SDRGPU_EARG; }
    SDRGPU_HIP(hipSetDevice(h->p.device));
    SDRGPU_CHECK(h->p.win.ensure(sizeof(float) * nz));
    SDRGPU_HIP(hipMemcpy(h->p.win.p, window, sizeof(float) * nz, hipMemcpyHostToDevice));
    h->p.nz = nz;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_fft_create(sdrgpu_fft** out, int device, int fftSize, int nz, int windowType) {
    if (!out) { set_error("fft_create: null handle"); return SDRGPU_EARG; }
    *out = nullptr;
    int logN = 0;
    while ((1 << logN) < fftSize) logN++;
    if (fftSize < 64 || fftSize > (1 << 20) || (1 << logN) != fftSize) {
        set_error("fft_create: size %d must be a power of two in [64, 2^20]", fftSize);
        return SDRGPU_EARG;
    }
    SDRGPU_HIP(hipSetDevice(device));
    sdrgpu_fft* h = new sdrgpu_fft();
    FftPlan& p = h->p;
    p.device = device; p.N = fftSize; p.logN = logN;
    int rc;
    if (fftSize <= 4096) {
        p.N1 = p.N2 = 0;
        rc = make_twiddles(p.tw1, fftSize);
    } else {
        p.N1 = 1 << ((logN + 1) / 2);   // N1 >= N2, both <= 1024
        p.N2 = fftSize / p.N1;
        rc = make_twiddles(p.tw1, p.N1);
        if (rc >= 0) rc = make_twiddles(p.tw2, p.N2);
        // chunk so the pass-A -> pass-B intermediate (+ the input it came from) stays
        // resident in the Infinity Cache: 64 MB of intermediate per chunk
        p.chunkFrames = std::max(1, (int)((64ll << 20) / ((long long)fftSize * 8)));
        if (rc >= 0) rc = p.scratch.ensure((size_t)p.chunkFrames * fftSize * sizeof(float2));
    }
    if (rc >= 0 && hipStreamCreateWithFlags(&p.own, hipStreamNonBlocking) != hipSuccess) {
        set_error("fft_create: hipStreamCreate failed");
        rc = SDRGPU_EHIP;
    }
    if (rc >= 0) rc = sdrgpu_fft_set_window_type(h, windowType, nz);
    if (rc < 0) { sdrgpu_fft_destroy(h); return rc; }
    *out = h;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_fft_set_window(sdrgpu_fft* h, const float* window, int nz) {
    if (!h || !window) { set_error("fft_set_window: null argument"); return SDRGPU_EARG; }
    return fft_upload_window(h, window, nz);
}

extern "C" int sdrgpu_fft_set_window_type(sdrgpu_fft* h, int windowType, int nz) {
    if (!h) { set_error("fft_set_window_type: null handle"); return SDRGPU_EARG; }
    if (nz <= 0 || nz > h->p.N) { set_error("fft: nz %d out of range (N %d)", nz, h->p.N); return SDRGPU_EARG; }
    std::vector<float> w(nz);
    SDRGPU_CHECK(create_window(windowType, w.data(), nz, 1));   // IQFrontEnd::updateFFTSize: centred
    return fft_upload_window(h, w.data(), nz);
}

extern "C" int sdrgpu_fft_size(sdrgpu_fft* h) { return h ? h->p.N : SDRGPU_EARG; }

extern "C" int sdrgpu_fft_execute_dev(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out,
                                      void* stream) {
    if (!h || !in || !out || frames < 0 || frameStride < 0) { set_error("fft_execute: bad argument"); return SDRGPU_EARG; }
    if (frames == 0) return 0;
    FftPlan& p = h->p;
    SDRGPU_HIP(hipSetDevice(p.device));
    hipStream_t s = stream ? (hipStream_t)stream : p.own;
    const float2* x = (const float2*)in;
    if (p.N1 == 0) {
        SDRGPU_CHECK(dispatch_single(p, x, frameStride, frames, out, s));
        return frames;
    }
    for (int f0 = 0; f0 < frames; f0 += p.chunkFrames) {
        int nf = std::min(p.chunkFrames, frames - f0);
        SDRGPU_CHECK(dispatch_passA(p, x + (long long)f0 * frameStride, frameStride, nf, s));
        SDRGPU_CHECK(dispatch_passB(p, nf, out + (long long)f0 * p.N, s));
    }
    return frames;
}

extern "C" int sdrgpu_fft_logmag(sdrgpu_fft* h, const void* in, float* out) {
    if (!h || !in) { set_error("fft_logmag: null argument"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    SDRGPU_HIP(hipSetDevice(p.device));
    size_t inB = sizeof(float2) * p.nz, outB = sizeof(float) * p.N;
    SDRGPU_CHECK(p.pin_in.ensure(inB));
    SDRGPU_CHECK(p.dev_in.ensure(inB));
    SDRGPU_CHECK(p.dev_out.ensure(outB));
    std::memcpy(p.pin_in.p, in, inB);
    SDRGPU_HIP(hipMemcpyAsync(p.dev_in.p, p.pin_in.p, inB, hipMemcpyHostToDevice, p.own));
    SDRGPU_CHECK(sdrgpu_fft_execute_dev(h, p.dev_in.p, p.nz, 1, p.dev_out.as<float>(), p.own));
    if (out) {
        SDRGPU_CHECK(p.pin_out.ensure(outB));
        SDRGPU_HIP(hipMemcpyAsync(p.pin_out.p, p.dev_out.p, outB, hipMemcpyDeviceToHost, p.own));
        SDRGPU_HIP(hipStreamSynchronize(p.own));
        std::memcpy(out, p.pin_out.p, outB);
    } else {
        SDRGPU_HIP(hipStreamSynchronize(p.own));
    }
    return p.N;
}

extern "C" int sdrgpu_fft_destroy(sdrgpu_fft* h) {
    if (!h) return SDRGPU_OK;
    (void)hipSetDevice(h->p.device);
    if (h->p.own) (void)hipStreamDestroy(h->p.own);
    delete h;
    return SDRGPU_OK;
}
