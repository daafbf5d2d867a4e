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
#include <cstdlib>
#include <algorithm>
#include <utility>
#include "sdrgpu_internal.h"
#include "fft_stages.h"
#include "fir_rows.h"
#include "fir_tail.h"

#ifndef SDRGPU_PB_NT
#define SDRGPU_PB_NT 1   // 64k pass B: streaming dB row stores (A/B builds: 0)
#endif
// cache policy of pass A's input loads (A/B builds; 2 = streaming)
#ifndef SDRGPU_PA_CP
#define SDRGPU_PA_CP 2
#endif
namespace sdrgpu {

// K3, volk_32fc_s32f_power_spectrum_32f(out, X, 1.0, N): 10*log10(re^2 + im^2).
// VOLK evaluates 10 * log10f(p) in fp32, which adds about one ulp of the dB value on top of the
// FFT's own error (median 1 ulp vs the correctly rounded dB of the exact DFT). Here the exponent
// of p is split off exactly (p = m 2^e, m in [0.5, 1)), only log2(m) is taken in fp32 (absolute
// error ~1e-7), and e + log2(m) is scaled by 10 log10(2) in fp64 and rounded once: the dB row
// then carries the FFT's error only (median 0 ulp, same class as pocketfft + an exact log;
// tests/test_gpu_parity.py::test_spectrum_ulp_distribution). Three fp64 ops per bin in a
// memory-bound epilogue. p = 0 gives -inf like log10f.
__device__ __forceinline__ float db_of(float2 X) {
    const float p = X.x * X.x + X.y * X.y;
    int e;
    const float m = frexpf(p, &e);
    const double l = (double)e + (double)__builtin_amdgcn_logf(m);   // v_log_f32: log2, m normal or 0
    return (float)(3.0102999566398119521 * l);
}

// Persistent tile loop shared by the three spectrum kernels. Each workgroup walks tiles
// blockIdx.x, +gridDim.x, ...; the 16 raw loads of tile i+1 (Frag) are issued before tile i
// is transformed and stored, so HBM latency overlaps the LDS exchange, the math and the
// stores of the previous tile (one register fragment in flight per thread).
template <int L, class Frag, bool T16 = false, class Issue, class Finish, class Store>
__device__ __forceinline__ void tile_loop(float2* lds, const float2* __restrict__ tw, int tile, int ntiles, int sF, int tF,
                                          int sL, int tL, Issue&& issue, Finish&& finish, Store&& store,
                                          const float2* tw16 = nullptr) {
    // One tile per workgroup (grid = tiles). A persistent variant with a ping-pong register
    // prefetch of the next tile was measured at the same 64k throughput with a quarter of the
    // occupancy (and spills at N1 = 1024), so the simple form is kept.
    constexpr int LS = Lds<L>::LS;
    if (tile >= ntiles) return;
    Frag fr;
    issue(fr, tile);
    float2 v[16];
    finish(fr, v);
    stage_first<L>(lds + sF * LS, v, tF);
    __syncthreads();
    stages_rest<L, T16>(lds, tw, sL, tL, [&](int k, float2 y, int slot) {
        if constexpr (std::is_invocable_v<Store&, int, int, float2, int>) store(tile, k, y, slot);
        else store(tile, k, y);
    }, tw16);
}

struct FragW {   // raw input + window values for 16 samples
    float2 x[16];
    float w[16];
};
struct FragC {
    float2 x[16];
};

// ---- single pass (N <= 4096): S frames per tile -------------------------------
template <int L, int S>
__global__ __launch_bounds__(S * L / 16) void fft_single_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz,
    const float2* __restrict__ tw, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int T = L / 16;
    const int tid = threadIdx.x;
    const int s = tid / T, t = tid % T;           // frame-contiguous mapping for load and store
    const int ntiles = (frames + S - 1) / S;
    tile_loop<L, FragW>(
        lds, tw, blockIdx.x, ntiles, s, t, s, t,
        [&](FragW& fr, int tile) {
            const int f = min(tile * S + s, frames - 1);
            const float2* x = in + (long long)f * frameStride;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int n = t + r * T;
                const int nc = n < nz ? n : nz - 1;
                fr.x[r] = x[nc];
                fr.w[r] = n < nz ? win[nc] : 0.0f;
            }
        },
        [&](const FragW& fr, float2 (&v)[16]) {
#pragma unroll
            for (int r = 0; r < 16; r++) v[r] = make_float2(fr.x[r].x * fr.w[r], fr.x[r].y * fr.w[r]);
        },
        [&](int tile, int k, float2 y) {
            const int f = tile * S + s;
            if (f < frames) out[(long long)f * L + k] = db_of(y);
        });
}

// raw buffer resource over `bytes` bytes from p: loads past the end return 0, stores past it are dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// ---- pass A: S columns x N1 rows per tile ---------------------------------------
// Column c of the frame viewed as N1 x N2: x[n1*N2 + c0 + c]. The column index is the
// fastest-varying thread coordinate in both the load and the store, so each wave reads
// and writes whole 128-B row segments (S = 16 columns x 8 B).
// Four-step twiddle W_N^(n2 k1), n2 = S*b + c: one load of the exact fp64-generated value
// from the N-entry Tfull[k1][n2] table (contiguous per 16 lanes, L2-resident). A product of
// two table values (W_N^(S b k1) x W_N^(c k1)) saved a little table space but added an
// fp32 rounding: the 64k spectrum's rms dB error on a tonal signal was 2.1x pocketfft's.
template <int L, int S, int CP = SDRGPU_PA_CP>   // CP: cache policy of the 256-point input loads
__device__ __forceinline__ void passA_tile(
    float2* lds, int tile, const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win,
    int nz, int N2, int logN, const float2* __restrict__ tw, const float2* __restrict__ tfull,
    float2* __restrict__ scratch, const float2* __restrict__ headp = nullptr, int nh = 0) {
    const int tid = threadIdx.x;
    const int c = tid % S, t = tid / S;
    constexpr int T = L / 16;
    const int nb = N2 / S;                        // column blocks per frame
    const int ntiles = nb * frames;
    if constexpr (L == 256) {
        // 256-point columns: both stages are radix 16, so the whole column is one LDS exchange.
        // Every global read is issued up front (input, window, the exact four-step twiddles of
        // this thread's 16 outputs and the WG's copy of the stage twiddles, which live in LDS),
        // so the WG waits for memory once instead of three times.
        if (tile >= ntiles) return;
        constexpr int LS = Lds<L>::LS;
        float2* twl = lds + S * LS;
        const int b = tile % nb;
        const long long f = tile / nb;
        const int col = b * S + c;
        // Buffer loads/stores: one wave-uniform resource per array and ONE per-lane byte offset
        // (o0) shared by every access of the thread; the row step r * 16 * N2 rides in the
        // scalar soffset. (Plain global accesses kept a 64-bit address pair per row live and
        // spilled at the 4-waves/SIMD register budget.)
        // split stream (fft_execute_split): frame 0 = [headp (nh) || in], frame f >= 1 at in + f stride - nh
        const float2* x = in + f * frameStride - (f > 0 ? nh : 0);
        const unsigned o0 = (unsigned)(t * N2 + col);
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)win, (short)0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc((void*)tfull, (short)0, 0x7fffffff, 0x00020000);
        const int rowB = T * N2 * 8;   // bytes between the rows t + 16 r and t + 16 (r + 1)
        float2 xv[16], tt[16];
        float wv[16];
        if (nh > 0 && f == 0) {   // the frame straddling two buffers (workgroup-uniform)
            // sample n comes from headp[n] (n < nh) or in[n - nh]: two range-checked loads (resources
            // of nh and nz - nh elements; the one out of range returns 0) summed, so no branch per
            // sample. The row step is in the per-lane offset: the range check ignores soffset.
            const __amdgpu_buffer_rsrc_t rh = brsrc(headp, (unsigned)nh * 8u);
            const __amdgpu_buffer_rsrc_t rb = brsrc(in, (unsigned)(nz - nh) * 8u);
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const unsigned n = o0 + (unsigned)(r * T * N2);
                const bool live = (int)n < nz;
                const float2 a = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rh, n * 8, 0, 0));
                const float2 b = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rb, (n - (unsigned)nh) * 8, 0, 0));
                const float we = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, (live ? n : 0u) * 4, 0, 0));
                xv[r] = make_float2(a.x + b.x, a.y + b.y);
                wv[r] = live ? we : 0.0f;
            }
        } else if (nz >= L * N2) {   // no zero padding (wave-uniform)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                xv[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, o0 * 8, r * rowB, CP));
                wv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, o0 * 4, r * rowB / 2, 0));
            }
        } else {              // zero-padded tail: clamped (in-bounds) loads, then select
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const unsigned n = o0 + (unsigned)(r * T * N2);
                const bool live = (int)n < nz;
                const unsigned nc = live ? n : 0u;
                const float2 xe = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, nc * 8, 0, 0));
                const float we = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, nc * 4, 0, 0));
                xv[r] = live ? xe : make_float2(0.0f, 0.0f);
                wv[r] = live ? we : 0.0f;
            }
        }
        for (int i = tid; i < L; i += S * T) twl[i] = tw[i];
        float2* tw16 = twl + L;   // twl[r t] as tw16[16 r + t]: conflict-free across t (stage_lds)
        stage16_twiddles<L>(tw16, tw, tid, S * T);
#pragma unroll
        for (int r = 0; r < 16; r++)   // exact W_N^(n2 k1), k1 = t + 16 r: same offsets as the input rows
            tt[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rt, o0 * 8, r * rowB, 0));
        float2 v[16];
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = make_float2(xv[r].x * wv[r], xv[r].y * wv[r]);
        float2* seq = lds + c * LS;
        stage_first<L>(seq, v, t);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = seq[pad16s<16>(t, r)];
#pragma unroll
        for (int r = 1; r < 16; r++) v[r] = cmul(v[r], tw16[16 * r + t]);
        dft16(v);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(scratch + (f << logN)), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const float2 y = cmul(v[r], tt[r]);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, y), rs,
                                                  o0 * 8, r * rowB, 0);
        }
        return;
    }
    tile_loop<L, FragW>(
        lds, tw, tile, ntiles, c, t, c, t,
        [&](FragW& fr, int tile) {
            const int b = tile % nb;
            const long long f = tile / nb;
            const int col = b * S + c;
            const float2* x = in + f * frameStride;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const long long n = (long long)(t + r * T) * N2 + col;
                const bool live = n < nz;
                const long long nc = live ? n : 0;   // frame[0]: always in bounds
                fr.x[r] = x[nc];
                fr.w[r] = live ? win[nc] : 0.0f;
            }
        },
        [&](const FragW& fr, float2 (&v)[16]) {
#pragma unroll
            for (int r = 0; r < 16; r++) v[r] = make_float2(fr.x[r].x * fr.w[r], fr.x[r].y * fr.w[r]);
        },
        [&](int tile, int k1, float2 y) {
            const int b = tile % nb;
            const long long f = tile / nb;
            const float2 t0 = tfull[(long long)k1 * N2 + b * S + c];   // exact W_N^(n2 k1)
            scratch[(f << logN) + (long long)k1 * N2 + b * S + c] = cmul(y, t0);
        });
}

template <int L, int S>
__global__ __launch_bounds__(S * L / 16) __attribute__((amdgpu_waves_per_eu(4))) void fft_passA_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz, int N2,
    int logN, const float2* __restrict__ tw, const float2* __restrict__ tfull,
    float2* __restrict__ scratch, const float2* __restrict__ headp, int nh, SideCopy side) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int ntiles = (N2 / S) * frames;
    if ((int)blockIdx.x >= ntiles) {   // spare workgroups: the caller's side copies (fft_execute_split)
        const int w = blockIdx.x - ntiles, nw = gridDim.x - ntiles;
        for (int k = 0; k < side.count; k++)
            for (int i = w * blockDim.x + threadIdx.x; i < side.n[k]; i += nw * blockDim.x) side.dst[k][i] = side.src[k][i];
        return;
    }
    passA_tile<L, S>(lds, blockIdx.x, in, frameStride, frames, win, nz, N2, logN, tw, tfull, scratch, headp, nh);
}

// ---- pass A, paired columns: S columns x N1 rows per tile, two adjacent columns per lane --
// Same transform as fft_passA_kernel with a third of its vector-memory instructions per
// element (the 64k pass A was issue-bound on them): 16-B loads of two
// adjacent columns (and an 8-B window pair), stage twiddles staged once per workgroup in
// LDS, and one 16-B load of the exact four-step twiddle pair W_N^(n2 k1) from an N-entry
// [k1][n2] table (L2-resident) instead of a product of two table values. Requires an even
// frame stride and a 16-B aligned input (checked on the host).
template <int L, int R, int NS, int V, bool T16 = false>
__device__ __forceinline__ void stage_lds_v(float2* seq0, const float2* twl, int t, const float2* tw16 = nullptr) {
    constexpr int T = L / 16, BPT = 16 / R, LS = Lds<L>::LS;
    float2 v[V][BPT][R];
#pragma unroll
    for (int q = 0; q < V; q++)
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = t + b * T, jm = j % NS;
#pragma unroll
            for (int r = 0; r < R; r++) v[q][b][r] = seq0[q * LS + pad16s<L / R>(j, r)];
            if constexpr (T16 && R == 16 && NS == 16) {   // conflict-free layout (stage_lds, fft_stages.h)
#pragma unroll
                for (int r = 1; r < R; r++) v[q][b][r] = cmul(v[q][b][r], tw16[16 * r + jm]);
            } else {
#pragma unroll
                for (int r = 1; r < R; r++) v[q][b][r] = cmul(v[q][b][r], twl[r * jm * (L / (NS * R))]);
            }
            dft<R>(v[q][b]);
        }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < V; q++)
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = t + b * T, idxD = (j / NS) * NS * R + (j % NS);
#pragma unroll
            for (int r = 0; r < R; r++) seq0[q * LS + pad16s<NS>(idxD, r)] = v[q][b][r];
        }
    __syncthreads();
}

template <int L, int R, int NS, int V, class Store>
__device__ __forceinline__ void stage_last_v(const float2* seq0, const float2* twl, int t, Store&& st) {
    constexpr int T = L / 16, BPT = 16 / R, LS = Lds<L>::LS;
    float2 v[V][BPT][R];
#pragma unroll
    for (int q = 0; q < V; q++)
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = t + b * T, jm = j % NS;
#pragma unroll
            for (int r = 0; r < R; r++) v[q][b][r] = seq0[q * LS + pad16s<L / R>(j, r)];
#pragma unroll
            for (int r = 1; r < R; r++) v[q][b][r] = cmul(v[q][b][r], twl[r * jm * (L / (NS * R))]);
            dft<R>(v[q][b]);
        }
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T, idxD = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; r++) {
            float2 y[V];
#pragma unroll
            for (int q = 0; q < V; q++) y[q] = v[q][b][r];
            st(idxD + r * NS, y);
        }
    }
}

// stages 2.. of V length-L sequences (seq q at seq0 + q*LS) with LDS twiddles
template <int L, int V, class Store>
__device__ __forceinline__ void stages_rest_v(float2* seq0, const float2* twl, int t, Store&& st) {
    if constexpr (L == 64) {
        stage_last_v<L, 4, 16, V>(seq0, twl, t, st);
    } else if constexpr (L == 128) {
        stage_last_v<L, 8, 16, V>(seq0, twl, t, st);
    } else if constexpr (L == 256) {
        stage_last_v<L, 16, 16, V>(seq0, twl, t, st);
    } else {
        stage_lds_v<L, 16, 16, V>(seq0, twl, t);
        if constexpr (L == 512) stage_last_v<L, 2, 256, V>(seq0, twl, t, st);
        else if constexpr (L == 1024) stage_last_v<L, 4, 256, V>(seq0, twl, t, st);
        else if constexpr (L == 2048) stage_last_v<L, 8, 256, V>(seq0, twl, t, st);
        else stage_last_v<L, 16, 256, V>(seq0, twl, t, st);
    }
}

template <int L, int S>
__device__ __forceinline__ void passA2_tile(
    float2* lds, int tile, const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win,
    int nz, int N2, int logN, const float2* __restrict__ tw, const float2* __restrict__ tfull, float2* __restrict__ scratch) {
    constexpr int P = S / 2, T = L / 16, NT = P * T, LS = Lds<L>::LS;
    float2* twl = lds + S * LS;
    const int tid = threadIdx.x;
    const int cp = tid % P, t = tid / P;
    for (int i = tid; i < L; i += NT) twl[i] = tw[i];
    const int nb = N2 / S;
    const int b = tile % nb;
    const long long f = tile / nb;
    const int col = b * S + 2 * cp;
    const float2* x = in + f * frameStride;
    float4 q[16];
    float2 w[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const long long n = (long long)(t + r * T) * N2 + col;
        if (n + 1 < nz) {
            q[r] = *reinterpret_cast<const float4*>(x + n);
            w[r] = *reinterpret_cast<const float2*>(win + n);
        } else {   // zero-padded tail (n >= nz) or the one pair straddling nz
            const bool live = n < nz;
            const float2 e = x[live ? n : 0];
            const float we = live ? win[n] : 0.0f;
            q[r] = make_float4(e.x, e.y, 0.0f, 0.0f);
            w[r] = make_float2(we, 0.0f);
        }
    }
    float2 v0[16], v1[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        v0[r] = make_float2(q[r].x * w[r].x, q[r].y * w[r].x);
        v1[r] = make_float2(q[r].z * w[r].y, q[r].w * w[r].y);
    }
    dft16(v0);
    dft16(v1);
    float2* seq0 = lds + 2 * cp * LS;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        seq0[pad16lo(t, r)] = v0[r];
        seq0[LS + pad16lo(t, r)] = v1[r];
    }
    __syncthreads();
    float2* dst = scratch + (f << logN);
    stages_rest_v<L, 2>(seq0, twl, t, [&](int k1, float2 (&y)[2]) {
        const long long o = (long long)k1 * N2 + col;
        const float4 tt = *reinterpret_cast<const float4*>(tfull + o);
        const float2 a = cmul(y[0], make_float2(tt.x, tt.y)), c = cmul(y[1], make_float2(tt.z, tt.w));
        *reinterpret_cast<float4*>(dst + o) = make_float4(a.x, a.y, c.x, c.y);
    });
}

template <int L, int S>
__global__ __launch_bounds__(S / 2 * L / 16) void fft_passA2_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz, int N2,
    int logN, const float2* __restrict__ tw, const float2* __restrict__ tfull, float2* __restrict__ scratch) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    passA2_tile<L, S>(lds, blockIdx.x, in, frameStride, frames, win, nz, N2, logN, tw, tfull, scratch);
}

// ---- 1M passes (N1 = N2 = 1024), persistent and software-pipelined ----------------------------
// The 1M column FFT needs 16 x 1024 x 8 B of LDS per tile (139 KB), so one workgroup per CU: in a
// one-shot kernel each CU alternates "load the tile" and "transform + store it", and HBM idles during
// the transform. Here each CU's workgroup walks tiles blockIdx.x, +gridDim.x, ... and issues the next
// tile's input + window loads (96 VGPRs) before it transforms the current one, so the loads fly
// during the LDS stages and the stores. The stage twiddles are staged in LDS once per workgroup, and
// the four-step twiddle W_N^(c k1) is generated in fp64 and rounded once (the same single rounding as
// a table): for column c and this thread's outputs k1 = t + 64 m, W^(c t) and W^(64 c) come from two
// 256-entry fp64 tables (W_N^(256 j), W_N^j; c t, 64 c < 2^16) and W^(c (t + 64 m)) = W^(c t)
// (W^(64 c))^m by an fp64 recurrence over m (15 products: relative error ~1e-15, far below the fp32
// rounding). That removes the 8 MB [k1][n2] table read (8 B per sample of L2 / Infinity-Cache
// traffic). Measured alternatives (rounds 2-4; kept in git history, not here): 8-column
// tiles (2.24-2.70 ms), spill-free laundered offsets (same time), the merged pass-B(c-1) + pass-A(c)
// launches (1.80 vs 1.73 ms), two workgroups per CU (2.16 ms).
__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

typedef unsigned bu2 __attribute__((ext_vector_type(2)));
typedef unsigned bu4 __attribute__((ext_vector_type(4)));

// tile -> (frame, block) of the 1M pass B: G8 adjacent row blocks on one XCD at once. Workgroups x,
// x + 8, ... (same XCD, same round) take blocks b, b + 1, ..., whose 32-B dB segments share 128-B
// lines, so a line is written whole in one L2.
template <int G8>
__device__ __forceinline__ void tile_fb(int T, int nb, int& b, long long& f) {
    const int g = T / (8 * G8), w = T % (8 * G8);
    const int P = g * 8 + (w & 7), h = w >> 3;
    const int npf = nb / G8;
    f = P / npf;
    b = G8 * (P % npf) + h;
}

// ---- 1M pass B: 8 rows of 1024 per tile (two workgroups per CU), each workgroup walking tiles with
// the next tile's 16 row values per thread loaded while the current tile is transformed and stored.
// The intermediate is pass A's tile-major layout [block][k1][16 columns]: a row piece of 16 columns is
// 128 contiguous bytes. Row blocks XCD-grouped by 4 (1.93 vs 1.97 ms per C2 step; ungrouped 2.06).
// Sequence stride LSB = 1090 float2 (even; Lds<1024>::LS = 1089 elsewhere). After stage 1 a
// half-wave holds 8 sequences x 2 (read2/write2, banks by float2 index mod 16) or 4 (ds_read_b64, mod
// 32) consecutive butterflies: at stride 1089 (= 1 mod 32) sequence s and butterfly t + 1 share the
// banks of s + 1 and t -- the middle stage's accesses 2-way, the last stage's reads 4-way, 3.7
// conflict cycles per LDS instruction measured (r6e SQ counters, tools/lds_bank_model.py reproduces
// it); at 1090 (= 2 mod 32) the middle stage is conflict-free and the last stage's reads 2-way.
#ifndef SDRGPU_PB1M_LS
#define SDRGPU_PB1M_LS 1090   // (A/B builds: 1089)
#endif
constexpr int kPassB1mLS = SDRGPU_PB1M_LS;
__global__ __launch_bounds__(512) void fft_passB_1m_kernel(const float2* __restrict__ scratch, int frames, int N1, int logN,
                                                           const float2* __restrict__ tw, float* __restrict__ out) {
    constexpr int L = 1024, T = L / 16, S = 8, XG = 4, LSB = kPassB1mLS;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* twl = lds + S * LSB;   // stage twiddles, staged once per workgroup
    float2* tw16 = twl + L;                // the middle stage's, bank-conflict-free (stage_lds)
    const int tid = threadIdx.x;
    for (int i = tid; i < L; i += S * T) twl[i] = tw[i];   // (first barrier below orders both)
    for (int i = tid; i < 256; i += S * T) tw16[i] = tw[(i >> 4) * (i & 15) * (L / 256)];
    const int sF = tid / T, tF = tid % T;
    const int nb = N1 / S;
    const int ntiles = nb * frames;
    float2 fr[16];
    auto issue = [&](int tile) {
        int b;
        long long f;
        tile_fb<XG>(tile, nb, b, f);
        const __amdgpu_buffer_rsrc_t rs = brsrc(scratch + (f << logN), 0x7fffffffu);
        const unsigned o = (unsigned)((tF / 16) * L * 16 + (b * S + sF) * 16 + tF % 16) * 8u;
#pragma unroll
        for (int r = 0; r < 16; r++) fr[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, o, r * 4 * L * 16 * 8, 0));
    };
    int tile = blockIdx.x;
    if (tile < ntiles) issue(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        float2 v[16];
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = fr[r];
        if (tile + (int)gridDim.x < ntiles) issue(tile + gridDim.x);
        // the LDS addresses below are loop-invariant; recomputing them per tile (laundered thread
        // index) keeps ~40 hoisted address registers from spilling the prefetched tile
        int tv = tid;
        asm volatile("" : "+v"(tv));
        const int sF2 = tv / T, tF2 = tv % T, sL2 = tv % S, tL2 = tv / S;
        __syncthreads();   // the previous tile's last LDS reads are done
        stage_first<L>(lds + sF2 * LSB, v, tF2);
        __syncthreads();
        int b;
        long long f;
        tile_fb<XG>(tile, nb, b, f);
        const __amdgpu_buffer_rsrc_t ro = brsrc(out + (f << logN) + b * S, 0x7fffffffu);
        stages_rest<L, true, LSB>(lds, twl, sL2, tL2, [&](int k2, float2 y) {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, db_of(y)), ro, (unsigned)(sL2 + N1 * k2) * 4u, 0, 0);
        }, tw16);
    }
}

// ---- 1M pass A: 16 paired columns x 1024 rows per tile, one workgroup per CU -----------------------
// The input rows are read once: streaming (slc) loads, so they do not push the 4 MB window out of L2
// (PMC fetch 18.15 -> 17.50 B/sample, C2 1.848 -> 1.798 ms). Each tile's 128 KB of output is written
// contiguously in the tile-major layout [block][k1][16] (1 KB per store instruction instead of eight
// 128-B row pieces: 1.89 vs 1.94 ms).
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1))) void fft_passA_1m_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz, int N2,
    int logN, const float2* __restrict__ tw, const double2* __restrict__ wt, float2* __restrict__ scratch) {
    constexpr int L = 1024, S = 16, P = S / 2, T = L / 16, NT = P * T, LS = Lds<L>::LS, CP = 2;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* twl = lds + S * LS;
    float2* tw16 = twl + L;   // the middle stage's twiddles, bank-conflict-free (stage_lds)
    const int tid = threadIdx.x;
    const int cp = tid % P, t = tid / P;
    for (int i = tid; i < L; i += NT) twl[i] = tw[i];   // (first barrier below orders both)
    for (int i = tid; i < 256; i += NT) tw16[i] = tw[(i >> 4) * (i & 15) * (L / 256)];
    const int nb = N2 / S;
    const int ntiles = nb * frames;
    // The input / window resources end at nz, so the zero-padded tail loads return 0 (nz even: a
    // column pair never straddles nz, checked on the host). The row step goes into the per-lane
    // offset, not the scalar one: the buffer range check covers voffset (+ the instruction offset)
    // only, so rows past nz addressed through soffset were NOT zeroed -- they read the next frame
    // and past the window's allocation (a first version did that: wrong and run-to-run varying
    // rows)
    const __amdgpu_buffer_rsrc_t rw = brsrc(win, (unsigned)nz * 4u);
    const int rowB = T * N2 * 8;   // bytes between rows t + 64 r and t + 64 (r + 1)
    float4 q[16];
    float2 w[16];
    auto issue = [&](int tile) {
        const int b = tile % nb;
        const long long f = tile / nb;
        const unsigned o = (unsigned)(t * N2 + b * S + 2 * cp);
        const __amdgpu_buffer_rsrc_t rx = brsrc(in + f * frameStride, (unsigned)nz * 8u);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            q[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, o * 8 + r * rowB, 0, CP));
            w[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rw, o * 4 + r * rowB / 2, 0, 0));
        }
    };
    int tile = blockIdx.x;
    if (tile < ntiles) issue(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        float2 v0[16], v1[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
            v0[r] = make_float2(q[r].x * w[r].x, q[r].y * w[r].x);
            v1[r] = make_float2(q[r].z * w[r].y, q[r].w * w[r].y);
        }
        if (tile + (int)gridDim.x < ntiles) issue(tile + gridDim.x);   // next tile's loads fly now
        dft16(v0);
        dft16(v1);
        int tv = tid;   // laundered thread index: the LDS addresses are recomputed per tile, not hoisted
        asm volatile("" : "+v"(tv));
        const int cp2 = tv % P, t2 = tv / P;
        float2* seq0 = lds + 2 * cp2 * LS;
        __syncthreads();   // the previous tile's last LDS reads are done (and twl is staged)
#pragma unroll
        for (int r = 0; r < 16; r++) {
            seq0[pad16lo(t2, r)] = v0[r];
            seq0[LS + pad16lo(t2, r)] = v1[r];
        }
        __syncthreads();
        stage_lds_v<L, 16, 16, 2, true>(seq0, twl, t2, tw16);   // middle stage, radix 16 (two barriers inside)
        const int b = tile % nb;
        const long long f = tile / nb;
        const int col = b * S + 2 * cp;
        const __amdgpu_buffer_rsrc_t rs = brsrc(scratch + (f << logN), 0x7fffffffu);
        // Stores carry the row step in the per-lane offset and a ZERO soffset. A >64-bit buffer
        // store with an SGPR soffset gets no wait state before the next VALU write of its data
        // VGPRs (hipcc's hazard check skips that form, and two 8-B stores get merged into it): it
        // wrote already-overwritten data, rows of some lanes changing from run to run (DESIGN.md
        // §3). The offset is advanced through an opaque register so the 16 row offsets are not all
        // precomputed (register pressure).
        double2 cur[2], step[2];
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            const int c = col + qq;
            const int e0 = c * t2, d = 64 * c;   // < 2^16
            cur[qq] = zmul(wt[e0 >> 8], wt[256 + (e0 & 255)]);
            step[qq] = zmul(wt[d >> 8], wt[256 + (d & 255)]);
        }
        // last stage (radix 4, NS = 256): outputs k1 = t + 64 m, m = b4 + 4 r, kept in registers
        float2 y[2][16];
#pragma unroll
        for (int qq = 0; qq < 2; qq++)
#pragma unroll
            for (int b4 = 0; b4 < 4; b4++) {
                const int j = t2 + b4 * T;
                float2 u[4];
#pragma unroll
                for (int r = 0; r < 4; r++) u[r] = seq0[qq * LS + pad16s<L / 4>(j, r)];
#pragma unroll
                for (int r = 1; r < 4; r++) u[r] = cmul(u[r], twl[r * j]);
                dft4v(u);
#pragma unroll
                for (int r = 0; r < 4; r++) y[qq][b4 + 4 * r] = u[r];
            }
        unsigned vo = (unsigned)(b * L * S + t * S + 2 * cp) * 8u;
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const float2 a = cmul(y[0][m], make_float2((float)cur[0].x, (float)cur[0].y));
            const float2 c = cmul(y[1][m], make_float2((float)cur[1].x, (float)cur[1].y));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bu4, make_float4(a.x, a.y, c.x, c.y)), rs, vo, 0, 0);
            vo += (unsigned)(T * S * 8);
            asm volatile("" : "+v"(vo));
            if (m < 15) {
                cur[0] = zmul(cur[0], step[0]);
                cur[1] = zmul(cur[1], step[1]);
            }
        }
    }
}

// ---- pass B: S rows of length N2 per tile, dB out, transposed store -----------------
// Stage 1 maps threads row-contiguous (coalesced row reads); the last stage maps the row
// index fastest so the transposed dB store writes S consecutive floats per k2.
// DPP move of a float: lanes outside row_mask keep `old`
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float old, float src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, src),
                                                                 CTRL, ROWMASK, 0xF, false));
}

// lane exchange with the partner lane ^ D (D = 1, 2, 4, 8: within a 16-lane DPP row)
template <int D>
__device__ __forceinline__ float xchg(float v, int lane) {
    if constexpr (D == 1) return dpp_f<0xB1, 0xF>(v, v);             // quad_perm [1,0,3,2]
    else if constexpr (D == 2) return dpp_f<0x4E, 0xF>(v, v);        // quad_perm [2,3,0,1]
    else {                                                            // row_shr:D / row_shl:D
        const float dn = dpp_f<0x110 + D, 0xF>(v, v), up = dpp_f<0x100 + D, 0xF>(v, v);
        return (lane & D) ? dn : up;
    }
}
// one transpose-reduce step over the value pairs (v[i], v[i + H]): the lane whose bit D is 0
// keeps the lower half and takes its partner's, the other keeps the upper half
template <int D, int H>
__device__ __forceinline__ void tr_step(float (&v)[16], int lane) {
    const bool hi = (lane & D) != 0;
#pragma unroll
    for (int i = 0; i < H; i++) {
        const float send = hi ? v[i] : v[i + H];
        const float keep = hi ? v[i + H] : v[i];
        v[i] = fmaxf(keep, xchg<D>(send, lane));
    }
}

// ZM: also the waterfall's full-span zoom row (fft_scaler::doZoom with viewOffset 0 and the whole
// bandwidth in view, gui/widgets/fft_scaler.h:27-64) at factor S: out width N / S, zoom[o] = max of
// the S consecutive bins [S o, S o + S) = the bins b*S + sL of one k2, held by the S lanes sL of a
// half-wave. Each lane keeps its 16 dB values (k2 = tL + 16 r); a 16-value transpose-reduce over
// the lane bits 0..3 (DPP, VALU only) leaves in every lane the max over its 16-lane row of one r,
// one swizzle (xor 16) folds the two rows, and lanes 16..31 store the half-wave's 16 zoom values
// with one instruction.
template <int L, int S, bool ZM = false>
__device__ __forceinline__ void passB_tile(
    float2* lds, int tile, const float2* __restrict__ scratch, int frames, int N1, int logN, const float2* __restrict__ tw,
    float* __restrict__ out, float* __restrict__ zoom = nullptr) {
    constexpr int T = L / 16;
    const int tid = threadIdx.x;
    const int sF = tid / T, tF = tid % T;
    const int sL = tid % S, tL = tid / S;
    const int nb = N1 / S;
    const int ntiles = nb * frames;
    float dbv[16];   // ZM: this lane's dB values, r = k2 >> 4
    constexpr bool T16 = L >= 256;   // the radix-16 NS = 16 stage's twiddles from LDS, conflict-free
    float2* tw16 = lds + S * Lds<L>::LS;
    if constexpr (T16) stage16_twiddles<L>(tw16, tw, tid, S * T);   // (tile_loop's barrier orders it)
    tile_loop<L, FragC, T16>(
        lds, tw, tile, ntiles, sF, tF, sL, tL,
        [&](FragC& fr, int tile) {
            const int b = tile % nb;
            const long long f = tile / nb;
            const float2* src = scratch + (f << logN) + (long long)(b * S + sF) * L + tF;
#pragma unroll
            for (int r = 0; r < 16; r++) fr.x[r] = src[r * T];
        },
        [&](const FragC& fr, float2 (&v)[16]) {
#pragma unroll
            for (int r = 0; r < 16; r++) v[r] = fr.x[r];
        },
        [&](int tile, int k2, float2 y, int slot) {
            const int b = tile % nb;
            const long long f = tile / nb;
            const float d = db_of(y);
            // dB rows are written once and never read back here: streaming stores (whole 128-B
            // lines: S = 32 consecutive floats per row), so they do not evict the intermediate
            float* o = &out[(f << logN) + b * S + sL + (long long)N1 * k2];
            if constexpr (SDRGPU_PB_NT) __builtin_nontemporal_store(d, o);
            else *o = d;
            if constexpr (ZM) dbv[slot] = d;   // stage_last<256, 16, 16>: slot r <-> k2 = tL + 16 r
        }, tw16);
    if constexpr (ZM) {
        static_assert(S == 32 && L == 256, "zoom: one half-wave per zoomed bin, k2 = tL + 16 r");
        if (tile >= ntiles) return;
        const int lane = tid & 63;
        tr_step<1, 8>(dbv, lane);
        tr_step<2, 4>(dbv, lane);
        tr_step<4, 2>(dbv, lane);
        tr_step<8, 1>(dbv, lane);
        // lane bits (b0 b1 b2 b3) now select r = 8 b0 + 4 b1 + 2 b2 + b3; fold the two rows: lane
        // i ^ 16 holds the same r (ds_swizzle xor 16 within 32 lanes: and 0x1F, xor 0x10)
        const float m = fmaxf(dbv[0], __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, dbv[0]), 0x401F)));
        if (sL >= 16) {
            const int j = sL - 16;
            const int r = ((j & 1) << 3) | ((j & 2) << 1) | ((j & 4) >> 1) | ((j & 8) >> 3);
            const int b = tile % nb;
            const long long f = tile / nb;
            zoom[(f << logN) / S + b + (long long)(N1 / S) * (tL + 16 * r)] = m;
        }
    }
}

template <int L, int S, bool ZM>
__global__ __launch_bounds__(S * L / 16) void fft_passB_kernel(
    const float2* __restrict__ scratch, int frames, int N1, int logN, const float2* __restrict__ tw,
    float* __restrict__ out, float* __restrict__ zoom) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    passB_tile<L, S, ZM>(lds, blockIdx.x, scratch, frames, N1, logN, tw, out, zoom);
}

// ---- merged launch: pass B of chunk c (first nB workgroups) + pass A of chunk c+1 --------
// The two halves share nothing (pass A writes the other scratch buffer), so one launch
// replaces two dependent kernel boundaries per chunk; the pass-B workgroups are dispatched
// first and pass A fills the CUs as they drain. Needs equal thread counts (SA*LA == SB*LB).
template <int LA, int SA, int LB, int SB, bool PAIRED, bool ZM>
__global__ __launch_bounds__((PAIRED ? SA / 2 : SA) * LA / 16) __attribute__((amdgpu_waves_per_eu(4))) void fft_merged_kernel(
    int nB, const float2* __restrict__ scratchB, int framesB, float* __restrict__ outB, float* __restrict__ zoomB,
    const float2* __restrict__ in, long long frameStride, int framesA, const float* __restrict__ win, int nz,
    int logN, const float2* __restrict__ tw1, const float2* __restrict__ tw2, const float2* __restrict__ tfull,
    float2* __restrict__ scratchA) {
    static_assert((PAIRED ? SA / 2 : SA) * LA == SB * LB, "merged pass kernels need equal workgroup sizes");
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if ((int)blockIdx.x < nB) {
        passB_tile<LB, SB, ZM>(lds, blockIdx.x, scratchB, framesB, LA, logN, tw2, outB, zoomB);
    } else if constexpr (PAIRED) {
        passA2_tile<LA, SA>(lds, blockIdx.x - nB, in, frameStride, framesA, win, nz, LB, logN, tw1, tfull, scratchA);
    } else {
        passA_tile<LA, SA>(lds, blockIdx.x - nB, in, frameStride, framesA, win, nz, LB, logN, tw1, tfull, scratchA);
    }
}

// ---- spectrum launches that also run a VFO's first stage over the same batch ---------------
// (sdrgpu_fft_execute_vfo_dev / _zoom_vfo_dev on the 64k plan: 256 x 256, 32-column / 32-row
// tiles, 512 threads.) The IQ batch is read from HBM once: each pass-A frame's 8 column tiles are
// dispatched next to one workgroup that computes the VFO stage-1 outputs of the same 65,536
// samples (2,048 outputs of the D = 32, 143-tap decimator = 16 row-kernel segments of 128, one per
// D-lane group of its 8 waves), so the second reader of every line finds it in the Infinity Cache
// (or L2) instead of HBM (splitter.h:46-60 fans the block out with one memcpy per consumer; here no
// consumer copies it). Pass A's input loads keep the default cache policy (CP) for that reason.
// The stage's outputs are bit-identical to fir_rows_kernel's (the same fir_rows_segment; only the
// row batch is smaller, to fit the spectrum's 128-VGPR budget, which leaves the summation order
// unchanged). The launch that carries the last pass B also has the stage's history workgroup.
struct VfoWork {
    FirArgs a;       // stage 1 (vfo_stage1_prepare)
    int frame0;      // global frame index of this launch's first pass-A frame
    int hist;        // this launch's last workgroup writes the stage's next-call history
};

// The segments are those fir_rows_kernel runs (32 outputs, launch_rows): a segment's xlator phasors
// are nco(segment start) x e^{i w D r}, so the segment boundaries are part of the arithmetic, and equal
// boundaries give equal bits. Quarter q of frame g's stage-1 outputs: 16 segments of 32 outputs, one
// per D-lane group, one row batch each -- a workgroup that lives one load round, like the column
// tiles beside it.
__device__ __forceinline__ void vfo_quarter_block(const VfoWork& v, int g, int q) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long seg = (long long)(v.frame0 + g) * 64 + q * 16 + wave * 2 + (lane >> 5);
    fir_rows_segment<32, 5, true, false, 32, 32, true>(v.a, seg, lane);
}

// XCD-grouped frames. Workgroups x, x + 8, x + 16, ... run on one XCD (round-robin dispatch, speed
// only), so after the nB pass-B tiles workgroup nB + 8 k + x takes item k % 12 of frame 8 (k / 12) + x:
// a frame's 4 stage-1 quarter workgroups (items 0-3, dispatched first) and its 8 column tiles share
// one XCD's L2 and live the same load round, so the second reader of each IQ line finds it in that
// L2 instead of crossing the fabric. C5 PMC 36.7 -> 30.4 B/sample (fetch 23.5 -> 17.1), group 1.743
// -> 1.696 ms (r4g). Measured and removed: a frame's 9 workgroups consecutive over all
// XCDs (fetch 26.1 B), one whole-frame stage-1 workgroup per frame (L2 turned over), the passes
// interleaved per XCD (noise), streaming pass-A input loads (the quarters' L2 hits need the lines).
template <bool ZM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void fft_vfo_kernel(
    int nB, const float2* __restrict__ scratchB, int framesB, float* __restrict__ outB, float* __restrict__ zoomB,
    const float2* __restrict__ in, long long frameStride, int framesA, const float* __restrict__ win, int nz,
    int logN, const float2* __restrict__ tw1, const float2* __restrict__ tw2, const float2* __restrict__ tfull,
    float2* __restrict__ scratchA, VfoWork v) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if (v.hist && blockIdx.x == gridDim.x - 1) {   // the stage's history carry (fir.h:80)
        (void)fir_hist_block<float2, true, false>(v.a);
        return;
    }
    if ((int)blockIdx.x < nB) {
        passB_tile<256, 32, ZM>(lds, blockIdx.x, scratchB, framesB, 256, logN, tw2, outB, zoomB);
        return;
    }
    const int i = blockIdx.x - nB, k = i >> 3, kk = k % 12;
    const int g = 8 * (k / 12) + (i & 7);
    if (g >= framesA) return;   // (padding of the last group of 8 frames)
    if (kk < 4) {
        vfo_quarter_block(v, g, kk);
        return;
    }
    passA_tile<256, 32, 0>(lds, g * 8 + kk - 4, in, frameStride, framesA, win, nz, 256, logN, tw1, tfull, scratchA);
}

// ---- one-pass 64k spectrum: no intermediate leaves the CU ----------------------------------------
// N = 65536 as four 16,384-point transforms (one radix-4 decimation-in-frequency step). Item (f, r)
// computes the bins 4 m + r of frame f:
//   X[4 m + r] = sum_{n < M} W_M^(n m) y_r[n],   y_r[n] = W_N^(n r) sum_{j < 4} W_4^(j r) w[n + M j] x[n + M j],
// M = 16384. The 16k transform is M = 32 x 32 x 16 on one CU (512 threads, one workgroup per CU):
//   stage 1 (registers): thread t holds y_r[t + 512 i], i < 32, straight from its loads (the four
//     quarters combined as they arrive); a radix-32 DFT over i and the twiddle W_M^(t k2) W_N^(t r)
//     = W_N^(t (4 k2 + r)) give A[t][k2];
//   stage 2 (LDS): per (k2, t0), a radix-32 DFT over t1 of A[t0 + 16 t1][k2], twiddle W_512^(t0 q1);
//   stage 3 (LDS): per (k2, q1), a radix-16 DFT over t0 -> Y[k2 + 32 q1 + 1024 q2], dB, store.
// A frame's two workgroups (quarters 0-1 and 2-3, the pair's bins 4 m + r0, 4 m + r0 + 1 adjacent so
// the dB rows leave as 8-byte pairs) sit on one XCD (blocks of 8 frames under round-robin dispatch, for
// speed only), so the frame is fetched from HBM once per reader and its second read is mostly served by
// that XCD's L2. The rows stream into LDS by LDS-DMA through a ring of row sets (below). The default
// since round 5 (C5 group 1.51 ms, 20.9 B/sample of fabric traffic, against 1.63 ms and 30.4 B for the
// two-pass launches). Rejected forms: one item per
// workgroup (1.89 ms), a persistent software-pipelined quarter-per-workgroup walk (2.06 ms, spills), the
// VFO half inside the row loop (1.60-1.91 ms).
// LDS image: 32 rows k2 of 544 used float2 (stage 1: column pad16(t); stage 2: column 17 q1 +
// (t0 ^ ((k2 >> 1) & 15))), row stride 560 (= 16 mod 32): every stage-2/3 access of a half-wave hits
// 32 distinct 8-byte bank pairs.
namespace op1 {
constexpr int M = 16384;
constexpr int RS = 560;                 // LDS row stride (float2)
constexpr int TW512 = 32 * RS;          // W_512^(t0 q1) at [q1][t0]
constexpr int W128 = TW512 + 512;       // W_128^(r i), i < 32
constexpr int W128D = (W128 + 64) * 8;   // (bytes) fp64 W_128^(r i), r = r0, r0 + 1, i < 32
constexpr int LDS_BYTES = W128D + 64 * 16;
constexpr int TAB = 512 + 128;          // device table: [q1][t0] W_512^(t0 q1), [r][i] W_128^(r i)
constexpr int TAB64 = 2048 + 128;       // fp64 table: W_N^m (m < 2048), [r][i] W_128^(r i)
}

// x w, rounded on its own: never contracted into the radix-4 adds that follow (left to the compiler,
// whether it fused x w + u into one fma differed between kernel instantiations, so the one-pass rows
// with and without the fused VFO differed in the last bit)
__device__ __forceinline__ float2 wmul(float2 x, float w) {
#pragma clang fp contract(off)
    return make_float2(x.x * w, x.y * w);
}

// 32-point DFT as 2 x 16 (even / odd halves), natural order in and out
__device__ __forceinline__ void dft32(float2* v) {
    constexpr float C[16] = {1.0f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                             0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                             0.19509032201612826785f, 0.0f, -0.19509032201612826785f, -0.38268343236508977173f,
                             -0.55557023301960222474f, -0.70710678118654752440f, -0.83146961230254523708f,
                             -0.92387953251128675613f, -0.98078528040323044913f};
    float2 e[16], o[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        e[i] = v[2 * i];
        o[i] = v[2 * i + 1];
    }
    dft16(e);
    dft16(o);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        float2 t = o[k];
        if (k == 8) t = mul_negi(t);
        else if (k) t = cmul(t, make_float2(C[k], -C[(k + 8) & 15] * (k < 8 ? -1.0f : 1.0f)));   // W_32^k
        v[k] = cadd(e[k], t);
        v[k + 16] = csub(e[k], t);
    }
}

// Stage-1 twiddles W_N^(t (4 k2 + r)) by an fp64 recurrence W_N^(t r) (W_N^(4 t))^k2 from two values of
// an fp64 table, rounded once (against one exact table value each, 128 KB per item from L2: 1.942 ->
// 1.893 ms, r41pb).
constexpr int k1pSlots = 5;   // LDS-DMA ring slots (24 KiB row sets) in the image region
constexpr int k1pPB = 2;   // (PAD) sample rows per load batch: 4 PB loads of x and of w, two batches in flight
#ifndef SDRGPU_1P_ABL
#define SDRGPU_1P_ABL 0   // (ablation builds, wrong results, timing only) 1: no loads, 2: no transforms, 4: no VFO,
                          // 8: fp32 stage-1 twiddles, 16: no dB / stores
#endif
// The ring's first k1pSlots - 1 row sets are issued before the VFO half, so they land while it computes
// (C5 group 1.518 -> 1.499 ms, same bits, r6g; A/B builds: 0)
#ifndef SDRGPU_1P_EARLYDMA
#define SDRGPU_1P_EARLYDMA 1
#endif
#ifndef SDRGPU_1P_EARLYW128
#define SDRGPU_1P_EARLYW128 1   // (A/B builds: 0) quarter r0 + 1's W_128 products during quarter r0's stage-3
                                // reads: C5 group 1.4748 / 1.4833 vs 1.4782 / 1.4880 ms (r7t, r7u), same bits
#endif
#ifdef SDRGPU_1P_TIMING   // (measurement builds) per-workgroup phase stamps of wave 0
__device__ unsigned long long g_1p_t[16384 * 8];
#define T1P(k)                                                                                    \
    do {                                                                                          \
        if (threadIdx.x == 0 && blockIdx.x < 16384) g_1p_t[blockIdx.x * 8 + (k)] = clock64();     \
    } while (0)
#else
#define T1P(k) do {} while (0)
#endif
// (the quarter pair of a workgroup: its VFO share, 32 segments of the frame's 64)
__device__ __forceinline__ void vfo_half_block(const VfoWork& v, int g, int p) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll 1
    for (int k = 0; k < 2; k++) {
        const long long seg = (long long)(v.frame0 + g) * 64 + p * 32 + k * 16 + wave * 2 + (lane >> 5);
        fir_rows_segment<32, 5, true, false, 32, 32, true>(v.a, seg, lane);
    }
}
template <bool ZM, bool VFO, bool PAD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1))) void fft_1p_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz,
    const float2* __restrict__ tab, const double2* __restrict__ tab64, float* __restrict__ out, float* __restrict__ zpart,
    VfoWork v) {
    using op1::M;
    using op1::RS;
    using op1::TW512;
    using op1::W128;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if constexpr (VFO) {
        if (v.hist && blockIdx.x == gridDim.x - 1) {   // the stage's history carry (fir.h:80)
            (void)fir_hist_block<float2, true, false>(v.a);
            return;
        }
    }
    const int b = blockIdx.x, k = b >> 3;
    const int f = 8 * (k >> 1) + (b & 7), p = k & 1, r0 = 2 * p;   // quarters r0, r0 + 1 of frame f
    if (f >= frames) return;
    T1P(0);
    // the frame's first reader (HBM): half of the VFO's stage 1. (Measured and rejected, r5: the VFO
    // inside the row loop -- from the LDS ring, 1.91 ms; as two batches of segments right after the
    // ring fetched their lines, 1.60 ms; after the loop / between the transforms, spilled)
    constexpr bool kDma = !PAD && !(SDRGPU_1P_ABL & 1);   // whole frames: the LDS-DMA row ring below
    constexpr bool kVfo = VFO && !(SDRGPU_1P_ABL & 4);
    if constexpr (kVfo && !(kDma && SDRGPU_1P_EARLYDMA)) vfo_half_block(v, f, p);
    T1P(1);
    // Index arithmetic is recomputed from a laundered thread index where it is used: left alone, the
    // compiler hoists the loop-invariant load / LDS / store addresses and spills them.
    auto tid = [] {
        int u = threadIdx.x;
        asm volatile("" : "+v"(u));
        return u;
    };
    {
        const int t = threadIdx.x;
        lds[TW512 + t] = tab[t];
        if (t < 64) reinterpret_cast<double2*>(reinterpret_cast<char*>(lds) + op1::W128D)[t] = tab64[2048 + 32 * (r0 + (t >> 5)) + (t & 31)];
    }
    // stage 1: y_r for r = r0 (even) and r0 + 1 (odd) from the four quarters: y_r = A_r + W_4^r q_r with
    // A_r = u0 + s_r u2, q_r = u1 + s_r u3, s_r = (-1)^r; W_4^r in {1, -i, -1, i} as (fx, fy), one of
    // them 0, the other +-1 (exact products). The pair's bins 4 m + r0, 4 m + r0 + 1 are adjacent: the
    // dB rows leave as 8-byte pairs.
    const float fxa = p ? -1.0f : 1.0f, fyb = p ? 1.0f : -1.0f;   // W_4^r0 = (fxa, 0), W_4^(r0+1) = (0, fyb)
    auto combine2 = [&](const float2 (&u)[4], float2& ya, float2& yb) {
        const float2 aa = cadd(u[0], u[2]), qa = cadd(u[1], u[3]), ab = csub(u[0], u[2]), qb = csub(u[1], u[3]);
        ya = make_float2(fmaf(fxa, qa.x, aa.x), fmaf(fxa, qa.y, aa.y));     // aa + W_4^r0 qa (exact products)
        yb = make_float2(fmaf(-fyb, qb.y, ab.x), fmaf(fyb, qb.x, ab.y));    // ab + W_4^(r0+1) qb
    };
    const unsigned lim = PAD ? (unsigned)nz : 65536u;     // (PAD: range-checked loads, 0 past nz)
    const __amdgpu_buffer_rsrc_t rw = brsrc(win, lim * 4u);
    const __amdgpu_buffer_rsrc_t rx = brsrc(in + (long long)f * frameStride, lim * 8u);
    constexpr int PB = k1pPB, NB = 32 / PB;
    float2 za[32], zb[32];
    float2 xv[2][PB][4];   // the load ring: two batches of PB sample rows x 4 quarters
    float wv[2][PB][4];
    auto issue = [&](auto bbc) {
        constexpr int bb = decltype(bbc)::value;
        const int t = tid();
#pragma unroll
        for (int ii = 0; ii < PB; ii++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int n0 = 512 * (PB * bb + ii) + M * j;
                if constexpr (PAD) {   // the offset in the per-lane part: the range check ignores soffset
                    xv[bb & 1][ii][j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, (t + n0) * 8, 0, 0));
                    wv[bb & 1][ii][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, (t + n0) * 4, 0, 0));
                } else {               // the row offset rides in soffset
                    xv[bb & 1][ii][j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, t * 8, n0 * 8, 0));
                    wv[bb & 1][ii][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, t * 4, n0 * 4, 0));
                }
            }
    };
    // combine batch bb into za / zb, then reuse its ring slot for batch bb + 2
    auto step = [&](auto bbc) {
        constexpr int bb = decltype(bbc)::value;
#pragma unroll
        for (int ii = 0; ii < PB; ii++) {
            float2 u[4];
#pragma unroll
            for (int j = 0; j < 4; j++) u[j] = wmul(xv[bb & 1][ii][j], wv[bb & 1][ii][j]);
            combine2(u, za[PB * bb + ii], zb[PB * bb + ii]);

        }
        if constexpr (bb + 2 < NB) issue(std::integral_constant<int, bb + 2>{});
        __builtin_amdgcn_sched_barrier(0);
    };
    if constexpr (SDRGPU_1P_ABL & 1) {
#pragma unroll
        for (int i = 0; i < 32; i++) {
            za[i] = make_float2((float)(tid() + i), (float)i);
            zb[i] = make_float2((float)i, (float)(tid() - i));
        }
    } else if constexpr (PAD) {   // zero-padded or unaligned frames: range-checked register loads through the ring
        issue(std::integral_constant<int, 0>{});
        issue(std::integral_constant<int, 1>{});
        static_for<0, NB>(step);
    } else {
        // Whole frames: the rows stream into LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
        // instruction, 16 B per lane, no VGPRs) through a ring of k1pSlots row sets in the (still
        // unused) image region. A row set = row i of the four quarters: x 4 x 4 KiB, w 4 x 2 KiB = 24
        // wave instructions, 3 per wave. 8- and 4-byte register loads reached ~25 GB/s per CU here
        // (the r5 phase stamps: the load phase was 60% of a workgroup's life); 16-B accesses are the
        // L2 path's full rate. Each wave waits for its own pieces of row set i (counted vmcnt: the
        // younger row sets stay in flight), a raw s_barrier makes every wave's pieces visible and
        // frees slot i - 1, the wave issues row set i + k1pSlots - 1 into that slot, then every thread
        // reads its sample t of the four quarters (ds_read_b64 / _b32, conflict-free) and combines.
        constexpr int S = k1pSlots, SLOT = 24576;
        typedef __attribute__((address_space(3))) char lchar;
        const unsigned ldsBase = (unsigned)(size_t)(lchar*)lds;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        // this wave's 3 pieces of every row set (wave-uniform): global byte base of row 0, row step,
        // offset in the slot. x pieces: 128 samples of one quarter (16 B = 2 samples per lane); w
        // pieces: 256 values (16 B = 4 per lane)
        const char* gb[3];
        unsigned rstep[3], loff[3];
        const float2* xf = in + (long long)f * frameStride;
#pragma unroll
        for (int e = 0; e < 3; e++) {
            const int m = 3 * wave + e;
            const int jx = m >> 2, cx = m & 3, jw = (m - 16) >> 1, cw = (m - 16) & 1;
            gb[e] = m < 16 ? reinterpret_cast<const char*>(xf + M * jx + 128 * cx)
                           : reinterpret_cast<const char*>(win + M * jw + 256 * cw);
            rstep[e] = m < 16 ? 512u * 8u : 512u * 4u;
            loff[e] = m < 16 ? (unsigned)(4096 * jx + 1024 * cx) : (unsigned)(16384 + 2048 * jw + 1024 * cw);
        }
        // LDS-DMA in inline asm: the compiler neither counts it (the waits below are explicit) nor
        // drains it with a vmcnt(0) before every LDS read it cannot prove disjoint (it did with the
        // builtin: no row set stayed in flight); M0 set and restored in the same statement
        // (the row pointers advance by one row step per row set, laundered: left alone, the compiler
        // precomputes all 96 pointers and spills them to VGPR lanes)
        auto dma = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const unsigned lane16 = (unsigned)(tid() & 63) * 16u;
#pragma unroll
            for (int e = 0; e < 3; e++) {
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
        if constexpr (kVfo && SDRGPU_1P_EARLYDMA) vfo_half_block(v, f, p);   // (its loads wait behind the ring's)
        static_for<0, 32>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int younger = (S - 2 < 31 - i) ? S - 2 : 31 - i;   // row sets issued after i, in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * younger) : "memory");   // this wave's pieces of row set i
            __builtin_amdgcn_s_barrier();   // every wave's pieces landed; every read of slot i - 1 done
            asm volatile("" ::: "memory");
            if constexpr (i + S - 1 < 32) dma(std::integral_constant<int, i + S - 1>{});
            const int t = tid();
            const char* slot = reinterpret_cast<const char*>(lds) + (i % S) * SLOT;
            float2 u[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float2 xx = *reinterpret_cast<const float2*>(slot + 4096 * j + 8 * t);
                const float ww = *reinterpret_cast<const float*>(slot + 16384 + 2048 * j + 4 * t);
                u[j] = wmul(xx, ww);
            }
            combine2(u, za[i], zb[i]);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    T1P(2);
    float* zf = ZM ? zpart + ((long long)f << 12) : nullptr;   // [f][workgroup][2048]
    const __amdgpu_buffer_rsrc_t ro = brsrc(out + ((long long)f << 16), 65536u * 4u);
    // the 16k transform of quarter r = r0 + h from its stage-1 registers z. Quarter r0's dB values wait in
    // registers (dA) for quarter r0 + 1's, and the two leave as one 8-byte store per bin pair.
    float dA[2][16];
    // (the VFO instantiations only: the others spill two registers with it)
    constexpr bool kEarlyW = SDRGPU_1P_EARLYW128 && VFO;
    auto w128mul = [&](float2 (&z)[32], int hh) {
        const double2* w128 = reinterpret_cast<const double2*>(reinterpret_cast<const char*>(lds) + op1::W128D) + 32 * hh;
#pragma unroll
        for (int i = 1; i < 32; i++) {
            const double2 q = zmul(make_double2(z[i].x, z[i].y), w128[i]);
            z[i] = make_float2((float)q.x, (float)q.y);
        }
    };
    auto transform = [&](auto hc, float2 (&z)[32]) {
        constexpr int h = decltype(hc)::value;
        const int r = r0 + h;
        __syncthreads();   // (h = 0: the tables staged; h = 1: quarter r0's stage-3 reads of the image are done)
        {   // stage-1 finish: W_128^(r i), radix 32, W_N^(t (4 k2 + r)), into the LDS image
            const int t = tid();
            // W_128^(r i) = W_N^(512 r i) as an fp64 product of the fp64 twiddle, rounded once. As an fp32
            // product with an fp32 table (two roundings) the near-peak bins of tonal frames were 1-2 ulp
            // off more often than pocketfft's (AES17: 7 of 22 bins beyond 1 ulp vs pocketfft's 4; 2 in
            // this form), +2.7% kernel time (r5x-r5z; applied at the combine instead: +5%)
            // (also for quarter 0, where W = 1 and the product is exact: a branch around it spilled)
            if constexpr (!(kEarlyW && h == 1)) w128mul(z, h);
            dft32(z);
            // W_N^(t r) (W_N^(4 t))^k2 as two independent fp64 chains over even / odd k2 (a serial chain of
            // 31 fp64 complex products was the stage's critical path)
            const double2 st = tab64[4 * t];
            double2 ce = tab64[t * r], co = zmul(ce, st);
            const double2 st2 = zmul(st, st);
            float2* row = lds + pad16(t);
            if constexpr (SDRGPU_1P_ABL & 8) {
                const float2 cf = make_float2((float)ce.x, (float)ce.y), sf = make_float2((float)st.x, (float)st.y);
#pragma unroll
                for (int k2 = 0; k2 < 32; k2++) row[k2 * RS] = cmul(z[k2], k2 & 1 ? sf : cf);
            } else
#pragma unroll
            for (int k2 = 0; k2 < 32; k2 += 2) {
                row[k2 * RS] = cmul(z[k2], make_float2((float)ce.x, (float)ce.y));
                row[(k2 + 1) * RS] = cmul(z[k2 + 1], make_float2((float)co.x, (float)co.y));
                if (k2 < 30) {
                    ce = zmul(ce, st2);
                    co = zmul(co, st2);
                }
            }
        }
        __syncthreads();
        if constexpr (h == 0) T1P(5);
        {   // stage 2: (k2, t0) = (t >> 4, t & 15)
            const int t = tid();
            const int k2 = t >> 4, t0 = t & 15;
            float2 a[32];
            const float2* src = lds + k2 * RS + t0;
#pragma unroll
            for (int t1 = 0; t1 < 32; t1++) a[t1] = src[17 * t1];
            dft32(a);
#pragma unroll
            for (int q1 = 1; q1 < 32; q1++) a[q1] = cmul(a[q1], lds[TW512 + 16 * q1 + t0]);
            __syncthreads();
            float2* dst = lds + k2 * RS + (t0 ^ ((k2 >> 1) & 15));
#pragma unroll
            for (int q1 = 0; q1 < 32; q1++) dst[17 * q1] = a[q1];
        }
        __syncthreads();
        T1P(6 + h);
        // stage 3: (k2, q1) = (e & 31, e >> 5), e = t, t + 512. The thread holds the same (k2, q1) bins
        // of both quarters, so quarter r0 + 1 stores (dA, dB) at float 4 (k2 + 32 q1 + 1024 q2) + r0
        // (8-byte aligned: r0 even) through a buffer resource, the q2 step in soffset
        static_for<0, 2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            const int t = tid();
            const int pe = t + 512 * e, k2 = pe & 31, q1 = pe >> 5, sw = (k2 >> 1) & 15;
            float2 c3[16];
            const float2* src = lds + k2 * RS + 17 * q1;
#pragma unroll
            for (int t0 = 0; t0 < 16; t0++) c3[t0] = src[t0 ^ sw];
            // quarter r0 + 1's W_128 products (registers only) while these reads are in flight
            if constexpr (kEarlyW && h == 0 && e == 0) w128mul(zb, 1);
            dft16(c3);
            if constexpr (SDRGPU_1P_ABL & 16) {
                if constexpr (h == 1) {
                    float acc = 0.0f;
#pragma unroll
                    for (int q2 = 0; q2 < 16; q2++) acc += c3[q2].x + c3[q2].y;
                    out[(f << 16) + pe] = acc;
                }
            } else if constexpr (h == 0) {
#pragma unroll
                for (int q2 = 0; q2 < 16; q2++) dA[e][q2] = db_of(c3[q2]);
            } else {
                float dv[16];
                const unsigned vo = (unsigned)(4 * (k2 + 32 * q1) + r0) * 4u;
#pragma unroll
                for (int q2 = 0; q2 < 16; q2++) {
                    dv[q2] = db_of(c3[q2]);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(bu2, make_float2(dA[e][q2], dv[q2])), ro, vo,
                                                          q2 * 4096 * 4, 0);
                }
                if constexpr (ZM) {   // max over both quarters and the 8 lanes k2 & 7: zoom column (k2 >> 3) + 4 q1 + 128 q2
#pragma unroll
                    for (int q2 = 0; q2 < 16; q2++) dv[q2] = fmaxf(dA[e][q2], dv[q2]);
                    const int lane = t & 63;
                    tr_step<1, 8>(dv, lane);
                    tr_step<2, 4>(dv, lane);
                    tr_step<4, 2>(dv, lane);
                    // lane bits (b0 b1 b2) now select q2 = 8 b0 + 4 b1 + 2 b2 + i in dv[i], i < 2
                    const int q2 = ((lane & 1) << 3) | ((lane & 2) << 1) | (lane & 4) >> 1;
                    float* zp = zf + ((long long)p << 11) + (k2 >> 3) + 4 * q1 + 128 * q2;
                    zp[0] = dv[0];
                    zp[128] = dv[1];
                }
            }
        });
    };
    if constexpr (SDRGPU_1P_ABL & 2) {
        float2 acc = make_float2(0.0f, 0.0f);
#pragma unroll
        for (int i = 0; i < 32; i++) acc = cadd(acc, cadd(za[i], zb[i]));
        out[(f << 16) + tid()] = acc.x + acc.y;
        return;
    }
    transform(std::integral_constant<int, 0>{}, za);
    T1P(3);
    transform(std::integral_constant<int, 1>{}, zb);
    T1P(4);
}

#ifdef SDRGPU_1P_TIMING
extern "C" int sdrgpu_debug_1p_times(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_1p_t), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

// zoom[f][o] = max over the two workgroups' partial maxima (fft_1p_kernel's ZM): 4 columns per thread
// as 16-B loads / stores (one element per thread took 20.8 us per 2^28-sample step); 256 threads per
// workgroup (both launches below)
static_assert(TAIL_NT_BIG == 256, "zoom_fold_block's indexing and the fold's block count assume 256 threads");
__device__ __forceinline__ void zoom_fold_block(const float* __restrict__ zpart, int frames, float* __restrict__ zoom, int blk) {
    const long long i = ((long long)blk * 256 + threadIdx.x) * 4;
    if (i >= (long long)frames * 2048) return;
    const long long f = i >> 11, o = i & 2047;
    const float4 a = *reinterpret_cast<const float4*>(zpart + (f << 12) + o);
    const float4 b = *reinterpret_cast<const float4*>(zpart + (f << 12) + 2048 + o);
    const float4 m = make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
    if (((uintptr_t)zoom & 15) == 0) {   // (wave-uniform)
        *reinterpret_cast<float4*>(zoom + i) = m;
    } else {
        zoom[i] = m.x; zoom[i + 1] = m.y; zoom[i + 2] = m.z; zoom[i + 3] = m.w;
    }
}
__global__ __launch_bounds__(256) void fft_1p_zoom_kernel(const float* __restrict__ zpart, int frames, float* __restrict__ zoom) {
    zoom_fold_block(zpart, frames, zoom, blockIdx.x);
}
// The VFO's later stages (fir_tail_kernel's workgroups, first) and the zoom fold (the rest) in one launch:
// the tail is latency-bound (dependent fmaf chains, barriers between stages), the fold moves 96 MB per C5
// step, so the fold's workgroups fill the CUs the tail leaves idle (both need only the one-pass
// launch's outputs). Same code, same bits as the two launches.
__global__ __launch_bounds__(TAIL_NT_BIG) void fft_1p_tail_fold_kernel(TailArgs t, const float* __restrict__ zpart, int frames,
                                                                         float* __restrict__ zoom) {
    extern __shared__ __attribute__((aligned(16))) float2 XS[];
    __shared__ TailGeom gs[TAIL_MAXS];
    const int w = blockIdx.x;
    if (w < t.G) fir_tail_block<TAIL_K_BIG, TAIL_NT_BIG>(t, w, w == t.G - 1, XS, gs);
    else zoom_fold_block(zpart, frames, zoom, w - t.G);
}

// ---- the front end's per-block launch: pass A (frame straddling two pushes read in place) + the
// VFO's first stage + its history carry + the tail copy, one launch (sdrgpu_frontend_*): the block is
// small (a reference-size block has ~5 frames and 9,600 stage-1 outputs), so the stage's segments
// are the small-call ones (32 outputs, one row batch each: 300 segments, 19 workgroups of 16).
struct VfoCall {
    FirArgs a;
    int blocks;      // stage-1 workgroups (16 segments each)
};
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void fft_passA_vfo_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz, int N2,
    int logN, const float2* __restrict__ tw, const float2* __restrict__ tfull, float2* __restrict__ scratch,
    const float2* __restrict__ headp, int nh, SideCopy side, VfoCall v) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int ntiles = (N2 / 32) * frames;
    int b = blockIdx.x;
    if (b < ntiles) {
        passA_tile<256, 32>(lds, b, in, frameStride, frames, win, nz, N2, logN, tw, tfull, scratch, headp, nh);
        return;
    }
    b -= ntiles;
    if (b < v.blocks) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        fir_rows_segment<32, 5, true, false, 32, 32, true>(v.a, ((long long)b * 8 + wave) * 2 + (lane >> 5), lane);
        return;
    }
    b -= v.blocks;
    if (b == 0) {   // the stage's history carry (fir.h:80)
        fir_hist_copy<float2, true, false>(v.a);
        return;
    }
    const int w = b - 1, nw = gridDim.x - ntiles - v.blocks - 1;   // spare workgroups: the side copies
    for (int k = 0; k < side.count; k++)
        for (int i = w * blockDim.x + threadIdx.x; i < side.n[k]; i += nw * blockDim.x) side.dst[k][i] = side.src[k][i];
}

// ... and its pass-B launch: the pass-B tiles + the VFO's tail workgroups (fir_tail_block on the
// first 256 threads of a 512-thread block), one launch for both (the tail needs only the stage-1
// output the pass-A launch wrote)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void fft_passB_tail_kernel(
    const float2* __restrict__ scratch, int frames, int N1, int logN, const float2* __restrict__ tw, float* __restrict__ out,
    TailArgs t) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ TailGeom gs[TAIL_MAXS];
    const int ntiles = (N1 / 32) * frames;
    if ((int)blockIdx.x < ntiles) {
        passB_tile<256, 32, false>(lds, blockIdx.x, scratch, frames, N1, logN, tw, out, nullptr);
        return;
    }
    const int w = blockIdx.x - ntiles;
    fir_tail_block<TAIL_K, TAIL_NT>(t, w, w == t.G - 1, lds, gs);
}

// ---------------------------------------------------------------- host side
struct FftPlan {
    int device = 0, N = 0, logN = 0, nz = 0;
    int N1 = 0, N2 = 0;               // two-pass split (N1 * N2 = N); N1 = 0 -> single pass
    DevBuf win, tw1, tw2, tfull, scratch, scratch2;
    int chunkFrames = 1;
    int sa = 16, sb = 32;             // pass-A columns / pass-B rows per workgroup (32 / 32 on the 64k plan)
    float2* cur = nullptr;            // scratch buffer of the chunk being launched
    int sa2 = 0;                      // paired pass-A columns per workgroup (0: paired kernel off)
    int gridA = 0, gridB = 0;         // the persistent 1M passes' grids (resident workgroups)
    DevBuf wt;                        // fp64 W_N^(256 j), W_N^j (j < 256) for the 1M pass A
    hipStream_t own = nullptr;
    PinnedBuf pin_in, pin_out;
    DevBuf dev_in, dev_out;
    // merged pass-B(c) + pass-A(c+1) launches (64k split): one launch boundary per chunk
    // instead of two; 1.87 -> 1.73 ms per 2^28 samples (A/B on one box). SDRGPU_FFT_MERGE=0 off.
    int merge = 1;
    StreamOrder order;                // scratch is per plan: calls on different streams are serialised
    sdrgpu_zoom* zoom = nullptr;      // execute_zoom's unfused zoom (sizes other than N / 32)
    int zoomSize = 0;
    Fft64Plan* f64 = nullptr;         // sdrgpu_fft_set_precision(h, 1): the fp64-interior kernels (fft64.hip)
    // sdrgpu_fft_set_timing: HIP events around each call's spectrum launch group (the fused VFO
    // stage included, the VFO's later stages not), a ring of kTimed calls read by sdrgpu_fft_group_times
    static constexpr int kTimed = 256;
    bool timing = false;
    hipEvent_t tev[kTimed][2] = {};
    long long tcalls = 0;
    int vfoFuse = 1;                  // the VFO's first stage inside the spectrum launches
    int onepass = 0;                  // the 64k plan's one-pass kernel (fft_1p_kernel): 0 never, 1 always, 2 calls of
                                      // >= k1pMinFrames frames (SDRGPU_FFT_1P, tuning)
    DevBuf tab1p, tab1p64, zpart;
    // sdrgpu_fft_set_tail_stream: the fused VFO's later stages and the zoom fold of
    // sdrgpu_fft_execute_(zoom_)vfo_dev run on this stream, overlapping the next call's spectrum launch.
    // Their inputs (the VFO's stage-1 outputs, the zoom partials) are double-buffered per call parity;
    // call k + 2's spectrum launch waits for call k's tail (tdone) before rewriting its buffers.
    hipStream_t tailStream = nullptr;
    DevBuf s1T[2], zpartT[2];
    hipEvent_t gdone[2] = {}, tdone[2] = {};
    bool tdoneRec[2] = {};
    long long tcallsT = 0;
};
static int time_mark(FftPlan& p, int which, hipStream_t s) {
    if (!p.timing) return SDRGPU_OK;
    SDRGPU_HIP(hipEventRecord(p.tev[p.tcalls % FftPlan::kTimed][which], s));
    if (which == 1) p.tcalls++;
    return SDRGPU_OK;
}

// t[m] = exp(-2 pi i (m * step) / L) for m < count (fp64 -> float)
static int make_twiddles(DevBuf& b, int L, int count = -1, int step = 1) {
    if (count < 0) count = L;
    std::vector<float2> t(count);
    for (int m = 0; m < count; m++) {
        double a = -2.0 * M_PI * (double)((long long)m * step % L) / (double)L;
        t[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    SDRGPU_CHECK(b.ensure(sizeof(float2) * count));
    SDRGPU_HIP(hipMemcpy(b.p, t.data(), sizeof(float2) * count, hipMemcpyHostToDevice));
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
static int launch_passA(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s,
                        const float2* headp = nullptr, int nh = 0, const SideCopy* side = nullptr) {
    auto k = fft_passA_kernel<L, S>;
    size_t lds = sizeof(float2) * (S * Lds<L>::LS + (L == 256 ? L + 256 : 0));   // + stage twiddles (256-point columns)
    SDRGPU_CHECK(set_lds(k, lds));
    SideCopy sc{};
    int spare = 0;
    if (side && side->count > 0) {
        sc = *side;
        int mx = 0;
        for (int i = 0; i < sc.count; i++) mx = std::max(mx, sc.n[i]);
        spare = std::min(64, (mx + S * L / 16 * 4 - 1) / (S * L / 16 * 4));   // ~4 elements per thread
        spare = std::max(spare, 1);
    }
    const int g = (p.N2 / S) * frames + spare;
    hipLaunchKernelGGL(k, dim3(g), dim3(S * L / 16), lds, s, in, stride, frames, p.win.as<float>(), p.nz, p.N2,
                       p.logN, p.tw1.as<float2>(), p.tfull.as<float2>(), p.cur, headp, nh, sc);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int L, int S>
static int launch_passA2(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    if (p.N2 % S) { set_error("fft: N2 %d not a multiple of %d columns", p.N2, S); return SDRGPU_ESTATE; }
    auto k = fft_passA2_kernel<L, S>;
    size_t lds = sizeof(float2) * (S * Lds<L>::LS + L);
    SDRGPU_CHECK(set_lds(k, lds));
    const int g = (p.N2 / S) * frames;
    hipLaunchKernelGGL(k, dim3(g), dim3(S / 2 * L / 16), lds, s, in, stride, frames, p.win.as<float>(), p.nz, p.N2,
                       p.logN, p.tw1.as<float2>(), p.tfull.as<float2>(), p.cur);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int L, int S, bool ZM = false>
static int launch_passB(const FftPlan& p, int frames, float* out, hipStream_t s, float* zoom = nullptr) {
    auto k = fft_passB_kernel<L, S, ZM>;
    size_t lds = sizeof(float2) * (S * Lds<L>::LS + (L >= 256 ? 256 : 0));   // + passB_tile's tw16
    SDRGPU_CHECK(set_lds(k, lds));
    const int g = (p.N1 / S) * frames;
    hipLaunchKernelGGL(k, dim3(g), dim3(S * L / 16), lds, s, p.cur, frames, p.N1, p.logN,
                       p.tw2.as<float2>(), out, zoom);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

// merged pass B (chunk c) + pass A (chunk c+1) launches of the 64k split (256 x 256, 32 columns / 32
// rows, one-column pass A). The 1M split's merged form (paired pass A, pass B at 8 rows to match its
// 512 threads) measured 12% SLOWER: pass B loses half its occupancy to pass A's 147 KB of LDS, so the
// 1M transform keeps separate launches.
template <bool ZM>
static int launch_merged(const FftPlan& p, const float2* scratchB, int framesB, float* outB, const float2* in,
                         long long stride, int framesA, float2* scratchA, hipStream_t s, float* zoomB = nullptr) {
    auto k = fft_merged_kernel<256, 32, 256, 32, false, ZM>;
    const size_t lds = sizeof(float2) * (32 * Lds<256>::LS + 256 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    const int nB = 8 * framesB, nA = 8 * framesA;
    hipLaunchKernelGGL(k, dim3(nB + nA), dim3(512), lds, s, nB, scratchB, framesB, outB, zoomB, in, stride, framesA,
                       p.win.as<float>(), p.nz, p.logN, p.tw1.as<float2>(), p.tw2.as<float2>(), p.tfull.as<float2>(),
                       scratchA);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}
static bool merged_supported(const FftPlan& p, bool paired) {
    return !paired && p.N1 == 256 && p.N2 == 256 && p.sa == 32 && p.sb == 32;
}

template <typename K>
static int resident_grid(const FftPlan& p, K k, int threads, size_t lds, int& grid) {
    if (!grid) {
        int per = 0, cus = 0;
        SDRGPU_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, threads, lds));
        SDRGPU_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p.device));
        grid = std::max(1, per) * cus;
    }
    return SDRGPU_OK;
}

// the persistent 1M passes for one chunk (pass B reads pass A's tile-major intermediate)
static int dispatch_1m(FftPlan& p, const float2* xc, long long stride, int nf, float* o, hipStream_t s) {
    {
        auto k = fft_passA_1m_kernel;
        const size_t lds = sizeof(float2) * (16 * Lds<1024>::LS + 1024 + 256);
        SDRGPU_CHECK(set_lds(k, lds));
        SDRGPU_CHECK(resident_grid(p, k, 512, lds, p.gridA));
        const int ntiles = (p.N2 / 16) * nf;
        hipLaunchKernelGGL(k, dim3(std::min(p.gridA, ntiles)), dim3(512), lds, s, xc, stride, nf, p.win.as<float>(), p.nz,
                           p.N2, p.logN, p.tw1.as<float2>(), p.wt.as<double2>(), p.cur);
        SDRGPU_HIP(hipGetLastError());
    }
    auto k = fft_passB_1m_kernel;
    const size_t lds = sizeof(float2) * (8 * kPassB1mLS + 1024 + 256);   // 80,000 B: two workgroups per CU
    SDRGPU_CHECK(set_lds(k, lds));
    SDRGPU_CHECK(resident_grid(p, k, 512, lds, p.gridB));
    const int ntiles = (p.N1 / 8) * nf;
    hipLaunchKernelGGL(k, dim3(std::min(p.gridB, ntiles)), dim3(512), lds, s, p.cur, nf, p.N1, p.logN, p.tw2.as<float2>(), o);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

static bool pipe1m_ok(const FftPlan& p, bool paired) { return paired && p.N1 == 1024 && p.N2 == 1024 && (p.nz % 2) == 0; }

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

// pass-A column FFT length N1 with SA columns per workgroup (8*SA-byte row segments)
static int dispatch_passA(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    switch (p.N1) {
    case 64: return launch_passA<64, 16>(p, in, stride, frames, s);
    case 128: return launch_passA<128, 16>(p, in, stride, frames, s);
    case 256:
        if (p.sa == 32) return launch_passA<256, 32>(p, in, stride, frames, s);
        return launch_passA<256, 16>(p, in, stride, frames, s);
    case 512: return launch_passA<512, 8>(p, in, stride, frames, s);
    case 1024: return launch_passA<1024, 16>(p, in, stride, frames, s);
    }
    set_error("fft: unsupported N1 %d", p.N1);
    return SDRGPU_EARG;
}

// paired-column pass A (16-B accesses; +13% on the 1M transform, slower than the one-column kernel
// at N1 = 256): N1 >= 512, when the input allows 16-B loads
static int dispatch_passA2(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    switch (p.N1) {
    case 512: return launch_passA2<512, 16>(p, in, stride, frames, s);
    case 1024: return launch_passA2<1024, 16>(p, in, stride, frames, s);
    }
    set_error("fft: unsupported paired N1 %d", p.N1);
    return SDRGPU_EARG;
}

static int dispatch_passB(const FftPlan& p, int frames, float* out, hipStream_t s, float* zoom = nullptr) {
    if (zoom) return launch_passB<256, 32, true>(p, frames, out, s, zoom);   // (zoom_fusable checked the plan)
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
    SDRGPU_SET_DEVICE(h->p.device);
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
    SDRGPU_SET_DEVICE(device);
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
        // resident in the Infinity Cache: 128 MB of intermediate per chunk (64 and 192-256 MB
        // measured 2-5% slower for 64k with merged launches; 1M: 2.32 vs 2.39 ms at 64 MB)
        long long chunkMB = 128;
        // the 1M plan (N1 = N2 = 1024): 64 MB = 8 frames, two persistent pass-A tiles per workgroup:
        // C2 1.770 -> 1.724 ms (r4u), 64 / 96 / 128 / 256 MB 1.742 / 1.802 / 1.77 / 2.10 (r4v, r4u; 3
        // and 2 interleaved runs); tile counts that are not a multiple of the grid (4 / 6 frames) are slower
        if (p.N1 == 1024 && p.N2 == 1024) chunkMB = 64;
        if (const char* e = tuning_env("SDRGPU_FFT_CHUNK_MB")) chunkMB = std::max(1, atoi(e));
        // 64k (256 x 256): 32 columns / 32 rows per workgroup (256-B pass-A row segments, 128-B
        // pass-B dB segments, 512 threads, 2 workgroups per CU): the merged spectrum launches
        // take 1.44 vs 1.58 ms per 2^28 samples with 16 / 16 (A/B on one box)
        if (p.N1 == 256 && p.N2 == 256) p.sa = p.sb = 32;
        if (const char* e = tuning_env("SDRGPU_FFT_MERGE")) p.merge = atoi(e);
        p.chunkFrames = std::max(1, (int)((chunkMB << 20) / ((long long)fftSize * 8)));
        // paired-column pass A: +13% on the 1M transform (N1 = 1024), but slower than the
        // one-column kernel at N1 = 256 (64k: 2.05-2.10 vs 1.86 ms per 2^28 samples, A/B on
        // one box), so it is the default only for N1 >= 512
        p.sa2 = p.N1 >= 512 ? 16 : 0;
        // 64k: the one-pass transform (fft_1p_kernel) is the default since r5 (C5 group 1.45 vs 1.63 ms
        // per 2^28 samples for the two-pass launches, A/B on one box); SDRGPU_FFT_1P=0 keeps the latter
        p.onepass = fftSize == 65536 ? 2 : 0;
        if (const char* e = tuning_env("SDRGPU_FFT_1P")) p.onepass = atoi(e);
        if (rc >= 0 && fftSize == 65536) {   // fft_1p_kernel's exact twiddles (op1::TAB)
            std::vector<float2> t(op1::TAB);
            auto w = [&](long long m) {
                const double a = -2.0 * M_PI * (double)(m % fftSize) / (double)fftSize;
                return make_float2((float)std::cos(a), (float)std::sin(a));
            };
            for (int q1 = 0; q1 < 32; q1++)
                for (int t0 = 0; t0 < 16; t0++) t[16 * q1 + t0] = w(128LL * t0 * q1);
            for (int r = 0; r < 4; r++)
                for (int i = 0; i < 32; i++) t[512 + 32 * r + i] = w(512LL * r * i);
            std::vector<double2> t64(op1::TAB64);   // fp64: W_N^m, m < 2048 (the stage-1 twiddle recurrence); W_128^(r i)
            auto w64 = [&](long long m) {
                const double a = -2.0 * M_PI * (double)(m % fftSize) / (double)fftSize;
                return make_double2(std::cos(a), std::sin(a));
            };
            for (int m = 0; m < 2048; m++) t64[m] = w64(m);
            for (int r = 0; r < 4; r++)
                for (int i = 0; i < 32; i++) t64[2048 + 32 * r + i] = w64(512LL * r * i);
            rc = p.tab1p.ensure(sizeof(float2) * t.size());
            if (rc >= 0) rc = p.tab1p64.ensure(sizeof(double2) * t64.size());
            if (rc >= 0 && (hipMemcpy(p.tab1p.p, t.data(), sizeof(float2) * t.size(), hipMemcpyHostToDevice) != hipSuccess ||
                            hipMemcpy(p.tab1p64.p, t64.data(), sizeof(double2) * t64.size(), hipMemcpyHostToDevice) != hipSuccess)) {
                set_error("fft: twiddle upload failed");
                rc = SDRGPU_EHIP;
            }
        }
        if (rc >= 0 && p.N1 == 1024 && p.N2 == 1024) {   // fp64 W_N^(256 j), W_N^j for the 1M pass A
            std::vector<double2> t(512);
            for (int j = 0; j < 256; j++) {
                const double a = -2.0 * M_PI * (double)(256 * j) / (double)fftSize;
                const double b = -2.0 * M_PI * (double)j / (double)fftSize;
                t[j] = make_double2(std::cos(a), std::sin(a));
                t[256 + j] = make_double2(std::cos(b), std::sin(b));
            }
            rc = p.wt.ensure(sizeof(double2) * t.size());
            if (rc >= 0 && hipMemcpy(p.wt.p, t.data(), sizeof(double2) * t.size(), hipMemcpyHostToDevice) != hipSuccess) {
                set_error("fft: twiddle upload failed");
                rc = SDRGPU_EHIP;
            }
        }
        if (rc >= 0) {   // Tfull[k1][n2] = W_N^(n2 k1), exact argument mod N (both pass-A kernels)
            std::vector<float2> t((size_t)fftSize);
            for (int k1 = 0; k1 < p.N1; k1++)
                for (int n2 = 0; n2 < p.N2; n2++) {
                    const long long m = ((long long)n2 * k1) % fftSize;
                    const double a = -2.0 * M_PI * (double)m / (double)fftSize;
                    t[(size_t)k1 * p.N2 + n2] = make_float2((float)std::cos(a), (float)std::sin(a));
                }
            rc = p.tfull.ensure(sizeof(float2) * t.size());
            if (rc >= 0 && hipMemcpy(p.tfull.p, t.data(), sizeof(float2) * t.size(), hipMemcpyHostToDevice) != hipSuccess) {
                set_error("fft: twiddle upload failed");
                rc = SDRGPU_EHIP;
            }
        }
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

// Spectrum arithmetic: 0 = fp32 kernels (default), 1 = fp64 interior (fft64.hip: the fp32 window
// product as the reference forms it, then fp64 butterflies, twiddles, |X|^2 and dB, rounded once)
extern "C" int sdrgpu_fft_set_precision(sdrgpu_fft* h, int mode) {
    if (!h || mode < 0 || mode > 1) { set_error("fft_set_precision: bad argument"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    SDRGPU_HIP(hipDeviceSynchronize());   // no call of the plan in flight while its kernels change
    if (mode == 0 && p.f64) {
        fft64_destroy(p.f64);
        p.f64 = nullptr;
    } else if (mode == 1 && !p.f64) {
        SDRGPU_CHECK(fft64_create(&p.f64, p.N));
    }
    return SDRGPU_OK;
}
extern "C" int sdrgpu_fft_get_precision(sdrgpu_fft* h) { return h ? (h->p.f64 ? 1 : 0) : SDRGPU_EARG; }

static bool zoom_fusable(const FftPlan& p, int zoomSize) {
    return p.N1 == 256 && p.N2 == 256 && p.sa == 32 && p.sb == 32 && zoomSize * 32 == p.N;
}

// the one-pass 64k launch (+ the zoom fold): 2 workgroups per frame (quarter pairs), XCD-grouped in
// blocks of 8 frames, + the VFO stage's history workgroup
template <bool ZM, bool VFO>
static int launch_1p(FftPlan& p, const float2* in, long long stride, int frames, float* out, float* zoom, VfoWork v,
                     hipStream_t s, bool fold = true, DevBuf* zpb = nullptr) {
    // LDS-DMA rows need whole frames, an even frame stride and a 16-B aligned base (16-B pieces);
    // anything else streams through the range-checked register ring
    const bool pad = p.nz < 65536 || (stride & 1) || ((uintptr_t)in & 15);
    DevBuf& zp = zpb ? *zpb : p.zpart;
    if (ZM) SDRGPU_CHECK(zp.ensure(sizeof(float) * 2 * 2048 * (size_t)frames));   // the two workgroups' partial rows
    const int g = 16 * ((frames + 7) / 8) + (VFO && v.hist ? 1 : 0);
    auto k = pad ? fft_1p_kernel<ZM, VFO, true> : fft_1p_kernel<ZM, VFO, false>;
    SDRGPU_CHECK(set_lds(k, op1::LDS_BYTES));
    hipLaunchKernelGGL(k, dim3(g), dim3(512), op1::LDS_BYTES, s, in, stride, frames, p.win.as<float>(), p.nz,
                       p.tab1p.as<float2>(), p.tab1p64.as<double2>(), out, ZM ? zp.as<float>() : nullptr, v);
    SDRGPU_HIP(hipGetLastError());
    if (ZM && fold) {
        const long long n = (long long)frames * 2048 / 4;
        hipLaunchKernelGGL(fft_1p_zoom_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, zp.as<float>(),
                           frames, zoom);
        SDRGPU_HIP(hipGetLastError());
    }
    return SDRGPU_OK;
}
// Below k1pMinFrames frames a call runs the two-pass launches: with two workgroups per frame, each two
// 16k transforms long, a reference-size block (4.7 frames) took 33 us against 27 us for the two-pass
// launches (per-call trace r6c vs r4); the one-pass kernel fills the device from ~128 frames.
constexpr int k1pMinFrames = 64;
static bool onepass_ok(const FftPlan& p, int frames) {
    return p.N == 65536 && p.tab1p.p && !p.f64 && (p.onepass == 1 || (p.onepass == 2 && frames >= k1pMinFrames));
}

// frames -> dB rows (and, with zoom != nullptr on a zoom_fusable plan, the full-span zoom rows)
static int fft_execute_body(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out, float* zoom,
                            hipStream_t s);
static int fft_execute(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out, float* zoom,
                       hipStream_t s) {
    SDRGPU_CHECK(time_mark(h->p, 0, s));
    const int rc = fft_execute_body(h, in, frameStride, frames, out, zoom, s);
    if (rc < 0) return rc;
    SDRGPU_CHECK(time_mark(h->p, 1, s));
    return rc;
}
static int fft_execute_body(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out, float* zoom,
                            hipStream_t s) {
    FftPlan& p = h->p;
    const float2* x = (const float2*)in;
    if (p.f64) return fft64_execute(p.f64, x, frameStride, frames, p.win.as<float>(), p.nz, out, s);   // (zoom: unfused)
    if (p.N1 == 0) {
        SDRGPU_CHECK(dispatch_single(p, x, frameStride, frames, out, s));
        return frames;
    }
    if (onepass_ok(p, frames)) {
        const int rc = zoom ? launch_1p<true, false>(p, x, frameStride, frames, out, zoom, VfoWork{}, s)
                            : launch_1p<false, false>(p, x, frameStride, frames, out, nullptr, VfoWork{}, s);
        if (rc < 0) return rc;
        return frames;
    }
    const long long zw = p.N / 32;   // zoom row width when fused
    auto zoomAt = [&](long long f0) { return zoom ? zoom + f0 * zw : nullptr; };
    // 16-B loads need an even frame stride and a 16-B aligned base
    const bool paired = p.sa2 > 0 && (frameStride % 2) == 0 && ((uintptr_t)in & 15) == 0;
    const int nchunks = (frames + p.chunkFrames - 1) / p.chunkFrames;
    // the intermediate grows with the largest chunk seen (a single-frame drop-in plan holds 0.5 MB)
    SDRGPU_CHECK(p.scratch.ensure((size_t)std::min(p.chunkFrames, frames) * p.N * sizeof(float2)));
    if (p.merge && nchunks > 1 && merged_supported(p, paired)) {
        // A(0); [B(c-1) + A(c)] for c = 1..; B(last). Scratch alternates between two buffers.
        SDRGPU_CHECK(p.scratch2.ensure(p.scratch.bytes));
        float2* sc[2] = {p.scratch.as<float2>(), p.scratch2.as<float2>()};
        p.cur = sc[0];
        SDRGPU_CHECK(dispatch_passA(p, x, frameStride, std::min(p.chunkFrames, frames), s));
        for (int c = 1; c < nchunks; c++) {
            const int fB = (c - 1) * p.chunkFrames, nfB = p.chunkFrames;
            const int fA = c * p.chunkFrames, nfA = std::min(p.chunkFrames, frames - fA);
            const float2* xa = x + (long long)fA * frameStride;
            float* ob = out + (long long)fB * p.N;
            if (zoom) SDRGPU_CHECK(launch_merged<true>(p, sc[(c - 1) & 1], nfB, ob, xa, frameStride, nfA, sc[c & 1], s, zoomAt(fB)));
            else SDRGPU_CHECK(launch_merged<false>(p, sc[(c - 1) & 1], nfB, ob, xa, frameStride, nfA, sc[c & 1], s));
        }
        const int fL = (nchunks - 1) * p.chunkFrames;
        p.cur = sc[(nchunks - 1) & 1];
        SDRGPU_CHECK(dispatch_passB(p, frames - fL, out + (long long)fL * p.N, s, zoomAt(fL)));
        return frames;
    }
    p.cur = p.scratch.as<float2>();
    for (int c = 0; c < nchunks; c++) {
        const int f0 = c * p.chunkFrames;
        const int nf = std::min(p.chunkFrames, frames - f0);
        const float2* xc = x + (long long)f0 * frameStride;
        if (pipe1m_ok(p, paired)) {
            SDRGPU_CHECK(dispatch_1m(p, xc, frameStride, nf, out + (long long)f0 * p.N, s));
            continue;
        }
        if (paired) SDRGPU_CHECK(dispatch_passA2(p, xc, frameStride, nf, s));
        else SDRGPU_CHECK(dispatch_passA(p, xc, frameStride, nf, s));
        SDRGPU_CHECK(dispatch_passB(p, nf, out + (long long)f0 * p.N, s, zoomAt(f0)));
    }
    return frames;
}

extern "C" int sdrgpu_fft_execute_dev(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out,
                                      void* stream) {
    if (!h || !in || !out || frames < 0 || frameStride < 0) { set_error("fft_execute: bad argument"); return SDRGPU_EARG; }
    if (frames == 0) return 0;
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    hipStream_t s = stream ? (hipStream_t)stream : p.own;
    SDRGPU_CHECK(p.order.follow(s));
    OrderScope od(p.order, s);
    return fft_execute(h, in, frameStride, frames, out, nullptr, s);
}

int sdrgpu::fft_execute_split(sdrgpu_fft* h, const float2* head, int nh, const float2* body, long long stride, int frames,
                              float* out, const SideCopy& side, hipStream_t s, const VfoStage1* vfo, sdrgpu_block* vfoBlock,
                              void* vfoOut, int* vfoN) {
    if (!h || !body || frames <= 0 || nh < 0 || (nh > 0 && !head)) return SDRGPU_ESTATE;
    FftPlan& p = h->p;
    // the 64k plan's default tiles (256 x 256, 32 columns / 32 rows, one-column pass A); one chunk
    if (p.f64 || !(p.N1 == 256 && p.N2 == 256 && p.sa == 32 && p.sb == 32 && p.sa2 == 0) || frames > p.chunkFrames || nh >= p.nz)
        return SDRGPU_ESTATE;
    SDRGPU_CHECK(p.scratch.ensure((size_t)frames * p.N * sizeof(float2)));
    p.cur = p.scratch.as<float2>();
    SDRGPU_CHECK(time_mark(p, 0, s));
    if (!vfo) {
        SDRGPU_CHECK((launch_passA<256, 32>(p, body, stride, frames, s, head, nh, &side)));
        SDRGPU_CHECK(dispatch_passB(p, frames, out, s));
        SDRGPU_CHECK(time_mark(p, 1, s));
        return frames;
    }
    const size_t ldsFFT = sizeof(float2) * (32 * Lds<256>::LS + 256 + 256);
    {   // pass A + the VFO's stage 1 + its history carry + the tail copy
        VfoCall v{vfo->a, (int)((((long long)vfo->M + 31) / 32 + 15) / 16)};
        auto k = fft_passA_vfo_kernel;
        SDRGPU_CHECK(set_lds(k, ldsFFT));
        int spare = 0;
        if (side.count > 0) {
            int mx = 0;
            for (int i = 0; i < side.count; i++) mx = std::max(mx, side.n[i]);
            spare = std::max(1, std::min(64, (mx + 512 * 4 - 1) / (512 * 4)));   // ~4 elements per thread
        }
        const int g = 8 * frames + v.blocks + 1 + spare;
        hipLaunchKernelGGL(k, dim3(g), dim3(512), ldsFFT, s, body, stride, frames, p.win.as<float>(), p.nz, p.N2, p.logN,
                           p.tw1.as<float2>(), p.tfull.as<float2>(), p.cur, head, nh, side, v);
        SDRGPU_HIP(hipGetLastError());
    }
    // pass B + the VFO's later stages (one tail launch's workgroups) where the chain has that form
    TailArgs t;
    size_t ldsTail = 0;
    int tail = vfo_tail_prepare(vfoBlock, *vfo, vfoOut, &t, &ldsTail);
    if (tail < 0) return tail;
    if (tail && (t.NT != TAIL_NT || t.K != TAIL_K)) tail = 0;   // (a big call's workgroups: the later stages run after pass B)
    if (tail) {
        auto k = fft_passB_tail_kernel;
        const size_t lds = std::max(ldsFFT, ldsTail);
        SDRGPU_CHECK(set_lds(k, lds));
        hipLaunchKernelGGL(k, dim3(8 * frames + t.G), dim3(512), lds, s, p.cur, frames, p.N1, p.logN, p.tw2.as<float2>(), out, t);
        SDRGPU_HIP(hipGetLastError());
        *vfoN = vfo_tail_commit(vfoBlock, *vfo, t);
        SDRGPU_CHECK(time_mark(p, 1, s));
        return frames;
    }
    SDRGPU_CHECK(dispatch_passB(p, frames, out, s));
    SDRGPU_CHECK(time_mark(p, 1, s));
    const int n = vfo_stage1_finish(vfoBlock, *vfo, vfoOut, s);
    if (n < 0) return n;
    *vfoN = n;
    return frames;
}

int sdrgpu::fft_set_onepass(sdrgpu_fft* h, int onepass) {
    if (!h) return SDRGPU_EARG;
    h->p.onepass = onepass;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_fft_set_kernel(sdrgpu_fft* h, int mode) {
    if (!h || mode < 0 || mode > 2) { set_error("fft_set_kernel: bad argument"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    const int prev = p.N == 65536 ? p.onepass : 2;
    if (p.N == 65536) p.onepass = mode;   // (read at call time: calls in flight keep their form)
    return prev;
}

int sdrgpu::fft_execute_owned(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out, hipStream_t s) {
    if (!h || !in || !out || frames < 0 || frameStride < 0) { set_error("fft_execute: bad argument"); return SDRGPU_EARG; }
    if (frames == 0) return 0;
    return fft_execute(h, in, frameStride, frames, out, nullptr, s);
}

// Rows + the waterfall's full-span zoom rows: fft_scaler(0, bw, bw, N, zoomSize).doZoom of every
// row (gui/widgets/fft_scaler.h:27-64: max over the bins [round(f0), round(f0 + N / zoomSize))).
// On the 64k plan with zoomSize = N / 32 the zoom is fused into pass B's dB store (the rows are
// not read again); any other size runs the zoom kernel over the rows afterwards.
extern "C" int sdrgpu_fft_execute_zoom_dev(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out,
                                           float* zoomOut, int zoomSize, void* stream) {
    if (!h || !in || !out || !zoomOut || frames < 0 || frameStride < 0 || zoomSize <= 0 || zoomSize > h->p.N) {
        set_error("fft_execute_zoom: bad argument");
        return SDRGPU_EARG;
    }
    if (frames == 0) return 0;
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    hipStream_t s = stream ? (hipStream_t)stream : p.own;
    SDRGPU_CHECK(p.order.follow(s));
    OrderScope od(p.order, s);
    if (zoom_fusable(p, zoomSize) && !p.f64) return fft_execute(h, in, frameStride, frames, out, zoomOut, s);
    SDRGPU_CHECK(fft_execute(h, in, frameStride, frames, out, nullptr, s));
    if (!p.zoom || p.zoomSize != zoomSize) {
        if (p.zoom) sdrgpu_zoom_destroy(p.zoom);
        p.zoom = nullptr;
        SDRGPU_CHECK(sdrgpu_zoom_create(&p.zoom, p.device, 0.0, 1.0, 1.0, p.N, zoomSize));
        p.zoomSize = zoomSize;
    }
    SDRGPU_CHECK(sdrgpu_zoom_execute_dev(p.zoom, out, frames, zoomOut, s));
    return frames;
}

// The fused launch group (fft_vfo_kernel): A(0)+V(0); [B(c-1) + A(c)+V(c)] for c = 1..; B(last) +
// the stage's history workgroup. Scratch alternates between two buffers as in fft_execute.
template <bool ZM>
static int launch_vfo(FftPlan& p, const float2* scratchB, int framesB, float* outB, float* zoomB, const float2* in,
                      int framesA, float2* scratchA, VfoWork v, hipStream_t s) {
    auto k = fft_vfo_kernel<ZM>;
    const size_t lds = sizeof(float2) * (32 * Lds<256>::LS + 256 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    const int nB = 8 * framesB;
    const int g = nB + 96 * ((framesA + 7) / 8) + (v.hist ? 1 : 0);
    hipLaunchKernelGGL(k, dim3(g), dim3(512), lds, s, nB, scratchB, framesB, outB, zoomB, in, (long long)p.N, framesA,
                       p.win.as<float>(), p.nz, p.logN, p.tw1.as<float2>(), p.tw2.as<float2>(), p.tfull.as<float2>(),
                       scratchA, v);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}
static int dispatch_vfo(FftPlan& p, bool zm, const float2* scratchB, int framesB, float* outB, float* zoomB,
                        const float2* in, int framesA, float2* scratchA, const VfoWork& v, hipStream_t s) {
    return zm ? launch_vfo<true>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
              : launch_vfo<false>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
}
static bool vfo_fusable(const FftPlan& p, float* zoom, int zoomSize) {
    return p.vfoFuse && !p.f64 && p.N1 == 256 && p.N2 == 256 && p.sa == 32 && p.sb == 32 && p.sa2 == 0 && p.nz == p.N &&
           (zoom == nullptr || zoom_fusable(p, zoomSize));
}
// Returns the VFO's output count: its later stages (vfo_stage1_finish) need only the stage-1 outputs,
// complete once the last pass-A launch is done; they run after the group on the call's stream (on a
// side stream beside the last launch they measured slower: 1.725 vs 1.705 ms, r4i).
static int fft_execute_vfo(FftPlan& p, const float2* x, int frames, float* out, float* zoom, const VfoStage1& st0,
                           sdrgpu_block* vfo, void* vfoOut, hipStream_t s) {
    VfoStage1 st = st0;
    if (p.tailStream && zoom && onepass_ok(p, frames)) {
        // the tail on its own stream (sdrgpu_fft_set_tail_stream): the stage-1 outputs and the zoom partials
        // go to this call parity's buffers, free once call k - 2's tail is done
        const int b = (int)(p.tcallsT & 1);
        if (p.tdoneRec[b]) SDRGPU_HIP(hipStreamWaitEvent(s, p.tdone[b], 0));
        SDRGPU_CHECK(p.s1T[b].ensure(sizeof(float2) * (size_t)std::max(st.M, 1)));
        st.out = p.s1T[b].p;
        st.a.out = p.s1T[b].p;
        TailArgs t;
        size_t ldsTail = 0;
        int tail = vfo_tail_prepare(vfo, st, vfoOut, &t, &ldsTail);
        if (tail < 0) return tail;
        if (tail && (t.NT != TAIL_NT_BIG || t.K != TAIL_K_BIG)) tail = 0;
        if (tail) {
            VfoWork v{st.a, 0, 1};
            SDRGPU_CHECK(time_mark(p, 0, s));
            SDRGPU_CHECK((launch_1p<true, true>(p, x, p.N, frames, out, zoom, v, s, false, &p.zpartT[b])));
            SDRGPU_CHECK(time_mark(p, 1, s));
            SDRGPU_HIP(hipEventRecord(p.gdone[b], s));
            SDRGPU_HIP(hipStreamWaitEvent(p.tailStream, p.gdone[b], 0));
            auto k = fft_1p_tail_fold_kernel;
            SDRGPU_CHECK(set_lds(k, ldsTail));
            const int nzb = (int)(((long long)frames * 2048 / 4 + 255) / 256);
            hipLaunchKernelGGL(k, dim3(t.G + nzb), dim3(TAIL_NT_BIG), ldsTail, p.tailStream, t, p.zpartT[b].as<float>(),
                               frames, zoom);
            SDRGPU_HIP(hipGetLastError());
            SDRGPU_HIP(hipEventRecord(p.tdone[b], p.tailStream));
            p.tdoneRec[b] = true;
            p.tcallsT++;
            return vfo_tail_commit(vfo, st, t);
        }
        st = st0;   // (no big-call tail: the same-stream path below)
    }
    if (onepass_ok(p, frames)) {
        VfoWork v{st.a, 0, 1};
        // with zoom rows and a big-call tail, the zoom fold rides in the tail's launch
        TailArgs t;
        size_t ldsTail = 0;
        int tail = zoom ? vfo_tail_prepare(vfo, st, vfoOut, &t, &ldsTail) : 0;
        if (tail < 0) return tail;
        if (tail && (t.NT != TAIL_NT_BIG || t.K != TAIL_K_BIG)) tail = 0;
        SDRGPU_CHECK(time_mark(p, 0, s));
        const int rc = zoom ? launch_1p<true, true>(p, x, p.N, frames, out, zoom, v, s, !tail)
                            : launch_1p<false, true>(p, x, p.N, frames, out, nullptr, v, s);
        if (rc < 0) return rc;
        SDRGPU_CHECK(time_mark(p, 1, s));
        if (tail) {
            auto k = fft_1p_tail_fold_kernel;
            SDRGPU_CHECK(set_lds(k, ldsTail));
            const int nz = (int)(((long long)frames * 2048 / 4 + 255) / 256);
            hipLaunchKernelGGL(k, dim3(t.G + nz), dim3(TAIL_NT_BIG), ldsTail, s, t, p.zpart.as<float>(), frames, zoom);
            SDRGPU_HIP(hipGetLastError());
            return vfo_tail_commit(vfo, st, t);
        }
        return vfo_stage1_finish(vfo, st, vfoOut, s);
    }
    const int cf = p.chunkFrames;
    const int nchunks = (frames + cf - 1) / cf;
    SDRGPU_CHECK(p.scratch.ensure((size_t)std::min(cf, frames) * p.N * sizeof(float2)));
    SDRGPU_CHECK(p.scratch2.ensure(p.scratch.bytes));
    float2* sc[2] = {p.scratch.as<float2>(), p.scratch2.as<float2>()};
    const long long zw = p.N / 32;
    auto zoomAt = [&](long long f0) { return zoom ? zoom + f0 * zw : nullptr; };
    VfoWork v{st.a, 0, 0};
    SDRGPU_CHECK(time_mark(p, 0, s));
    SDRGPU_CHECK(dispatch_vfo(p, zoom != nullptr, nullptr, 0, nullptr, nullptr, x, std::min(cf, frames), sc[0], v, s));
    for (int c = 1; c < nchunks; c++) {
        const int fB = (c - 1) * cf, fA = c * cf, nfA = std::min(cf, frames - fA);
        v.frame0 = fA;
        SDRGPU_CHECK(dispatch_vfo(p, zoom != nullptr, sc[(c - 1) & 1], cf, out + (long long)fB * p.N, zoomAt(fB),
                                  x + (long long)fA * p.N, nfA, sc[c & 1], v, s));
    }
    const int fL = (nchunks - 1) * cf;
    v.hist = 1;
    SDRGPU_CHECK(dispatch_vfo(p, zoom != nullptr, sc[(nchunks - 1) & 1], frames - fL, out + (long long)fL * p.N, zoomAt(fL),
                              nullptr, 0, nullptr, v, s));
    SDRGPU_CHECK(time_mark(p, 1, s));
    return vfo_stage1_finish(vfo, st, vfoOut, s);
}

// Spectrum (+ the waterfall's zoom rows) + one RxVFO over the same device batch of back-to-back
// frames (fftRate = fs / N: the IQFrontEnd's reshaper keeps every sample, iq_frontend.h:56-60), the
// VFO reading the batch in place like every consumer of the front end's splitter
// (iq_frontend.cpp:15-52). On the 64k plan with the VFO's D = 32 first stage (the RxVFO's plan_256
// at 61.44 MS/s) the batch is read from HBM once: the stage runs inside the spectrum launches
// (fft_vfo_kernel) and only the VFO's later stages run after them. Otherwise: the spectrum launch
// group, then the VFO. Returns the VFO's output count (vfoOut).
static int fft_execute_zoom_vfo_body(sdrgpu_fft* h, const void* in, int frames, float* out, float* zoomOut, int zoomSize,
                                     sdrgpu_block* vfo, void* vfoOut, hipStream_t s, int fuse, const VfoStage1& st);
extern "C" int sdrgpu_fft_execute_zoom_vfo_dev(sdrgpu_fft* h, const void* in, int frames, float* out, float* zoomOut,
                                               int zoomSize, sdrgpu_block* vfo, void* vfoOut, void* stream) {
    if (!h || !in || !out || !vfo || !vfoOut || frames < 0 || (zoomOut && (zoomSize <= 0 || zoomSize > h->p.N))) {
        set_error("fft_execute_vfo: bad argument");
        return SDRGPU_EARG;
    }
    FftPlan& p = h->p;
    const long long count = (long long)frames * p.N;
    if (count > 0x7fffffffLL) { set_error("fft_execute_vfo: %lld samples per call (max 2^31 - 1)", count); return SDRGPU_EARG; }
    // back-to-back frames: the spectrum must cover every sample the VFO consumes, on one device
    if (p.nz != p.N) { set_error("fft_execute_vfo: plan nz %d != N %d (frames must be back to back)", p.nz, p.N); return SDRGPU_EARG; }
    if (!vfo->impl) { set_error("fft_execute_vfo: null VFO block handle"); return SDRGPU_EARG; }
    if (vfo->impl->device != p.device) {
        set_error("fft_execute_vfo: VFO on device %d, spectrum plan on device %d", vfo->impl->device, p.device);
        return SDRGPU_EARG;
    }
    if (frames == 0) return 0;
    SDRGPU_SET_DEVICE(p.device);
    hipStream_t s = stream ? (hipStream_t)stream : p.own;
    SDRGPU_CHECK(p.order.follow(s));
    OrderScope od(p.order, s);
    // tail-stream mode: the VFO's work of a call ends on the tail stream; its next call on `s` needs
    // only what `s` itself ordered (stage 1's history), so a VFO last used by this plan's tail is
    // not waited for here (that wait would serialise the overlap)
    const bool tmode = p.tailStream && zoomOut && p.tailStream != s;
    if (!(tmode && vfo->impl->order.last == p.tailStream)) SDRGPU_CHECK(vfo->impl->order.follow(s));
    OrderScope ov(vfo->impl->order, tmode ? p.tailStream : s);
    VfoStage1 st;
    const int fuse = vfo_fusable(p, zoomOut, zoomSize) ? vfo_stage1_prepare(vfo, in, (int)count, &st) : 0;
    if (fuse < 0) return fuse;
    const long long before = p.tcallsT;
    const int n = fft_execute_zoom_vfo_body(h, in, frames, out, zoomOut, zoomSize, vfo, vfoOut, s, fuse, st);
    if (n >= 0 && tmode && p.tcallsT == before) {
        // (this call took a path that ran everything on `s`: the tail stream's consumers wait for it)
        SDRGPU_HIP(hipEventRecord(p.gdone[0], s));
        SDRGPU_HIP(hipStreamWaitEvent(p.tailStream, p.gdone[0], 0));
    }
    return n;
}

static int fft_execute_zoom_vfo_body(sdrgpu_fft* h, const void* in, int frames, float* out, float* zoomOut, int zoomSize,
                                     sdrgpu_block* vfo, void* vfoOut, hipStream_t s, int fuse, const VfoStage1& st) {
    FftPlan& p = h->p;
    const long long count = (long long)frames * p.N;
    if (fuse) return fft_execute_vfo(p, (const float2*)in, frames, out, zoomOut, st, vfo, vfoOut, s);
    if (zoomOut && !(zoom_fusable(p, zoomSize) && !p.f64)) {
        SDRGPU_CHECK(fft_execute(h, in, p.N, frames, out, nullptr, s));
        if (!p.zoom || p.zoomSize != zoomSize) {
            if (p.zoom) sdrgpu_zoom_destroy(p.zoom);
            p.zoom = nullptr;
            SDRGPU_CHECK(sdrgpu_zoom_create(&p.zoom, p.device, 0.0, 1.0, 1.0, p.N, zoomSize));
            p.zoomSize = zoomSize;
        }
        SDRGPU_CHECK(sdrgpu_zoom_execute_dev(p.zoom, out, frames, zoomOut, s));
    } else {
        SDRGPU_CHECK(fft_execute(h, in, p.N, frames, out, zoomOut, s));
    }
    return block_run_owned(vfo, in, (int)count, vfoOut, s);
}

extern "C" int sdrgpu_fft_execute_vfo_dev(sdrgpu_fft* h, const void* in, int frames, float* out, sdrgpu_block* vfo,
                                          void* vfoOut, void* stream) {
    return sdrgpu_fft_execute_zoom_vfo_dev(h, in, frames, out, nullptr, 0, vfo, vfoOut, stream);
}

// Timing of the spectrum launch group (HIP events on the call's stream; off by default)
extern "C" int sdrgpu_fft_set_timing(sdrgpu_fft* h, int on) {
    if (!h) { set_error("fft_set_timing: null handle"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    if (on && !p.tev[0][0])
        for (auto& e : p.tev) {
            SDRGPU_HIP(hipEventCreate(&e[0]));
            SDRGPU_HIP(hipEventCreate(&e[1]));
        }
    p.timing = on != 0;
    p.tcalls = 0;
    return SDRGPU_OK;
}
// the group times (ms) of the last min(n, calls, 256) timed calls, oldest first; waits for them
extern "C" int sdrgpu_fft_group_times(sdrgpu_fft* h, float* ms, int n) {
    if (!h || !ms || n < 0) { set_error("fft_group_times: bad argument"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    const long long k = std::min<long long>({(long long)n, p.tcalls, (long long)FftPlan::kTimed});
    for (long long i = 0; i < k; i++) {
        auto& e = p.tev[(p.tcalls - k + i) % FftPlan::kTimed];
        SDRGPU_HIP(hipEventSynchronize(e[1]));
        SDRGPU_HIP(hipEventElapsedTime(&ms[i], e[0], e[1]));
    }
    return (int)k;
}

extern "C" int sdrgpu_fft_logmag(sdrgpu_fft* h, const void* in, float* out) {
    if (!h || !in) { set_error("fft_logmag: null argument"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    size_t inB = sizeof(float2) * p.nz, outB = sizeof(float) * p.N;
    SDRGPU_CHECK(p.pin_in.ensure(inB));
    SDRGPU_CHECK(p.dev_in.ensure(inB));
    SDRGPU_CHECK(p.dev_out.ensure(outB));
    // registered host buffers (sdrgpu_host_register) are DMA'd directly, others staged
    const void* src = in;
    if (!host_pinned(in, inB)) {
        std::memcpy(p.pin_in.p, in, inB);
        src = p.pin_in.p;
    }
    SDRGPU_HIP(hipMemcpyAsync(p.dev_in.p, src, inB, hipMemcpyHostToDevice, p.own));
    SDRGPU_CHECK(sdrgpu_fft_execute_dev(h, p.dev_in.p, p.nz, 1, p.dev_out.as<float>(), p.own));
    if (out && host_pinned(out, outB)) {
        SDRGPU_HIP(hipMemcpyAsync(out, p.dev_out.p, outB, hipMemcpyDeviceToHost, p.own));
        SDRGPU_HIP(hipStreamSynchronize(p.own));
    } else if (out) {
        SDRGPU_CHECK(p.pin_out.ensure(outB));
        SDRGPU_HIP(hipMemcpyAsync(p.pin_out.p, p.dev_out.p, outB, hipMemcpyDeviceToHost, p.own));
        SDRGPU_HIP(hipStreamSynchronize(p.own));
        std::memcpy(out, p.pin_out.p, outB);
    } else {
        SDRGPU_HIP(hipStreamSynchronize(p.own));
    }
    return p.N;
}

extern "C" int sdrgpu_fft_set_tail_stream(sdrgpu_fft* h, void* stream) {
    if (!h) { set_error("fft_set_tail_stream: null handle"); return SDRGPU_EARG; }
    FftPlan& p = h->p;
    SDRGPU_SET_DEVICE(p.device);
    if (p.tailStream && p.tailStream != (hipStream_t)stream)   // tails in flight keep their buffers until done
        for (int b = 0; b < 2; b++)
            if (p.tdoneRec[b]) SDRGPU_HIP(hipEventSynchronize(p.tdone[b]));
    if (stream && !p.gdone[0])
        for (int b = 0; b < 2; b++) {
            SDRGPU_HIP(hipEventCreateWithFlags(&p.gdone[b], hipEventDisableTiming));
            SDRGPU_HIP(hipEventCreateWithFlags(&p.tdone[b], hipEventDisableTiming));
        }
    if ((hipStream_t)stream != p.tailStream) {
        p.tdoneRec[0] = p.tdoneRec[1] = false;
        p.tcallsT = 0;
    }
    p.tailStream = (hipStream_t)stream;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_fft_destroy(sdrgpu_fft* h) {
    if (!h) return SDRGPU_OK;
    (void)hipSetDevice(h->p.device);
    for (int b = 0; b < 2; b++) {
        if (h->p.tdoneRec[b]) (void)hipEventSynchronize(h->p.tdone[b]);
        if (h->p.gdone[b]) (void)hipEventDestroy(h->p.gdone[b]);
        if (h->p.tdone[b]) (void)hipEventDestroy(h->p.tdone[b]);
    }
    if (h->p.own) (void)hipStreamDestroy(h->p.own);
    if (h->p.zoom) sdrgpu_zoom_destroy(h->p.zoom);
    if (h->p.f64) fft64_destroy(h->p.f64);
    for (auto& e : h->p.tev)
        for (auto& ev : e)
            if (ev) (void)hipEventDestroy(ev);
    delete h;
    return SDRGPU_OK;
}
