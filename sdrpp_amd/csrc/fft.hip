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

// ---- 1M pass A, persistent and software-pipelined (N1 = 1024, paired columns) --------------
// The 1M column FFT needs S x 1024 x 8 B of LDS per tile (139 KB at S = 16), so one workgroup per
// CU: in the one-shot kernel above each CU alternates "load the tile" and "transform + store it",
// and HBM idles during the transform. Here a CU's workgroup walks tiles blockIdx.x, +gridDim.x, ...
// and issues the next tile's input + window loads (96 VGPRs) before it transforms the current one,
// so the loads fly during the LDS stages and the stores. The stage twiddles are staged in LDS once
// per workgroup, and the four-step twiddle W_N^(c k1) is generated in fp64 and rounded once
// (the same single rounding as the table it replaces): for column c and this thread's outputs
// k1 = t + 64 m, W^(c t) and W^(64 c) come from two 256-entry fp64 tables (W_N^(256 j), W_N^j;
// c t, 64 c < 2^16) and W^(c (t + 64 m)) = W^(c t) (W^(64 c))^m by an fp64 recurrence over m
// (15 products: relative error ~1e-15, far below the fp32 rounding). That removes the 8 MB
// [k1][n2] table read (8 B per sample of L2 / Infinity-Cache traffic).
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef float nt_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 nt_load4(const float2* p) {   // streaming (non-temporal) 16-B load
    const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 nt_load2(const float2* p) {
    const nt_f2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f2*>(p));
    return make_float2(v.x, v.y);
}
__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

typedef unsigned bu2 __attribute__((ext_vector_type(2)));
typedef unsigned bu4 __attribute__((ext_vector_type(4)));

// the radix-16 middle stage (NS = 16) of the 1M pass A for one column, thread t: read + twiddle +
// DFT into v, then (after the caller's barrier) the in-place write
__device__ __forceinline__ void mid16_read(const float2* seq, const float2* tw16, int t, float2 (&v)[16]) {
    constexpr int L = 1024;
    const int jm = t % 16;
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = seq[pad16s<L / 16>(t, r)];
#pragma unroll
    for (int r = 1; r < 16; r++) v[r] = cmul(v[r], tw16[16 * r + jm]);   // (stage_lds's tw16 layout)
    dft16(v);
}
__device__ __forceinline__ void mid16_write(float2* seq, int t, const float2 (&v)[16]) {
    const int idxD = (t / 16) * 256 + (t % 16);
#pragma unroll
    for (int r = 0; r < 16; r++) seq[pad16s<16>(idxD, r)] = v[r];
}

// tile -> (frame, block) of the persistent 1M passes. G (the grid, a multiple of 8 G8 and of 8) > 1
// groups G8 adjacent blocks on one XCD at once: workgroups x, x + 8, ... (same XCD, same round)
// take blocks b, b + 1, ..., whose row / dB segments share 128-B lines (64-B pass-A segments at 8
// columns, 32-B dB segments at 8 rows), so a line is filled / written whole in one L2.
template <int G8>
__device__ __forceinline__ void tile_fb(int T, int nb, int& b, long long& f) {
    if constexpr (G8 <= 1) {
        b = T % nb;
        f = T / nb;
    } else {
        const int g = T / (8 * G8), w = T % (8 * G8);
        const int P = g * 8 + (w & 7), h = w >> 3;
        const int npf = nb / G8;
        f = P / npf;
        b = G8 * (P % npf) + h;
    }
}

// VAR (tuning, SDRGPU_FFT_1M_VAR): bit 0 middle stage one column at a time, bit 3 row offsets
// advanced through opaque registers (together: no spills, same time as the default, r3 A/B),
// bit 6 XCD-grouped column blocks (S = 8); bits 4 / 5 measurement only (below). Measured and
// removed (r3, C2 step, 3 interleaved runs, one box): the last stage + 8-B stores one column at a
// time (2.22 vs 1.95 ms), the four-step fp64 tables staged in LDS (2.17 vs 1.95 ms).
// ---- 1M pass B, persistent and software-pipelined (N2 = 1024) -------------------------------
// Same transform as fft_passB_kernel<1024, S>, each workgroup walking tiles with the next tile's
// 16 row values per thread loaded while the current tile is transformed and stored.
template <int S, int CP, int VAR = 0>   // VAR (measurement only): 16 loads tile 0 only, 32 stores dropped
__device__ __forceinline__ void passB_1m_body(int tile0, int step, const float2* __restrict__ scratch, int frames,
                                              int N1, int logN, const float2* __restrict__ tw, float* __restrict__ out) {
    constexpr int L = 1024, T = L / 16;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int XG = (VAR & 64) ? 32 / S : 1;   // XCD grouping of row blocks (bit 6): 128-B dB lines
    constexpr bool TMAJ = VAR & 128;              // bit 7: the tile-major intermediate of pass A at 16 columns
    float2* twl = lds + S * Lds<L>::LS;   // stage twiddles, staged once per workgroup
    float2* tw16 = twl + L;                // the middle stage's, bank-conflict-free (stage_lds)
    const int tid = threadIdx.x;
    for (int i = tid; i < L; i += S * T) twl[i] = tw[i];   // (first barrier below orders both)
    for (int i = tid; i < 256; i += S * T) tw16[i] = tw[(i >> 4) * (i & 15) * (L / 256)];
    const int sF = tid / T, tF = tid % T;
    const int nb = N1 / S;
    const int ntiles = nb * frames;
    float2 fr[16];
#define SDRGPU_PB1M_ISSUE(TILE)                                                                                       \
    do {                                                                                                              \
        int b_;                                                                                                       \
        long long f_;                                                                                                 \
        tile_fb<XG>((TILE), nb, b_, f_);                                                                              \
        if (VAR & 16) { b_ = 0; f_ = 0; }                                                                             \
        const __amdgpu_buffer_rsrc_t rs_ = brsrc(scratch + (f_ << logN), 0x7fffffffu);                                \
        const unsigned o_ = TMAJ ? (unsigned)((tF / 16) * L * 16 + (b_ * S + sF) * 16 + tF % 16) * 8u                 \
                                 : (unsigned)((b_ * S + sF) * L + tF) * 8u;                                            \
        _Pragma("unroll") for (int r = 0; r < 16; r++)                                                               \
            fr[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs_, o_, r * (TMAJ ? 4 * L * 16 * 8 : T * 8), CP)); \
    } while (0)
    int tile = tile0;
    if (tile < ntiles) SDRGPU_PB1M_ISSUE(tile);
    for (; tile < ntiles; tile += step) {
        float2 v[16];
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = fr[r];
        if (tile + step < ntiles) SDRGPU_PB1M_ISSUE(tile + step);
        // the LDS addresses below are loop-invariant; recomputing them per tile (laundered thread
        // index) keeps ~40 hoisted address registers from spilling the prefetched tile
        int tv = tid;
        asm volatile("" : "+v"(tv));
        const int sF2 = tv / T, tF2 = tv % T, sL2 = tv % S, tL2 = tv / S;
        __syncthreads();   // the previous tile's last LDS reads are done
        stage_first<L>(lds + sF2 * Lds<L>::LS, v, tF2);
        __syncthreads();
        int b;
        long long f;
        tile_fb<XG>(tile, nb, b, f);
        const __amdgpu_buffer_rsrc_t ro = brsrc(out + (f << logN) + b * S, (VAR & 32) ? 0u : 0x7fffffffu);
        stages_rest<L, true>(lds, twl, sL2, tL2, [&](int k2, float2 y) {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, db_of(y)), ro, (unsigned)(sL2 + N1 * k2) * 4u, 0, CP);
        }, tw16);
    }
}
#undef SDRGPU_PB1M_ISSUE

template <int S, int CP, int VAR = 0>
__global__ __launch_bounds__(S * 1024 / 16) void fft_passB_1m_kernel(const float2* __restrict__ scratch, int frames, int N1,
                                                                    int logN, const float2* __restrict__ tw,
                                                                    float* __restrict__ out) {
    passB_1m_body<S, CP, VAR>(blockIdx.x, gridDim.x, scratch, frames, N1, logN, tw, out);
}

// MERGED (round 4, fft_merged_1m launches): the workgroup first runs its share of the previous
// chunk's pass-B tiles (mb), then this pass A. Both walk tiles blockIdx.x + k gridDim.x; they share
// nothing (pass A writes the other scratch buffer). Pass B's twiddles sit inside pass A's data
// region: pass A's first barrier orders its first LDS write after every pass-B read. (The pass-A
// code stays in the kernel body: moved into a device function, the compiler's allocation changed
// and the kernel spilled 24 VGPRs.)
struct MergeB {
    const float2* scratch;
    int frames, N1;
    float* out;
    const float2* tw;
};
template <int S, int CP, int VAR, bool MERGED = false>   // CP: cache-policy bits of the streaming accesses (0, or 2 = nt; tuning)
__global__ __launch_bounds__(S / 2 * 1024 / 16) __attribute__((amdgpu_waves_per_eu(S < 16 ? 2 : 1))) void fft_passA_1m_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz, int N2,
    int logN, const float2* __restrict__ tw, const double2* __restrict__ wt, float2* __restrict__ scratch, MergeB mb) {
    if constexpr (MERGED) {
        if (mb.frames) passB_1m_body<8, 0, 64 | 128>(blockIdx.x, gridDim.x, mb.scratch, mb.frames, mb.N1, logN, mb.tw, mb.out);
        if (!frames) return;
    }
    constexpr int L = 1024, P = S / 2, T = L / 16, NT = P * T, LS = Lds<L>::LS;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr bool MIDCOL = VAR & 1, LAUNDER = VAR & 8;
    constexpr bool NOLOAD = VAR & 16, NOSTORE = VAR & 32;   // (measurement only: wrong results)
    constexpr int XG = ((VAR & 64) && S < 16) ? 16 / S : 1;   // XCD grouping of column blocks (bit 6): 128-B row lines
    // bit 7: tile-major intermediate [b][k1][c] (each tile's 128 KB written contiguously; pass B
    // then reads 128-B pieces of 16 columns) instead of row-major [k1][n2]
    constexpr bool TMAJ = VAR & 128;
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
    // LAUNDER: the 16 row offsets are advanced through opaque registers; left to itself the
    // compiler may precompute all 32 and spill them, and every reload from scratch then waits
    // (vmcnt, in order) for the prefetch loads issued before it
#define SDRGPU_PA1M_ISSUE(TILE)                                                                                         \
    do {                                                                                                                \
        int b_;                                                                                                         \
        long long f_;                                                                                                   \
        tile_fb<XG>((TILE), nb, b_, f_);                                                                                \
        if (NOLOAD) { b_ = 0; f_ = 0; }                                                                                 \
        const unsigned o_ = (unsigned)(t * N2 + b_ * S + 2 * cp);                                                       \
        const __amdgpu_buffer_rsrc_t rx_ = brsrc(in + f_ * frameStride, (unsigned)nz * 8u);                            \
        unsigned vq_ = o_ * 8, vw_ = o_ * 4;                                                                            \
        _Pragma("unroll") for (int r = 0; r < 16; r++) {                                                                \
            if constexpr (LAUNDER) {                                                                                    \
                q[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx_, vq_, 0, CP));              \
                w[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rw, vw_, 0, 0));                 \
                vq_ += (unsigned)rowB;                                                                                  \
                vw_ += (unsigned)rowB / 2;                                                                              \
                asm volatile("" : "+v"(vq_), "+v"(vw_));                                                                \
            } else {                                                                                                    \
                q[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx_, o_ * 8 + r * rowB, 0, CP)); \
                w[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rw, o_ * 4 + r * rowB / 2, 0, 0)); \
            }                                                                                                           \
        }                                                                                                               \
    } while (0)
    int tile = blockIdx.x;
    if (tile < ntiles) SDRGPU_PA1M_ISSUE(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        float2 v0[16], v1[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
            v0[r] = make_float2(q[r].x * w[r].x, q[r].y * w[r].x);
            v1[r] = make_float2(q[r].z * w[r].y, q[r].w * w[r].y);
        }
        if (tile + (int)gridDim.x < ntiles) SDRGPU_PA1M_ISSUE(tile + (int)gridDim.x);   // next tile's loads fly now
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
        // middle stage (radix 16, NS = 16). MIDCOL: one column at a time, 16 values live instead
        // of 32. Column 1's region is disjoint from column 0's, so its read needs no barrier of its
        // own.
        float2 m16[16];
        if constexpr (MIDCOL) {
            mid16_read(seq0, tw16, t2, m16);
            __syncthreads();   // every column-0 read is done
            mid16_write(seq0, t2, m16);
            mid16_read(seq0 + LS, tw16, t2, m16);
            __syncthreads();   // every column-1 read done
            mid16_write(seq0 + LS, t2, m16);
            __syncthreads();
        } else {
            stage_lds_v<L, 16, 16, 2, true>(seq0, twl, t2, tw16);   // (two barriers inside)
        }
        int b;
        long long f;
        tile_fb<XG>(tile, nb, b, f);
        const int col = b * S + 2 * cp;
        const __amdgpu_buffer_rsrc_t rs = brsrc(scratch + (f << logN), NOSTORE ? 0u : 0x7fffffffu);
        // Stores carry the row step in the per-lane offset and a ZERO soffset. A >64-bit buffer
        // store with an SGPR soffset gets no wait state before the next VALU write of its data
        // VGPRs (hipcc's hazard check skips that form, and two 8-B stores get merged into it): it
        // wrote already-overwritten data, rows of some lanes changing from run to run (DESIGN.md
        // §3). The offset is advanced through an opaque register so the 16 row offsets are not all
        // precomputed (register pressure).
        {
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
            unsigned vo = TMAJ ? (unsigned)(b * L * S + t * S + 2 * cp) * 8u : (unsigned)(t * N2 + col) * 8u;
            const unsigned mstep = TMAJ ? (unsigned)(T * S * 8) : (unsigned)rowB;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                const float2 a = cmul(y[0][m], make_float2((float)cur[0].x, (float)cur[0].y));
                const float2 c = cmul(y[1][m], make_float2((float)cur[1].x, (float)cur[1].y));
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bu4, make_float4(a.x, a.y, c.x, c.y)), rs, vo, 0, 0);
                vo += mstep;
                asm volatile("" : "+v"(vo));
                if (m < 15) {
                    cur[0] = zmul(cur[0], step[0]);
                    cur[1] = zmul(cur[1], step[1]);
                }
            }
        }
    }
}
#undef SDRGPU_PA1M_ISSUE

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
// boundaries give equal bits. (XG 0-2) one workgroup per frame: 64 segments, 4 per D-lane group.
__device__ __forceinline__ void vfo_frame_block(const VfoWork& v, int g) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;   // 8 waves x 2 groups
    for (int k = 0; k < 4; k++) {
        const long long seg = (long long)(v.frame0 + g) * 64 + k * 16 + wave * 2 + (lane >> 5);
        fir_rows_segment<32, 5, true, false, 32, 32, true>(v.a, seg, lane);
    }
}
// (XG 3, the default) quarter q of frame g's stage-1 outputs: 16 segments of 32 outputs, one per D-lane
// group, one row batch each -- a workgroup that lives one load round, like the column tiles beside it
__device__ __forceinline__ void vfo_quarter_block(const VfoWork& v, int g, int q) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long seg = (long long)(v.frame0 + g) * 64 + q * 16 + wave * 2 + (lane >> 5);
    fir_rows_segment<32, 5, true, false, 32, 32, true>(v.a, seg, lane);
}

// XG: XCD-grouped frames. Workgroups x, x + 8, x + 16, ... run on one XCD (round-robin dispatch), so
// workgroup 8 k + x takes item k % 9 of frame 8 (k / 9) + x: a frame's stage-1 workgroup (item 0,
// dispatched first) and its 8 column tiles share one XCD's L2, and the second reader of each IQ line
// finds it there instead of crossing the fabric to the Infinity Cache. Ungrouped, a frame's 9
// consecutive workgroups land on all eight XCDs.
// XG 3 (the default): a frame's stage 1 as 4 quarter workgroups of 16 one-row-batch segments: they
// live one load round, as the 8 column tiles beside them do, so all 12 read the frame's lines at the
// same time and the second read is served by the XCD's L2. C5 PMC 36.7 -> 30.4 B/sample (fetch 23.5
// -> 17.1), group 1.743 -> 1.696 ms (3 interleaved runs, r4g).
// XG 2 (tuning): also interleaves the two passes -- XCD x's workgroups take, per group of 17, one
// frame's 8 pass-B row tiles and then one frame's 9 pass-A items, instead of every pass-B tile of
// the launch first (the Infinity-Cache reads of pass B beside the HBM reads of pass A all launch
// long, rather than one phase after the other).
template <bool ZM, int CP, int XG = 0>
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
    int g, r;                        // pass-A frame g: 8 column tiles (r < 8), its VFO block (r = 8)
    if constexpr (XG == 3) {
        if ((int)blockIdx.x < nB) {
            passB_tile<256, 32, ZM>(lds, blockIdx.x, scratchB, framesB, 256, logN, tw2, outB, zoomB);
            return;
        }
        const int i = blockIdx.x - nB, k = i >> 3, kk = k % 12;
        g = 8 * (k / 12) + (i & 7);
        if (g >= framesA) return;
        if (kk < 4) {
            vfo_quarter_block(v, g, kk);
            return;
        }
        passA_tile<256, 32, CP>(lds, g * 8 + kk - 4, in, frameStride, framesA, win, nz, 256, logN, tw1, tfull, scratchA);
        return;
    } else if constexpr (XG == 2) {
        const int i = blockIdx.x, k = i >> 3, kk = k % 17;
        const int gs = 8 * (k / 17) + (i & 7);   // frame slot of this XCD lane
        if (kk < 8) {
            if (gs < framesB) passB_tile<256, 32, ZM>(lds, gs * 8 + kk, scratchB, framesB, 256, logN, tw2, outB, zoomB);
            return;
        }
        g = gs;
        r = kk == 8 ? 8 : kk - 9;
        if (g >= framesA) return;
    } else {
    if ((int)blockIdx.x < nB) {
        passB_tile<256, 32, ZM>(lds, blockIdx.x, scratchB, framesB, 256, logN, tw2, outB, zoomB);
        return;
    }
    const int i = blockIdx.x - nB;   // (nB = 8 x pass-B frames: XCD lane of i = that of blockIdx.x)
    if constexpr (XG == 1) {
        const int k = i >> 3, kk = k % 9;
        g = 8 * (k / 9) + (i & 7);
        r = kk == 0 ? 8 : kk - 1;
        if (g >= framesA) return;    // (padding of the last group of 8 frames)
    } else {
        g = i / 9;
        r = i % 9;
    }
    }
    if (r == 8) vfo_frame_block(v, g);
    else passA_tile<256, 32, CP>(lds, g * 8 + r, in, frameStride, framesA, win, nz, 256, logN, tw1, tfull, scratchA);
}

// ---- one-pass 64k spectrum (round 4): no intermediate leaves the CU ---------------------------
// N = 65536 as four 16,384-point transforms (one radix-4 decimation-in-frequency step). Workgroup
// (f, r) computes the bins 4 m + r of frame f:
//   X[4 m + r] = sum_{n < M} W_M^(n m) y_r[n],   y_r[n] = W_N^(n r) sum_{j < 4} W_4^(j r) w[n + M j] x[n + M j],
// M = 16384. The 16k transform is M = 32 x 32 x 16 on one CU:
//   stage 1 (registers): thread t holds y_r[t + 512 i], i < 32, straight from its loads (the four
//     quarters combined as they arrive); a radix-32 DFT over i and the twiddle W_M^(t k2) W_N^(t r)
//     = W_N^(t (4 k2 + r)) (one exact fp64-built table value) give A[t][k2];
//   stage 2 (LDS): per (k2, t0), a radix-32 DFT over t1 of A[t0 + 16 t1][k2], twiddle W_512^(t0 q1);
//   stage 3 (LDS): per (k2, q1), a radix-16 DFT over t0 -> Y[k2 + 32 q1 + 1024 q2], dB, store.
// The four workgroups of a frame are consecutive on one XCD (round-robin dispatch: workgroup b runs
// on XCD b mod 8), so the frame is fetched from HBM once and read by the other three from that XCD's
// L2. Fabric traffic per sample is then the input (8 B) and the dB row (4 B): the two-pass transform's
// 16 B of intermediate are gone. With a VFO (VFO = true) each workgroup first runs quarter r of the
// VFO stage 1 (vfo_quarter_block: the same segments as fir_rows_kernel, so bit-identical), which is
// the frame's first reader. Zoom (ZM): each workgroup writes the max of its 8 bins of every 32-bin
// zoom column to zpart[f][r][o]; fft_1p_zoom_kernel folds the four.
// LDS image: 32 rows k2 of 544 used float2 (stage 1: column pad16(t); stage 2: column 17 q1 +
// (t0 ^ ((k2 >> 1) & 15))), row stride 560 (= 16 mod 32): every stage-2/3 access of a half-wave hits
// 32 distinct 8-byte bank pairs.
namespace op1 {
constexpr int M = 16384;
constexpr int RS = 560;                 // LDS row stride (float2)
constexpr int TW512 = 32 * RS;          // W_512^(t0 q1) at [q1][t0]
constexpr int W128 = TW512 + 512;       // W_128^(r i), i < 32
constexpr int LDS_BYTES = (W128 + 32) * 8;
constexpr int TAB = 4 * M + 512 + 128;  // device table: [r][k2][t] W_N^(t (4 k2 + r)), [q1][t0], [r][i]
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

// stage-1 twiddles W_N^(t (4 k2 + r)): 0 = one exact table value each (128 KB per workgroup from L2);
// 1 = an fp64 recurrence W_N^(t r) (W_N^(4 t))^k2 from two values of an fp64 table, rounded once
// (group 1.942 -> 1.893 ms, r41pb; the 1p tests pass with both)
#ifndef SDRGPU_1P_TW
#define SDRGPU_1P_TW 1
#endif
#ifndef SDRGPU_1P_PB
#define SDRGPU_1P_PB 4   // sample rows per load batch
#endif
#ifdef SDRGPU_1P_TIMING   // (measurement builds) per-workgroup phase timestamps, wave 0
__device__ unsigned long long g_1p_t[16384 * 8];
#define T1P(k) do { if (threadIdx.x == 0 && blockIdx.x < 16384) g_1p_t[blockIdx.x * 8 + (k)] = clock64(); } while (0)
#else
#define T1P(k) do {} while (0)
#endif
#ifndef SDRGPU_1P_VFO_UNROLL
#define SDRGPU_1P_VFO_UNROLL 0   // (A/B) fft_1p256_kernel's two stage-1 segments per lane group unrolled
#endif
#ifndef SDRGPU_1P_NT
#define SDRGPU_1P_NT 0   // (A/B) fft_1p256_kernel's dB rows as streaming stores
#endif
#ifndef SDRGPU_1P_WIDE
#define SDRGPU_1P_WIDE 0
#endif
#ifndef SDRGPU_1P_VFO_LAST
#define SDRGPU_1P_VFO_LAST 0   // (A/B) the VFO quarter after the transform instead of before it
#endif
#ifndef SDRGPU_1P_PB2
#define SDRGPU_1P_PB2 2   // (HALF) sample rows per load batch at the 128-VGPR budget
#endif
// HALF (SDRGPU_FFT_1P=2): the LDS image holds 16 rows k2 at a time (76 KB: two workgroups per CU, 128
// VGPRs): stage 1's 32 outputs stay in registers, and rows 0-15, then 16-31, go through stages 2 and 3
template <bool ZM, bool VFO, bool HALF = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(HALF ? 4 : 1))) void fft_1p_kernel(
    const float2* __restrict__ in, long long frameStride, int frames, const float* __restrict__ win, int nz,
    const float2* __restrict__ tab, const double2* __restrict__ tab64, float* __restrict__ out, float* __restrict__ zpart,
    VfoWork v) {
    using op1::M;
    using op1::RS;
    constexpr int TW512 = (HALF ? 16 : 32) * RS, W128 = TW512 + 512;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if constexpr (VFO) {
        if (v.hist && blockIdx.x == gridDim.x - 1) {   // the stage's history carry (fir.h:80)
            (void)fir_hist_block<float2, true, false>(v.a);
            return;
        }
    }
    const int b = blockIdx.x, k = b >> 3;
    const int f = 8 * (k >> 2) + (b & 7), r = k & 3;
    if (f >= frames) return;
    T1P(0);
    if constexpr (VFO && !SDRGPU_1P_VFO_LAST) vfo_quarter_block(v, f, r);
    T1P(1);
    const int t = threadIdx.x;
    float2* tw512 = lds + TW512;
    float2* w128 = lds + W128;
    tw512[t] = tab[4 * M + t];
    if (t < 32) w128[t] = tab[4 * M + 512 + 32 * r + t];
    // stage 1: y_r[t + 512 i] from the four quarters. W_4^(j r): (u0 + s u2) + W_4^r (u1 + s u3), s = (-1)^r
    const float s = (r & 1) ? -1.0f : 1.0f;
    const float fx = r == 0 ? 1.0f : (r == 2 ? -1.0f : 0.0f), fy = r == 1 ? -1.0f : (r == 3 ? 1.0f : 0.0f);
    const float2* xf = in + (long long)f * frameStride;
    float2 z[32];
    auto combine = [&](int i, const float2 (&xv)[4], const float (&wv)[4]) {
        float2 u[4];
#pragma unroll
        for (int j = 0; j < 4; j++) u[j] = make_float2(xv[j].x * wv[j], xv[j].y * wv[j]);
        const float2 a = make_float2(fmaf(s, u[2].x, u[0].x), fmaf(s, u[2].y, u[0].y));
        const float2 q = make_float2(fmaf(s, u[3].x, u[1].x), fmaf(s, u[3].y, u[1].y));
        // W_4^r q with W_4^r in {1, -i, -1, i}: one of fx, fy is 0, the other +-1 (exact products)
        z[i] = make_float2(a.x + (fx * q.x - fy * q.y), a.y + (fx * q.y + fy * q.x));
    };
    double2 c0, st;   // (SDRGPU_1P_TW 1) W_N^(t r), W_N^(4 t): loaded first, used after the loads
    if constexpr (SDRGPU_1P_TW == 1 && !HALF) {
        c0 = tab64[t * r];
        st = tab64[4 * t];
    }
    // batches of PB sample rows (4 PB loads of x and of w each), the next batch's loads in flight while
    // this one is combined (two batches of registers; issued all at once, the loads spill)
    constexpr int PB = HALF ? SDRGPU_1P_PB2 : SDRGPU_1P_PB, NB = 32 / PB;
    auto pipeline = [&](auto&& ld) {
        float2 xv[2][PB][4];
        float wv[2][PB][4];
        auto issue = [&](int bb, float2 (&xb)[PB][4], float (&wb)[PB][4]) {
#pragma unroll
            for (int ii = 0; ii < PB; ii++)
#pragma unroll
                for (int j = 0; j < 4; j++) ld(512 * (PB * bb + ii) + M * j, xb[ii][j], wb[ii][j]);
        };
        issue(0, xv[0], wv[0]);
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            if (bb + 1 < NB) issue(bb + 1, xv[(bb + 1) & 1], wv[(bb + 1) & 1]);
#pragma unroll
            for (int ii = 0; ii < PB; ii++) combine(PB * bb + ii, xv[bb & 1][ii], wv[bb & 1][ii]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // SDRGPU_1P_WIDE: half the load instructions (the vmcnt cap of 63 per wave bounds the bytes in
    // flight): lanes 2u and 2u + 1 load rows i and i + 1 of the adjacent sample pair (t, t + 1) as one
    // 16-B load each (8-B for the window) and swap the halves the other lane needs (DPP)
    auto pipeline2 = [&](auto&& ld2) {
        constexpr int PP = PB / 2;
        const int lane = t & 63;
        const bool odd = (t & 1) != 0;
        float4 xr[2][PP][4];
        float2 wr[2][PP][4];
        auto issue = [&](int bb, float4 (&xb)[PP][4], float2 (&wb)[PP][4]) {
#pragma unroll
            for (int pp = 0; pp < PP; pp++)
#pragma unroll
                for (int j = 0; j < 4; j++) ld2(512 * (PB * bb + 2 * pp) + M * j, xb[pp][j], wb[pp][j]);
        };
        issue(0, xr[0], wr[0]);
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            if (bb + 1 < NB) issue(bb + 1, xr[(bb + 1) & 1], wr[(bb + 1) & 1]);
#pragma unroll
            for (int pp = 0; pp < PP; pp++) {
                float2 x0[4], x1[4];
                float w0[4], w1[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    // even lane: (x(t, i), x(t + 1, i)); odd lane: (x(t - 1, i + 1), x(t, i + 1))
                    const float4 X = xr[bb & 1][pp][j];
                    const float2 Wv = wr[bb & 1][pp][j];
                    const float r0 = xchg<1>(odd ? X.x : X.z, lane), r1 = xchg<1>(odd ? X.y : X.w, lane);
                    x0[j] = odd ? make_float2(r0, r1) : make_float2(X.x, X.y);
                    x1[j] = odd ? make_float2(X.z, X.w) : make_float2(r0, r1);
                    const float rw = xchg<1>(odd ? Wv.x : Wv.y, lane);
                    w0[j] = odd ? rw : Wv.x;
                    w1[j] = odd ? Wv.y : rw;
                }
                combine(PB * bb + 2 * pp, x0, w0);
                combine(PB * bb + 2 * pp + 1, x1, w1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    if (SDRGPU_1P_WIDE && nz >= 65536 && ((uintptr_t)xf & 15) == 0) {
        const __amdgpu_buffer_rsrc_t rx = brsrc(xf, 65536u * 8u), rw = brsrc(win, 65536u * 4u);
        const int o = t + 511 * (t & 1);   // the pair's first sample, in row i (even lane) or i + 1 (odd lane)
        pipeline2([&](int n0, float4& xo, float2& wo) {
            xo = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, o * 8, n0 * 8, 0));
            wo = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rw, o * 4, n0 * 4, 0));
        });
    } else if (nz >= 65536) {   // no zero padding (workgroup-uniform): the row offset rides in soffset
        const __amdgpu_buffer_rsrc_t rx = brsrc(xf, 65536u * 8u), rw = brsrc(win, 65536u * 4u);
        pipeline([&](int n0, float2& xo, float& wo) {
            xo = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, t * 8, n0 * 8, 0));
            wo = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, t * 4, n0 * 4, 0));
        });
    } else {             // zero-padded frame: range-checked loads, the offset in the per-lane part (past nz: 0)
        const __amdgpu_buffer_rsrc_t rx = brsrc(xf, (unsigned)nz * 8u), rw = brsrc(win, (unsigned)nz * 4u);
        pipeline([&](int n0, float2& xo, float& wo) {
            xo = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, (t + n0) * 8, 0, 0));
            wo = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, (t + n0) * 4, 0, 0));
        });
    }
    T1P(2);
    __syncthreads();   // (w128, tw512)
#pragma unroll
    for (int i = 1; i < 32; i++) z[i] = cmul(z[i], w128[i]);   // W_128^(r i) = W_N^(512 r i)
    dft32(z);
    float* of = out + ((long long)f << 16);
    if constexpr (HALF) {
        double2 c = tab64[t * r];   // (loaded here: at 128 VGPRs they do not stay live through the loads)
        st = tab64[4 * t];
#pragma unroll
        for (int k2 = 0; k2 < 32; k2++) {
            z[k2] = cmul(z[k2], make_float2((float)c.x, (float)c.y));
            if (k2 < 31) c = zmul(c, st);
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int kl = 0; kl < 16; kl++) lds[kl * RS + pad16(t)] = z[16 * h + kl];
            __syncthreads();
            // stage 2 on rows k2 = 16 h + kl: (kl, t0) = (t >> 4, t & 15), the first 256 threads
            const int kl2 = (t >> 4) & 15, t0 = t & 15, k22 = 16 * h + kl2;
            float2 a[32];
            if (t < 256) {
#pragma unroll
                for (int t1 = 0; t1 < 32; t1++) a[t1] = lds[kl2 * RS + t0 + 17 * t1];
                dft32(a);
#pragma unroll
                for (int q1 = 1; q1 < 32; q1++) a[q1] = cmul(a[q1], lds[TW512 + 16 * q1 + t0]);
            }
            __syncthreads();
            if (t < 256) {
                const int sw = t0 ^ ((k22 >> 1) & 15);
#pragma unroll
                for (int q1 = 0; q1 < 32; q1++) lds[kl2 * RS + 17 * q1 + sw] = a[q1];
            }
            __syncthreads();
            // stage 3: (kl, q1) = (t & 15, t >> 4)
            const int kl = t & 15, q1 = t >> 4, k2 = 16 * h + kl, sw = (k2 >> 1) & 15;
            float2 c3[16];
#pragma unroll
            for (int t0 = 0; t0 < 16; t0++) c3[t0] = lds[kl * RS + 17 * q1 + (t0 ^ sw)];
            dft16(c3);
            float dv[16];
#pragma unroll
            for (int q2 = 0; q2 < 16; q2++) {
                dv[q2] = db_of(c3[q2]);
                of[4 * (k2 + 32 * q1 + 1024 * q2) + r] = dv[q2];
            }
            if constexpr (ZM) {   // max over the 8 lanes kl & 7 (zoom column (k2 >> 3) + 4 q1 + 128 q2)
                const int lane = t & 63;
                tr_step<1, 8>(dv, lane);
                tr_step<2, 4>(dv, lane);
                tr_step<4, 2>(dv, lane);
                const int q2 = ((lane & 1) << 3) | ((lane & 2) << 1) | (lane & 4) >> 1;
                float* zp = zpart + ((long long)(4 * f + r) << 11) + (k2 >> 3) + 4 * q1 + 128 * q2;
                zp[0] = dv[0];
                zp[128] = dv[1];
            }
            if (h == 0) __syncthreads();   // (stage 3's reads before the next rows land)
        }
        if constexpr (VFO && SDRGPU_1P_VFO_LAST) vfo_quarter_block(v, f, r);
        return;
    }
    if constexpr (SDRGPU_1P_TW == 1) {
        double2 c = c0;
#pragma unroll
        for (int k2 = 0; k2 < 32; k2++) {
            lds[k2 * RS + pad16(t)] = cmul(z[k2], make_float2((float)c.x, (float)c.y));
            if (k2 < 31) c = zmul(c, st);
        }
    } else {
#pragma unroll
        for (int k2 = 0; k2 < 32; k2++) lds[k2 * RS + pad16(t)] = cmul(z[k2], tab[(32 * r + k2) * 512 + t]);   // W_N^(t (4 k2 + r))
    }
    __syncthreads();
    T1P(3);
    // stage 2: (k2, t0) = (t >> 4, t & 15)
    {
        const int k2 = t >> 4, t0 = t & 15;
        float2 a[32];
#pragma unroll
        for (int t1 = 0; t1 < 32; t1++) a[t1] = lds[k2 * RS + t0 + 17 * t1];
        dft32(a);
#pragma unroll
        for (int q1 = 1; q1 < 32; q1++) a[q1] = cmul(a[q1], tw512[16 * q1 + t0]);
        __syncthreads();
        const int sw = t0 ^ ((k2 >> 1) & 15);
#pragma unroll
        for (int q1 = 0; q1 < 32; q1++) lds[k2 * RS + 17 * q1 + sw] = a[q1];
    }
    __syncthreads();
    T1P(4);
    // stage 3: (k2, q1) = (p & 31, p >> 5), p = t, t + 512
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int p = t + 512 * h, k2 = p & 31, q1 = p >> 5, sw = (k2 >> 1) & 15;
        float2 c[16];
#pragma unroll
        for (int t0 = 0; t0 < 16; t0++) c[t0] = lds[k2 * RS + 17 * q1 + (t0 ^ sw)];
        dft16(c);
        float dv[16];
#pragma unroll
        for (int q2 = 0; q2 < 16; q2++) {
            dv[q2] = db_of(c[q2]);
            of[4 * (k2 + 32 * q1 + 1024 * q2) + r] = dv[q2];
        }
        if constexpr (ZM) {   // max over the 8 lanes k2 & 7 (zoom column (k2 >> 3) + 4 q1 + 128 q2)
            const int lane = t & 63;
            tr_step<1, 8>(dv, lane);
            tr_step<2, 4>(dv, lane);
            tr_step<4, 2>(dv, lane);
            // lane bits (b0 b1 b2) now select q2 = 8 b0 + 4 b1 + 2 b2 + i in dv[i], i < 2
            const int q2 = ((lane & 1) << 3) | ((lane & 2) << 1) | (lane & 4) >> 1;
            float* zp = zpart + ((long long)(4 * f + r) << 11) + (k2 >> 3) + 4 * q1 + 128 * q2;
            zp[0] = dv[0];
            zp[128] = dv[1];
        }
    }
    T1P(5);
    if constexpr (VFO && SDRGPU_1P_VFO_LAST) vfo_quarter_block(v, f, r);
}
#ifdef SDRGPU_1P_TIMING
extern "C" int sdrgpu_debug_1p_times(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_1p_t), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

// SDRGPU_FFT_1P=3: the half-image transform with 256-thread workgroups (2 per CU at 76 KB of LDS and up
// to 256 VGPRs each: one workgroup's loads wait while the other one computes). Thread t takes the stage-1
// columns t and t + 256; stages 2 and 3 as in the HALF mode (the 256 threads are stage 2's butterflies).
// SV (SDRGPU_FFT_1P=4): the VFO quarters as workgroups of their own, a frame's 4 quarters dispatched
// before its 4 transform workgroups on the same XCD (they fetch the frame; the transforms read it from L2)
template <bool ZM, bool VFO, bool SV = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void fft_1p256_kernel(const float2* __restrict__ in, long long frameStride, int frames,
                                                        const float* __restrict__ win, int nz, const float2* __restrict__ tab,
                                                        const double2* __restrict__ tab64, float* __restrict__ out,
                                                        float* __restrict__ zpart, VfoWork v) {
    using op1::M;
    using op1::RS;
    constexpr int TW512 = 16 * RS, W128 = TW512 + 512;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if constexpr (VFO) {
        if (v.hist && blockIdx.x == gridDim.x - 1) {   // the stage's history carry (fir.h:80)
            (void)fir_hist_block<float2, true, false>(v.a);
            return;
        }
    }
    const int b = blockIdx.x, k = b >> 3;
    const int kq = SV ? (k & 7) : (k & 3) + 4;
    const int f = 8 * (SV ? k >> 3 : k >> 2) + (b & 7), r = kq & 3;
    if (f >= frames) return;
    const int t = threadIdx.x;
    if constexpr (VFO) {   // quarter r of the stage: 16 segments, 8 per pass of the 4 waves
      if (!SV || kq < 4) {
        const int lane = t & 63, wave = t >> 6;
#if SDRGPU_1P_VFO_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
        for (int sub = 0; sub < 2; sub++)
            fir_rows_segment<32, 5, true, false, 32, 32, true>(
                v.a, (long long)(v.frame0 + f) * 64 + r * 16 + sub * 8 + wave * 2 + (lane >> 5), lane);
        if (SV) return;
      }
    }
    lds[TW512 + t] = tab[4 * M + t];
    lds[TW512 + 256 + t] = tab[4 * M + 256 + t];
    if (t < 32) lds[W128 + t] = tab[4 * M + 512 + 32 * r + t];
    const float s = (r & 1) ? -1.0f : 1.0f;
    const float fx = r == 0 ? 1.0f : (r == 2 ? -1.0f : 0.0f), fy = r == 1 ? -1.0f : (r == 3 ? 1.0f : 0.0f);
    const float2* xf = in + (long long)f * frameStride;
    float2 z[2][32];
    auto combine = [&](int u, int i, const float2 (&xv)[4], const float (&wv)[4]) {
        float2 uu[4];
#pragma unroll
        for (int j = 0; j < 4; j++) uu[j] = make_float2(xv[j].x * wv[j], xv[j].y * wv[j]);
        const float2 a = make_float2(fmaf(s, uu[2].x, uu[0].x), fmaf(s, uu[2].y, uu[0].y));
        const float2 q = make_float2(fmaf(s, uu[3].x, uu[1].x), fmaf(s, uu[3].y, uu[1].y));
        z[u][i] = make_float2(a.x + (fx * q.x - fy * q.y), a.y + (fx * q.y + fy * q.x));
    };
    constexpr int NB = 32;   // one sample row (both columns, four quarters) per batch
    auto pipeline = [&](auto&& ld) {
        float2 xv[2][2][4];
        float wv[2][2][4];
        auto issue = [&](int i, float2 (&xb)[2][4], float (&wb)[2][4]) {
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int j = 0; j < 4; j++) ld(256 * u + 512 * i + M * j, xb[u][j], wb[u][j]);
        };
        issue(0, xv[0], wv[0]);
#pragma unroll
        for (int i = 0; i < NB; i++) {
            if (i + 1 < NB) issue(i + 1, xv[(i + 1) & 1], wv[(i + 1) & 1]);
#pragma unroll
            for (int u = 0; u < 2; u++) combine(u, i, xv[i & 1][u], wv[i & 1][u]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    if (nz >= 65536) {
        const __amdgpu_buffer_rsrc_t rx = brsrc(xf, 65536u * 8u), rw = brsrc(win, 65536u * 4u);
        pipeline([&](int n0, float2& xo, float& wo) {
            xo = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, t * 8, n0 * 8, 0));
            wo = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, t * 4, n0 * 4, 0));
        });
    } else {
        const __amdgpu_buffer_rsrc_t rx = brsrc(xf, (unsigned)nz * 8u), rw = brsrc(win, (unsigned)nz * 4u);
        pipeline([&](int n0, float2& xo, float& wo) {
            xo = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, (t + n0) * 8, 0, 0));
            wo = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, (t + n0) * 4, 0, 0));
        });
    }
    __syncthreads();   // (the LDS tables)
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int tu = t + 256 * u;
#pragma unroll
        for (int i = 1; i < 32; i++) z[u][i] = cmul(z[u][i], lds[W128 + i]);
        dft32(z[u]);
        if constexpr (SDRGPU_1P_TW == 1) {
            double2 c = tab64[tu * r];
            const double2 st = tab64[4 * tu];
#pragma unroll
            for (int k2 = 0; k2 < 32; k2++) {
                z[u][k2] = cmul(z[u][k2], make_float2((float)c.x, (float)c.y));
                if (k2 < 31) c = zmul(c, st);
            }
        } else {
#pragma unroll
            for (int k2 = 0; k2 < 32; k2++) z[u][k2] = cmul(z[u][k2], tab[(32 * r + k2) * 512 + tu]);
        }
    }
    float* of = out + ((long long)f << 16);
#pragma unroll
    for (int h = 0; h < 2; h++) {
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int kl = 0; kl < 16; kl++) lds[kl * RS + pad16(t + 256 * u)] = z[u][16 * h + kl];
        __syncthreads();
        {   // stage 2: (kl, t0) = (t >> 4, t & 15)
            const int kl = t >> 4, t0 = t & 15, k2 = 16 * h + kl;
            float2 a[32];
#pragma unroll
            for (int t1 = 0; t1 < 32; t1++) a[t1] = lds[kl * RS + t0 + 17 * t1];
            dft32(a);
#pragma unroll
            for (int q1 = 1; q1 < 32; q1++) a[q1] = cmul(a[q1], lds[TW512 + 16 * q1 + t0]);
            __syncthreads();
            const int sw = t0 ^ ((k2 >> 1) & 15);
#pragma unroll
            for (int q1 = 0; q1 < 32; q1++) lds[kl * RS + 17 * q1 + sw] = a[q1];
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 2; e++) {   // stage 3: (kl, q1) = (p & 15, p >> 4), p = t, t + 256
            const int p = t + 256 * e, kl = p & 15, q1 = p >> 4, k2 = 16 * h + kl, sw = (k2 >> 1) & 15;
            float2 c3[16];
#pragma unroll
            for (int t0 = 0; t0 < 16; t0++) c3[t0] = lds[kl * RS + 17 * q1 + (t0 ^ sw)];
            dft16(c3);
            float dv[16];
#pragma unroll
            for (int q2 = 0; q2 < 16; q2++) {
                dv[q2] = db_of(c3[q2]);
                if constexpr (SDRGPU_1P_NT) __builtin_nontemporal_store(dv[q2], &of[4 * (k2 + 32 * q1 + 1024 * q2) + r]);
                else of[4 * (k2 + 32 * q1 + 1024 * q2) + r] = dv[q2];
            }
            if constexpr (ZM) {
                const int lane = t & 63;
                tr_step<1, 8>(dv, lane);
                tr_step<2, 4>(dv, lane);
                tr_step<4, 2>(dv, lane);
                const int q2 = ((lane & 1) << 3) | ((lane & 2) << 1) | (lane & 4) >> 1;
                float* zp = zpart + ((long long)(4 * f + r) << 11) + (k2 >> 3) + 4 * q1 + 128 * q2;
                zp[0] = dv[0];
                zp[128] = dv[1];
            }
        }
        if (h == 0) __syncthreads();
    }
}

// zoom[f][o] = max over the four workgroups' partial maxima (fft_1p_kernel's ZM)
__global__ __launch_bounds__(256) void fft_1p_zoom_kernel(const float* __restrict__ zpart, int frames, float* __restrict__ zoom) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)frames * 2048) return;
    const long long f = i >> 11, o = i & 2047;
    const float* p = zpart + (f << 13) + o;
    zoom[i] = fmaxf(fmaxf(p[0], p[2048]), fmaxf(p[4096], p[6144]));
}

// ---- the C5 launch group as ONE persistent launch with per-frame dataflow (round 4, tuning:
// SDRGPU_FFT_VFO_PERSIST). Each workgroup reads its XCD id (HW_REG_XCC_ID) and takes items from that
// XCD's queue: frame f = 8 j + x belongs to XCD x; its 12 first-pass items (4 stage-1 quarters, 8
// column tiles) come at queue step j and its 8 pass-B row tiles at step j + lag, so pass B of a frame
// runs on the XCD that wrote its intermediate, a few frames later, from that XCD's L2 / the Infinity
// Cache -- no launch boundaries, no chunk drains, and the intermediate's working set is ~lag frames
// per XCD instead of a 128-MB chunk. The intermediate lives in a ring of R frame slots per XCD.
// Dependencies (same XCD, so one L2 is the coherence point; the producer drains its stores before
// counting, the consumer drops its L1 before reading):
//   pass-B tile of f   waits for the 8 column tiles of f   (aDone[f] == 8)
//   column tile of f   waits for the 8 pass-B tiles of f - 8 R, the slot's previous user (bDone == 8)
// Every wait points at an item dequeued earlier by a running workgroup, so there is no deadlock for
// any residency; every spin is bounded (on timeout the kernel raises err[0] and goes on).
constexpr int kPersistRing = 32;   // slots per XCD
struct PersistWork {
    VfoWork v;
    int frames, lag;
    int* q;          // [8] per-XCD item counters (zeroed per call)
    int* aDone;      // [frames]
    int* bDone;      // [frames]
    int* err;        // [1] spin timeouts
};
__device__ __forceinline__ bool persist_wait(const int* c, int target, int* err) {
    for (int k = 0; k < (1 << 22); k++) {
        if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
        __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_fetch_add(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
}
// (the item bodies as separate functions: inlined into one loop their registers add up and the
// kernel spilled 37 VGPRs at the 128-VGPR budget)
__device__ __attribute__((noinline)) void persist_quarter(const VfoWork& v, int f, int q) { vfo_quarter_block(v, f, q); }
__device__ __attribute__((noinline)) void persist_tile_a(float2* lds, int r, const float2* x, long long N, const float* win,
                                                         int nz, int logN, const float2* tw1, const float2* tfull, float2* slot) {
    passA_tile<256, 32, 0>(lds, r, x, N, 1, win, nz, 256, logN, tw1, tfull, slot);
}
template <bool ZM>
__device__ __attribute__((noinline)) void persist_tile_b(float2* lds, int r, const float2* slot, int logN, const float2* tw2,
                                                         float* o, float* z) {
    passB_tile<256, 32, ZM>(lds, r, slot, 1, 256, logN, tw2, o, z);
}
template <bool ZM, bool INL = false>   // INL (tuning): the item bodies inlined (spills 37 VGPRs)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void fft_vfo_persist_kernel(
    const float2* __restrict__ in, float* __restrict__ out, float* __restrict__ zoom, const float* __restrict__ win, int nz,
    int logN, const float2* __restrict__ tw1, const float2* __restrict__ tw2, const float2* __restrict__ tfull,
    float2* __restrict__ ring, PersistWork w) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ int item;
    const int tid = threadIdx.x;
    if (blockIdx.x == 0) (void)fir_hist_copy<float2, true, false>(w.v.a);   // the stage's history carry (fir.h:80)
    const int x = (int)(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7);   // HW_REG_XCC_ID[2:0]
    const int J = (w.frames - x + 7) / 8;   // this XCD's frames: f = 8 j + x, j < J
    const int L = w.lag;
    const int a = J < L ? J : L, b = J < L ? L : J, c2 = J < L ? 0 : 20;
    const int total = 20 * J;
    const long long N = 1LL << logN;
    // the next item's index is drawn while the current one runs (an atomic round trip per item would
    // otherwise serialise with the work)
    int nxt = 0;
    if (tid == 0) nxt = __hip_atomic_fetch_add(&w.q[x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        __syncthreads();   // (the previous item's last LDS reads and its use of `item` are done)
        if (tid == 0) {
            item = nxt;
            if (nxt < total) nxt = __hip_atomic_fetch_add(&w.q[x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        int i = item;
        if (i >= total) break;
        int st, k;   // queue step, item within it: k < 12 first pass (0-3 quarters, 4-11 tiles), k >= 12 pass B
        if (i < 12 * a) {
            st = i / 12; k = i % 12;
        } else if ((i -= 12 * a) < c2 * (b - a)) {
            st = a + i / c2; k = i % c2;
        } else {
            i -= c2 * (b - a);
            st = b + i / 8; k = 12 + i % 8;
        }
        if (k < 12) {
            const int j = st, f = 8 * j + x;
            if (k < 4) {
                if constexpr (INL) vfo_quarter_block(w.v, f, k);
                else persist_quarter(w.v, f, k);
                continue;
            }
            float2* slot = ring + (long long)(x * kPersistRing + j % kPersistRing) * N;
            if (j >= kPersistRing) {   // the slot's previous frame must be out of pass B
                if (tid == 0) (void)persist_wait(&w.bDone[f - 8 * kPersistRing], 8, w.err);
                __syncthreads();
            }
            if constexpr (INL) passA_tile<256, 32, 0>(lds, k - 4, in + (long long)f * N, N, 1, win, nz, 256, logN, tw1, tfull, slot);
            else persist_tile_a(lds, k - 4, in + (long long)f * N, N, win, nz, logN, tw1, tfull, slot);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's intermediate stores are in L2
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(&w.aDone[f], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const int j = st - L, f = 8 * j + x;
            const float2* slot = ring + (long long)(x * kPersistRing + j % kPersistRing) * N;
            if (tid == 0) (void)persist_wait(&w.aDone[f], 8, w.err);
            __syncthreads();
            asm volatile("buffer_inv sc0" ::: "memory");   // no stale L1 lines of the slot's previous frame
            if constexpr (INL)
                passB_tile<256, 32, ZM>(lds, k - 12, slot, 1, 256, logN, tw2, out + (long long)f * N,
                                        ZM ? zoom + (long long)f * (N / 32) : nullptr);
            else persist_tile_b<ZM>(lds, k - 12, slot, logN, tw2, out + (long long)f * N, ZM ? zoom + (long long)f * (N / 32) : nullptr);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (its slot reads are done before the slot is freed)
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(&w.bDone[f], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
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
    fir_tail_block(t, w, w == t.G - 1, lds, gs);
}

// ---------------------------------------------------------------- host side
struct FftPlan {
    int device = 0, N = 0, logN = 0, nz = 0;
    int N1 = 0, N2 = 0;               // two-pass split (N1 * N2 = N); N1 = 0 -> single pass
    DevBuf win, tw1, tw2, tfull, scratch;
    int chunkFrames = 1;
    int sa = 16, sb = 32;             // pass-A columns / pass-B rows per workgroup (tuning)
    float2* cur = nullptr;            // scratch buffer of the chunk being launched
    int sa2 = 0;                      // paired pass-A columns per workgroup (0: paired kernel off)
    int pipe1m = 1;                   // N1 = N2 = 1024: persistent software-pipelined passes (SDRGPU_FFT_1M=0 off)
    int gridA = 0, gridB = 0, gridM = 0;   // their grids (resident workgroups); gridM: the merged 1M launches
    int merge1m = 0;                  // SDRGPU_FFT_MERGE_1M (tuning): merged pass-B(c-1) + pass-A(c) launches
    // pass-A variant (SDRGPU_FFT_1M_VAR, tuning: fft_passA_1m_kernel's VAR). Default 128: the
    // tile-major intermediate (each pass-A tile's 128 KB written contiguously, 1 KB per store
    // instruction instead of eight 128-B row pieces; pass B reads 16-column pieces of 128 B):
    // 1.89 vs 1.94 ms per C2 step (3 interleaved runs, one box)
    int var1m = 128;
    int var1mB = 64;                  // pass-B variant (SDRGPU_FFT_1M_VARB, tuning: 64 XCD grouping; 16 / 32 measurement only)
    // columns / rows per workgroup of the 1M passes (SDRGPU_FFT_1M_SA / SB, tuning). Pass B at 8
    // rows (2 workgroups per CU) with XCD-grouped row blocks (4 blocks whose 32-B dB segments share
    // 128-B lines on one XCD): 1.93 vs 1.97 ms per C2 step (3 interleaved runs on each of two boxes);
    // without the grouping 2.06. Pass A at 8 columns: 2.24 (XCD-grouped) / 2.70 ms.
    int sA1m = 16, sB1m = 8;
    DevBuf wt;                        // fp64 W_N^(256 j), W_N^j (j < 256) for the 1M pass A
    hipStream_t own = nullptr;
    PinnedBuf pin_in, pin_out;
    DevBuf dev_in, dev_out;
    // two-stream chunk pipeline: pass A of chunk i+1 (caller stream) overlaps pass B of chunk
    // i (second stream), scratch double-buffered. Measured SLOWER (64k: 2.16 vs 1.86 ms, 1M:
    // 2.98 vs 2.39 ms per step; the concurrent passes evict each other's Infinity-Cache
    // working set), so it is off unless SDRGPU_FFT_PIPE=1.
    int pipe = 0;
    // merged pass-B(c) + pass-A(c+1) launches (64k split): one launch boundary per chunk
    // instead of two; 1.87 -> 1.73 ms per 2^28 samples (A/B on one box). SDRGPU_FFT_MERGE=0 off.
    int merge = 1;
    StreamOrder order;                // scratch is per plan: calls on different streams are serialised
    sdrgpu_zoom* zoom = nullptr;      // execute_zoom's unfused zoom (sizes other than N / 32)
    int zoomSize = 0;
    hipStream_t s2 = nullptr;
    hipEvent_t evFork = nullptr, evJoin = nullptr, evA[2] = {nullptr, nullptr}, evB[2] = {nullptr, nullptr};
    // SDRGPU_FFT_VFO_SIDE=1 (tuning): the fused VFO's later stages on the side stream, beside the last
    // pass-B launch. Measured slower: C5 step 1.725 vs 1.705 ms (3 interleaved runs, r4i; the overlap
    // stretches the last launch more than it hides), so they run after it on the call's stream
    int vfoSide = 0;
    int vfoPersist = 0;   // SDRGPU_FFT_VFO_PERSIST (tuning): the group as one persistent dataflow launch
    int persistLag = 6;   // SDRGPU_FFT_PERSIST_LAG (tuning): queue steps between a frame's two passes
    DevBuf persistCtl;    // its counters: q[8], aDone[frames], bDone[frames], err
    int gridP = 0;
    DevBuf scratch2;
    Fft64Plan* f64 = nullptr;         // sdrgpu_fft_set_precision(h, 1): the fp64-interior kernels (fft64.hip)
    // sdrgpu_fft_set_timing: HIP events around each call's spectrum launch group (the fused VFO
    // stage included, the VFO's later stages not), a ring of kTimed calls read by sdrgpu_fft_group_times
    static constexpr int kTimed = 256;
    bool timing = false;
    hipEvent_t tev[kTimed][2] = {};
    long long tcalls = 0;
    int vfoCP = 0;                    // fused VFO launches: pass-A input cache policy (SDRGPU_FFT_VFO_CP, tuning)
    int vfoFuse = 1;                  // SDRGPU_FFT_VFO_FUSE=0 (tuning): spectrum and VFO as separate launch groups
    int fuseTail = 1;                 // SDRGPU_FFT_FUSE_TAIL=0 (tuning): the front end's VFO tail as a launch of its own
    // fft_vfo_kernel's launch order (SDRGPU_FFT_VFO_XCD, tuning): 0 a frame's 9 workgroups consecutive;
    // 1 XCD-grouped (group 1.732 -> 1.694 ms, r4d); 2 + passes interleaved (1.684 -> 1.679, noise, r4f);
    // 3 XCD-grouped with quarter-frame stage-1 workgroups (1.743 -> 1.696 ms, r4g), the default
    int vfoXcd = 3;
    // the 64k plan: one-pass spectrum launches (fft_1p_kernel), SDRGPU_FFT_1P (tuning)
    int onepass = 0;
    DevBuf tab1p, tab1p64, zpart;
};
// the plan's side stream and its events (the two-stream pipeline; the fused VFO's later stages)
static int ensure_side(FftPlan& p) {
    if (p.s2) return SDRGPU_OK;
    SDRGPU_HIP(hipStreamCreateWithFlags(&p.s2, hipStreamNonBlocking));
    SDRGPU_HIP(hipEventCreateWithFlags(&p.evFork, hipEventDisableTiming));
    SDRGPU_HIP(hipEventCreateWithFlags(&p.evJoin, hipEventDisableTiming));
    for (int k = 0; k < 2; k++) {
        SDRGPU_HIP(hipEventCreateWithFlags(&p.evA[k], hipEventDisableTiming));
        SDRGPU_HIP(hipEventCreateWithFlags(&p.evB[k], hipEventDisableTiming));
    }
    return SDRGPU_OK;
}
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

template <int LA, int SA, int LB, int SB, bool PAIRED, bool ZM = false>
static int launch_merged(const FftPlan& p, const float2* scratchB, int framesB, float* outB, const float2* in,
                         long long stride, int framesA, float2* scratchA, hipStream_t s, float* zoomB = nullptr) {
    auto k = fft_merged_kernel<LA, SA, LB, SB, PAIRED, ZM>;
    size_t lds = sizeof(float2) * std::max(SA * Lds<LA>::LS + ((PAIRED || LA == 256) ? LA : 0) + (LA == 256 && !PAIRED ? 256 : 0),
                                           SB * Lds<LB>::LS + (LB >= 256 ? 256 : 0));
    SDRGPU_CHECK(set_lds(k, lds));
    const int nB = (LA / SB) * framesB, nA = (LB / SA) * framesA;
    hipLaunchKernelGGL(k, dim3(nB + nA), dim3(SB * LB / 16), lds, s, nB, scratchB, framesB, outB, zoomB, in, stride, framesA,
                       p.win.as<float>(), p.nz, p.logN, p.tw1.as<float2>(), p.tw2.as<float2>(), p.tfull.as<float2>(),
                       scratchA);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int S, int CP, int VAR>
static int launch_passA_1m(FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    if (p.N2 % S) { set_error("fft: N2 %d not a multiple of %d columns", p.N2, S); return SDRGPU_ESTATE; }
    auto k = fft_passA_1m_kernel<S, CP, VAR>;
    size_t lds = sizeof(float2) * (S * Lds<1024>::LS + 1024 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    if (!p.gridA) {
        int per = 0, cus = 0;
        SDRGPU_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, S / 2 * 64, lds));
        SDRGPU_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p.device));
        p.gridA = std::max(1, per) * cus;
    }
    const int ntiles = (p.N2 / S) * frames;
    hipLaunchKernelGGL(k, dim3(std::min(p.gridA, ntiles)), dim3(S / 2 * 64), lds, s, in, stride, frames, p.win.as<float>(),
                       p.nz, p.N2, p.logN, p.tw1.as<float2>(), p.wt.as<double2>(), p.cur, MergeB{});
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

template <int S, int CP, int VAR = 0>
static int launch_passB_1m(FftPlan& p, int frames, float* out, hipStream_t s) {
    auto k = fft_passB_1m_kernel<S, CP, VAR>;
    size_t lds = sizeof(float2) * (S * Lds<1024>::LS + 1024 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    if (!p.gridB) {
        int per = 0, cus = 0;
        SDRGPU_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, S * 64, lds));
        SDRGPU_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p.device));
        p.gridB = std::max(1, per) * cus;
    }
    const int ntiles = (p.N1 / S) * frames;
    hipLaunchKernelGGL(k, dim3(std::min(p.gridB, ntiles)), dim3(S * 64), lds, s, p.cur, frames, p.N1, p.logN,
                       p.tw2.as<float2>(), out);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

// one merged 1M launch (fft_passA_1m_kernel<16, 2, 128, MERGED>): pass B of framesB frames of scratchB
// (0: none), then pass A of framesA frames into scratchA (0: none)
static int launch_merged_1m(FftPlan& p, const float2* scratchB, int framesB, float* outB, const float2* in, long long stride,
                            int framesA, float2* scratchA, hipStream_t s) {
    auto k = fft_passA_1m_kernel<16, 2, 128, true>;
    const size_t lds = sizeof(float2) * (16 * Lds<1024>::LS + 1024 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    if (!p.gridM) {
        int per = 0, cus = 0;
        SDRGPU_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, 512, lds));
        SDRGPU_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p.device));
        p.gridM = std::max(1, per) * cus;
    }
    const int tiles = std::max((p.N1 / 8) * framesB, (p.N2 / 16) * framesA);
    hipLaunchKernelGGL(k, dim3(std::min(p.gridM, tiles)), dim3(512), lds, s, in, stride, framesA, p.win.as<float>(), p.nz,
                       p.N2, p.logN, p.tw1.as<float2>(), p.wt.as<double2>(), scratchA,
                       MergeB{scratchB, framesB, p.N1, outB, p.tw2.as<float2>()});
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}

// the persistent 1M passes for one chunk, with the tuning variants. Pass B reads the layout pass A
// wrote: tile-major (pass A VAR 128, the default) or row-major (every other variant).
static int dispatch_1m(FftPlan& p, const float2* xc, long long stride, int nf, float* o, hipStream_t s) {
    if (p.pipe1m == 2) {   // (tuning) non-temporal streaming accesses, row-major
        SDRGPU_CHECK((launch_passA_1m<16, 2, 0>(p, xc, stride, nf, s)));
        return launch_passB_1m<16, 2>(p, nf, o, s);
    }
    if (p.pipe1m == 3 || p.pipe1m == 4) {   // (tuning) default layout with cached input loads (3), nt pass B loads (4)
        if (p.pipe1m == 3) SDRGPU_CHECK((launch_passA_1m<16, 0, 128>(p, xc, stride, nf, s)));
        else SDRGPU_CHECK((launch_passA_1m<16, 2, 128>(p, xc, stride, nf, s)));
        return p.pipe1m == 4 ? launch_passB_1m<8, 2, 64 | 128>(p, nf, o, s) : launch_passB_1m<8, 0, 64 | 128>(p, nf, o, s);
    }
    bool tm = false;
    if (p.sA1m == 8) {
        if (p.var1m == 73) SDRGPU_CHECK((launch_passA_1m<8, 0, 73>(p, xc, stride, nf, s)));
        else if (p.var1m & 64) SDRGPU_CHECK((launch_passA_1m<8, 0, 64>(p, xc, stride, nf, s)));
        else SDRGPU_CHECK((launch_passA_1m<8, 0, 0>(p, xc, stride, nf, s)));
    } else {
        switch (p.var1m) {
        // default: the input rows are read once, non-temporal (slc), so they do not push the 4 MB
        // window out of L2 (PMC fetch 18.15 -> 17.50 B/sample, C2 1.848 -> 1.798 ms, 3 interleaved
        // runs; non-temporal pass-B loads of the intermediate measured 2.41 ms: it must stay cached)
        case 128: SDRGPU_CHECK((launch_passA_1m<16, 2, 128>(p, xc, stride, nf, s))); tm = true; break;
        case 137: SDRGPU_CHECK((launch_passA_1m<16, 0, 137>(p, xc, stride, nf, s))); tm = true; break;
        case 144: SDRGPU_CHECK((launch_passA_1m<16, 0, 144>(p, xc, stride, nf, s))); tm = true; break;   // (measurement)
        case 160: SDRGPU_CHECK((launch_passA_1m<16, 0, 160>(p, xc, stride, nf, s))); tm = true; break;
        case 176: SDRGPU_CHECK((launch_passA_1m<16, 0, 176>(p, xc, stride, nf, s))); tm = true; break;
        case 9: SDRGPU_CHECK((launch_passA_1m<16, 0, 9>(p, xc, stride, nf, s))); break;
        case 16: SDRGPU_CHECK((launch_passA_1m<16, 0, 16>(p, xc, stride, nf, s))); break;
        case 32: SDRGPU_CHECK((launch_passA_1m<16, 0, 32>(p, xc, stride, nf, s))); break;
        case 48: SDRGPU_CHECK((launch_passA_1m<16, 0, 48>(p, xc, stride, nf, s))); break;
        default: SDRGPU_CHECK((launch_passA_1m<16, 0, 0>(p, xc, stride, nf, s))); break;
        }
    }
    if (tm) {
        switch (p.var1mB) {   // (16 / 32 / 48: measurement only)
        case 16: return launch_passB_1m<8, 0, 64 | 128 | 16>(p, nf, o, s);
        case 32: return launch_passB_1m<8, 0, 64 | 128 | 32>(p, nf, o, s);
        case 48: return launch_passB_1m<8, 0, 64 | 128 | 48>(p, nf, o, s);
        }
        return p.sB1m == 8 ? launch_passB_1m<8, 0, 64 | 128>(p, nf, o, s) : launch_passB_1m<16, 0, 128>(p, nf, o, s);
    }
    if (p.sB1m == 8) return (p.var1mB & 64) ? launch_passB_1m<8, 0, 64>(p, nf, o, s) : launch_passB_1m<8, 0, 0>(p, nf, o, s);
    switch (p.var1mB) {
    case 64: return launch_passB_1m<16, 0, 64>(p, nf, o, s);
    case 16: return launch_passB_1m<16, 0, 16>(p, nf, o, s);
    case 32: return launch_passB_1m<16, 0, 32>(p, nf, o, s);
    case 48: return launch_passB_1m<16, 0, 48>(p, nf, o, s);
    default: return launch_passB_1m<16, 0>(p, nf, o, s);
    }
}

static bool pipe1m_ok(const FftPlan& p, bool paired) { return p.pipe1m && paired && p.N1 == 1024 && p.N2 == 1024 && (p.nz % 2) == 0; }

// merged pass B (chunk c) + pass A (chunk c+1) launches: the 64k split (256 x 256, one-column
// pass A). The 1M split's merged form (paired pass A, pass B at 8 rows to match its 512
// threads) measured 12% SLOWER (2.68 vs 2.39 ms per 256 frames): pass B loses half its
// occupancy to pass A's 147 KB of LDS, so the 1M transform keeps separate launches.
static int dispatch_merged(const FftPlan& p, const float2* scratchB, int framesB, float* outB, const float2* in,
                           long long stride, int framesA, float2* scratchA, hipStream_t s, float* zoomB = nullptr) {
    if (zoomB) return launch_merged<256, 32, 256, 32, false, true>(p, scratchB, framesB, outB, in, stride, framesA, scratchA, s, zoomB);
    if (p.sa == 64) return launch_merged<256, 64, 256, 64, false>(p, scratchB, framesB, outB, in, stride, framesA, scratchA, s);
    if (p.sa == 32) return launch_merged<256, 32, 256, 32, false>(p, scratchB, framesB, outB, in, stride, framesA, scratchA, s);
    return launch_merged<256, 16, 256, 16, false>(p, scratchB, framesB, outB, in, stride, framesA, scratchA, s);
}
static bool merged_supported(const FftPlan& p, bool paired) {
    return !paired && p.N1 == 256 && p.N2 == 256 && (p.sa == 16 || ((p.sa == 32 || p.sa == 64) && p.sb == p.sa));
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

// pass-A column FFT length N1 with SA columns per workgroup (8*SA-byte row segments)
static int dispatch_passA(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    switch (p.N1) {
    case 64: return launch_passA<64, 16>(p, in, stride, frames, s);
    case 128: return launch_passA<128, 16>(p, in, stride, frames, s);
    case 256:
        if (p.sa == 64) return launch_passA<256, 64>(p, in, stride, frames, s);
        if (p.sa == 32) return launch_passA<256, 32>(p, in, stride, frames, s);
        return launch_passA<256, 16>(p, in, stride, frames, s);
    case 512: return launch_passA<512, 8>(p, in, stride, frames, s);
    case 1024:
        if (p.sa == 16) return launch_passA<1024, 16>(p, in, stride, frames, s);
        return launch_passA<1024, 8>(p, in, stride, frames, s);   // (sa 8 only on request)
    }
    set_error("fft: unsupported N1 %d", p.N1);
    return SDRGPU_EARG;
}

// paired-column pass A (16-B accesses); used when the input allows 16-B loads
static int dispatch_passA2(const FftPlan& p, const float2* in, long long stride, int frames, hipStream_t s) {
    switch (p.N1) {
    case 64: return launch_passA2<64, 32>(p, in, stride, frames, s);
    case 128: return launch_passA2<128, 32>(p, in, stride, frames, s);
    case 256:
        if (p.sa2 == 64) return launch_passA2<256, 64>(p, in, stride, frames, s);
        if (p.sa2 == 16) return launch_passA2<256, 16>(p, in, stride, frames, s);
        return launch_passA2<256, 32>(p, in, stride, frames, s);
    case 512: return launch_passA2<512, 16>(p, in, stride, frames, s);
    case 1024:
        if (p.sa2 == 8) return launch_passA2<1024, 8>(p, in, stride, frames, s);   // (tuning; 2.68 vs 2.10 ms)
        return launch_passA2<1024, 16>(p, in, stride, frames, s);
    }
    set_error("fft: unsupported N1 %d", p.N1);
    return SDRGPU_EARG;
}

static int dispatch_passB(const FftPlan& p, int frames, float* out, hipStream_t s, float* zoom = nullptr) {
    if (zoom) return launch_passB<256, 32, true>(p, frames, out, s, zoom);   // (zoom_fusable checked the plan)
    switch (p.N2) {
    case 64: return launch_passB<64, 32>(p, frames, out, s);
    case 128: return launch_passB<128, 32>(p, frames, out, s);
    case 256:
        if (p.sb == 64) return launch_passB<256, 64>(p, frames, out, s);
        if (p.sb == 16) return launch_passB<256, 16>(p, frames, out, s);
        return launch_passB<256, 32>(p, frames, out, s);
    case 512: return launch_passB<512, 16>(p, frames, out, s);
    case 1024:
        if (p.sb == 8) return launch_passB<1024, 8>(p, frames, out, s);   // (tuning; equal time)
        return launch_passB<1024, 16>(p, frames, out, s);
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
        if (const char* e = tuning_env("SDRGPU_FFT_N1")) {   // (tuning) another split, N1, N2 in [64, 1024]
            const int n1 = atoi(e);
            if (n1 >= 64 && n1 <= 1024 && (n1 & (n1 - 1)) == 0 && fftSize / n1 >= 64 && fftSize / n1 <= 1024) p.N1 = n1;
        }
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
        if (const char* e = tuning_env("SDRGPU_FFT_SA")) p.sa = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_SB")) p.sb = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_PIPE")) p.pipe = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_MERGE")) p.merge = atoi(e);
        p.chunkFrames = std::max(1, (int)((chunkMB << 20) / ((long long)fftSize * 8)));
        // paired-column pass A: +13% on the 1M transform (N1 = 1024), but slower than the
        // one-column kernel at N1 = 256 (64k: 2.05-2.10 vs 1.86 ms per 2^28 samples, A/B on
        // one box), so it is the default only for N1 >= 512
        p.sa2 = p.N1 >= 512 ? 16 : 0;
        if (const char* e = tuning_env("SDRGPU_FFT_SA2")) p.sa2 = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_1M")) p.pipe1m = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_MERGE_1M")) p.merge1m = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_1M_VAR")) p.var1m = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_1M_VARB")) p.var1mB = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_1M_SA")) p.sA1m = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_1M_SB")) p.sB1m = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_VFO_CP")) p.vfoCP = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_VFO_FUSE")) p.vfoFuse = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_VFO_XCD")) p.vfoXcd = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_VFO_SIDE")) p.vfoSide = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_VFO_PERSIST")) p.vfoPersist = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FFT_PERSIST_LAG")) p.persistLag = std::max(1, atoi(e));
        if (const char* e = tuning_env("SDRGPU_FFT_1P")) p.onepass = atoi(e);
        if (rc >= 0 && fftSize == 65536) {   // fft_1p_kernel's exact twiddles (op1::TAB)
            std::vector<float2> t(op1::TAB);
            auto w = [&](long long m) {
                const double a = -2.0 * M_PI * (double)(m % fftSize) / (double)fftSize;
                return make_float2((float)std::cos(a), (float)std::sin(a));
            };
            for (int r = 0; r < 4; r++)
                for (int k2 = 0; k2 < 32; k2++)
                    for (int tt = 0; tt < 512; tt++) t[(size_t)(32 * r + k2) * 512 + tt] = w((long long)tt * (4 * k2 + r));
            for (int q1 = 0; q1 < 32; q1++)
                for (int t0 = 0; t0 < 16; t0++) t[4 * op1::M + 16 * q1 + t0] = w(128LL * t0 * q1);
            for (int r = 0; r < 4; r++)
                for (int i = 0; i < 32; i++) t[4 * op1::M + 512 + 32 * r + i] = w(512LL * r * i);
            std::vector<double2> t64(2048);   // W_N^m, m < 2048, fp64 (SDRGPU_1P_TW 1)
            for (int m = 0; m < 2048; m++) {
                const double a = -2.0 * M_PI * (double)m / (double)fftSize;
                t64[m] = make_double2(std::cos(a), std::sin(a));
            }
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
    if (const char* e = tuning_env("SDRGPU_FFT_FUSE_TAIL")) p.fuseTail = atoi(e);
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

// the one-pass 64k launch (+ the zoom fold): 4 workgroups per frame, XCD-grouped in blocks of 8 frames
template <bool ZM, bool VFO>
static int launch_1p(FftPlan& p, const float2* in, long long stride, int frames, float* out, float* zoom, VfoWork v,
                     hipStream_t s) {
    const bool half = p.onepass >= 2, w256 = p.onepass >= 3, sv = VFO && p.onepass == 4;
    auto k = sv ? fft_1p256_kernel<ZM, VFO, true> : w256 ? fft_1p256_kernel<ZM, VFO> : half ? fft_1p_kernel<ZM, VFO, true>
                                                                                             : fft_1p_kernel<ZM, VFO, false>;
    const int ldsB = half ? (16 * op1::RS + 512 + 32) * 8 : op1::LDS_BYTES;
    SDRGPU_CHECK(set_lds(k, ldsB));
    if (ZM) SDRGPU_CHECK(p.zpart.ensure(sizeof(float) * 4 * 2048 * (size_t)frames));
    const int g = (sv ? 64 : 32) * ((frames + 7) / 8) + (VFO && v.hist ? 1 : 0);
    hipLaunchKernelGGL(k, dim3(g), dim3(w256 ? 256 : 512), ldsB, s, in, stride, frames, p.win.as<float>(), p.nz,
                       p.tab1p.as<float2>(), p.tab1p64.as<double2>(), out, ZM ? p.zpart.as<float>() : nullptr, v);
    SDRGPU_HIP(hipGetLastError());
    if (ZM) {
        const long long n = (long long)frames * 2048;
        hipLaunchKernelGGL(fft_1p_zoom_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p.zpart.as<float>(),
                           frames, zoom);
        SDRGPU_HIP(hipGetLastError());
    }
    return SDRGPU_OK;
}
static bool onepass_ok(const FftPlan& p) { return p.onepass && p.N == 65536 && p.tab1p.p && !p.f64; }

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
    if (onepass_ok(p)) {
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
        if (paired) SDRGPU_CHECK(dispatch_passA2(p, x, frameStride, std::min(p.chunkFrames, frames), s));
        else SDRGPU_CHECK(dispatch_passA(p, x, frameStride, std::min(p.chunkFrames, frames), s));
        for (int c = 1; c < nchunks; c++) {
            const int fB = (c - 1) * p.chunkFrames, nfB = p.chunkFrames;
            const int fA = c * p.chunkFrames, nfA = std::min(p.chunkFrames, frames - fA);
            SDRGPU_CHECK(dispatch_merged(p, sc[(c - 1) & 1], nfB, out + (long long)fB * p.N,
                                         x + (long long)fA * frameStride, frameStride, nfA, sc[c & 1], s, zoomAt(fB)));
        }
        const int fL = (nchunks - 1) * p.chunkFrames;
        p.cur = sc[(nchunks - 1) & 1];
        SDRGPU_CHECK(dispatch_passB(p, frames - fL, out + (long long)fL * p.N, s, zoomAt(fL)));
        return frames;
    }
    const bool pipe = p.pipe && nchunks > 1 && !zoom;
    if (pipe) {
        SDRGPU_CHECK(ensure_side(p));
        SDRGPU_CHECK(p.scratch2.ensure(p.scratch.bytes));
        SDRGPU_HIP(hipEventRecord(p.evFork, s));
        SDRGPU_HIP(hipStreamWaitEvent(p.s2, p.evFork, 0));
    }
    if (pipe1m_ok(p, paired) && !pipe && !zoom && p.merge1m && nchunks > 1 && p.var1m == 128 && p.sA1m == 16 && p.sB1m == 8 &&
        p.var1mB == 64) {
        // A(0); [B(c - 1) + A(c)] for c = 1 ..; B(last): the chunks alternate between two scratch buffers
        SDRGPU_CHECK(p.scratch2.ensure(p.scratch.bytes));
        float2* sc[2] = {p.scratch.as<float2>(), p.scratch2.as<float2>()};
        const int cf = p.chunkFrames;
        SDRGPU_CHECK(launch_merged_1m(p, nullptr, 0, nullptr, x, frameStride, std::min(cf, frames), sc[0], s));
        for (int c = 1; c < nchunks; c++) {
            const int fB = (c - 1) * cf, fA = c * cf;
            SDRGPU_CHECK(launch_merged_1m(p, sc[(c - 1) & 1], cf, out + (long long)fB * p.N, x + (long long)fA * frameStride,
                                          frameStride, std::min(cf, frames - fA), sc[c & 1], s));
        }
        const int fL = (nchunks - 1) * cf;
        SDRGPU_CHECK(launch_merged_1m(p, sc[(nchunks - 1) & 1], frames - fL, out + (long long)fL * p.N, nullptr, 0, 0, nullptr, s));
        return frames;
    }
    for (int c = 0; c < nchunks; c++) {
        const int f0 = c * p.chunkFrames;
        const int nf = std::min(p.chunkFrames, frames - f0);
        const float2* xc = x + (long long)f0 * frameStride;
        const int b = pipe ? (c & 1) : 0;
        p.cur = b ? p.scratch2.as<float2>() : p.scratch.as<float2>();
        if (pipe && c >= 2) SDRGPU_HIP(hipStreamWaitEvent(s, p.evB[b], 0));   // buffer b free again
        if (pipe1m_ok(p, paired) && !pipe) {
            SDRGPU_CHECK(dispatch_1m(p, xc, frameStride, nf, out + (long long)f0 * p.N, s));
            continue;
        }
        if (paired) SDRGPU_CHECK(dispatch_passA2(p, xc, frameStride, nf, s));
        else SDRGPU_CHECK(dispatch_passA(p, xc, frameStride, nf, s));
        hipStream_t sb = s;
        if (pipe) {
            SDRGPU_HIP(hipEventRecord(p.evA[b], s));
            SDRGPU_HIP(hipStreamWaitEvent(p.s2, p.evA[b], 0));
            sb = p.s2;
        }
        SDRGPU_CHECK(dispatch_passB(p, nf, out + (long long)f0 * p.N, sb, zoomAt(f0)));
        if (pipe) SDRGPU_HIP(hipEventRecord(p.evB[b], p.s2));
    }
    if (pipe) SDRGPU_HIP(hipStreamWaitEvent(s, p.evB[(nchunks - 1) & 1], 0));   // join
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
    const int tail = p.fuseTail ? vfo_tail_prepare(vfoBlock, *vfo, vfoOut, &t, &ldsTail) : 0;
    if (tail < 0) return tail;
    if (tail) {
        auto k = fft_passB_tail_kernel;
        const size_t lds = std::max(ldsFFT, ldsTail);
        SDRGPU_CHECK(set_lds(k, lds));
        hipLaunchKernelGGL(k, dim3(8 * frames + t.G), dim3(512), lds, s, p.cur, frames, p.N1, p.logN, p.tw2.as<float2>(), out, t);
        SDRGPU_HIP(hipGetLastError());
        *vfoN = vfo_tail_commit(vfoBlock, t);
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
template <bool ZM, int CP, int XG = 0>
static int launch_vfo(FftPlan& p, const float2* scratchB, int framesB, float* outB, float* zoomB, const float2* in,
                      int framesA, float2* scratchA, VfoWork v, hipStream_t s) {
    auto k = fft_vfo_kernel<ZM, CP, XG>;
    const size_t lds = sizeof(float2) * (32 * Lds<256>::LS + 256 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    const int nB = 8 * framesB;
    const int g = (XG == 2 ? 136 * ((std::max(framesA, framesB) + 7) / 8)
                           : nB + (XG == 3 ? 96 * ((framesA + 7) / 8) : XG ? 72 * ((framesA + 7) / 8) : 9 * framesA)) +
                  (v.hist ? 1 : 0);
    hipLaunchKernelGGL(k, dim3(g), dim3(512), lds, s, nB, scratchB, framesB, outB, zoomB, in, (long long)p.N, framesA,
                       p.win.as<float>(), p.nz, p.logN, p.tw1.as<float2>(), p.tw2.as<float2>(), p.tfull.as<float2>(),
                       scratchA, v);
    SDRGPU_HIP(hipGetLastError());
    return SDRGPU_OK;
}
static int dispatch_vfo(FftPlan& p, bool zm, const float2* scratchB, int framesB, float* outB, float* zoomB,
                        const float2* in, int framesA, float2* scratchA, const VfoWork& v, hipStream_t s) {
    if (p.vfoXcd == 3) {
        if (p.vfoCP == 2)   // (tuning) streaming pass-A input loads: the stage's L2 hits, no Infinity-Cache allocation
            return zm ? launch_vfo<true, 2, 3>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
                      : launch_vfo<false, 2, 3>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
        return zm ? launch_vfo<true, 0, 3>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
                  : launch_vfo<false, 0, 3>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
    }
    if (p.vfoXcd == 2) return zm ? launch_vfo<true, 0, 2>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
                                 : launch_vfo<false, 0, 2>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
    if (p.vfoXcd) return zm ? launch_vfo<true, 0, 1>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
                            : launch_vfo<false, 0, 1>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
    if (zm) return p.vfoCP == 2 ? launch_vfo<true, 2>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
                                : launch_vfo<true, 0>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
    return p.vfoCP == 2 ? launch_vfo<false, 2>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s)
                        : launch_vfo<false, 0>(p, scratchB, framesB, outB, zoomB, in, framesA, scratchA, v, s);
}
static bool vfo_fusable(const FftPlan& p, float* zoom, int zoomSize) {
    return p.vfoFuse && !p.f64 && p.N1 == 256 && p.N2 == 256 && p.sa == 32 && p.sb == 32 && p.sa2 == 0 && p.nz == p.N &&
           (zoom == nullptr || zoom_fusable(p, zoomSize));
}
// Returns the VFO's output count: its later stages (vfo_stage1_finish) need only the stage-1 outputs,
// complete once the last pass-A launch is done, so they run on the plan's side stream beside the last
// launch (pass B of the last chunk + the stage's history), and the call's stream joins them.
// the group as one fft_vfo_persist_kernel launch (SPX devices: 8 XCDs, read by HW_REG_XCC_ID)
static int fft_execute_vfo_persist(FftPlan& p, const float2* x, int frames, float* out, float* zoom, const VfoStage1& st,
                                   hipStream_t s) {
    SDRGPU_CHECK(p.scratch.ensure((size_t)8 * kPersistRing * p.N * sizeof(float2)));
    const size_t ctl = sizeof(int) * (8 + 2 * (size_t)frames + 1);
    SDRGPU_CHECK(p.persistCtl.ensure(ctl));
    int* c = p.persistCtl.as<int>();
    SDRGPU_HIP(hipMemsetAsync(c, 0, ctl, s));
    PersistWork w{VfoWork{st.a, 0, 0}, frames, p.persistLag, c, c + 8, c + 8 + frames, c + 8 + 2 * frames};
    auto k = p.vfoPersist == 2 ? (zoom ? fft_vfo_persist_kernel<true, true> : fft_vfo_persist_kernel<false, true>)
                               : (zoom ? fft_vfo_persist_kernel<true> : fft_vfo_persist_kernel<false>);
    const size_t lds = sizeof(float2) * (32 * Lds<256>::LS + 256 + 256);
    SDRGPU_CHECK(set_lds(k, lds));
    if (!p.gridP) {
        int per = 0, cus = 0;
        SDRGPU_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, 512, lds));
        SDRGPU_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p.device));
        p.gridP = std::max(1, std::min(per, 2)) * cus;
    }
    SDRGPU_CHECK(time_mark(p, 0, s));
    hipLaunchKernelGGL(k, dim3(p.gridP), dim3(512), lds, s, x, out, zoom, p.win.as<float>(), p.nz, p.logN,
                       p.tw1.as<float2>(), p.tw2.as<float2>(), p.tfull.as<float2>(), p.scratch.as<float2>(), w);
    SDRGPU_HIP(hipGetLastError());
    return time_mark(p, 1, s);
}
// spin timeouts of the last persistent launch (synchronises the plan's stream; tests)
extern "C" int sdrgpu_fft_persist_errors(sdrgpu_fft* h, int frames) {
    if (!h || !h->p.persistCtl.p) return 0;
    int e = 0;
    SDRGPU_HIP(hipDeviceSynchronize());
    SDRGPU_HIP(hipMemcpy(&e, h->p.persistCtl.as<int>() + 8 + 2 * frames, sizeof(int), hipMemcpyDeviceToHost));
    return e;
}

static int fft_execute_vfo(FftPlan& p, const float2* x, int frames, float* out, float* zoom, const VfoStage1& st,
                           sdrgpu_block* vfo, void* vfoOut, hipStream_t s) {
    if (p.vfoPersist) {
        int cus = 0;
        SDRGPU_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p.device));
        if (cus == 256) {
            SDRGPU_CHECK(fft_execute_vfo_persist(p, x, frames, out, zoom, st, s));
            return vfo_stage1_finish(vfo, st, vfoOut, s);
        }
    }
    if (onepass_ok(p)) {
        VfoWork v{st.a, 0, 1};
        SDRGPU_CHECK(time_mark(p, 0, s));
        const int rc = zoom ? launch_1p<true, true>(p, x, p.N, frames, out, zoom, v, s)
                            : launch_1p<false, true>(p, x, p.N, frames, out, nullptr, v, s);
        if (rc < 0) return rc;
        SDRGPU_CHECK(time_mark(p, 1, s));
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
    int m = 0;
    if (p.vfoSide) {
        SDRGPU_CHECK(ensure_side(p));
        SDRGPU_HIP(hipEventRecord(p.evFork, s));
        SDRGPU_HIP(hipStreamWaitEvent(p.s2, p.evFork, 0));
        m = vfo_stage1_finish(vfo, st, vfoOut, p.s2);
        if (m < 0) return m;
        SDRGPU_HIP(hipEventRecord(p.evJoin, p.s2));
    }
    const int fL = (nchunks - 1) * cf;
    v.hist = 1;
    SDRGPU_CHECK(dispatch_vfo(p, zoom != nullptr, sc[(nchunks - 1) & 1], frames - fL, out + (long long)fL * p.N, zoomAt(fL),
                              nullptr, 0, nullptr, v, s));
    SDRGPU_CHECK(time_mark(p, 1, s));
    if (p.vfoSide) {
        SDRGPU_HIP(hipStreamWaitEvent(s, p.evJoin, 0));
        return m;
    }
    return vfo_stage1_finish(vfo, st, vfoOut, s);
}

// Spectrum (+ the waterfall's zoom rows) + one RxVFO over the same device batch of back-to-back
// frames (fftRate = fs / N: the IQFrontEnd's reshaper keeps every sample, iq_frontend.h:56-60), the
// VFO reading the batch in place like every consumer of the front end's splitter
// (iq_frontend.cpp:15-52). On the 64k plan with the VFO's D = 32 first stage (the RxVFO's plan_256
// at 61.44 MS/s) the batch is read from HBM once: the stage runs inside the spectrum launches
// (fft_vfo_kernel) and only the VFO's later stages run after them. Otherwise: the spectrum launch
// group, then the VFO. Returns the VFO's output count (vfoOut).
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
    if (vfo->impl && vfo->impl->device != p.device) {
        set_error("fft_execute_vfo: VFO on device %d, spectrum plan on device %d", vfo->impl->device, p.device);
        return SDRGPU_EARG;
    }
    if (frames == 0) return 0;
    SDRGPU_SET_DEVICE(p.device);
    hipStream_t s = stream ? (hipStream_t)stream : p.own;
    SDRGPU_CHECK(p.order.follow(s));
    OrderScope od(p.order, s);
    SDRGPU_CHECK(vfo->impl->order.follow(s));
    OrderScope ov(vfo->impl->order, s);
    VfoStage1 st;
    const int fuse = vfo_fusable(p, zoomOut, zoomSize) ? vfo_stage1_prepare(vfo, in, (int)count, &st) : 0;
    if (fuse < 0) return fuse;
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

extern "C" int sdrgpu_fft_destroy(sdrgpu_fft* h) {
    if (!h) return SDRGPU_OK;
    (void)hipSetDevice(h->p.device);
    if (h->p.own) (void)hipStreamDestroy(h->p.own);
    if (h->p.zoom) sdrgpu_zoom_destroy(h->p.zoom);
    if (h->p.f64) fft64_destroy(h->p.f64);
    for (auto& e : h->p.tev)
        for (auto& ev : e)
            if (ev) (void)hipEventDestroy(ev);
    if (h->p.s2) {
        (void)hipStreamSynchronize(h->p.s2);
        (void)hipStreamDestroy(h->p.s2);
        (void)hipEventDestroy(h->p.evFork);
        (void)hipEventDestroy(h->p.evJoin);
        for (int k = 0; k < 2; k++) {
            (void)hipEventDestroy(h->p.evA[k]);
            (void)hipEventDestroy(h->p.evB[k]);
        }
    }
    delete h;
    return SDRGPU_OK;
}
