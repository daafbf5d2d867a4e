// Critically sampled M-channel polyphase channelizer (BASELINE config C4).
//
// Definition: channel k is FrequencyXlator(-k fs/M)
// (channel/frequency_xlator.h:43-50, exact NCO) -> DecimatingFIR<complex_t, float>(h, M)
// (filter/decimating_fir.h:45-68) with a Q*M-tap prototype h. With buf = [history || in] and
// D = M, output m of channel k is
//   y_k[m] = sum_j h[j] buf[offset + mM + j] exp(-2 pi i k n_j / M),  j = qM + r,
// and because n_j = mM + j + const, the rotation depends on r only:
//   y_k[m] = sum_c W_M^(k c) v_m[c],   v_m[(rot + r) mod M] = sum_q h[qM + r] buf[offset + (m+q)M + r].
// So one launch does, per output frame m: M branch FIRs of Q taps (the polyphase bank of
// multirate/polyphase_bank.h:32, branch r = bank phase M-1-r) and one M-point forward FFT.
// That is ~4Q + 5 log2 M flop per input sample (64 + 50 at M = 1024, Q = 16), far below the
// HBM ridge, so the kernel is HBM-bound: 8 B in + 8 B out per sample. A dense
// DFT-as-GEMM (512 flop/sample) would make it compute-bound; fp32 MFMA has no higher peak
// than packed-fp32 VALU on gfx950, so the FFT form is the faster one.
//
// Kernel layout: one thread per branch r (NT = M threads), 16 frames per batch. A thread
// keeps its Q taps and a 16-deep circular window of its branch's samples in registers; each
// batch loads one new sample per frame (coalesced: consecutive r), forms 16 branch outputs
// into the batch's 16 LDS sequences (rotated by `rot`), then the workgroup runs 16 M-point
// Stockham FFTs in LDS and stores the channel vectors, out[m][k]. (Prefetching the next
// batch across the FFT spills at 1024 threads; with 16 loads in flight per thread at batch
// start the chip already has ~32 MB outstanding per batch time, above the HBM rate.)
#include <algorithm>
#include <cstring>
#include <vector>
#include "sdrgpu_internal.h"
#include "fft_stages.h"
#ifndef SDRGPU_CHAN_PF
#define SDRGPU_CHAN_PF 1   // FFT-form channelizer: next batch's samples loaded during this batch's FFTs (A/B: 0)
#endif
#ifndef SDRGPU_CHAN_PF2
// the second branch's first 8 frames prefetched as well (204 VGPRs; all 16: 82 spilled): C4 1.158 (no
// prefetch) -> 1.074 (first branch) -> 1.064 ms (+ 8 frames), 3 interleaved runs, r4z
#define SDRGPU_CHAN_PF2 8
#endif
#ifndef SDRGPU_CHAN_NT
#define SDRGPU_CHAN_NT 1   // FFT-form channelizer: streaming output row stores (A/B builds: 0)
#endif

namespace sdrgpu {

constexpr int CHAN_Q = 16;   // taps per branch (prototype padded to Q*M)

template <int L>
__global__ __launch_bounds__(L) void chan_kernel(const float2* __restrict__ hist, const float2* __restrict__ in, int H,
                                                 int count, const float* __restrict__ taps, long long offset0, int rot,
                                                 int frames, int fpw, const float2* __restrict__ tw,
                                                 float2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int Q = CHAN_Q, T = L / 16, LS = Lds<L>::LS;
    const int r = threadIdx.x;
    float2* twl = lds + 16 * LS;                       // FFT twiddles staged once in LDS
    twl[r] = tw[r];                                    // (L threads, L twiddles; first barrier orders it)
    float2* tw16 = twl + L;                            // middle stage's, bank-conflict-free (stage_lds)
    stage16_twiddles<L>(tw16, tw, r, L);
    const int m0 = blockIdx.x * fpw;
    const int m1 = min(m0 + fpw, frames);
    auto fetch = [&](long long b) -> float2 {          // buf[b] of [hist (H) || in (count)], 0 outside
        if (b < H) return hist[b];
        const long long i = b - H;
        return i < count ? in[i] : make_float2(0.f, 0.f);
    };
    const long long base = offset0 + r;
    float2 xs[16];                                     // xs[(m - m0) & 15] = buf[base + m L]
#pragma unroll
    for (int q = 0; q < 15; q++) xs[q] = fetch(base + (long long)(m0 + q) * L);
    xs[15] = make_float2(0.f, 0.f);
    for (int mb = m0; mb < m1; mb += 16) {
        // re-materialise the lane's LDS/FFT indices per batch instead of letting the compiler
        // hoist ~50 loop-invariant addresses out of the loop (they spill at 128 VGPRs)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int sF = tid / T, tF = tid % T;          // FFT role: sequence sF (a frame), thread tF
        const int c = (rot + tid) & (L - 1);
        float2 nx[16];                                 // newest tap row of each frame of the batch
        float h[Q];                                    // (re-read per batch from L2: not live across the FFT)
#pragma unroll
        for (int q = 0; q < Q; q++) h[q] = taps[q * L + r];
        // interior batch (all 16 rows inside `in`): per-row uniform base + the lane's r, so the
        // 16 loads share one offset register instead of 16 64-bit addresses
        const long long lo = offset0 + (long long)(mb + 15) * L, hi = offset0 + (long long)(mb + 31) * L + L;
        if (mb + 16 <= m1 && lo >= H && hi <= (long long)H + count) {
            const float2* __restrict__ src = in + (lo - H);
#pragma unroll
            for (int f = 0; f < 16; f++) nx[f] = src[(long long)f * L + tid];
        } else {
#pragma unroll
            for (int f = 0; f < 16; f++) nx[f] = (mb + f < m1) ? fetch(base + (long long)(mb + f + 15) * L) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int f = 0; f < 16; f++) {
            xs[(f + 15) & 15] = nx[f];
            float2 u = make_float2(0.f, 0.f);
#pragma unroll
            for (int q = 0; q < Q; q++) {
                const float2 x = xs[(f + q) & 15];
                u.x = fmaf(h[q], x.x, u.x);
                u.y = fmaf(h[q], x.y, u.y);
            }
            lds[f * LS + pad16(c)] = u;
        }
        __syncthreads();
        float2 v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = lds[sF * LS + pad16s<T>(tF, i)];
        __syncthreads();
        stage_first<L>(lds + sF * LS, v, tF);
        __syncthreads();
        const int m = mb + sF;
        float2* o = out + (long long)m * L;
        stages_rest<L, (L >= 256)>(lds, twl, sF, tF, [&](int k, float2 y) {
            if (m < m1) o[k] = y;
        }, tw16);
        __syncthreads();
    }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// The M = 1024 DFT of the 16 branch vectors of a batch as dense matrix products on the f32
// matrix cores (the "filterbank cast as batched MFMA GEMM" form of BASELINE C4). With
// c = 32 a + b and k = k1 + 32 k2, W_1024^(kc) = W_32^(k1 a) W_1024^(k1 b) W_32^(k2 b), so per
// frame (viewed as the 32 x 32 matrix X[a][b] = v[32 a + b]):
//   Z = F X  (F[k1][a] = W_32^(k1 a)),  Z'[k1][b] = Z[k1][b] W_1024^(k1 b),  Y = Z' F  (F symmetric),
// and Y[k1][k2] is channel k1 + 32 k2: two complex 32 x 32 x 32 products = 2 x 128
// v_mfma_f32_16x16x4_f32 per frame (512 flop per sample against the FFT's ~50). Wave w of the
// 8 owns frames w and w + 8 of the batch: all its LDS traffic stays inside its own sequences,
// so the stages need no workgroup barrier. MFMA operand layout (as fir_mfma_kernel): A[i][k]
// from lane (i = lane & 15, k = lane >> 4), B[k][j] from lane (j = lane & 15, k = lane >> 4),
// accumulator e of a lane = D[4 (lane >> 4) + e][lane & 15]. The W_32 operand of lane (i, kk)
// at k-step s of block x is W_32^((16 x + i)(4 s + kk)) in both products.
// Cross-lane LDS hand-off inside one wave: the HIP memory model does not order one lane's LDS
// store before another lane's later LDS load, so every write phase of chan_dft_gemm is closed by
// a wave-scope release fence + wave barrier + acquire fence (no workgroup barrier is needed: each
// wave touches only its own sequences). Costs a few cycles per phase.
__device__ __forceinline__ void wave_lds_handoff() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int L>
__device__ __forceinline__ void chan_dft_gemm(float2* lds, const float2* twl, int tid, int mb, int m1, float2* __restrict__ out) {
    static_assert(L == 1024, "DFT-GEMM channelizer: 1024 = 32 x 32");
    constexpr int LS = Lds<L>::LS;
    const int lane = tid & 63, wv = tid >> 6;
    const int i = lane & 15, kk = lane >> 4;
    // W_32^n = W_1024^(32 n), read from the staged twiddles at each k-step (as registers the 16
    // values per lane push the kernel past 256 VGPRs)
    auto Wv = [&](int x, int s) { return twl[32 * (((16 * x + i) * (4 * s + kk)) & 31)]; };
#pragma unroll 1
    for (int fr = 0; fr < 2; fr++) {
        const int sF = wv + 8 * fr;
        float2* X = lds + sF * LS;
        f32x4 ar[2][2], ai[2][2];   // [row block][column block]
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 2; y++) ar[x][y] = ai[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
        // Z = F X: A = F (rows k1 = 16 bi + i), B = X (k = a = 4 s + kk, columns b = 16 bj + i)
#pragma unroll
        for (int s = 0; s < 8; s++)
#pragma unroll
            for (int bj = 0; bj < 2; bj++) {
                const float2 xb = X[pad16(32 * (4 * s + kk) + 16 * bj + i)];
#pragma unroll
                for (int bi = 0; bi < 2; bi++) {
                    const float2 w = Wv(bi, s);
                    ar[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, xb.x, ar[bi][bj], 0, 0, 0);
                    ar[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(-w.y, xb.y, ar[bi][bj], 0, 0, 0);
                    ai[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, xb.y, ai[bi][bj], 0, 0, 0);
                    ai[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, xb.x, ai[bi][bj], 0, 0, 0);
                }
            }
        // Z'[k1][b] = Z[k1][b] W_1024^(k1 b) (k1 b < 1024), written over X[k1][b] once every lane
        // of this wave has read its operands of X above
        wave_lds_handoff();
#pragma unroll
        for (int bi = 0; bi < 2; bi++)
#pragma unroll
            for (int bj = 0; bj < 2; bj++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int k1 = 16 * bi + 4 * kk + e, b = 16 * bj + i;
                    X[pad16(32 * k1 + b)] = cmul(make_float2(ar[bi][bj][e], ai[bi][bj][e]), twl[k1 * b]);
                }
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 2; y++) ar[x][y] = ai[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
        wave_lds_handoff();   // Z' stored by other lanes, read below as A operands
        // Y = Z' F: A = Z' (rows k1 = 16 bi + i, k = b = 4 s + kk), B = F (columns k2 = 16 bj + i)
#pragma unroll
        for (int s = 0; s < 8; s++) {
            float2 za[2];
#pragma unroll
            for (int bi = 0; bi < 2; bi++) za[bi] = X[pad16(32 * (16 * bi + i) + 4 * s + kk)];
#pragma unroll
            for (int bi = 0; bi < 2; bi++)
#pragma unroll
                for (int bj = 0; bj < 2; bj++) {
                    const float2 g = Wv(bj, s);
                    ar[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(za[bi].x, g.x, ar[bi][bj], 0, 0, 0);
                    ar[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(-za[bi].y, g.y, ar[bi][bj], 0, 0, 0);
                    ai[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(za[bi].x, g.y, ai[bi][bj], 0, 0, 0);
                    ai[bi][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(za[bi].y, g.x, ai[bi][bj], 0, 0, 0);
                }
        }
        // channel k = k1 + 32 k2 into the sequence (natural order), then one coalesced row store
        wave_lds_handoff();   // every lane's Z' reads done before the sequence is overwritten
#pragma unroll
        for (int bi = 0; bi < 2; bi++)
#pragma unroll
            for (int bj = 0; bj < 2; bj++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int k1 = 16 * bi + 4 * kk + e, k2 = 16 * bj + i;
                    X[pad16(k1 + 32 * k2)] = make_float2(ar[bi][bj][e], ai[bi][bj][e]);
                }
        wave_lds_handoff();   // channel vector stored by other lanes, read for the row store
        const int m = mb + sF;
        if (m < m1) {
            float2* o = out + (long long)m * L;
#pragma unroll
            for (int q = 0; q < L / 64; q++) o[lane + 64 * q] = X[pad16(lane + 64 * q)];
        }
        wave_lds_handoff();   // row store's reads done before the next frame's sequence is used
    }
}

// Two branches per thread (L/2 threads): the kernel above needs ~180 VGPRs and spills at
// 1024 threads (128-VGPR cap); here each lane owns branches r and r + L/2 and plays two FFT
// roles in turn (sequences sF and sF + 8), with a 256-VGPR cap at L/2 threads. GEMM: the
// per-frame DFT runs as chan_dft_gemm (matrix cores) instead of the LDS FFT.
template <int L, bool GEMM = false>
__global__ __launch_bounds__(L / 2) void chan2_kernel(const float2* __restrict__ hist, const float2* __restrict__ in, int H,
                                                      int count, const float* __restrict__ taps, long long offset0,
                                                      int rot, int frames, int fpw, const float2* __restrict__ tw,
                                                      float2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int Q = CHAN_Q, T = L / 16, LS = Lds<L>::LS, NT = L / 2;
    float2* twl = lds + 16 * LS;
    twl[threadIdx.x] = tw[threadIdx.x];
    twl[threadIdx.x + NT] = tw[threadIdx.x + NT];
    float2* tw16 = twl + L;   // the middle FFT stage's twiddles, bank-conflict-free (stage_lds)
    stage16_twiddles<L>(tw16, tw, threadIdx.x, NT);
    const int m0 = blockIdx.x * fpw;
    const int m1 = min(m0 + fpw, frames);
    auto fetch = [&](long long b) -> float2 {
        if (b < H) return hist[b];
        const long long i = b - H;
        return i < count ? in[i] : make_float2(0.f, 0.f);
    };
    float2 xs[2][16];
#pragma unroll
    for (int h2 = 0; h2 < 2; h2++) {
        const long long base = offset0 + threadIdx.x + h2 * NT;
#pragma unroll
        for (int q = 0; q < 15; q++) xs[h2][q] = fetch(base + (long long)(m0 + q) * L);
        xs[h2][15] = make_float2(0.f, 0.f);
    }
    // PF (SDRGPU_CHAN_PF build flag, A/B; not with GEMM, whose DFT already holds 236 VGPRs): the next
    // batch's 16 samples of the first branch are loaded while this batch's FFTs run (both branches: 72
    // VGPRs spilled)
    constexpr bool PFK = SDRGPU_CHAN_PF && !GEMM;
    float2 pf[1][16];
    auto load_batch = [&](int mb, int tid, auto& dst, int h0, int h1) {
        const long long lo = offset0 + (long long)(mb + 15) * L, hi = offset0 + (long long)(mb + 31) * L + L;
        const bool inner = mb + 16 <= m1 && lo >= H && hi <= (long long)H + count;
#pragma unroll
        for (int h2 = h0; h2 < h1; h2++) {
            const int r = tid + h2 * NT;
            if (inner) {
                const float2* __restrict__ src = in + (lo - H);
#pragma unroll
                for (int f = 0; f < 16; f++) dst[h2 - h0][f] = src[(long long)f * L + r];
            } else {
                const long long base = offset0 + r;
#pragma unroll
                for (int f = 0; f < 16; f++)
                    dst[h2 - h0][f] = (mb + f < m1) ? fetch(base + (long long)(mb + f + 15) * L) : make_float2(0.f, 0.f);
            }
        }
    };
    // (SDRGPU_CHAN_PF2, A/B: the second branch's first PF2 frames prefetched as well)
    constexpr int PF2 = PFK ? SDRGPU_CHAN_PF2 : 0;
    float2 pf2[PF2 > 0 ? PF2 : 1];
    auto load2 = [&](int mb, int tid) {   // branch 1, frames < PF2
        if constexpr (PF2 > 0) {
            const long long lo = offset0 + (long long)(mb + 15) * L, hi = offset0 + (long long)(mb + 31) * L + L;
            const bool inner = mb + 16 <= m1 && lo >= H && hi <= (long long)H + count;
            const int r = tid + NT;
            if (inner) {
                const float2* __restrict__ src = in + (lo - H);
#pragma unroll
                for (int f = 0; f < PF2; f++) pf2[f] = src[(long long)f * L + r];
            } else {
                const long long base = offset0 + r;
#pragma unroll
                for (int f = 0; f < PF2; f++) pf2[f] = (mb + f < m1) ? fetch(base + (long long)(mb + f + 15) * L) : make_float2(0.f, 0.f);
            }
        }
    };
    if constexpr (PFK) if (m0 < m1) { load_batch(m0, threadIdx.x, pf, 0, 1); load2(m0, threadIdx.x); }
    for (int mb = m0; mb < m1; mb += 16) {
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        float2 cur[2][16];
        if constexpr (PFK) {
#pragma unroll
            for (int f = 0; f < 16; f++) cur[0][f] = pf[0][f];
            float2 (&c1)[1][16] = *reinterpret_cast<float2 (*)[1][16]>(&cur[1]);
            load_batch(mb, tid, c1, 1, 2);
            if constexpr (PF2 > 0) {
#pragma unroll
                for (int f = 0; f < PF2; f++) cur[1][f] = pf2[f];
            }
        } else {
            load_batch(mb, tid, cur, 0, 2);
        }
#pragma unroll
        for (int h2 = 0; h2 < 2; h2++) {
            const int r = tid + h2 * NT;
            const int c = (rot + r) & (L - 1);
            float h[Q];
#pragma unroll
            for (int q = 0; q < Q; q++) h[q] = taps[q * L + r];
            const float2 (&nx)[16] = cur[h2];
#pragma unroll
            for (int f = 0; f < 16; f++) {
                xs[h2][(f + 15) & 15] = nx[f];
                float2 u = make_float2(0.f, 0.f);
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    const float2 x = xs[h2][(f + q) & 15];
                    u.x = fmaf(h[q], x.x, u.x);
                    u.y = fmaf(h[q], x.y, u.y);
                }
                lds[f * LS + pad16(c)] = u;
            }
        }
        __syncthreads();
        if constexpr (PFK) if (mb + 16 < m1) { load_batch(mb + 16, tid, pf, 0, 1); load2(mb + 16, tid); }
        if constexpr (GEMM) {
            chan_dft_gemm<L>(lds, twl, tid, mb, m1, out);
            __syncthreads();
            continue;
        }
#pragma unroll 1
        for (int half = 0; half < 2; half++) {
            const int sF = tid / T + 8 * half, tF = tid % T;
            float2 v[16];
#pragma unroll
            for (int i = 0; i < 16; i++) v[i] = lds[sF * LS + pad16s<T>(tF, i)];
            __syncthreads();
            stage_first<L>(lds + sF * LS, v, tF);
            __syncthreads();
            const int m = mb + sF;
            float2* o = out + (long long)m * L;
            stages_rest<L, (L >= 256)>(lds, twl, sF, tF, [&](int k, float2 y) {
                if (m < m1) {
                    if constexpr (SDRGPU_CHAN_NT) {   // channel rows are written once: streaming stores
                        typedef float f2v __attribute__((ext_vector_type(2)));
                        __builtin_nontemporal_store(f2v{y.x, y.y}, reinterpret_cast<f2v*>(o + k));
                    } else {
                        o[k] = y;
                    }
                }
            }, tw16);
            __syncthreads();
        }
    }
}

__global__ void chan_hist_kernel(const float2* __restrict__ hist, const float2* __restrict__ in,
                                 float2* __restrict__ next, int H, int count) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= H) return;
    const long long b = (long long)count + k;          // last H samples of [hist || in]
    next[k] = b < H ? hist[b] : in[b - H];
}

struct ChannelizerBlock : Block {
    int M = 0, ntaps = 0, Hp = 0, offset = 0, fpw = 256;
    // two branches per thread (chan2_kernel, no spill): 1.17 vs 1.63 ms per 2^28 samples
    // against the one-branch kernel on one box; chan_kernel is the one-branch form
    bool two = true;
    int dft = 0;             // 0: LDS FFT (chan2_kernel); 1: DFT-GEMM on the matrix cores (M = 1024)
    long long phase = 0;     // absolute input index mod M of the next sample
    DevBuf taps, tw, hist[2];
    int cur = 0;

    int setup(int dev, int channels, const float* t, int n) {
        device = dev;
        in_dtype = out_dtype = SDRGPU_C64;
        if (channels != 256 && channels != 512 && channels != 1024) {
            set_error("channelizer: %d channels unsupported (256, 512 or 1024)", channels);
            return SDRGPU_EARG;
        }
        if (!t || n < 1 || n > CHAN_Q * channels) {
            set_error("channelizer: %d taps out of range [1, %d]", n, CHAN_Q * channels);
            return SDRGPU_EARG;
        }
        M = channels;
        ntaps = n;
        Hp = CHAN_Q * M - 1;
        SDRGPU_CHECK(init_stream());
        std::vector<float> pq((size_t)CHAN_Q * M, 0.0f);       // [q][r] = h[q M + r]
        for (int j = 0; j < n; j++) pq[j] = t[j];
        SDRGPU_CHECK(taps.ensure(sizeof(float) * pq.size()));
        SDRGPU_HIP(hipMemcpy(taps.p, pq.data(), sizeof(float) * pq.size(), hipMemcpyHostToDevice));
        std::vector<float2> w(M);
        for (int i = 0; i < M; i++) {
            const double a = -2.0 * M_PI * (double)i / (double)M;
            w[i] = make_float2((float)std::cos(a), (float)std::sin(a));
        }
        SDRGPU_CHECK(tw.ensure(sizeof(float2) * M));
        SDRGPU_HIP(hipMemcpy(tw.p, w.data(), sizeof(float2) * M, hipMemcpyHostToDevice));
        for (int k = 0; k < 2; k++) SDRGPU_CHECK(hist[k].ensure(sizeof(float2) * Hp));
        return reset();
    }
    // DecimatingFIR output count (decimating_fir.h:45-68) x M channels
    int out_count(int count) override { return count > offset ? (count - offset + M - 1) / M * M : 0; }
    int reset() override {
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemset(hist[cur].p, 0, sizeof(float2) * Hp));
        offset = 0;
        phase = 0;
        return SDRGPU_OK;
    }
    template <int L>
    int launch(const void* in, int count, int frames, long long offset0, int rot, void* out, hipStream_t s) {
        auto k = two ? chan2_kernel<L> : chan_kernel<L>;
        if constexpr (L == 1024) {
            if (dft == 1) k = chan2_kernel<L, true>;
        }
        const size_t lds = sizeof(float2) * (16 * Lds<L>::LS + L + 256);   // sequences, twiddles, tw16
        SDRGPU_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        const int grid = (frames + fpw - 1) / fpw;
        hipLaunchKernelGGL(k, dim3(grid), dim3(two || dft ? L / 2 : L), lds, s, hist[cur].as<float2>(), (const float2*)in, Hp, count,
                           taps.as<float>(), offset0, rot, frames, fpw, tw.as<float2>(), (float2*)out);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count < 0) { set_error("channelizer: negative count"); return SDRGPU_EARG; }
        SDRGPU_SET_DEVICE(device);
        const int outN = out_count(count);
        const int frames = outN / M;
        const int H = ntaps - 1;                                   // the reference FIR's history
        if (frames > 0) {
            // buf' (history H) index b <-> padded buf index b + (Hp - H); absolute sample index
            // of buf'[b] is phase - H + b, so the NCO rotation of tap row r is (rot + r) mod M
            const long long offset0 = (long long)offset + (Hp - H);
            const int rot = (int)((((phase - H + offset) % M) + M) % M);
            int rc;
            if (M == 1024) rc = launch<1024>(in, count, frames, offset0, rot, out, s);
            else if (M == 512) rc = launch<512>(in, count, frames, offset0, rot, out, s);
            else rc = launch<256>(in, count, frames, offset0, rot, out, s);
            SDRGPU_CHECK(rc);
        }
        if (count > 0) {
            hipLaunchKernelGGL(chan_hist_kernel, dim3((Hp + 255) / 256), dim3(256), 0, s, hist[cur].as<float2>(),
                               (const float2*)in, hist[cur ^ 1].as<float2>(), Hp, count);
            SDRGPU_HIP(hipGetLastError());
            cur ^= 1;
        }
        offset = offset + frames * M - count;
        phase = (phase + count) % M;
        return outN;
    }
};

}  // namespace sdrgpu

using namespace sdrgpu;

extern "C" int sdrgpu_channelizer_create(sdrgpu_block** h, int device, int channels, const float* taps, int ntaps) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* b = new ChannelizerBlock();
    const int rc = b->setup(device, channels, taps, ntaps);
    if (rc < 0) { delete b; return rc; }
    *h = new sdrgpu_block{b};
    return SDRGPU_OK;
}

// C4's two forms: 0 = branch FIRs + LDS FFT (default, HBM-bound), 1 = branch FIRs + DFT as
// batched f32 MFMA GEMMs (1024 channels only)
extern "C" int sdrgpu_channelizer_set_dft(sdrgpu_block* h, int mode) {
    auto* b = h ? dynamic_cast<ChannelizerBlock*>(h->impl) : nullptr;
    if (!b) { set_error("channelizer_set_dft: not a channelizer"); return SDRGPU_EARG; }
    if (mode != 0 && mode != 1) { set_error("channelizer_set_dft: mode %d (0 FFT, 1 MFMA GEMM)", mode); return SDRGPU_EARG; }
    if (mode == 1 && b->M != 1024) { set_error("channelizer_set_dft: the MFMA GEMM form needs 1024 channels (have %d)", b->M); return SDRGPU_EARG; }
    b->dft = mode;
    return SDRGPU_OK;
}
