// Channel-chain kernels and stateful blocks: frequency xlator, FIR / decimating
// FIR (optionally with the xlator fused into its load and the FM quadrature
// demodulator fused into its store), power-of-two decimator, polyphase and
// rational resamplers, RxVFO, FM / broadcast-FM (mono) demodulators, ingest
// converters. Reference semantics are cited per block; DESIGN.md has the layout.
#include <cmath>
#include <cstring>
#include <algorithm>
#include <memory>
#include <numeric>
#include <type_traits>
#include "sdrgpu_internal.h"
#include "fir_rows.h"
#include "fir_tail.h"

namespace sdrgpu {

// ------------------------------------------------------------------- helpers
__global__ void nco_hi_kernel(float2* __restrict__ phi, int n, double theta0, double w) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    phi[j] = nco_phi(theta0, w, j);
}


// ------------------------------------------------------------ FIR engine
// out[m] = sum_{j<ntaps} buf[offset0 + m*D + j] * taps[j],  buf = hist(H) | in(count)
// (correlation order, filter/fir.h:62-83, decimating_fir.h:45-68).
// LDS holds one tile's input span "phase-major": span element s goes to phase
// p = s % D, row r = s / D, at p*RSP + (r % K)*RSK + r / K. Thread l computes K
// consecutive outputs from a K-deep register window that slides one row per tap
// step, so lanes read consecutive LDS words (conflict-free for any D) and every
// row load feeds K outputs.


// FIR tile kernel: one tile of NT*K outputs per workgroup.
//  1. The tile's input span (rows * D elements) is loaded with all PF loads per thread in
//     flight at once (interior tiles; the few tiles touching the history or the tail of the
//     call fetch element-wise), the fused xlator's NCO phasor is formed as
//     base(tid) * S[u] (S[u] = e^{i w u NT}, wave-uniform scalar loads) instead of two table
//     loads per element, and each element is stored into the phase-major, row-swizzled LDS
//     image X[p][r % K][r / K] with an address that advances by a constant per slot when
//     D | NT and K | NT/D (all plan stages), else with the general index split.
//  2. Each thread computes K consecutive outputs with a register window sliding one row per
//     tap; taps are staged once per workgroup in LDS (wave-uniform broadcast reads).
// History / tail samples come from [hist (H) || in (count)]; hist is stored translated.


template <typename DT, typename TT, int K, bool XL, bool QUAD, bool STEREO, bool TL>
__global__ __launch_bounds__(256) void fir_kernel(FirArgs a) {
    if (fir_hist_block<DT, XL>(a)) return;
    constexpr int PF = sizeof(DT) == 8 ? 36 : 40;   // load slots per thread issued together
    const int NT = blockDim.x;       // 64, 128 or 256 (host picks the largest tile that fits LDS)
    const int TM = NT * K;
    constexpr int QOFF = QUAD ? 1 : 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    DT* X = reinterpret_cast<DT*>(smem);
    __shared__ float2 lastY[QUAD ? 256 : 1];

    const int tid = threadIdx.x;
    const int tile = blockIdx.x;
    const int rows = TM + a.Q + K;                               // padded taps + prefetch rows
    const int span = rows * a.D;
    const DT* in = reinterpret_cast<const DT*>(a.in);
    const TT* __restrict__ taps = reinterpret_cast<const TT*>(a.taps);
    if constexpr (TL) {
        TT* tl = reinterpret_cast<TT*>(smem + a.tapsLdsOff);
        for (int i = tid; i < a.D * a.Q; i += NT) tl[i] = taps[i];
        taps = tl;                                                // (ordered by the barrier below)
    }
    auto lds_index = [&](int sx) {
        int p, r;
        if (a.dshift >= 0) {
            p = sx & (a.D - 1);
            r = sx >> a.dshift;
        } else {
            r = sx / a.D;
            p = sx - r * a.D;
        }
        return p * a.RSP + (r % K) * a.RSK + r / K;
    };

    const int mFirst = tile * a.TMS - QOFF;                      // output of local index 0
    const long long b0 = (long long)a.offset0 + (long long)mFirst * a.D;
    const bool interior = (b0 >= a.H) && (b0 + span <= (long long)a.H + a.count);
    int sxRest = tid;                                            // first slot fetched element-wise
    if (interior) {
        const DT* __restrict__ src = in + (b0 - a.H);
        DT pf[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int sx = tid + u * NT;
            if (sx < span) pf[u] = src[sx];
        }
        if constexpr (XL) {
            // phasor(i0 + tid + u NT) = nco(i0 + tid) * e^{i w u NT}
            const float2 ph0 = nco_at(a, b0 - a.H + tid);
            const float2* __restrict__ S = a.nstep;
#pragma unroll
            for (int u = 0; u < PF; u++) pf[u] = xlate_slot(pf[u], ph0, S[u]);
        }
        if (a.simple) {
            // D | NT and K | NT/D: the slot's phase is fixed, its row advances by NT/D
            int idx = lds_index(tid);
            const int inc = (NT / a.D) / K;
#pragma unroll
            for (int u = 0; u < PF; u++) {
                if (tid + u * NT < span) X[idx] = pf[u];
                idx += inc;
            }
        } else {
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int sx = tid + u * NT;
                if (sx < span) X[lds_index(sx)] = pf[u];
            }
        }
        sxRest = tid + PF * NT;                                  // remainder (rare: huge decimations)
    }
    for (int sx = sxRest; sx < span; sx += NT) X[lds_index(sx)] = fir_fetch<DT, XL>(a, b0 + sx);
    __syncthreads();

    DT acc[K];
#pragma unroll
    for (int i = 0; i < K; i++) acc[i] = zero_of<DT>();
    // a.Q is padded to a multiple of QC with zero taps. Row l*K + j + K*s of phase p sits at
    // Xj[j][s] (j = row % K), so a chunk's QC row reads are K base addresses + immediates.
    constexpr int QC = 8;
    const int l = tid;
    for (int p = 0; p < a.D; p++) {
        const DT* Xj[K];
#pragma unroll
        for (int j = 0; j < K; j++) Xj[j] = X + p * a.RSP + j * a.RSK + l;
        const TT* __restrict__ Hp = taps + p * a.Q;
        DT w[K];
#pragma unroll
        for (int i = 0; i < K; i++) w[i] = Xj[i][0];                // rows l*K + i
        // (unrolling this loop 4 chunks deep removes the window-carry moves but measured
        // 1.5% slower on C3: kept rolled)
        for (int q0 = 0; q0 < a.Q; q0 += QC) {
            TT hv[QC];
            DT nx[QC];
#pragma unroll
            for (int u = 0; u < QC; u++) hv[u] = Hp[q0 + u];
#pragma unroll
            for (int u = 0; u < QC; u++) nx[u] = Xj[u % K][1 + (q0 + u) / K];   // row l*K + K + q0 + u
#pragma unroll
            for (int u = 0; u < QC; u++) {
#pragma unroll
                for (int i = 0; i < K; i++) mac(acc[i], w[(i + u) % K], hv[u]);
                w[u % K] = nx[u];
            }
        }
    }

    if constexpr (QUAD) {
        // FM quadrature (demod/quadrature.h:41-56): out = arg(y[m] * conj(y[m-1])) / dev
        lastY[l] = acc[K - 1];
        const float2 din0 = a.din[0];                 // y[-1] of the stream: carried from the last call
        __syncthreads();
        float* out = reinterpret_cast<float*>(a.out);
        const float2 left = lastY[l > 0 ? l - 1 : 0];
#pragma unroll
        for (int i = 0; i < K; i++) {
            const int m = mFirst + l * K + i;
            if (m >= 0 && m >= tile * a.TMS && m < a.M) {
                float2 prev = (i > 0) ? acc[i > 0 ? i - 1 : 0] : left;
                if (m == 0) prev = din0;
                const float2 y = acc[i];
                const float br = prev.x, bi = -prev.y;
                const float re = (y.x * br) - (y.y * bi);
                const float im = (y.y * br) + (y.x * bi);
                out[m] = quad_atan2f(im, re) * a.invDev;
                if (m == a.M - 1) a.dinNext[0] = y;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; i++) {
            const int m = mFirst + l * K + i;
            if (m < a.M && m < (tile + 1) * a.TMS) {
                if constexpr (STEREO) {
                    reinterpret_cast<float2*>(a.out)[m] = make_float2(acc[i], acc[i]);   // LRToStereo(l = r)
                } else {
                    reinterpret_cast<DT*>(a.out)[m] = acc[i];
                }
            }
        }
    }
}

// ------------------------------------------------ MFMA FIR (complex data x real taps)
// With Qp = ceil(ntaps / D) taps per phase (C3: 256 taps / 8 = 32), each phase's correlation
//   y_p[m] = sum_q g_p[q] u_p[m + q],   u_p[n] = span[n D + p],   g_p[q] = h[q D + p]
// is a Toeplitz product and runs on the f32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32
// FMA chains at the vector-FMA peak, one VGPR per operand, no VALU issue):
//   Y[i][j] += sum_k A[i][k] B[k][j],   A[i][k] = u_p[o + 16 i + k],   B[k][j] = g_p[k - j]
// (zero outside [0, Qp)), so the 16 x 16 accumulator holds outputs o + 16 i + j and k runs over
// [0, 16 + Qp - 1) in steps of 4 (1.47x the essential MACs at Qp = 32). Re and im are two
// accumulators sharing B. A wave owns 256 consecutive outputs, a workgroup MF_TM = 1024.
// LDS: the span phase-major with one pad row per 16 (X[p][r + r / 16]: the 16 rows of one A
// load fall in distinct banks), and B as gz[p][t] = g_p[t - 15], t < 64 (host-built).
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int MF_KS = 12;                   // k steps of 4: k < 48 >= 16 + Qp - 1 for Qp <= 32
constexpr int MF_GZ = 64;                   // gz entries per phase
constexpr int mf_rows(int nw) { return 256 * nw + 4 * MF_KS; }   // span rows per phase

// HALF (round 4): only half of the D phases' span rows are in LDS at a time -- a thread's span
// loads all belong to one phase (NT % D == 0), so the threads of the upper phases keep theirs in
// registers while the MFMAs run over the lower phases, then store them into the same LDS. Half the
// LDS per workgroup: four workgroups (16 waves) per CU instead of two, the same MFMA chains in the
// same order (bit-identical outputs).
// DC (round 4): the decimation as a compile-time constant (0: a.D at run time). C3's D = 8 then has a
// constant span, so the PF load / store slots need no range guards (only the last is partial) and the
// LDS indices fold: the SQ counters showed the SIMD ~90% busy with MFMA + VALU issue (no co-issue on
// the f32 matrix path), so every VALU instruction saved is kernel time.
template <int NW, bool XL, bool QUAD, bool HALF = false, int DC = 0>   // NW waves per workgroup, 256 outputs each
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(HALF ? 4 : 1))) void fir_mfma_kernel(FirArgs a) {
    if (fir_hist_block<float2, XL>(a)) return;
    constexpr int NT = 64 * NW, MF_TM = 256 * NW, MF_ROWS = mf_rows(NW);
    constexpr int PF = (MF_ROWS * 8 + NT - 1) / NT;    // load slots per thread for D <= 8
    constexpr int QOFF = QUAD ? 1 : 0;
    constexpr int NH = HALF ? 2 : 1;                   // phase halves through LDS
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* X = reinterpret_cast<float2*>(smem);
    float* gz = reinterpret_cast<float*>(smem + a.tapsLdsOff);
    const int tid = threadIdx.x, tile = blockIdx.x;
    // D a power of two dividing NT (host-checked); RSP = MF_ROWS + MF_ROWS / 16 + 1 (run_mfma_nw)
    const int D = DC ? DC : a.D, RSP = DC ? MF_ROWS + MF_ROWS / 16 + 1 : a.RSP;
    const int dsh = DC ? __builtin_ctz((unsigned)(DC ? DC : 1)) : a.dshift;
    const int DH = D / NH;                            // phases in LDS at a time
    {
        const float* __restrict__ g = reinterpret_cast<const float*>(a.taps);
        for (int i = tid; i < D * MF_GZ; i += NT) gz[i] = g[i];
    }
    auto lds_index = [&](int sx) {   // (HALF: the phase's slot within its half)
        const int r = sx >> dsh, p = sx & (D - 1);
        return (p % DH) * RSP + r + (r >> 4);
    };
    const int mFirst = tile * a.TMS - QOFF;
    const long long b0 = (long long)a.offset0 + (long long)mFirst * D;
    const int span = MF_ROWS * D;
    const bool interior = (b0 >= a.H) && (b0 + span <= (long long)a.H + a.count);
    float2 pf[PF];
    if (interior) {
        // XL: the NCO phase of slot 0 is computed before the PF loads are issued (its sincos
        // temporaries would otherwise be live next to the 2 x PF loaded registers)
        float2 ph0 = make_float2(1.f, 0.f);
        if constexpr (XL) {
            ph0 = nco_at(a, b0 - a.H + tid);
            __builtin_amdgcn_sched_barrier(0);
        }
        // one wave-uniform buffer resource and ONE per-lane offset for all PF loads, the slot step
        // in the scalar offset (no per-slot 64-bit address registers; interior: no range check needed)
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float2*>(reinterpret_cast<const float2*>(a.in) + (b0 - a.H)), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int sx = tid + u * NT;
            if (sx < span) pf[u] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsrc, tid * 8, u * NT * 8, 0));
        }
        if constexpr (XL) {
            // the wave-uniform step table through the constant address space: scalar loads, so
            // the 2 x PF step values do not take VGPRs next to the PF loaded samples
            const __attribute__((address_space(4))) float* S = (const __attribute__((address_space(4))) float*)a.nstep;
#pragma unroll
            for (int u = 0; u < PF; u++) pf[u] = xlate_slot(pf[u], ph0, make_float2(S[2 * u], S[2 * u + 1]));
        }
    }
    const int lane = tid & 63, o = (tid >> 6) * 256;
    const int i = lane & 15, kk = lane >> 4;   // A row i / B column j = i, k offset kk
    f32x4_t cre = {0.f, 0.f, 0.f, 0.f}, cim = {0.f, 0.f, 0.f, 0.f};
    const int myHalf = (tid & (D - 1)) / DH;   // the phase half this thread's span slots belong to
    auto mfma_half = [&](int h) {
        for (int p = h * DH; p < (h + 1) * DH; p++) {
            const float2* Xp = X + (p - h * DH) * RSP;
            const float* gp = gz + p * MF_GZ + 15 - i + kk;   // B[k0 + kk][i] = g_p[k0 + kk - i]
            const int r0 = o + 16 * i + kk;
#pragma unroll
            for (int s = 0; s < MF_KS; s++) {
                const int r = r0 + 4 * s;
                const float2 xa = Xp[r + (r >> 4)];
                const float bb = gp[4 * s];
                cre = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.x, bb, cre, 0, 0, 0);
                cim = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.y, bb, cim, 0, 0, 0);
                // HALF: the upper half's PF samples are still live through these MFMAs; fence
                // the LDS loads in groups of 4 k steps so they are not all hoisted (no spill)
                if constexpr (HALF) if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    // the interior and edge tiles run separate half loops: pf is not live across the edge path's
    // NCO fetches (one shared loop keeps it live there and spills the HALF kernel)
    if (interior) {
#pragma unroll
        for (int h = 0; h < NH; h++) {
            if (h > 0) __syncthreads();   // every MFMA read of the previous half is done
            if (myHalf == h) {
                // slot u: phase tid % D fixed, row advancing by NT / D (+ its pad rows)
                int idx = lds_index(tid);
                const int inc = (NT >> dsh) + (NT >> dsh) / 16;
#pragma unroll
                for (int u = 0; u < PF; u++) {
                    if (tid + u * NT < span) X[idx] = pf[u];
                    idx += inc;
                }
            }
            // (HALF runs only for D <= 8, where the PF slots cover the span: host-checked)
            if constexpr (!HALF)
                for (int sx = tid + PF * NT; sx < span; sx += NT) X[lds_index(sx)] = fir_fetch<float2, XL>(a, b0 + sx);
            __syncthreads();
            mfma_half(h);
        }
    } else {
        for (int h = 0; h < NH; h++) {
            if (h > 0) __syncthreads();
            for (int sx = tid; sx < span; sx += NT)
                if (((sx & (D - 1)) / DH) == h) X[lds_index(sx)] = fir_fetch<float2, XL>(a, b0 + sx);
            __syncthreads();
            mfma_half(h);
        }
    }
    // accumulator element e of this lane: row (lane >> 4) * 4 + e, column lane & 15
    if constexpr (QUAD) {
        // FM quadrature (demod/quadrature.h:41-56) on the tile's outputs staged in LDS (the span
        // is dead once every wave has passed the barrier); output 0 of the tile only supplies y[m-1]
        float2* Y = X;
        const float2 din0 = a.din[0];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 4; e++) Y[o + 16 * (kk * 4 + e) + i] = make_float2(cre[e], cim[e]);
        __syncthreads();
        float* out = reinterpret_cast<float*>(a.out);
#pragma unroll
        for (int e = 0; e < MF_TM / NT; e++) {
            const int ml = tid + e * NT;
            const int m = mFirst + ml;
            if (ml >= QOFF && m >= 0 && m < a.M) {
                const float2 y = Y[ml];
                const float2 prev = (m == 0) ? din0 : Y[ml - 1];
                const float br = prev.x, bi = -prev.y;
                const float re = (y.x * br) - (y.y * bi);
                const float im = (y.y * br) + (y.x * bi);
                out[m] = quad_atan2f(im, re) * a.invDev;
                if (m == a.M - 1) a.dinNext[0] = y;
            }
        }
    } else {
        float2* out = reinterpret_cast<float2*>(a.out);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int m = mFirst + o + 16 * (kk * 4 + e) + i;
            if (m < a.M && m < (tile + 1) * a.TMS) out[m] = make_float2(cre[e], cim[e]);
        }
    }
}

// Phase-split variant for larger decimations (VFO stage 1: D = 32, 143 taps -> Qp = 5): a tile
// is 256 outputs, the four waves split the D phases (wave w takes p = w, w + 4, ...), each
// accumulating the whole 16 x 16 output block over its phases with k < 4 * ks (ks = ceil((15 + Qp)
// / 4) steps), and the four partial blocks are summed through LDS. Small tiles keep the span in
// LDS for D up to 32 (75 KB at D = 32, 2 workgroups per CU) and for D = 8 let 7 share a CU.
template <bool XL, bool QUAD>
__global__ __launch_bounds__(256) void fir_mfma_ps_kernel(FirArgs a) {
    if (fir_hist_block<float2, XL>(a)) return;
    constexpr int NT = 256, TM = 256, PF = 36, QOFF = QUAD ? 1 : 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* X = reinterpret_cast<float2*>(smem);
    float* gz = reinterpret_cast<float*>(smem + a.tapsLdsOff);
    const int tid = threadIdx.x, tile = blockIdx.x;
    const int D = a.D, RSP = a.RSP, dsh = a.dshift, ks = a.Q;   // a.Q carries ks here
    {
        const float* __restrict__ g = reinterpret_cast<const float*>(a.taps);
        for (int i = tid; i < D * a.gzs; i += NT) gz[i] = g[i];
    }
    auto lds_index = [&](int sx) {
        const int r = sx >> dsh, p = sx & (D - 1);
        return p * RSP + r + (r >> 4);
    };
    const int rows = TM + 4 * ks;
    const int span = rows * D;
    const int mFirst = tile * a.TMS - QOFF;
    const long long b0 = (long long)a.offset0 + (long long)mFirst * D;
    const bool interior = (b0 >= a.H) && (b0 + span <= (long long)a.H + a.count);
    int sxRest = tid;
    if (interior) {
        const float2* __restrict__ src = reinterpret_cast<const float2*>(a.in) + (b0 - a.H);
        float2 pf[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int sx = tid + u * NT;
            if (sx < span) pf[u] = src[sx];
        }
        if constexpr (XL) {
            const float2 ph0 = nco_at(a, b0 - a.H + tid);
            const float2* __restrict__ S = a.nstep;
#pragma unroll
            for (int u = 0; u < PF; u++) pf[u] = xlate_slot(pf[u], ph0, S[u]);
        }
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int sx = tid + u * NT;
            if (sx < span) X[lds_index(sx)] = pf[u];
        }
        sxRest = tid + PF * NT;
    }
    for (int sx = sxRest; sx < span; sx += NT) X[lds_index(sx)] = fir_fetch<float2, XL>(a, b0 + sx);
    __syncthreads();

    const int lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, kk = lane >> 4;   // A row i / B column j = i, k offset kk
    f32x4_t cre = {0.f, 0.f, 0.f, 0.f}, cim = {0.f, 0.f, 0.f, 0.f};
    for (int p = w; p < D; p += 4) {
        const float2* Xp = X + p * RSP;
        const float* gp = gz + p * a.gzs + 15 - i + kk;   // B[k0 + kk][i] = g_p[k0 + kk - i]
        const int r0 = 16 * i + kk;
#pragma unroll
        for (int s = 0; s < MF_KS; s++) {   // unrolled so the operand reads are issued ahead
            if (s < ks) {
                const int r = r0 + 4 * s;
                const float2 xa = Xp[r + (r >> 4)];
                const float bb = gp[4 * s];
                cre = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.x, bb, cre, 0, 0, 0);
                cim = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.y, bb, cim, 0, 0, 0);
            }
        }
    }
    // partial blocks of the four waves -> LDS (the span is dead after the barrier), summed per output
    float2* P = X;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 4; e++) P[w * TM + 16 * (kk * 4 + e) + i] = make_float2(cre[e], cim[e]);
    __syncthreads();
    auto ysum = [&](int ml) {
        const float2 q0 = P[ml], q1 = P[TM + ml], q2 = P[2 * TM + ml], q3 = P[3 * TM + ml];
        return make_float2((q0.x + q1.x) + (q2.x + q3.x), (q0.y + q1.y) + (q2.y + q3.y));
    };
    const int ml = tid, m = mFirst + ml;
    if constexpr (QUAD) {
        if (ml >= QOFF && m >= 0 && m < a.M) {
            const float2 y = ysum(ml);
            const float2 prev = (m == 0) ? a.din[0] : ysum(ml - 1);
            const float br = prev.x, bi = -prev.y;
            const float re = (y.x * br) - (y.y * bi);
            const float im = (y.y * br) + (y.x * bi);
            reinterpret_cast<float*>(a.out)[m] = quad_atan2f(im, re) * a.invDev;
            if (m == a.M - 1) a.dinNext[0] = y;
        }
    } else {
        if (m < a.M && m < (tile + 1) * a.TMS) reinterpret_cast<float2*>(a.out)[m] = ysum(ml);
    }
}

template <int D, int QP, bool XL, bool QUAD, int RS = rows_rs<D>()>
__global__ __launch_bounds__(256) void fir_rows_kernel(FirArgs a) {
    if (fir_hist_block<float2, XL, false>(a)) return;
    constexpr int NG = 64 / D;
    const int lane = threadIdx.x & 63;
    fir_rows_segment<D, QP, XL, QUAD, RS>(a, ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * NG + lane / D, lane);
}

template <typename DT, bool XL>
__global__ void fir_hist_kernel(const DT* __restrict__ hist, const DT* __restrict__ in, DT* __restrict__ next, int H,
                                int count, const float2* __restrict__ phi, const float2* __restrict__ plo) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= H) return;
    const long long b = (long long)count + k;
    DT v;
    if (b < H) {
        v = hist[b];
    } else {
        const long long i = b - H;
        v = in[i];
        if constexpr (XL) v = cmulf(v, nco_tab(phi, plo, i));
    }
    next[k] = v;
}


// --------------------------------------------------------------- xlator
__global__ void xlator_kernel(const float2* __restrict__ in, float2* __restrict__ out, long long n,
                              const float2* __restrict__ phi, const float2* __restrict__ plo) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = cmulf(in[i], nco_tab(phi, plo, i));
}

// host side of the NCO tables
constexpr int NCO_PF = 64;   // >= the FIR kernel's load slots per thread
struct Nco {
    double w = 0.0;
    PhaseAcc phase;     // phase of the next input sample
    DevBuf plo, phi;
    DevBuf step;        // [3][NCO_PF]: e^{i w u NT}, NT = 64, 128, 256 (fp64 -> float)
    DevBuf rstep;       // [2][ROWS_STEP]: e^{i w D u}, D = 8, 32 (fir_rows_kernel's row step)
    const float2* rstep_for(int D) const { return rstep.as<float2>() + (D == 8 ? 0 : ROWS_STEP); }
    const float2* step_for(int NT) const { return step.as<float2>() + (NT == 64 ? 0 : NT == 128 ? 1 : 2) * NCO_PF; }
    int set_w(double w_) {
        w = w_;
        {
            std::vector<float2> st(3 * NCO_PF);
            const int nts[3] = {64, 128, 256};
            for (int k = 0; k < 3; k++)
                for (int u = 0; u < NCO_PF; u++) {
                    const double a = std::fmod(w * (double)u * (double)nts[k], 2.0 * M_PI);
                    st[k * NCO_PF + u] = make_float2((float)std::cos(a), (float)std::sin(a));
                }
            SDRGPU_CHECK(step.ensure(sizeof(float2) * st.size()));
            SDRGPU_HIP(hipMemcpy(step.p, st.data(), sizeof(float2) * st.size(), hipMemcpyHostToDevice));
            std::vector<float2> rs(2 * ROWS_STEP);
            for (int k = 0; k < 2; k++)
                for (int u = 0; u < ROWS_STEP; u++) {
                    const double a = std::fmod(w * (double)u * (k ? 32.0 : 8.0), 2.0 * M_PI);
                    rs[k * ROWS_STEP + u] = make_float2((float)std::cos(a), (float)std::sin(a));
                }
            SDRGPU_CHECK(rstep.ensure(sizeof(float2) * rs.size()));
            SDRGPU_HIP(hipMemcpy(rstep.p, rs.data(), sizeof(float2) * rs.size(), hipMemcpyHostToDevice));
        }
        std::vector<float2> t(NCO_LO);
        for (int k = 0; k < NCO_LO; k++) {
            const double a = std::fmod(w * (double)k, 2.0 * M_PI);
            t[k] = make_float2((float)std::cos(a), (float)std::sin(a));
        }
        SDRGPU_CHECK(plo.ensure(sizeof(float2) * NCO_LO));
        SDRGPU_HIP(hipMemcpy(plo.p, t.data(), sizeof(float2) * NCO_LO, hipMemcpyHostToDevice));
        return SDRGPU_OK;
    }
    // coarse table for a call of `count` samples starting at the current phase
    int prepare(int count, hipStream_t s) {
        const int nhi = (count >> NCO_LO_BITS) + 2;
        SDRGPU_CHECK(phi.ensure(sizeof(float2) * nhi));
        hipLaunchKernelGGL(nco_hi_kernel, dim3((nhi + 255) / 256), dim3(256), 0, s, phi.as<float2>(), nhi,
                           phase.value(), w);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
};

// ----------------------------------------------------------- quadrature
// demod/quadrature.h:41-56: arg(y * conj(d)) / dev (one expression for every kernel using it)
__device__ __forceinline__ float quad_value(float2 y, float2 d, float invDev) {
    const float br = d.x, bi = -d.y;
    const float re = (y.x * br) - (y.y * bi);
    const float im = (y.y * br) + (y.x * bi);
    return quad_atan2f(im, re) * invDev;
}
__global__ void quad_kernel(const float2* __restrict__ in, float* __restrict__ out, int n, const float2* __restrict__ din,
                            float2* __restrict__ dinNext, float invDev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 y = in[i];
    out[i] = quad_value(y, i ? in[i - 1] : din[0], invDev);
    if (i == n - 1) dinNext[0] = y;
}

// BroadcastFM mono for short calls (a reference block: 307,200 / 256 = 1,200 samples at
// 240 kS/s): the quadrature and the audio FIR (+ LRToStereo) in one launch instead of two
// 5-7 us ones. Workgroup b computes outputs [256 b, 256 b + 256) from the quadrature values of
// its window of [hist || quad(in)] (halo recomputed), with the FIR's tap order and fmaf chain
// (fir_kernel at D = 1), so the outputs are bit-identical to the two-launch path; the last
// workgroup writes the next call's FIR history and y[-1].
constexpr int WFM_TM = 256;
__global__ __launch_bounds__(WFM_TM) void wfm_short_kernel(
    const float2* __restrict__ in, int count, const float2* __restrict__ din, float2* __restrict__ dinNext,
    const float* __restrict__ hist, float* __restrict__ histNext, const float* __restrict__ taps, int Q, int H,
    float invDev, float2* __restrict__ out) {
    extern __shared__ float X[];
    const int tid = threadIdx.x;
    auto qv = [&](long long b) -> float {   // [hist || quad(in)][b], zero past the end
        if (b < H) return hist[b];
        const long long i = b - H;
        if (i >= count) return 0.0f;
        return quad_value(in[i], i ? in[i - 1] : din[0], invDev);
    };
    if (blockIdx.x == gridDim.x - 1) {
        for (int k = tid; k < H; k += WFM_TM) histNext[k] = qv((long long)count + k);
        if (tid == 0) dinNext[0] = in[count - 1];
        return;
    }
    const int m0 = blockIdx.x * WFM_TM;
    for (int j = tid; j < WFM_TM + Q; j += WFM_TM) X[j] = qv((long long)m0 + j);
    __syncthreads();
    const int m = m0 + tid;
    if (m >= count) return;
    float acc = 0.0f;
    for (int q = 0; q < Q; q++) acc = fmaf(X[tid + q], taps[q], acc);
    out[m] = make_float2(acc, acc);
}

// BroadcastFM mono for big calls (C5: 1,048,576 samples at 240 kS/s per step): the same fused form
// with K = 4 outputs per thread (1,024 per workgroup). The quadrature values of the window go to LDS in
// fir_tail's row layout (element e at row e mod K, column e / K: a thread's K-output register window
// reads consecutive columns, conflict-free), rows r and r + K/2 interleaved as float pairs, so the
// thread's outputs i and i + K / 2 run as one packed fp32 FMA (v_pk_fma_f32; each lane is the fmaf of the
// scalar chain, same bits) over the padded taps in tap order (fir_kernel at D = 1): the window pair of
// outputs (i, i + K/2) at tap u is rows ((i + u) mod K, (i + u + K/2) mod K), one stored pair, swapped
// (op_sel) when (i + u) mod K >= K/2. No quadrature round trip through HBM (quad_kernel +
// fir_kernel<float, float, 4>: 5.3 + 15.6 us per C5 step, r5m; scalar chains in this kernel 15.7 us).
#ifndef SDRGPU_WFM_BK
#define SDRGPU_WFM_BK 4   // outputs per thread (r6o: 14.6 vs 15.1 us per C5 step at 8, same bits; A/B builds: 8)
#endif
constexpr int WFM_BK = SDRGPU_WFM_BK, WFM_BNT = 256, WFM_BCH = WFM_BK * WFM_BNT;
__global__ __launch_bounds__(WFM_BNT) void wfm_big_kernel(
    const float2* __restrict__ in, int count, const float2* __restrict__ din, float2* __restrict__ dinNext,
    const float* __restrict__ hist, float* __restrict__ histNext, const float* __restrict__ taps, int Q, int H,
    float invDev, float2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float X[];
    constexpr int K = WFM_BK;
    const int tid = threadIdx.x;
    auto qv = [&](long long b) -> float {   // [hist || quad(in)][b], zero past the end
        if (b < H) return hist[b];
        const long long i = b - H;
        if (i >= count) return 0.0f;
        return quad_value(in[i], i ? in[i - 1] : din[0], invDev);
    };
    if (blockIdx.x == gridDim.x - 1) {
        for (int k = tid; k < H; k += WFM_BNT) histNext[k] = qv((long long)count + k);
        if (tid == 0) dinNext[0] = in[count - 1];
        return;
    }
    const long long m0 = (long long)blockIdx.x * WFM_BCH;
    const int RSK = WFM_BNT + Q / K + 2;   // columns per row (Q is a multiple of 8, <= 256: host-checked)
    float* T = X + K * RSK;                // the taps
    const f2v* P = reinterpret_cast<const f2v*>(X);   // P[r * RSK + c] = (row r, row r + K/2) at column c, r < K/2
    auto at = [&](int j) { return 2 * ((j % (K / 2)) * RSK + j / K) + (j / (K / 2)) % 2; };   // float index of element j
    for (int q = tid; q < Q; q += WFM_BNT) T[q] = taps[q];
    // the window [m0, m0 + K RSK) of [hist || quad(in)]: interior workgroups issue all their sample
    // loads at once (one memory round trip), the first and last take the element-wise path
    constexpr int NF = (K * (WFM_BNT + 256 / K + 2) + WFM_BNT - 1) / WFM_BNT;
    if (m0 >= H + 1 && m0 + K * RSK - H <= count) {
        float2 y[NF], yp[NF];
        const float2* src = in + (m0 - H);
#pragma unroll
        for (int k = 0; k < NF; k++) {
            const int j = tid + k * WFM_BNT;
            const int jj = j < K * RSK ? j : 0;
            y[k] = src[jj];
            yp[k] = src[jj - 1];
        }
#pragma unroll
        for (int k = 0; k < NF; k++) {
            const int j = tid + k * WFM_BNT;
            if (j < K * RSK) X[at(j)] = quad_value(y[k], yp[k], invDev);
        }
    } else {
        for (int j = tid; j < K * RSK; j += WFM_BNT) X[at(j)] = qv(m0 + j);
    }
    __syncthreads();
    f2v acc[K / 2], w[K / 2];   // acc[i] = outputs (i, i + K/2); w[r] = window rows (r, r + K/2)
#pragma unroll
    for (int i = 0; i < K / 2; i++) {
        acc[i] = f2v{0.f, 0.f};
        w[i] = P[i * RSK + tid];
    }
    for (int q0 = 0; q0 < Q; q0 += K) {
        float hv[K];
        f2v nx[K / 2];
#pragma unroll
        for (int u = 0; u < K; u++) hv[u] = T[q0 + u];   // (LDS broadcasts)
#pragma unroll
        for (int r = 0; r < K / 2; r++) nx[r] = P[r * RSK + tid + 1 + q0 / K];
#pragma unroll
        for (int u = 0; u < K; u++) {
#pragma unroll
            for (int i = 0; i < K / 2; i++) {
                const int r = (i + u) % K;
                const f2v x = r < K / 2 ? w[r] : __builtin_shufflevector(w[r - K / 2], w[r - K / 2], 1, 0);
                acc[i] = __builtin_elementwise_fma(x, f2v{hv[u], hv[u]}, acc[i]);
            }
            if (u < K / 2) w[u].x = nx[u].x;   // row u slides to the next column
            else w[u - K / 2].y = nx[u - K / 2].y;
        }
    }
    float a[K];
#pragma unroll
    for (int i = 0; i < K / 2; i++) {
        a[i] = acc[i].x;
        a[i + K / 2] = acc[i].y;
    }
    const long long m = m0 + (long long)tid * K;
    if (m + K <= count) {
        float4* o = reinterpret_cast<float4*>(out + m);   // (out: 8-byte stereo frames; 16-B aligned pairs)
        if (((uintptr_t)out & 15) == 0) {
#pragma unroll
            for (int i = 0; i < K; i += 2) o[i / 2] = make_float4(a[i], a[i], a[i + 1], a[i + 1]);
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < K; i++)
        if (m + i < count) out[m + i] = make_float2(a[i], a[i]);
}

template <int K, int NT>
__global__ __launch_bounds__(NT) void fir_tail_kernel(TailArgs t) {
    extern __shared__ __attribute__((aligned(16))) float2 XS[];
    __shared__ TailGeom gs[TAIL_MAXS];
    fir_tail_block<K, NT>(t, blockIdx.x, blockIdx.x == gridDim.x - 1, XS, gs);
}

// ------------------------------------------------ polyphase resampler
// multirate/polyphase_resampler.h:69-99 in closed form: with pos = offset*interp + phase,
// output m uses pos_m = pos0 + m*decim -> (offset_m, phase_m) = divmod(pos_m, interp).
template <typename DT>
__global__ void poly_kernel(const DT* __restrict__ hist, const DT* __restrict__ in, const float* __restrict__ bank,
                            DT* __restrict__ out, int H, int tpp, int interp, int decim, long long pos0, int M) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const long long pos = pos0 + (long long)m * decim;
    const long long off = pos / interp;
    const int ph = (int)(pos % interp);
    const float* hb = bank + (size_t)ph * tpp;
    DT acc = zero_of<DT>();
    for (int j = 0; j < tpp; j++) {
        const long long b = off + j;
        const DT x = b < H ? hist[b] : in[b - H];
        mac(acc, x, hb[j]);
    }
    out[m] = acc;
}

// ------------------------------------------------------------ converters
__device__ __forceinline__ float convert_one(int kind, const void* __restrict__ in, long long i) {
    switch (kind) {
    case SDRGPU_CONV_U8: return (((const uint8_t*)in)[i] - 128 + 0.5f) / (128.0f - 0.5f);
    case SDRGPU_CONV_I16: return (((const int16_t*)in)[i] + 0.5f) / (32768.0f - 0.5f);
    case SDRGPU_CONV_I24: {
        const uint8_t* p = (const uint8_t*)in + 3 * i;
        int32_t v = (int32_t)((uint32_t)(p[0] | (p[1] << 8) | (p[2] << 16)) << 8) >> 8;
        return (v + 0.5f) / (8388608.0f - 0.5f);
    }
    case SDRGPU_CONV_I32: return (float)((((const int32_t*)in)[i] + 0.5) / (2147483648.0 - 0.5));
    case SDRGPU_CONV_F64: return (float)((const double*)in)[i];
    case SDRGPU_CONV_I8: return ((float)((const int8_t*)in)[i]) * (float)(1.0 / 128.0f);
    default: return ((const float*)in)[i];   // SDRGPU_CONV_F32: IEEE float samples as they are
    }
}
__global__ void convert_kernel(int kind, const void* __restrict__ in, long long n, float* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = convert_one(kind, in, i);
}
// one-channel WAV (file_source worker_1ch, main.cpp:294-430): I = Q = the converted sample
__global__ void convert_mono_kernel(int kind, const void* __restrict__ in, long long n, float2* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = convert_one(kind, in, i);
    out[i] = make_float2(v, v);
}

// ================================================================ host blocks
int DevBuf::ensure(size_t want) {
    if (want <= bytes) return SDRGPU_OK;
    release();
    size_t sz = std::max<size_t>(want, 256);
    if (hipMalloc(&p, sz) != hipSuccess) {
        p = nullptr;
        set_error("hipMalloc(%zu) failed", sz);
        return SDRGPU_ENOMEM;
    }
    bytes = sz;
    return SDRGPU_OK;
}
void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}
int PinnedBuf::ensure(size_t want) {
    if (want <= bytes) return SDRGPU_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    size_t sz = std::max<size_t>(want, 256);
    if (hipHostMalloc(&p, sz, hipHostMallocDefault) != hipSuccess) {
        p = nullptr;
        set_error("hipHostMalloc(%zu) failed", sz);
        return SDRGPU_ENOMEM;
    }
    bytes = sz;
    return SDRGPU_OK;
}
PinnedBuf::~PinnedBuf() {
    if (p) (void)hipHostFree(p);
}

int StreamOrder::follow(hipStream_t s) {
    if (last == nullptr || last == s) return SDRGPU_OK;
    if (multi) {
        SDRGPU_HIP(hipStreamWaitEvent(s, ev, 0));
        return SDRGPU_OK;
    }
    SDRGPU_HIP(hipDeviceSynchronize());   // first stream change: the previous stream may be gone
    if (!ev) SDRGPU_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    multi = true;
    return SDRGPU_OK;
}
int StreamOrder::done(hipStream_t s) {
    if (multi) SDRGPU_HIP(hipEventRecord(ev, s));
    last = s;
    return SDRGPU_OK;
}
StreamOrder::~StreamOrder() {
    if (ev) (void)hipEventDestroy(ev);
}

Block::~Block() {
    if (own) (void)hipStreamDestroy(own);
}
int Block::init_stream() {
    SDRGPU_SET_DEVICE(device);
    SDRGPU_HIP(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
    return SDRGPU_OK;
}

// ------------------------------------------------------------------ FIR block
struct FirBlock : Block {
    int ttype = SDRGPU_F32, ntaps = 0, D = 1, offset = 0, Q = 1;
    bool xl = false, quad = false, stereo = false;
    Nco nco;                // XL: fused frequency xlator
    float invDev = 1.0f;    // QUAD
    DevBuf taps, hist[2], din[2];
    int cur = 0;            // ping-pong index

    int setup(int dev, int dtype_, int ttype_, const float* t, int n, int decim) {
        device = dev;
        in_dtype = dtype_;
        out_dtype = quad ? SDRGPU_F32 : (stereo ? SDRGPU_C64 : dtype_);
        ttype = ttype_;
        if (decim < 1) { set_error("fir: decimation %d < 1", decim); return SDRGPU_EARG; }
        D = decim;
        if (const char* e = tuning_env("SDRGPU_FIR_MFMA_NW")) mfNW = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FIR_MFMA_HALF")) mfHalf = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FIR_MFMA_DC")) mfDc = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FIR_MFMA_PS")) usePS = atoi(e);
        if (const char* e = tuning_env("SDRGPU_FIR_ROWS")) useRows = atoi(e);
        SDRGPU_CHECK(init_stream());
        SDRGPU_CHECK(set_taps(t, n));
        return SDRGPU_OK;
    }
    // FIR::setTaps (fir.h:31-52): history kept aligned to the newest sample;
    // DecimatingFIR::setTaps resets the decimation phase (decimating_fir.h:19-26)
    int set_taps(const float* t, int n) {
        if (!t || n < 1 || n > 64001) { set_error("fir: tap count %d out of range [1, 64001]", n); return SDRGPU_EARG; }
        SDRGPU_SET_DEVICE(device);
        const size_t es = esize(in_dtype);
        const int oldH = ntaps > 0 ? ntaps - 1 : 0, newH = n - 1;
        std::vector<unsigned char> oldHist((size_t)oldH * es), newHist((size_t)std::max(newH, 1) * es, 0);
        if (oldH > 0) SDRGPU_HIP(hipMemcpy(oldHist.data(), hist[cur].p, oldHist.size(), hipMemcpyDeviceToHost));
        const int keep = std::min(oldH, newH);
        if (keep > 0) std::memcpy(newHist.data() + (size_t)(newH - keep) * es, oldHist.data() + (size_t)(oldH - keep) * es, keep * es);
        for (int k = 0; k < 2; k++) SDRGPU_CHECK(hist[k].ensure(newHist.size()));
        SDRGPU_HIP(hipMemcpy(hist[cur].p, newHist.data(), newHist.size(), hipMemcpyHostToDevice));
        host_taps.assign(t, t + (size_t)n * (ttype == SDRGPU_C64 ? 2 : 1));
        ntaps = n;
        offset = 0;
        SDRGPU_CHECK(upload_taps());
        if (quad) {
            for (int k = 0; k < 2; k++) SDRGPU_CHECK(din[k].ensure(sizeof(float2)));
        }
        return SDRGPU_OK;
    }
    int set_decimation(int d) {
        if (d < 1) { set_error("fir: decimation %d < 1", d); return SDRGPU_EARG; }
        D = d;
        offset = 0;
        return upload_taps();
    }
    // device taps in [p][q] = h[q*D + p] order, zero past ntaps (phase-major like the LDS span)
    std::vector<float> host_taps;
    int upload_taps() {
        SDRGPU_SET_DEVICE(device);
        Q = (ntaps + D - 1) / D;
        Q = (Q + 7) / 8 * 8;      // kernel chunk QC = 8 (zero taps past ntaps)
        const int e = ttype == SDRGPU_C64 ? 2 : 1;
        std::vector<float> pq((size_t)D * Q * e, 0.0f);
        for (int p = 0; p < D; p++)
            for (int q = 0; q < Q; q++) {
                const int j = q * D + p;
                if (j < ntaps)
                    for (int k = 0; k < e; k++) pq[((size_t)p * Q + q) * e + k] = host_taps[(size_t)j * e + k];
            }
        SDRGPU_CHECK(taps.ensure(sizeof(float) * pq.size()));
        SDRGPU_HIP(hipMemcpy(taps.p, pq.data(), sizeof(float) * pq.size(), hipMemcpyHostToDevice));
        // matrix-core path (fir_mfma_kernel): complex data, real taps, 16..32 taps per phase,
        // D a power of two <= 8 (with 128 threads, a load slot advances by whole 16-row pad groups)
        const int Qr = (ntaps + D - 1) / D;
        const bool cplx = in_dtype == SDRGPU_C64 && ttype == SDRGPU_F32 && !stereo && (D & (D - 1)) == 0 && Qr <= 32 &&
                          useMfma != 0;
        mf = cplx && D <= 8 && (Qr >= 16 || useMfma == 2);
        // phase-split tiles for the larger decimations (and on request for the others)
        mfps = cplx && !mf && D >= 4 && D <= 32 && (usePS != 0);
        if (usePS == 2 && cplx && D >= 4 && D <= 32) { mfps = true; mf = false; }
        // row-streaming kernel for D = 32 with <= 8 taps per phase (VFO stage 1), ahead of the MFMA tiles
        rowsk = in_dtype == SDRGPU_C64 && ttype == SDRGPU_F32 && !stereo && rows_qp(D, Qr) > 0 &&
                !(quad && D == 32) && (useRows == 2 || (useRows == 1 && D == 32));
        if (mf || mfps) {
            // gz[p][t] = h[(t - 15) D + p], gzs entries per phase (t < 15 + 4 ks suffice)
            gzs = mf ? MF_GZ : 16 + 4 * ((15 + Qr + 3) / 4);
            std::vector<float> g((size_t)D * gzs, 0.0f);
            for (int p = 0; p < D; p++)
                for (int t = 15; t < gzs; t++) {
                    const int j = (t - 15) * D + p;
                    if (t - 15 < Qr && j < ntaps) g[(size_t)p * gzs + t] = host_taps[j];
                }
            SDRGPU_CHECK(gzTaps.ensure(sizeof(float) * g.size()));
            SDRGPU_HIP(hipMemcpy(gzTaps.p, g.data(), sizeof(float) * g.size(), hipMemcpyHostToDevice));
        }
        return SDRGPU_OK;
    }
    void* histNextArg = nullptr;   // the running call's history destination (FirArgs::histNext)
    bool ncoTable = false;         // the running call's kernels read the per-call NCO table
    bool mf = false;        // fir_mfma_kernel selected for the current taps / decimation
    bool mfps = false;      // fir_mfma_ps_kernel selected
    bool rowsk = false;     // fir_rows_kernel selected
    int useRows = 1;        // SDRGPU_FIR_ROWS (tuning): 0 off, 1 auto (D = 32), 2 also D = 8
    template <int D, int QP, bool QD, int RS = rows_rs<D>()>
    int launch_rows_rs(FirArgs& a, hipStream_t s) {
        const int q = QD ? 1 : 0;
        const long long segs = ((long long)a.M + q + (RS - q) - 1) / (RS - q);
        const int blocks = (int)((segs + 4 * (64 / D) - 1) / (4 * (64 / D)));   // 4 waves x 64/D groups
        const int g = blocks + (a.histNext ? 1 : 0);
        if (xl) hipLaunchKernelGGL((fir_rows_kernel<D, QP, true, QD, RS>), dim3(g), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((fir_rows_kernel<D, QP, false, QD, RS>), dim3(g), dim3(256), 0, s, a);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
    // D = 32: 32-output segments (one row batch each) at every call size, the segments the spectrum
    // launches cut for a fused first stage (fft.hip vfo_quarter_block: same segments, same bits); a
    // reference-size block (9,600 stage-1 outputs) is 300 segments, where 128-output ones were 75
    // segments in 10 workgroups (62 us)
    template <int D, int QP, bool QD>
    int launch_rows(FirArgs& a, hipStream_t s) {
        if constexpr (D == 32 && !QD) return launch_rows_rs<D, QP, QD, 32>(a, s);
        return launch_rows_rs<D, QP, QD>(a, s);
    }
    // taps per phase of the rows kernel: D = 32 exact (2..8), D = 8 padded to 16, 24 or 32
    static int rows_qp(int D, int Qr) {
        if (D == 32) return (Qr >= 2 && Qr <= 8) ? Qr : 0;
        if (D == 8) return Qr < 2 ? 0 : Qr <= 16 ? 16 : Qr <= 24 ? 24 : Qr <= 32 ? 32 : 0;
        return 0;
    }
    // the row kernel's launch arguments for one call (state as it stands: nothing changes here)
    FirArgs rows_args(const void* in, int count, void* out, int M) {
        FirArgs a{};
        a.histNext = histNextArg;
        a.hist = hist[cur].p; a.in = in; a.taps = taps.p; a.out = out;
        a.din = din[cur].as<float2>(); a.dinNext = din[cur ^ 1].as<float2>();
        a.phi = nco.phi.as<float2>(); a.plo = nco.plo.as<float2>(); a.ncoTheta0 = nco.phase.value(); a.ncoW = nco.w;
        a.ntaps = ntaps; a.H = ntaps - 1; a.count = count; a.D = D; a.Q = Q; a.offset0 = offset; a.M = M;
        a.invDev = invDev;
        a.nstep = xl ? nco.rstep_for(D) : nullptr;
        return a;
    }
    // A call whose row-kernel segments another launch runs (fft.hip's spectrum launches, VfoStage1):
    // D = 32 with the fused xlator, 5 taps per phase (the RxVFO's plan_256 stage 1), a history to
    // carry. Those launches use 128-output segments at any call size: a segment's length does not
    // change any output's bits (each output's partial runs over its own QP rows, in row order).
    bool rows_external(int count) {
        return rowsk && xl && !quad && D == 32 && rows_qp(D, (ntaps + D - 1) / D) == 5 && ntaps > 1 && out_count(count) > 0;
    }
    // the state update of run() after such a call
    void rows_commit(int count, int M) {
        cur ^= 1;
        offset = offset + M * D - count;
        nco.phase.advance(nco.w, count);
    }
    int run_rows(const void* in, int count, void* out, int M, hipStream_t s) {
        FirArgs a = rows_args(in, count, out, M);
        const int qp = rows_qp(D, (ntaps + D - 1) / D);
        if (D == 32 && !quad) {
            switch (qp) {
            case 2: return launch_rows<32, 2, false>(a, s);
            case 3: return launch_rows<32, 3, false>(a, s);
            case 4: return launch_rows<32, 4, false>(a, s);
            case 5: return launch_rows<32, 5, false>(a, s);
            case 6: return launch_rows<32, 6, false>(a, s);
            case 7: return launch_rows<32, 7, false>(a, s);
            case 8: return launch_rows<32, 8, false>(a, s);
            }
        } else if (D == 8) {
            switch (qp) {
            case 16: return quad ? launch_rows<8, 16, true>(a, s) : launch_rows<8, 16, false>(a, s);
            case 24: return quad ? launch_rows<8, 24, true>(a, s) : launch_rows<8, 24, false>(a, s);
            case 32: return quad ? launch_rows<8, 32, true>(a, s) : launch_rows<8, 32, false>(a, s);
            }
        }
        set_error("fir: rows kernel does not take (D %d, ntaps %d)", D, ntaps);
        return SDRGPU_EARG;
    }
    int gzs = MF_GZ;
    int usePS = 1;          // SDRGPU_FIR_MFMA_PS (tuning): 0 off, 1 auto (D >= 4 where fir_mfma_kernel is not used), 2 force
    template <bool XL, bool QD>
    int launch_mfma_ps(FirArgs& a, int tiles, size_t lds, hipStream_t s) {
        auto k = fir_mfma_ps_kernel<XL, QD>;
        SDRGPU_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k, dim3(tiles + (a.histNext ? 1 : 0)), dim3(256), lds, s, a);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
    int run_mfma_ps(const void* in, int count, void* out, int M, hipStream_t s) {
        FirArgs a{};
        a.histNext = histNextArg;
        a.hist = hist[cur].p; a.in = in; a.taps = gzTaps.p; a.out = out;
        a.din = din[cur].as<float2>(); a.dinNext = din[cur ^ 1].as<float2>();
        a.phi = nco.phi.as<float2>(); a.plo = nco.plo.as<float2>(); a.ncoTheta0 = nco.phase.value(); a.ncoW = nco.w;
        a.ntaps = ntaps; a.H = ntaps - 1; a.count = count; a.D = D; a.offset0 = offset; a.M = M;
        const int Qr = (ntaps + D - 1) / D;
        a.Q = (15 + Qr + 3) / 4;                        // k steps
        const int rows = 256 + 4 * a.Q;
        a.RSP = (rows + rows / 16) | 1;                 // odd: the D phases of one load slot in distinct banks
        a.TMS = quad ? 255 : 256;
        a.dshift = __builtin_ctz((unsigned)D);
        a.invDev = invDev;
        a.nstep = xl ? nco.step_for(256) : nullptr;
        const size_t xb = std::max(sizeof(float2) * (size_t)D * a.RSP, sizeof(float2) * 4 * 256);   // span / partials
        a.tapsLdsOff = (int)((xb + 15) / 16 * 16);
        a.gzs = gzs;
        const size_t lds = a.tapsLdsOff + sizeof(float) * D * gzs;   // D = 32, Qp = 5: 79.6 KB, 2 per CU
        if (lds > 150 * 1024) { set_error("fir: MFMA tile does not fit (D %d)", D); return SDRGPU_EARG; }
        const int tiles = (M + a.TMS - 1) / a.TMS;
        a.ntiles = tiles;
        if (xl) return quad ? launch_mfma_ps<true, true>(a, tiles, lds, s) : launch_mfma_ps<true, false>(a, tiles, lds, s);
        return quad ? launch_mfma_ps<false, true>(a, tiles, lds, s) : launch_mfma_ps<false, false>(a, tiles, lds, s);
    }
    int useMfma = 1;        // f32 MFMA tiles: 1 auto (>= 16 taps per phase)
    DevBuf gzTaps;
    template <int NW, bool XL, bool QD>
    int launch_mfma(FirArgs& a, int tiles, size_t lds, bool half, hipStream_t s) {
        auto k = half ? (a.D == 8 && mfDc ? fir_mfma_kernel<NW, XL, QD, true, 8> : fir_mfma_kernel<NW, XL, QD, true>)
                      : (a.D == 8 && mfDc ? fir_mfma_kernel<NW, XL, QD, false, 8> : fir_mfma_kernel<NW, XL, QD, false>);
        SDRGPU_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k, dim3(tiles + (a.histNext ? 1 : 0)), dim3(64 * NW), lds, s, a);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
    int mfNW = 4;           // SDRGPU_FIR_MFMA_NW (tuning): waves (x 256 outputs) per workgroup, 4 or 2 (2: 4 WG/CU, measured 13% slower on C3)
    // fir_mfma_kernel HALF: half the phases' span in LDS at a time, 4 workgroups per CU (105 VGPRs, no
    // spill); C3 kernel 0.842 -> 0.787 ms (3 interleaved runs, r4d). SDRGPU_FIR_MFMA_HALF=0 (tuning) off
    int mfHalf = 1;
    int mfDc = 1;           // SDRGPU_FIR_MFMA_DC=0 (tuning): D = 8 as a run-time value (fir_mfma_kernel DC)
    template <int NW>
    int run_mfma_nw(const void* in, int count, void* out, int M, hipStream_t s) {
        constexpr int MF_TM = 256 * NW, MF_ROWS = mf_rows(NW);
        FirArgs a{};
        a.histNext = histNextArg;
        a.hist = hist[cur].p; a.in = in; a.taps = gzTaps.p; a.out = out;
        a.din = din[cur].as<float2>(); a.dinNext = din[cur ^ 1].as<float2>();
        a.phi = nco.phi.as<float2>(); a.plo = nco.plo.as<float2>(); a.ncoTheta0 = nco.phase.value(); a.ncoW = nco.w;
        a.ntaps = ntaps; a.H = ntaps - 1; a.count = count; a.D = D; a.offset0 = offset; a.M = M;
        a.TMS = quad ? MF_TM - 1 : MF_TM;
        a.RSP = MF_ROWS + MF_ROWS / 16 + 1;
        a.dshift = __builtin_ctz((unsigned)D);
        a.invDev = invDev;
        a.nstep = xl ? nco.step_for(64 * NW) : nullptr;
        // HALF needs two phase halves (D >= 2) and the PF load slots covering the span (D <= 8)
        const bool half = mfHalf && D >= 2 && D <= 8;
        const size_t xb = std::max(sizeof(float2) * (size_t)(half ? D / 2 : D) * a.RSP, sizeof(float2) * (size_t)MF_TM);
        a.tapsLdsOff = (int)((xb + 15) / 16 * 16);
        const size_t lds = a.tapsLdsOff + sizeof(float) * D * MF_GZ;
        const int tiles = (M + a.TMS - 1) / a.TMS;
        a.ntiles = tiles;
        if (xl) return quad ? launch_mfma<NW, true, true>(a, tiles, lds, half, s) : launch_mfma<NW, true, false>(a, tiles, lds, half, s);
        return quad ? launch_mfma<NW, false, true>(a, tiles, lds, half, s) : launch_mfma<NW, false, false>(a, tiles, lds, half, s);
    }
    int run_mfma(const void* in, int count, void* out, int M, hipStream_t s) {
        return mfNW == 4 ? run_mfma_nw<4>(in, count, out, M, s) : run_mfma_nw<2>(in, count, out, M, s);
    }
    int out_count(int count) override { return count > offset ? (count - offset + D - 1) / D : 0; }
    int reset() override {
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemset(hist[cur].p, 0, (size_t)std::max(ntaps - 1, 1) * esize(in_dtype)));
        if (quad) SDRGPU_HIP(hipMemset(din[cur].p, 0, sizeof(float2)));
        offset = 0;
        nco.phase.reset();
        return SDRGPU_OK;
    }
    int forceK = 0;         // (A/B history: outputs per thread forced)
    int choose_k() const {
        if (forceK == 1 || forceK == 2 || forceK == 4 || forceK == 8) return forceK;
        // register blocking pays when a row feeds several taps per phase (unpadded Q large)
        const int Qr = (ntaps + D - 1) / D;
        if (Qr >= 16) return 4;
        if (Qr >= 6) return 2;
        return 1;
    }
    int NT = 256;
    int forceNT = 0;        // (A/B history: threads per tile forced)
    int ldsCap = 76;        // preferred LDS per tile (KB)
    template <typename DT, typename TT, int K, bool XL, bool QD, bool ST>
    int launch_t(FirArgs& a, int tiles, size_t lds, hipStream_t s) {
        // taps behind the span in LDS when they fit (<= 16 KB)
        const size_t tb = (size_t)D * Q * sizeof(TT);
        const bool tl = tb <= 16 * 1024 && lds + tb <= 160 * 1024;
        a.tapsLdsOff = (int)((lds + 15) / 16 * 16);
        if (tl) lds = a.tapsLdsOff + tb;
        auto k = tl ? fir_kernel<DT, TT, K, XL, QD, ST, true> : fir_kernel<DT, TT, K, XL, QD, ST, false>;
        SDRGPU_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        a.ntiles = tiles;
        a.simple = (NT % D == 0) && ((NT / D) % K == 0);
        a.nstep = xl ? nco.step_for(NT) : nullptr;
        // one tile per workgroup: a co-resident persistent grid with a register prefetch of the
        // next tile was measured 1.5x SLOWER on C3 (the hardware's own workgroup turnover
        // staggers the load/compute phases of the workgroups sharing a CU better)
        hipLaunchKernelGGL(k, dim3(tiles + (a.histNext ? 1 : 0)), dim3(NT), lds, s, a);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
    template <typename DT, typename TT, bool XL, bool QD, bool ST>
    int launch_k(FirArgs& a, int K, int tiles, size_t lds, hipStream_t s) {
        if (K == 8) return launch_t<DT, TT, 8, XL, QD, ST>(a, tiles, lds, s);
        if (K == 4) return launch_t<DT, TT, 4, XL, QD, ST>(a, tiles, lds, s);
        if (K == 2) return launch_t<DT, TT, 2, XL, QD, ST>(a, tiles, lds, s);
        return launch_t<DT, TT, 1, XL, QD, ST>(a, tiles, lds, s);
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count < 0) { set_error("fir: negative count"); return SDRGPU_EARG; }
        SDRGPU_SET_DEVICE(device);
        const int M = out_count(count);
        const int H = ntaps - 1;
        // the row kernel forms its coarse phasors itself (nco_inline); the tile kernels and the
        // separate history kernel of a call without outputs read the per-call table
        ncoTable = xl && count > 0 && (M == 0 || !rowsk);
        if (ncoTable) SDRGPU_CHECK(nco.prepare(count, s));
        // with outputs to compute, the FIR launch itself carries the history (fir_hist_block)
        histNextArg = (M > 0 && H > 0) ? hist[cur ^ 1].p : nullptr;
        if (M > 0 && rowsk) {
            SDRGPU_CHECK(run_rows(in, count, out, M, s));
        } else if (M > 0 && mf) {
            SDRGPU_CHECK(run_mfma(in, count, out, M, s));
        } else if (M > 0 && mfps) {
            SDRGPU_CHECK(run_mfma_ps(in, count, out, M, s));
        } else if (M > 0) {
            int K = choose_k();
            // LDS budget: span (TM + Q + K rows) * D elements + taps; shrink K, then the
            // tile's thread count, until it fits (large decimations: plan_8192 stage 0)
            size_t es = esize(in_dtype);
            size_t lds = 0;
            int RSK = 0, RSP = 0;
            // prefer a tile that leaves room for two workgroups per CU (<= 76 KB), else <= 150 KB
            const int K0 = K;
            for (size_t cap : {(size_t)ldsCap * 1024, (size_t)150 * 1024}) {
                K = K0;
                NT = (forceNT == 64 || forceNT == 128) ? forceNT : 256;
                for (;;) {
                    const int TM = NT * K;
                    const int rows = TM + Q + 2 * K;
                    RSK = (rows + K - 1) / K;
                    RSP = K * RSK + 1;
                    lds = es * (size_t)D * RSP;
                    if (lds <= cap) break;
                    if (K > 1) K /= 2;
                    else if (NT > 64) NT /= 2;
                    else break;
                }
                if (lds <= cap) break;
            }
            if (lds > 150 * 1024) {
                set_error("fir: tile does not fit LDS (ntaps %d, decim %d)", ntaps, D);
                return SDRGPU_EARG;
            }
            const int TM = NT * K;
            const int TMS = quad ? TM - 1 : TM;
            const int tiles = (M + TMS - 1) / TMS;
            FirArgs a{};
            a.histNext = histNextArg;
            a.hist = hist[cur].p; a.in = in; a.taps = taps.p; a.out = out;
            a.din = din[cur].as<float2>(); a.dinNext = din[cur ^ 1].as<float2>();
            a.phi = nco.phi.as<float2>(); a.plo = nco.plo.as<float2>(); a.ncoTheta0 = nco.phase.value(); a.ncoW = nco.w;
            a.ntaps = ntaps; a.H = H; a.count = count; a.D = D; a.Q = Q; a.offset0 = offset; a.M = M;
            a.TMS = TMS; a.RSK = RSK; a.RSP = RSP; a.invDev = invDev;
            a.dshift = (D & (D - 1)) ? -1 : __builtin_ctz((unsigned)D);
            int rc;
            if (in_dtype == SDRGPU_F32) {
                rc = stereo ? launch_k<float, float, false, false, true>(a, K, tiles, lds, s)
                            : launch_k<float, float, false, false, false>(a, K, tiles, lds, s);
            } else if (ttype == SDRGPU_C64) {
                rc = launch_k<float2, float2, false, false, false>(a, K, tiles, lds, s);
            } else if (xl && quad) {
                rc = launch_k<float2, float, true, true, false>(a, K, tiles, lds, s);
            } else if (xl) {
                rc = launch_k<float2, float, true, false, false>(a, K, tiles, lds, s);
            } else if (quad) {
                rc = launch_k<float2, float, false, true, false>(a, K, tiles, lds, s);
            } else {
                rc = launch_k<float2, float, false, false, false>(a, K, tiles, lds, s);
            }
            SDRGPU_CHECK(rc);
        }
        if (quad && M == 0) {
            SDRGPU_HIP(hipMemcpyAsync(din[cur ^ 1].p, din[cur].p, sizeof(float2), hipMemcpyDeviceToDevice, s));
        }
        if (H > 0 && M == 0) {
            const int nb = (H + 255) / 256;
            if (in_dtype == SDRGPU_F32) {
                hipLaunchKernelGGL((fir_hist_kernel<float, false>), dim3(nb), dim3(256), 0, s, hist[cur].as<float>(),
                                   (const float*)in, hist[cur ^ 1].as<float>(), H, count, nullptr, nullptr);
            } else if (xl) {
                hipLaunchKernelGGL((fir_hist_kernel<float2, true>), dim3(nb), dim3(256), 0, s, hist[cur].as<float2>(),
                                   (const float2*)in, hist[cur ^ 1].as<float2>(), H, count, nco.phi.as<float2>(),
                                   nco.plo.as<float2>());
            } else {
                hipLaunchKernelGGL((fir_hist_kernel<float2, false>), dim3(nb), dim3(256), 0, s, hist[cur].as<float2>(),
                                   (const float2*)in, hist[cur ^ 1].as<float2>(), H, count, nullptr, nullptr);
            }
            SDRGPU_HIP(hipGetLastError());
        }
        cur ^= 1;
        offset = offset + M * D - count;
        if (xl) nco.phase.advance(nco.w, count);
        return M;
    }
};

// --------------------------------------------------------------- xlator block
struct XlatorBlock : Block {
    Nco nco;
    int out_count(int count) override { return count; }
    int reset() override { nco.phase.reset(); return SDRGPU_OK; }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        SDRGPU_SET_DEVICE(device);
        if (count > 0) {
            SDRGPU_CHECK(nco.prepare(count, s));
            hipLaunchKernelGGL(xlator_kernel, dim3((count + 255) / 256), dim3(256), 0, s, (const float2*)in, (float2*)out,
                               (long long)count, nco.phi.as<float2>(), nco.plo.as<float2>());
            SDRGPU_HIP(hipGetLastError());
        }
        nco.phase.advance(nco.w, count);
        return count;
    }
};

// ------------------------------------------------------------ quadrature block
struct QuadBlock : Block {
    float invDev = 1.0f;
    DevBuf din[2];
    int cur = 0;
    int out_count(int count) override { return count; }
    int reset() override {
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemset(din[cur].p, 0, sizeof(float2)));
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        SDRGPU_SET_DEVICE(device);
        if (count <= 0) return 0;
        hipLaunchKernelGGL(quad_kernel, dim3((count + 255) / 256), dim3(256), 0, s, (const float2*)in, (float*)out, count,
                           din[cur].as<float2>(), din[cur ^ 1].as<float2>(), invDev);
        SDRGPU_HIP(hipGetLastError());
        cur ^= 1;
        return count;
    }
};

// ------------------------------------------------------------- polyphase block
struct PolyBlock : Block {
    int interp = 1, decim = 1, tpp = 1, phase = 0, offset = 0;
    DevBuf bank, hist[2];
    int cur = 0;
    int setup(int dev, int dtype, int ip, int dc, const float* taps, int n) {
        device = dev;
        in_dtype = out_dtype = dtype;
        if (ip < 1 || dc < 1 || !taps || n < 1) { set_error("polyphase: bad ratio/taps"); return SDRGPU_EARG; }
        interp = ip; decim = dc;
        SDRGPU_CHECK(init_stream());
        // multirate/polyphase_bank.h:15-47: phases[P-1-(i%P)][i/P] = taps[i]
        tpp = (n + interp - 1) / interp;
        std::vector<float> b((size_t)interp * tpp, 0.0f);
        for (int i = 0; i < interp * tpp; i++)
            b[(size_t)((interp - 1) - (i % interp)) * tpp + i / interp] = (i < n) ? taps[i] : 0.0f;
        SDRGPU_CHECK(bank.ensure(sizeof(float) * b.size()));
        SDRGPU_HIP(hipMemcpy(bank.p, b.data(), sizeof(float) * b.size(), hipMemcpyHostToDevice));
        for (int k = 0; k < 2; k++) SDRGPU_CHECK(hist[k].ensure(esize(dtype) * std::max(tpp - 1, 1)));
        return reset();
    }
    int out_count(int count) override {
        // while (offset < count) { out; phase += decim; offset += phase / interp; phase %= interp; }
        long long pos = (long long)offset * interp + phase;
        long long lim = (long long)count * interp;
        if (pos >= lim) return 0;
        return (int)((lim - 1 - pos) / decim + 1);
    }
    int reset() override {
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemset(hist[cur].p, 0, esize(in_dtype) * std::max(tpp - 1, 1)));
        phase = 0; offset = 0;
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        SDRGPU_SET_DEVICE(device);
        const int M = out_count(count);
        const int H = tpp - 1;
        const long long pos0 = (long long)offset * interp + phase;
        if (M > 0) {
            if (in_dtype == SDRGPU_F32)
                hipLaunchKernelGGL((poly_kernel<float>), dim3((M + 255) / 256), dim3(256), 0, s, hist[cur].as<float>(),
                                   (const float*)in, bank.as<float>(), (float*)out, H, tpp, interp, decim, pos0, M);
            else
                hipLaunchKernelGGL((poly_kernel<float2>), dim3((M + 255) / 256), dim3(256), 0, s, hist[cur].as<float2>(),
                                   (const float2*)in, bank.as<float>(), (float2*)out, H, tpp, interp, decim, pos0, M);
            SDRGPU_HIP(hipGetLastError());
        }
        if (H > 0) {
            const int nb = (H + 255) / 256;
            if (in_dtype == SDRGPU_F32)
                hipLaunchKernelGGL((fir_hist_kernel<float, false>), dim3(nb), dim3(256), 0, s, hist[cur].as<float>(),
                                   (const float*)in, hist[cur ^ 1].as<float>(), H, count, nullptr, nullptr);
            else
                hipLaunchKernelGGL((fir_hist_kernel<float2, false>), dim3(nb), dim3(256), 0, s, hist[cur].as<float2>(),
                                   (const float2*)in, hist[cur ^ 1].as<float2>(), H, count, nullptr, nullptr);
            SDRGPU_HIP(hipGetLastError());
            cur ^= 1;
        }
        long long pos = pos0 + (long long)M * decim;
        offset = (int)(pos / interp) - count;
        phase = (int)(pos % interp);
        return M;
    }
};

// ---------------------------------------------------------- chains of blocks
// Runs children back to back on one stream through device scratch buffers.
struct ChainBlock : Block {
    std::vector<std::unique_ptr<Block>> kids;
    DevBuf scratch[2];
    int out_count(int count) override {
        for (auto& k : kids) count = k->out_count(count);   // (does not mutate state)
        return count;
    }
    int reset() override {
        for (auto& k : kids) SDRGPU_CHECK(k->reset());
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (kids.empty()) {
            SDRGPU_HIP(hipMemcpyAsync(out, in, (size_t)count * esize(in_dtype), hipMemcpyDeviceToDevice, s));
            return count;
        }
        int nt = 0;
        const int tr = run_tail(in, count, out, s, &nt);
        if (tr < 0) return tr;
        if (tr > 0) return nt;
        return run_from(0, in, count, out, s);
    }
    // kids[i0..] on n samples at src (kid i0's input), the last one writing `out`
    int run_from(size_t i0, const void* src, int n, void* out, hipStream_t s) {
        if (i0 >= kids.size()) {
            if (src != out) SDRGPU_HIP(hipMemcpyAsync(out, src, (size_t)n * esize(out_dtype), hipMemcpyDeviceToDevice, s));
            return n;
        }
        // upper bound of intermediate sizes: each child's output never exceeds its input here
        for (size_t i = i0; i < kids.size(); i++) {
            void* dst;
            if (i + 1 == kids.size()) {
                dst = out;
            } else {
                const int m = kids[i]->out_count(n);
                SDRGPU_CHECK(scratch[i & 1].ensure((size_t)std::max(m, 1) * esize(kids[i]->out_dtype)));
                dst = scratch[i & 1].p;
            }
            n = kids[i]->run(src, n, dst, s);
            if (n < 0) return n;
            src = dst;
        }
        return n;
    }
    // Short calls: the first kid as usual, then every later kid -- when all are plain FIR blocks
    // (complex data, real taps, no fused xlator / quadrature) -- in one fir_tail_kernel launch.
    // Returns 1 (done, *nout = outputs), 0 (not applicable: the per-kid path runs) or an error.
    static constexpr int kTailMaxIn = 1 << 15;   // first kid's outputs (a reference block: 9,600)
    // SDRGPU_VFO_TAIL (tuning): 0 off; 1 calls up to kTailMaxIn; 2 (default) every size (big calls:
    // thousands of tail workgroups, each ~TAIL_PF * TAIL_NT stage-0 samples: the C5 step's three
    // later-stage launches become one, 1.760 -> 1.747 ms, 3 interleaved runs, r4j; 512 last-stage
    // outputs per workgroup to start from measured best of 32 / 64 / 128 / 512, r4l)
    int tailMode = -1;
    int tailBigOut = 512;   // big calls: last-stage outputs per workgroup to start from
    // big calls: the workgroup count and image size depend only on (n0, the stages' offsets), which
    // repeat call after call; the per-workgroup geometry scan is kept for the last key
    struct TailKey {
        int n0 = -1, S = 0;
        int off[TAIL_MAXS] = {}, H[TAIL_MAXS] = {}, Q[TAIL_MAXS] = {}, D[TAIL_MAXS] = {};
        int G = 0, maxEl = 0;
    } tailCache;
    // The tail launch's arguments for kids[1..] on n0 samples of kid 0's output: 1 (t, f, lds
    // filled), 0 (not applicable: the per-kid path runs).
    int tail_plan(int n0, TailArgs& t, FirBlock** f, size_t& lds) {
        if (tailMode < 0) {
            const char* e = tuning_env("SDRGPU_VFO_TAIL");
            tailMode = e ? atoi(e) : 2;
            if (const char* b = tuning_env("SDRGPU_TAIL_BIGOUT")) tailBigOut = std::max(32, atoi(b));
        }
        const int S = (int)kids.size() - 1;
        if (!tailMode || S < 2 || S > TAIL_MAXS) return 0;
        const bool big = n0 > kTailMaxIn;
        if (big && tailMode < 2) return 0;
        for (int i = 0; i < S; i++) {
            f[i] = dynamic_cast<FirBlock*>(kids[i + 1].get());
            if (!f[i] || f[i]->in_dtype != SDRGPU_C64 || f[i]->ttype != SDRGPU_F32 || f[i]->xl || f[i]->quad ||
                f[i]->stereo || f[i]->offset > f[i]->ntaps - 1 || f[i]->Q % 8 != 0 || (f[i]->D & (f[i]->D - 1)) ||
                f[i]->D > TAIL_NT / 8)
                return 0;
        }
        t = TailArgs{};
        t.S = S;
        t.K = big ? TAIL_K_BIG : TAIL_K;
        t.NT = big ? TAIL_NT_BIG : TAIL_NT;
        int n = n0;
        for (int i = 0; i < S; i++) {
            TailStage& st = t.st[i];
            st.hist = f[i]->hist[f[i]->cur].as<float2>();
            st.histNext = f[i]->hist[f[i]->cur ^ 1].as<float2>();
            st.taps = f[i]->taps.as<float>();
            st.H = f[i]->ntaps - 1;
            st.n = n;
            st.D = f[i]->D;
            st.dsh = __builtin_ctz((unsigned)st.D);
            st.Q = f[i]->Q;
            st.off = f[i]->offset;
            st.M = f[i]->out_count(n);
            n = st.M;
        }
        // ~128 last-stage outputs per workgroup, more workgroups while stage 0's image exceeds one
        // load batch (TAIL_PF per thread); big calls start from ~512 per workgroup
        int maxEl = 0;
        TailGeom g[TAIL_MAXS];
        // (the geometry depends on exactly these: every stage's offset, history, padded taps per phase
        // and decimation, and the stage count)
        bool cached = big && tailCache.n0 == n0 && tailCache.S == S;
        for (int i = 0; cached && i < S; i++)
            cached = tailCache.off[i] == t.st[i].off && tailCache.H[i] == t.st[i].H && tailCache.Q[i] == t.st[i].Q &&
                     tailCache.D[i] == t.st[i].D;
        if (cached) {
            t.G = tailCache.G;
            maxEl = tailCache.maxEl;
        } else {
            for (t.G = big ? std::max((n + tailBigOut - 1) / tailBigOut, 1) : std::min(std::max((n + 127) / 128, 1), 32);; t.G *= 2) {
                int nel0 = 0;
                maxEl = 0;
                for (int w = 0; w < t.G; w++) {
                    maxEl = std::max(maxEl, tail_geometry(t, w, g));
                    nel0 = std::max(nel0, g[0].nel);
                }
                if (nel0 <= TAIL_PF * t.NT) break;
                if ((!big && t.G >= 64) || t.G >= std::max(n, 1) || t.G >= (1 << 20)) return 0;
            }
            if (big) {
                tailCache.n0 = n0;
                tailCache.S = S;
                for (int i = 0; i < S; i++) {
                    tailCache.off[i] = t.st[i].off;
                    tailCache.H[i] = t.st[i].H;
                    tailCache.Q[i] = t.st[i].Q;
                    tailCache.D[i] = t.st[i].D;
                }
                tailCache.G = t.G;
                tailCache.maxEl = maxEl;
            }
        }
        t.ldsEl = maxEl;
        int tapF = 0;
        for (int i = 0; i < S; i++) {
            t.tapOff[i] = tapF;
            tapF += t.st[i].D * t.st[i].Q;
            if (i > 0 && t.st[i].H > TAIL_NT) return 0;   // one history load per thread
        }
        t.tapTotal = tapF;
        if (tapF > 2 * TAIL_NT) return 0;                 // two tap loads per thread
        lds = sizeof(float2) * (size_t)maxEl + sizeof(float) * (size_t)tapF;
        if (lds > TAIL_LDSMAX) return 0;
        return 1;
    }
    // the tail launch over kid 0's output s1 (n0 samples) into out, and the kids' state update
    int launch_tail(TailArgs& t, FirBlock** f, size_t lds, const void* s1, void* out, hipStream_t s) {
        t.in = reinterpret_cast<const float2*>(s1);
        t.out = reinterpret_cast<float2*>(out);
        if (t.K == TAIL_K_BIG && t.NT == TAIL_NT_BIG) hipLaunchKernelGGL((fir_tail_kernel<TAIL_K_BIG, TAIL_NT_BIG>), dim3(t.G), dim3(TAIL_NT_BIG), lds, s, t);
        else hipLaunchKernelGGL((fir_tail_kernel<TAIL_K, TAIL_NT>), dim3(t.G), dim3(TAIL_NT), lds, s, t);
        SDRGPU_HIP(hipGetLastError());
        for (int i = 0; i < t.S; i++) {   // FirBlock::run's state update
            f[i]->cur ^= 1;
            f[i]->offset = f[i]->offset + t.st[i].M * f[i]->D - t.st[i].n;
        }
        return t.st[t.S - 1].M;
    }
    int run_tail(const void* in, int count, void* out, hipStream_t s, int* nout) {
        TailArgs t;
        FirBlock* f[TAIL_MAXS];
        size_t lds = 0;
        const int n0 = kids.empty() ? 0 : kids[0]->out_count(count);
        const int ok = tail_plan(n0, t, f, lds);
        if (ok <= 0) return ok;
        SDRGPU_CHECK(scratch[0].ensure(sizeof(float2) * (size_t)std::max(n0, 1)));
        const int m0 = kids[0]->run(in, count, scratch[0].p, s);
        if (m0 < 0) return m0;
        if (m0 != n0) { set_error("chain: first stage produced %d samples, expected %d", m0, n0); return SDRGPU_ESTATE; }
        const int n = launch_tail(t, f, lds, scratch[0].p, out, s);
        if (n < 0) return n;
        *nout = n;
        return 1;
    }
    // kids[1..] on kid 0's output that another launch produced (vfo_stage1_finish): the tail launch
    // where it applies, else kid by kid
    int run_rest(const void* s1, int n0, void* out, hipStream_t s) {
        TailArgs t;
        FirBlock* f[TAIL_MAXS];
        size_t lds = 0;
        const int ok = tail_plan(n0, t, f, lds);
        if (ok < 0) return ok;
        if (ok) return launch_tail(t, f, lds, s1, out, s);
        return run_from(1, s1, n0, out, s);
    }
};

static std::unique_ptr<FirBlock> make_fir(int dev, int dtype, int ttype, const float* taps, int n, int decim, int* rc,
                                          bool xl = false, double w = 0.0, bool quad = false, float invDev = 1.0f,
                                          bool stereo = false) {
    auto f = std::make_unique<FirBlock>();
    f->xl = xl; f->quad = quad; f->invDev = invDev; f->stereo = stereo;
    *rc = f->setup(dev, dtype, ttype, taps, n, decim);
    if (*rc >= 0 && xl) *rc = f->nco.set_w(w);
    if (*rc >= 0) *rc = f->reset();
    return f;
}

// composition helpers for other translation units (loops.hip)
int chain_new(int dev, int in_dtype, int out_dtype, Block** out) {
    auto* c = new ChainBlock();
    c->device = dev; c->in_dtype = in_dtype; c->out_dtype = out_dtype;
    const int rc = c->init_stream();
    if (rc < 0) { delete c; return rc; }
    *out = c;
    return SDRGPU_OK;
}
int chain_append(Block* chain, Block* kid) {
    auto* c = dynamic_cast<ChainBlock*>(chain);
    if (!c || !kid) { delete kid; set_error("chain_append: bad argument"); return SDRGPU_EARG; }
    c->kids.emplace_back(kid);
    return SDRGPU_OK;
}
int chain_size(Block* chain) {
    auto* c = dynamic_cast<ChainBlock*>(chain);
    return c ? (int)c->kids.size() : -1;
}
Block* chain_kid(Block* chain, int i) {
    auto* c = dynamic_cast<ChainBlock*>(chain);
    return (c && i >= 0 && i < (int)c->kids.size()) ? c->kids[i].get() : nullptr;
}
Block* make_fir_block(int dev, int dtype, int ttype, const float* taps, int n, int decim, bool stereo, int* rc) {
    return make_fir(dev, dtype, ttype, taps, n, decim, rc, false, 0.0, false, 1.0f, stereo).release();
}
Block* make_quad_block(int dev, double deviationRad, int* rc) {
    auto* q = new QuadBlock();
    q->device = dev;
    q->in_dtype = SDRGPU_C64;
    q->out_dtype = SDRGPU_F32;
    q->invDev = (float)(1.0 / deviationRad);
    *rc = q->init_stream();
    for (int k = 0; k < 2 && *rc >= 0; k++) *rc = q->din[k].ensure(sizeof(float2));
    if (*rc >= 0) *rc = q->reset();
    return q;
}
Block* make_xlator_block(int dev, double offsetRad, int* rc) {
    auto* x = new XlatorBlock();
    x->device = dev;
    *rc = x->init_stream();
    if (*rc >= 0) *rc = x->nco.set_w(xlator_effective_omega(offsetRad));
    return x;
}

// PowerDecimator<T> (multirate/power_decimator.h): cascade of plan stages. With
// `xlFirst` the RxVFO's xlator is fused into the first (full-rate) stage.
static int build_power_decim(ChainBlock* c, int dev, int dtype, int ratio, bool xlFirst, double w) {
    if (ratio == 1) return SDRGPU_OK;
    int d[8], n[8];
    const float* t[8];
    int ns = decim_plan(ratio, d, n, t);
    if (ns < 0) return ns;
    for (int i = 0; i < ns; i++) {
        int rc;
        auto f = make_fir(dev, dtype, SDRGPU_F32, t[i], n[i], d[i], &rc, xlFirst && i == 0, w);
        if (rc < 0) return rc;
        c->kids.push_back(std::move(f));
    }
    return SDRGPU_OK;
}

// RationalResampler<T>::reconfigure (multirate/rational_resampler.h:121-167)
struct RationalPlan {
    int mode = 3, predec = 1, interp = 1, decim = 1;
    std::vector<float> taps;
};
static int plan_rational(double inSr, double outSr, RationalPlan& rp) {
    if (!(inSr > 0) || !(outSr > 0)) { set_error("rational resampler: bad samplerates"); return SDRGPU_EARG; }
    const int maxRatio = 8192;
    int predecPower = std::min<int>((int)std::floor(std::log2(inSr / outSr)), maxRatio);
    int predecRatio = std::min<int>(predecPower >= 0 && predecPower < 31 ? (1 << predecPower) : maxRatio, maxRatio);
    double intSr = inSr;
    bool useDecim = (inSr > outSr && predecPower > 0);
    if (useDecim) intSr = inSr / (double)predecRatio;
    rp.predec = useDecim ? predecRatio : 1;
    int IntSR = (int)std::round(intSr), OutSR = (int)std::round(outSr);
    int g = std::gcd(IntSR, OutSR);
    rp.interp = OutSR / g;
    rp.decim = IntSR / g;
    if (rp.interp == rp.decim) { rp.mode = useDecim ? 1 : 3; return SDRGPU_OK; }
    double tapSr = intSr * (double)rp.interp;
    double tapBw = std::min<double>(inSr, outSr) / 2.0;
    int n = taps_low_pass(tapBw, tapBw * 0.1, tapSr, 0, nullptr);
    if (n < 1) return n < 0 ? n : SDRGPU_EARG;
    rp.taps.resize(n);
    taps_low_pass(tapBw, tapBw * 0.1, tapSr, 0, rp.taps.data());
    for (auto& v : rp.taps) v *= (float)rp.interp;
    rp.mode = useDecim ? 0 : 2;
    return SDRGPU_OK;
}

static int build_rational(ChainBlock* c, int dev, int dtype, double inSr, double outSr, bool xlFirst, double w) {
    RationalPlan rp;
    SDRGPU_CHECK(plan_rational(inSr, outSr, rp));
    bool xlDone = false;
    if (rp.mode == 0 || rp.mode == 1) {
        SDRGPU_CHECK(build_power_decim(c, dev, dtype, rp.predec, xlFirst, w));
        xlDone = true;
    }
    if (xlFirst && !xlDone) {
        auto x = std::make_unique<XlatorBlock>();
        x->device = dev;
        SDRGPU_CHECK(x->init_stream());
        SDRGPU_CHECK(x->nco.set_w(w));
        c->kids.insert(c->kids.begin(), std::move(x));
    }
    if (rp.mode == 0 || rp.mode == 2) {
        auto p = std::make_unique<PolyBlock>();
        SDRGPU_CHECK(p->setup(dev, dtype, rp.interp, rp.decim, rp.taps.data(), (int)rp.taps.size()));
        c->kids.push_back(std::move(p));
    }
    return SDRGPU_OK;
}

// RxVFO (channel/rx_vfo.h:24-121)
struct VfoBlock : ChainBlock {
    double inSr = 0, outSr = 0, bw = 0, offset = 0;
    int build() {
        kids.clear();
        const double w = xlator_effective_omega(hz_to_rads(-offset, inSr));
        SDRGPU_CHECK(build_rational(this, device, SDRGPU_C64, inSr, outSr, true, w));
        if (bw != outSr) {
            double fw = bw / 2.0;
            int n = taps_low_pass(fw, fw * 0.1, outSr, 0, nullptr);
            if (n < 1) return n < 0 ? n : SDRGPU_EARG;
            std::vector<float> t(n);
            taps_low_pass(fw, fw * 0.1, outSr, 0, t.data());
            int rc;
            auto f = make_fir(device, SDRGPU_C64, SDRGPU_F32, t.data(), n, 1, &rc);
            if (rc < 0) return rc;
            kids.push_back(std::move(f));
        }
        return SDRGPU_OK;
    }
    // setOffset keeps the running NCO phase (frequency_xlator.h:25-29)
    int set_offset(double off) {
        offset = off;
        const double w = xlator_effective_omega(hz_to_rads(-offset, inSr));
        for (auto& k : kids) {
            if (auto* f = dynamic_cast<FirBlock*>(k.get()); f && f->xl) return f->nco.set_w(w);
            if (auto* x = dynamic_cast<XlatorBlock*>(k.get())) return x->nco.set_w(w);
        }
        return SDRGPU_OK;
    }
};

// ---- VFO stage 1 inside the spectrum launches (fir_rows.h VfoStage1) --------------------------
int vfo_stage1_prepare(sdrgpu_block* vfo, const void* in, int count, VfoStage1* st) {
    auto* c = vfo && vfo->impl ? dynamic_cast<ChainBlock*>(vfo->impl) : nullptr;
    if (!c || c->kids.empty() || count <= 0) return 0;
    auto* f = dynamic_cast<FirBlock*>(c->kids[0].get());
    if (!f || !f->rows_external(count)) return 0;
    SDRGPU_SET_DEVICE(f->device);
    const int M = f->out_count(count);
    SDRGPU_CHECK(c->scratch[0].ensure(sizeof(float2) * (size_t)M));
    f->histNextArg = f->hist[f->cur ^ 1].p;
    st->a = f->rows_args(in, count, c->scratch[0].p, M);
    st->M = M;
    st->count = count;
    st->out = c->scratch[0].p;
    return 1;
}
int vfo_tail_prepare(sdrgpu_block* vfo, const VfoStage1& st, void* out, TailArgs* t, size_t* lds) {
    auto* c = dynamic_cast<ChainBlock*>(vfo->impl);
    FirBlock* f[TAIL_MAXS];
    const int ok = c->tail_plan(st.M, *t, f, *lds);
    if (ok <= 0) return ok;
    t->in = reinterpret_cast<const float2*>(st.out);
    t->out = reinterpret_cast<float2*>(out);
    return 1;
}
// called once the launches that carry stage 1 and the tail are in: only then does any stage's state
// move on (a failed launch leaves the VFO as it was, as the header promises)
int vfo_tail_commit(sdrgpu_block* vfo, const VfoStage1& st, const TailArgs& t) {
    auto* c = dynamic_cast<ChainBlock*>(vfo->impl);
    dynamic_cast<FirBlock*>(c->kids[0].get())->rows_commit(st.count, st.M);
    for (int i = 0; i < t.S; i++) {   // FirBlock::run's state update (as launch_tail)
        auto* f = dynamic_cast<FirBlock*>(c->kids[i + 1].get());
        f->cur ^= 1;
        f->offset = f->offset + t.st[i].M * f->D - t.st[i].n;
    }
    return t.st[t.S - 1].M;
}
int vfo_stage1_finish(sdrgpu_block* vfo, const VfoStage1& st, void* out, hipStream_t s) {
    auto* c = dynamic_cast<ChainBlock*>(vfo->impl);
    auto* f = dynamic_cast<FirBlock*>(c->kids[0].get());
    f->rows_commit(st.count, st.M);
    return c->run_rest(st.out, st.M, out, s);
}

}  // namespace sdrgpu

using namespace sdrgpu;

// ================================================================== C ABI
static int wrap(sdrgpu_block** h, Block* b, int rc) {
    if (rc < 0) { delete b; return rc; }
    *h = new sdrgpu_block{b};
    return SDRGPU_OK;
}
#define NEED_HANDLE(h) do { if (!(h) || !(h)->impl) { set_error("null block handle"); return SDRGPU_EARG; } } while (0)

extern "C" int sdrgpu_xlator_create(sdrgpu_block** h, int device, double offsetRad) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* x = new XlatorBlock();
    x->device = device;
    int rc = x->init_stream();
    if (rc >= 0) rc = x->nco.set_w(xlator_effective_omega(offsetRad));
    return wrap(h, x, rc);
}
extern "C" int sdrgpu_xlator_set_offset(sdrgpu_block* h, double offsetRad) {
    NEED_HANDLE(h);
    auto* x = dynamic_cast<XlatorBlock*>(h->impl);
    if (!x) { set_error("not an xlator"); return SDRGPU_ESTATE; }
    return x->nco.set_w(xlator_effective_omega(offsetRad));
}

extern "C" int sdrgpu_fir_create(sdrgpu_block** h, int device, int dtype, int ttype, const float* taps, int ntaps, int decim) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    if ((dtype != SDRGPU_F32 && dtype != SDRGPU_C64) || (ttype != SDRGPU_F32 && ttype != SDRGPU_C64) ||
        (dtype == SDRGPU_F32 && ttype == SDRGPU_C64)) {
        set_error("fir_create: unsupported (dtype %d, ttype %d)", dtype, ttype);
        return SDRGPU_EARG;
    }
    int rc;
    auto f = make_fir(device, dtype, ttype, taps, ntaps, decim, &rc);
    return wrap(h, f.release(), rc);
}
extern "C" int sdrgpu_fir_set_taps(sdrgpu_block* h, const float* taps, int ntaps) {
    NEED_HANDLE(h);
    auto* f = dynamic_cast<FirBlock*>(h->impl);
    if (!f) { set_error("not a FIR"); return SDRGPU_ESTATE; }
    return f->set_taps(taps, ntaps);
}
extern "C" int sdrgpu_fir_set_decimation(sdrgpu_block* h, int decim) {
    NEED_HANDLE(h);
    auto* f = dynamic_cast<FirBlock*>(h->impl);
    if (!f) { set_error("not a FIR"); return SDRGPU_ESTATE; }
    return f->set_decimation(decim);
}

extern "C" int sdrgpu_quadrature_create(sdrgpu_block** h, int device, double deviationRad) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* q = new QuadBlock();
    q->device = device; q->in_dtype = SDRGPU_C64; q->out_dtype = SDRGPU_F32;
    q->invDev = (float)(1.0 / deviationRad);
    int rc = q->init_stream();
    for (int k = 0; k < 2 && rc >= 0; k++) rc = q->din[k].ensure(sizeof(float2));
    if (rc >= 0) rc = q->reset();
    return wrap(h, q, rc);
}
extern "C" int sdrgpu_quadrature_set_deviation(sdrgpu_block* h, double deviationRad) {
    NEED_HANDLE(h);
    if (auto* q = dynamic_cast<QuadBlock*>(h->impl)) { q->invDev = (float)(1.0 / deviationRad); return SDRGPU_OK; }
    if (auto* f = dynamic_cast<FirBlock*>(h->impl); f && f->quad) { f->invDev = (float)(1.0 / deviationRad); return SDRGPU_OK; }
    set_error("not a quadrature demodulator");
    return SDRGPU_ESTATE;
}

extern "C" int sdrgpu_power_decimator_create(sdrgpu_block** h, int device, int dtype, int ratio) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    if (ratio < 1 || (ratio & (ratio - 1)) || ratio > (8192)) {
        set_error("power_decimator: ratio %d must be a power of two <= 8192", ratio);   // checkRatio
        return SDRGPU_EARG;
    }
    auto* c = new ChainBlock();
    c->device = device; c->in_dtype = c->out_dtype = dtype;
    int rc = c->init_stream();
    if (rc >= 0) rc = build_power_decim(c, device, dtype, ratio, false, 0.0);
    return wrap(h, c, rc);
}

extern "C" int sdrgpu_polyphase_resampler_create(sdrgpu_block** h, int device, int dtype, int interp, int decim,
                                                 const float* taps, int ntaps) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* p = new PolyBlock();
    return wrap(h, p, p->setup(device, dtype, interp, decim, taps, ntaps));
}

// FrequencyXlator(w) -> RationalResampler<complex_t>(inSr -> outSr) with the xlator fused into the
// first decimation stage (BroadcastFM's RDS branch, broadcast_fm.h:164-171)
namespace sdrgpu {
Block* make_xlate_resample_block(int dev, double inSr, double outSr, double w, int* rc) {
    auto* c = new ChainBlock();
    c->device = dev; c->in_dtype = c->out_dtype = SDRGPU_C64;
    *rc = c->init_stream();
    if (*rc >= 0) *rc = build_rational(c, dev, SDRGPU_C64, inSr, outSr, true, w);
    return c;
}
}  // namespace sdrgpu

extern "C" int sdrgpu_rational_resampler_create(sdrgpu_block** h, int device, int dtype, double inSr, double outSr) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* c = new ChainBlock();
    c->device = device; c->in_dtype = c->out_dtype = dtype;
    int rc = c->init_stream();
    if (rc >= 0) rc = build_rational(c, device, dtype, inSr, outSr, false, 0.0);
    return wrap(h, c, rc);
}

extern "C" int sdrgpu_rxvfo_create(sdrgpu_block** h, int device, double inSr, double outSr, double bw, double offset) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* v = new VfoBlock();
    v->device = device; v->in_dtype = v->out_dtype = SDRGPU_C64;
    v->inSr = inSr; v->outSr = outSr; v->bw = bw; v->offset = offset;
    int rc = v->init_stream();
    if (rc >= 0) rc = v->build();
    return wrap(h, v, rc);
}
extern "C" int sdrgpu_rxvfo_set_offset(sdrgpu_block* h, double offset) {
    NEED_HANDLE(h);
    auto* v = dynamic_cast<VfoBlock*>(h->impl);
    if (!v) { set_error("not an RxVFO"); return SDRGPU_ESTATE; }
    return v->set_offset(offset);
}

extern "C" int sdrgpu_ddc_fm_create(sdrgpu_block** h, int device, double offsetRad, const float* taps, int ntaps, int decim,
                                    double deviationRad) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    int rc;
    auto f = make_fir(device, SDRGPU_C64, SDRGPU_F32, taps, ntaps, decim, &rc, true, xlator_effective_omega(offsetRad),
                      true, (float)(1.0 / deviationRad));
    return wrap(h, f.release(), rc);
}

// Fused DDC without the demodulator: FrequencyXlator(offsetRad) -> DecimatingFIR<complex_t,float>
// (frequency_xlator.h:43-50, decimating_fir.h:45-68), complex_t out. The same kernels as the fused
// DDC+FM block with the quadrature epilogue off (RxVFO's first stage has this shape too).
extern "C" int sdrgpu_ddc_create(sdrgpu_block** h, int device, double offsetRad, const float* taps, int ntaps, int decim) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    int rc;
    auto f = make_fir(device, SDRGPU_C64, SDRGPU_F32, taps, ntaps, decim, &rc, true, xlator_effective_omega(offsetRad));
    return wrap(h, f.release(), rc);
}

// FM<float> (demod/fm.h:25-133): quadrature(bw/2) -> optional LPF/HPF/BPF
extern "C" int sdrgpu_fm_create(sdrgpu_block** h, int device, double samplerate, double bandwidth, int lowPass, int highPass) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* c = new ChainBlock();
    c->device = device; c->in_dtype = SDRGPU_C64; c->out_dtype = SDRGPU_F32;
    int rc = c->init_stream();
    sdrgpu_block* qh = nullptr;
    if (rc >= 0) rc = sdrgpu_quadrature_create(&qh, device, hz_to_rads(bandwidth / 2.0, samplerate));
    if (rc >= 0) { c->kids.emplace_back(qh->impl); delete qh; }
    if (rc >= 0 && (lowPass || highPass)) {
        int n;
        std::vector<float> t;
        if (lowPass && highPass) {
            n = taps_band_pass_f(300.0, bandwidth / 2.0, 100.0, samplerate, 0, nullptr);
            if (n > 0) { t.resize(n); taps_band_pass_f(300.0, bandwidth / 2.0, 100.0, samplerate, 0, t.data()); }
        } else if (highPass) {
            n = taps_high_pass(300.0, 100.0, samplerate, 0, nullptr);
            if (n > 0) { t.resize(n); taps_high_pass(300.0, 100.0, samplerate, 0, t.data()); }
        } else {
            n = taps_low_pass(bandwidth / 2.0, (bandwidth / 2.0) * 0.1, samplerate, 0, nullptr);
            if (n > 0) { t.resize(n); taps_low_pass(bandwidth / 2.0, (bandwidth / 2.0) * 0.1, samplerate, 0, t.data()); }
        }
        rc = n < 1 ? (n < 0 ? n : SDRGPU_EARG) : SDRGPU_OK;
        if (rc >= 0) {
            auto f = make_fir(device, SDRGPU_F32, SDRGPU_F32, t.data(), n, 1, &rc);
            if (rc >= 0) c->kids.push_back(std::move(f));
        }
    }
    return wrap(h, c, rc);
}

// [quadrature, stereo FIR at D = 1] in one launch: wfm_short_kernel for calls up to kShortMax
// samples, wfm_big_kernel above
struct WfmBlock : ChainBlock {
    static constexpr int kShortMax = 1 << 15;
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (kids.size() != 2) return ChainBlock::run(in, count, out, s);
        auto* qb = static_cast<QuadBlock*>(kids[0].get());
        auto* fb = static_cast<FirBlock*>(kids[1].get());
        if (count <= 0 || fb->D != 1 || fb->Q % WFM_BK != 0 || fb->Q > 256) return ChainBlock::run(in, count, out, s);
        SDRGPU_SET_DEVICE(device);
        if (count > kShortMax) {
            const int blocks = (int)(((long long)count + WFM_BCH - 1) / WFM_BCH);
            const size_t lds = sizeof(float) * ((size_t)WFM_BK * (WFM_BNT + fb->Q / WFM_BK + 2) + fb->Q);
            hipLaunchKernelGGL(wfm_big_kernel, dim3(blocks + 1), dim3(WFM_BNT), lds, s, (const float2*)in, count,
                               qb->din[qb->cur].as<float2>(), qb->din[qb->cur ^ 1].as<float2>(), fb->hist[fb->cur].as<float>(),
                               fb->hist[fb->cur ^ 1].as<float>(), fb->taps.as<float>(), fb->Q, fb->ntaps - 1, qb->invDev,
                               (float2*)out);
            SDRGPU_HIP(hipGetLastError());
            qb->cur ^= 1;
            fb->cur ^= 1;
            return count;
        }
        const int blocks = (count + WFM_TM - 1) / WFM_TM;
        const size_t lds = sizeof(float) * (size_t)(WFM_TM + fb->Q);
        hipLaunchKernelGGL(wfm_short_kernel, dim3(blocks + 1), dim3(WFM_TM), lds, s, (const float2*)in, count,
                           qb->din[qb->cur].as<float2>(), qb->din[qb->cur ^ 1].as<float2>(), fb->hist[fb->cur].as<float>(),
                           fb->hist[fb->cur ^ 1].as<float>(), fb->taps.as<float>(), fb->Q, fb->ntaps - 1, qb->invDev,
                           (float2*)out);
        SDRGPU_HIP(hipGetLastError());
        qb->cur ^= 1;
        fb->cur ^= 1;
        return count;
    }
};

// BroadcastFM, stereo == false (demod/broadcast_fm.h:144-215): quadrature(dev) ->
// 228-tap (at 240 kS/s) audio LPF lowPass(15 kHz, 4 kHz) -> LRToStereo(l = r)
extern "C" int sdrgpu_wfm_create(sdrgpu_block** h, int device, double deviation, double samplerate, int lowPass) {
    if (!h) { set_error("null out-handle"); return SDRGPU_EARG; }
    auto* c = new WfmBlock();
    c->device = device; c->in_dtype = SDRGPU_C64; c->out_dtype = SDRGPU_C64;
    int rc = c->init_stream();
    sdrgpu_block* qh = nullptr;
    if (rc >= 0) rc = sdrgpu_quadrature_create(&qh, device, hz_to_rads(deviation, samplerate));
    if (rc >= 0) { c->kids.emplace_back(qh->impl); delete qh; }
    if (rc >= 0) {
        int n = taps_low_pass(15000.0, 4000.0, samplerate, 0, nullptr);
        std::vector<float> t(std::max(n, 1), 1.0f);
        if (lowPass && n > 0) taps_low_pass(15000.0, 4000.0, samplerate, 0, t.data());
        else n = 1;   // unfiltered MPX: identity tap, same stereo interleave
        auto f = make_fir(device, SDRGPU_F32, SDRGPU_F32, t.data(), n, 1, &rc, false, 0.0, false, 1.0f, true);
        if (rc >= 0) c->kids.push_back(std::move(f));
    }
    return wrap(h, c, rc);
}

extern "C" int sdrgpu_block_out_count(sdrgpu_block* h, int count) {
    NEED_HANDLE(h);
    return h->impl->out_count(count);
}

extern "C" int sdrgpu_block_process_dev(sdrgpu_block* h, const void* in, int count, void* out, void* stream) {
    NEED_HANDLE(h);
    if (count < 0 || (count > 0 && (!in || !out))) { set_error("process: bad buffers"); return SDRGPU_EARG; }
    Block* b = h->impl;
    const hipStream_t s = stream ? (hipStream_t)stream : b->own;
    SDRGPU_SET_DEVICE(b->device);
    SDRGPU_CHECK(b->order.follow(s));
    OrderScope od(b->order, s);
    return b->run(in, count, out, s);
}

int sdrgpu::block_run_owned(sdrgpu_block* h, const void* in, int count, void* out, hipStream_t s) {
    NEED_HANDLE(h);
    if (count < 0 || (count > 0 && (!in || !out))) { set_error("process: bad buffers"); return SDRGPU_EARG; }
    return h->impl->run(in, count, out, s);
}

extern "C" int sdrgpu_block_process(sdrgpu_block* h, const void* in, int count, void* out) {
    NEED_HANDLE(h);
    if (count < 0 || (count > 0 && (!in || !out))) { set_error("process: bad buffers"); return SDRGPU_EARG; }
    Block* b = h->impl;
    SDRGPU_SET_DEVICE(b->device);
    const size_t inB = (size_t)std::max(count, 1) * esize(b->in_dtype);
    const int mExp = b->out_count(count);
    const size_t outB = (size_t)std::max(mExp, 1) * esize(b->out_dtype);
    SDRGPU_CHECK(b->pin_in.ensure(inB));
    SDRGPU_CHECK(b->pin_out.ensure(outB));
    SDRGPU_CHECK(b->dev_in.ensure(inB));
    SDRGPU_CHECK(b->dev_out.ensure(outB));
    // buffers registered with sdrgpu_host_register are DMA'd directly; others go through the
    // handle's pinned staging buffers
    const bool inPinned = host_pinned(in, (size_t)count * esize(b->in_dtype));
    const bool outPinned = host_pinned(out, (size_t)mExp * esize(b->out_dtype));
    if (count > 0) {
        if (!inPinned) std::memcpy(b->pin_in.p, in, (size_t)count * esize(b->in_dtype));
    }
    SDRGPU_CHECK(b->order.follow(b->own));
    OrderScope od(b->order, b->own);
    if (count > 0)
        SDRGPU_HIP(hipMemcpyAsync(b->dev_in.p, inPinned ? in : b->pin_in.p, (size_t)count * esize(b->in_dtype),
                                  hipMemcpyHostToDevice, b->own));
    int m = b->run(b->dev_in.p, count, b->dev_out.p, b->own);
    if (m < 0) return m;
    void* dst = (outPinned && m <= mExp) ? out : b->pin_out.p;
    if (m > 0) SDRGPU_HIP(hipMemcpyAsync(dst, b->dev_out.p, (size_t)m * esize(b->out_dtype), hipMemcpyDeviceToHost, b->own));
    SDRGPU_HIP(hipStreamSynchronize(b->own));
    if (m > 0 && dst != out) std::memcpy(out, b->pin_out.p, (size_t)m * esize(b->out_dtype));
    return m;
}

extern "C" int sdrgpu_block_reset(sdrgpu_block* h) {
    NEED_HANDLE(h);
    int rc = h->impl->reset();
    if (rc >= 0) SDRGPU_HIP(hipDeviceSynchronize());
    return rc;
}

extern "C" int sdrgpu_block_destroy(sdrgpu_block* h) {
    if (!h) return SDRGPU_OK;
    if (h->impl) {
        (void)hipSetDevice(h->impl->device);
        (void)hipDeviceSynchronize();
        delete h->impl;
    }
    delete h;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_convert_dev(int device, int kind, const void* in, long long n, float* out, void* stream) {
    if (kind < SDRGPU_CONV_U8 || kind > SDRGPU_CONV_F32 || n < 0 || (n > 0 && (!in || !out))) {
        set_error("convert: bad argument");
        return SDRGPU_EARG;
    }
    SDRGPU_SET_DEVICE(device);
    if (n == 0) return 0;
    hipLaunchKernelGGL(convert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, kind, in, n, out);
    SDRGPU_HIP(hipGetLastError());
    return (int)std::min<long long>(n, 0x7fffffff);
}

extern "C" int sdrgpu_convert_mono_dev(int device, int kind, const void* in, long long n, void* out, void* stream) {
    if (kind < SDRGPU_CONV_U8 || kind > SDRGPU_CONV_F32 || n < 0 || (n > 0 && (!in || !out))) {
        set_error("convert_mono: bad argument");
        return SDRGPU_EARG;
    }
    SDRGPU_SET_DEVICE(device);
    if (n == 0) return 0;
    hipLaunchKernelGGL(convert_mono_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, kind, in, n,
                       (float2*)out);
    SDRGPU_HIP(hipGetLastError());
    return (int)std::min<long long>(n, 0x7fffffff);
}

extern "C" int sdrgpu_convert_mono(int device, int kind, const void* in, long long n, void* out) {
    static const int isz[] = {1, 2, 3, 4, 8, 1, 4};
    if (kind < SDRGPU_CONV_U8 || kind > SDRGPU_CONV_F32 || n < 0) { set_error("convert_mono: bad argument"); return SDRGPU_EARG; }
    if (n == 0) return 0;
    SDRGPU_SET_DEVICE(device);
    DevBuf din, dout;
    SDRGPU_CHECK(din.ensure((size_t)n * isz[kind]));
    SDRGPU_CHECK(dout.ensure((size_t)n * sizeof(float2)));
    SDRGPU_HIP(hipMemcpy(din.p, in, (size_t)n * isz[kind], hipMemcpyHostToDevice));
    SDRGPU_CHECK(sdrgpu_convert_mono_dev(device, kind, din.p, n, dout.p, nullptr));
    SDRGPU_HIP(hipMemcpy(out, dout.p, (size_t)n * sizeof(float2), hipMemcpyDeviceToHost));
    return (int)std::min<long long>(n, 0x7fffffff);
}

extern "C" int sdrgpu_convert(int device, int kind, const void* in, long long n, float* out) {
    static const int isz[] = {1, 2, 3, 4, 8, 1, 4};
    if (kind < SDRGPU_CONV_U8 || kind > SDRGPU_CONV_F32 || n < 0) { set_error("convert: bad argument"); return SDRGPU_EARG; }
    if (n == 0) return 0;
    SDRGPU_SET_DEVICE(device);
    void* din = nullptr;
    float* dout = nullptr;
    SDRGPU_HIP(hipMalloc(&din, (size_t)n * isz[kind]));
    if (hipMalloc((void**)&dout, (size_t)n * sizeof(float)) != hipSuccess) {
        (void)hipFree(din);
        set_error("convert: hipMalloc failed");
        return SDRGPU_ENOMEM;
    }
    int rc = SDRGPU_OK;
    if (hipMemcpy(din, in, (size_t)n * isz[kind], hipMemcpyHostToDevice) != hipSuccess) rc = SDRGPU_EHIP;
    if (rc >= 0) rc = sdrgpu_convert_dev(device, kind, din, n, dout, nullptr);
    if (rc >= 0 && hipMemcpy(out, dout, (size_t)n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) rc = SDRGPU_EHIP;
    (void)hipFree(din);
    (void)hipFree(dout);
    if (rc == SDRGPU_EHIP) set_error("convert: hipMemcpy failed");
    return rc < 0 ? rc : (int)std::min<long long>(n, 0x7fffffff);
}
