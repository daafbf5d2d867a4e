// Channel-chain device code shared by blocks.hip (the FIR / VFO kernels) and fft.hip (the spectrum
// launches that also run a VFO's first stage over the same batch, sdrgpu_fft_execute_vfo_dev):
// complex helpers, the two-level NCO, the FIR launch arguments and edge fetches, the history-carry
// workgroup, and the row-streaming decimating FIR segment.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <utility>

namespace sdrgpu {

// The contraction is spelled out: left to -ffp-contract=fast, a*b - c*d becomes fma(a, b, -cd) in one
// kernel and fma(-c, d, ab) in another (the SLP vectoriser's packed form picks the other product),
// and the spectrum launches' VFO stage 1 then differed from fir_rows_kernel's in the last bit
// (r4b: test_spectrum_vfo_fused). With explicit fmaf there is one rounding sequence everywhere.
__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}

// packed-fp32 pairs (v_pk_fma_f32 and friends: one instruction for both components, each the same IEEE
// operation as its scalar form)
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v to_v(float2 a) { return f2v{a.x, a.y}; }
__device__ __forceinline__ float2 to_f2(f2v a) { return make_float2(a.x, a.y); }

// fn(integral_constant<int, I>) for I in [A, B): a compile-time loop (a long `#pragma unroll` loop can
// stay rolled past the unroller's threshold, and a run-time ring index sends the ring to scratch)
template <int A, class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& fn, std::integer_sequence<int, I...>) {
    (fn(std::integral_constant<int, A + I>{}), ...);
}
template <int A, int B, class F>
__device__ __forceinline__ void static_for(F&& fn) {
    static_for_impl<A>(fn, std::make_integer_sequence<int, B - A>{});
}
// x * (ph0 * step): the xlator's per-slot product, each complex result pinned to plain VGPRs.
// Left to itself the SLP vectoriser packs a run of these into v_pk_fma pairs that compute both
// signs of every term (twice the live registers per slot: the PF-slot kernels spilled on it).
// The arithmetic is the same two cmulf's.
__device__ __forceinline__ float2 xlate_slot(float2 x, float2 ph0, float2 step) {
    float2 ph = cmulf(ph0, step);
    asm volatile("" : "+v"(ph.x), "+v"(ph.y));
    float2 r = cmulf(x, ph);
    asm volatile("" : "+v"(r.x), "+v"(r.y));
    return r;
}

// Two-level NCO table: phasor(i) = Phi[i >> 12] * Plo[i & 4095], with
// Plo[k] = exp(i w k) (fixed per configuration, fp64 -> float on the host) and
// Phi[j] = exp(i (theta0 + w 4096 j)) (per call, fp64 on the device). Two cached
// loads + one complex multiply per sample instead of an fp64 argument reduction
// and a sincos; error <= ~2 ulp of the phasor, no drift (theta0 is carried in
// double-double on the host).
constexpr int NCO_LO_BITS = 12;
constexpr int NCO_LO = 1 << NCO_LO_BITS;
__device__ __forceinline__ float2 nco_tab(const float2* __restrict__ phi, const float2* __restrict__ plo, long long i) {
    return cmulf(phi[i >> NCO_LO_BITS], plo[i & (NCO_LO - 1)]);
}
__device__ __forceinline__ float2 nco_phi(double theta0, double w, long long j) {
    const double TWO_PI = 6.283185307179586476925286766559;
    double a = fma(w * (double)NCO_LO, (double)j, theta0);
    a = fma(-rint(a / TWO_PI), TWO_PI, a);
    double sn, cs;
    sincos(a, &sn, &cs);
    return make_float2((float)cs, (float)sn);
}

template <typename T> __device__ __forceinline__ T zero_of();
template <> __device__ __forceinline__ float zero_of<float>() { return 0.0f; }
template <> __device__ __forceinline__ float2 zero_of<float2>() { return make_float2(0.f, 0.f); }

// atan2 of the FM quadrature (demod/quadrature.h:41-56: arg(y * conj(y[-1])) = complex_t::phase(), i.e.
// atan2f), for every kernel that forms it: OCML's atan2f, the device libm's correctly-signed,
// ~1-ulp counterpart of the reference's glibc atan2f (tests/test_ref_pinned.py pins it against the
// reference-code fixture). Round 3 measured a minimax polynomial with v_rcp_f32 instead (|error| <=
// 1.4 ulp(pi) absolute, far more ulps than that on small phase steps): C3 0.862 -> 0.850 ms, -1.3%
// (profiles/r3/c3_atan/). Not worth the parity concession: it stays an A/B build only
// (-DSDRGPU_POLY_ATAN2).
__device__ __forceinline__ float quad_atan2f(float y, float x) {
#ifndef SDRGPU_POLY_ATAN2
    return atan2f(y, x);
#else
    const float ax = fabsf(x), ay = fabsf(y);
    const bool swp = ay > ax;
    const float mn = swp ? ax : ay, mx = swp ? ay : ax;
    const float a = mn * __builtin_amdgcn_rcpf(mx == 0.0f ? 1.0f : mx);
    const float s = a * a;
    float p = 0.0028662257f;
    p = fmaf(p, s, -0.0161657367f);
    p = fmaf(p, s, 0.0429096138f);
    p = fmaf(p, s, -0.0752896400f);
    p = fmaf(p, s, 0.1065626393f);
    p = fmaf(p, s, -0.1420889944f);
    p = fmaf(p, s, 0.1999355085f);
    p = fmaf(p, s, -0.3333314528f);
    float r = fmaf(a * s, p, a);
    r = swp ? 1.57079632679489662f - r : r;
    r = signbit(x) ? 3.14159265358979324f - r : r;
    return copysignf(r, y);
#endif
}

// acc += x * h for the four (data, tap) type pairs of filter/fir.h:69-75
__device__ __forceinline__ void mac(float& acc, float x, float h) { acc = fmaf(x, h, acc); }
__device__ __forceinline__ void mac(float2& acc, float2 x, float h) { acc.x = fmaf(x.x, h, acc.x); acc.y = fmaf(x.y, h, acc.y); }
__device__ __forceinline__ void mac(float2& acc, float2 x, float2 h) {
    acc.x = fmaf(x.x, h.x, acc.x); acc.x = fmaf(-x.y, h.y, acc.x);
    acc.y = fmaf(x.x, h.y, acc.y); acc.y = fmaf(x.y, h.x, acc.y);
}

struct FirArgs {
    const void* hist;
    const void* in;
    const void* taps;   // [D][Q] (phase-major, zero-padded) elements of TT
    void* out;
    const float2* din;  // QUAD: y[-1] (carried)
    float2* dinNext;    // QUAD: y[M-1]
    const float2* phi;  // XL: per-call coarse phasors (only the separate history kernel reads them)
    const float2* plo;  // XL: fine phasors
    double ncoTheta0, ncoW;   // XL: the coarse phasor of index j is nco_phi(ncoTheta0, ncoW, j)
    int ntaps, H, count, D, Q, offset0, M, TMS, RSK, RSP;
    int dshift;         // log2(D) when D is a power of two, else -1
    int ntiles;         // tiles of TMS outputs (persistent grid walks them)
    int tapsLdsOff;     // TL: byte offset of the [D][Q] taps in dynamic LDS
    int simple;         // D | NT and K | NT/D: constant LDS stride per load slot
    const float2* nstep;  // XL: e^{i w u NT}, u < NCO_PF, for this launch's NT
    float invDev;
    int gzs;            // MFMA phase-split: gz entries per phase
    void* histNext;     // non-null: the launch has one extra, last workgroup that writes the next
                        // call's history (the last H samples of hist | in, translated) there
};

// XL phasor of input index i inside a FIR kernel: the coarse factor computed in place (the same
// fp64 expression as nco_hi_kernel's table, so the same bits) instead of read from a per-call
// table, which would need a launch of its own before every call. The row kernel (VFO stage 1:
// the C5 chain's only translating FIR) does this; the MFMA / LDS tile kernels keep the table:
// there every wave forms its own phasors and the fp64 sincos serialises with the matrix work
// (C3: +1.3% kernel time measured).
__device__ __forceinline__ float2 nco_inline(const FirArgs& a, long long i) {
    return cmulf(nco_phi(a.ncoTheta0, a.ncoW, i >> NCO_LO_BITS), a.plo[i & (NCO_LO - 1)]);
}
template <bool TAB = true>   // TAB: read the per-call table; else form the coarse phasor in place
__device__ __forceinline__ float2 nco_at(const FirArgs& a, long long i) {
    if constexpr (TAB) return nco_tab(a.phi, a.plo, i);
    else return nco_inline(a, i);
}

template <typename DT, bool XL, bool TAB = true>
__device__ __forceinline__ DT fir_fetch(const FirArgs& a, long long b) {
    const DT* hist = reinterpret_cast<const DT*>(a.hist);
    const DT* in = reinterpret_cast<const DT*>(a.in);
    // branch-free: one load from an address that exists (clamped), then a select, so the callers'
    // unrolled row loops keep all their edge fetches in flight instead of issuing one
    // branch-guarded load (and its NCO table loads) at a time. An edge segment of the VFO's
    // stage-1 FIR at the reference block size took 19 us that way: the whole launch's time.
    const long long i = b - a.H;
    const bool inH = b >= 0 && b < a.H, inI = i >= 0 && i < a.count;
    const DT* src = inH ? hist + b : (inI ? in + i : (a.count > 0 ? in : hist));
    DT x = *src;
    if constexpr (XL) {
        const float2 r = nco_at<TAB>(a, inI ? i : 0);
        if (inI) x = cmulf(x, r);
    }
    return (inH || inI) ? x : zero_of<DT>();
}

// The history carry of FIR::process (fir.h:80: memmove of the last ntaps - 1 inputs) as the
// launch's extra workgroup, so a call needs no separate history kernel: next[k] = [hist | in]
// [count + k], k < H (the xlator applied to `in` samples, as fir_fetch does).
template <typename DT, bool XL, bool TAB = true>
__device__ __forceinline__ void fir_hist_copy(const FirArgs& a) {
    const DT* hist = reinterpret_cast<const DT*>(a.hist);
    const DT* in = reinterpret_cast<const DT*>(a.in);
    DT* next = reinterpret_cast<DT*>(a.histNext);
    for (int k = threadIdx.x; k < a.H; k += blockDim.x) {
        const long long b = (long long)a.count + k;
        DT v;
        if (b < a.H) {
            v = hist[b];
        } else {
            v = in[b - a.H];
            if constexpr (XL) v = cmulf(v, nco_at<TAB>(a, b - a.H));
        }
        next[k] = v;
    }
}
template <typename DT, bool XL, bool TAB = true>
__device__ __forceinline__ bool fir_hist_block(const FirArgs& a) {
    if (a.histNext == nullptr || blockIdx.x != gridDim.x - 1) return false;
    fir_hist_copy<DT, XL, TAB>(a);
    return true;
}

// Row-streaming decimating FIR, no LDS (D = 32: VFO stage 1, 143 taps -> QP = 5 taps per phase;
// D = 8: C3, 256 taps -> QP = 32, with the FM quadrature fused on the outputs). Lane p of each
// D-lane group owns phase p. A group walks a segment of RS outputs row by row: row r is the D
// samples buf[b0 + D r .. + D - 1], one coalesced 8D-byte load per group. The lane keeps the
// QP - 1 open partial sums of its phase in registers (output o takes row o + q with tap
// h[D q + p]), so every row costs QP complex x real FMAs and closes one per-phase partial.
// Every D closed outputs the D per-phase partials are summed across the group by a log2(D)-step
// xor transpose-reduce (ds_swizzle), which leaves output D blk + p in lane p. Each sample is
// read once (plus QP - 1 halo rows per segment). With QUAD a segment starts one output early
// (that output only feeds y[m - 1] of the next) and stores RS - 1 outputs.
// D = 32 (no quadrature) runs 32-output segments at every call size (round 4: the spectrum launches
// compute the stage in one-load-round workgroups of such segments beside the column tiles, and the
// separate kernel must cut the same segments to give the same bits; round 1-3 used 128 above 2^19
// outputs). Earlier: segments of 64 or 256 outputs measured the same as 128; forcing 4 waves per SIMD
// (128 VGPRs) spills and ran 10% slower; loading batch t + 1 while batch t computes (2 waves per
// SIMD) was no faster. D = 8 (C3) measured equal to fir_mfma_kernel (0.84 vs 0.85 ms), so it
// runs only on request (SDRGPU_FIR_ROWS=2).
constexpr int ROWS_STEP = 512;  // e^{i w D u} table length (>= RS + QP - 1)
template <int D> constexpr int rows_rs() { return D == 32 ? 128 : 256; }
// One D-lane group's segment `seg` (lane = the thread's lane in its wave). BT0: rows per load batch
// (default: D = 32 keeps 64 rows, 32 KB per wave, in flight at 2 waves per SIMD, 0.6% faster than
// 32 rows at 3 -- the kernel waits on its row loads; QP = 32 fits 16). The batch size does not
// change any output: every output's partials are summed in row order either way, so a launch that
// runs the segments with a smaller register budget (the spectrum launches of fft.hip) produces the
// same bits.
// LOWREG: issue the cross-lane reduce steps one pair at a time (sched_barrier), so a 128-VGPR launch
// does not spill the swizzle temporaries the scheduler would otherwise hoist (same instructions, same
// bits).
template <int D, int QP, bool XL, bool QUAD, int RS = rows_rs<D>(), int BT0 = (QP > 16 ? 16 : (D == 32 ? 64 : 32)),
          bool LOWREG = false>
__device__ __forceinline__ void fir_rows_segment(const FirArgs& a, long long seg, int lane) {
    constexpr int QOFF = QUAD ? 1 : 0;
    // short segments (small calls) take one batch of RS rows
    constexpr int BT = BT0 < RS ? BT0 : RS;
    static_assert(RS % BT == 0 && BT % D == 0, "rows kernel: segment = whole batches of D rows");
    const int p = lane & (D - 1);
    const long long mseg = seg * (RS - QOFF) - QOFF;   // output of local index 0
    if (mseg + QOFF >= a.M) return;   // (the cross-lane steps stay inside one D-lane group)
    const float* __restrict__ taps = reinterpret_cast<const float*>(a.taps);   // [p][Q]
    float h[QP];
#pragma unroll
    for (int q = 0; q < QP; q++) h[q] = q < a.Q ? taps[p * a.Q + q] : 0.0f;
    constexpr int NR = RS + QP - 1;
    const long long b0 = (long long)a.offset0 + mseg * D;
    const bool interior = (b0 >= a.H) && (b0 + (long long)D * NR <= (long long)a.H + a.count);
    const float2* __restrict__ src = reinterpret_cast<const float2*>(a.in) + (b0 - a.H) + p;
    float2 ph0 = make_float2(1.f, 0.f);
    // the row-step table through the constant address space: scalar (SMEM) loads
    const __attribute__((address_space(4))) float* nstep = (const __attribute__((address_space(4))) float*)a.nstep;
    // phasor of the segment's first input sample (index b0 - H + p of `in`; negative inside the
    // history, where the formula still holds: coarse index floor(i / 4096), fine index i mod 4096)
    if constexpr (XL) ph0 = nco_inline(a, b0 - a.H + p);
    float2* __restrict__ out2 = reinterpret_cast<float2*>(a.out);
    float* __restrict__ outf = reinterpret_cast<float*>(a.out);
    // interior segments load unconditionally (BT row loads in flight); the few segments touching
    // the history or the end of the call fetch element-wise
    auto body = [&](auto fast) {
        constexpr bool F = decltype(fast)::value;
        auto row = [&](int r) -> float2 {   // raw row sample (history samples are stored translated)
            if constexpr (F) return src[D * r];
            else return fir_fetch<float2, false, false>(a, b0 + (long long)D * r + p);
        };
        // fused xlator: e^{i w (i0 + D r)} = ph0 e^{i w D r} on `in` samples. Edge segments (the
        // history at the front, the call's end) use the same phasors: forming each one in fp64
        // (nco_inline per sample) made the two edge segments of a reference-size block take
        // ~3x as long as the rest of the launch (r3 per-call trace)
        auto xlate = [&](float2 x, int r) -> float2 {
            if constexpr (XL) {
                const float2 y = cmulf(x, cmulf(ph0, make_float2(nstep[2 * r], nstep[2 * r + 1])));
                if constexpr (F) x = y;
                else x = (b0 + (long long)D * r + p >= a.H) ? y : x;
            }
            return x;
        };
        float2 P[QP];   // P[k], k >= 1: the open partial of output (r - k) before row r
#pragma unroll
        for (int k = 0; k < QP; k++) P[k] = make_float2(0.f, 0.f);
        auto step = [&](float2 x) -> float2 {
            float2 done = P[QP - 1];
            mac(done, x, h[QP - 1]);
#pragma unroll
            for (int k = QP - 1; k >= 2; k--) {
                P[k] = P[k - 1];
                mac(P[k], x, h[k - 1]);
            }
            P[1] = make_float2(x.x * h[0], x.y * h[0]);
            return done;
        };
        // one-batch segments (small calls) issue the prologue rows with the batch: one round
        // of row loads per segment instead of two dependent ones
        constexpr bool ONE = RS == BT;
        if constexpr (!ONE) {
            for (int r0 = 0; r0 < QP - 1; r0 += 8) {   // prologue: rows 0 .. QP - 2 close no output
                float2 pro[8];
#pragma unroll
                for (int r = 0; r < 8; r++) pro[r] = (r0 + r < QP - 1) ? row(r0 + r) : make_float2(0.f, 0.f);
#pragma unroll
                for (int r = 0; r < 8; r++)
                    if (r0 + r < QP - 1) (void)step(xlate(pro[r], r0 + r));
            }
        }
        float2 ylast = make_float2(0.f, 0.f);   // QUAD: the group's previous output
#pragma unroll 1
        for (int bt = 0; bt < RS / BT; bt++) {
            float2 v[BT];
            if constexpr (ONE) {
                float2 pro[QP > 1 ? QP - 1 : 1];
#pragma unroll
                for (int r = 0; r < QP - 1; r++) pro[r] = row(r);
#pragma unroll
                for (int i = 0; i < BT; i++) v[i] = row(QP - 1 + i);
#pragma unroll
                for (int r = 0; r < QP - 1; r++) (void)step(xlate(pro[r], r));
            } else {
#pragma unroll
                for (int i = 0; i < BT; i++) v[i] = row(QP - 1 + BT * bt + i);   // BT row loads in flight
            }
#pragma unroll
            for (int i = 0; i < BT; i++) v[i] = step(xlate(v[i], QP - 1 + BT * bt + i));
#pragma unroll
            for (int kb = 0; kb < BT / D; kb++) {
                float2* w = v + kb * D;
#define SDRGPU_RED_STEP(DX)                                                                        \
                if constexpr (D > (DX)) {                                                          \
                    const bool up = (p & (DX)) != 0;                                               \
                    _Pragma("unroll") for (int i = 0; i < (DX); i++) {                             \
                        const float2 snd = up ? w[i] : w[i + (DX)];                                \
                        const float2 keep = up ? w[i + (DX)] : w[i];                               \
                        const float rx = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(snd.x), ((DX) << 10) | 0x1F)); \
                        const float ry = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(snd.y), ((DX) << 10) | 0x1F)); \
                        w[i] = make_float2(keep.x + rx, keep.y + ry);                              \
                        if constexpr (LOWREG) __builtin_amdgcn_sched_barrier(0);                   \
                    }                                                                              \
                }
                if constexpr (D == 32) {
                    // xor 16 within a 32-lane group as one v_permlane16_swap per register pair: it swaps
                    // rows 1 / 3 of w[i] with rows 0 / 2 of w[i + 16], so lanes 0-15 (up = 0) then hold
                    // (own w[i], partner's w[i]) and lanes 16-31 (partner's w[i + 16], own w[i + 16]):
                    // the same sums as the swizzle step (a + b == b + a exactly), in place, without the
                    // send / keep selects and their temporaries (the spectrum launches run this at a
                    // 128-VGPR budget)
                    _Pragma("unroll") for (int i = 0; i < 16; i++) {
                        const auto sx = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[i].x), __float_as_uint(w[i + 16].x), false, false);
                        const auto sy = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[i].y), __float_as_uint(w[i + 16].y), false, false);
                        w[i] = make_float2(__uint_as_float(sx[0]) + __uint_as_float(sx[1]), __uint_as_float(sy[0]) + __uint_as_float(sy[1]));
                    }
                } else {
                    SDRGPU_RED_STEP(16)
                }
                SDRGPU_RED_STEP(8)
                SDRGPU_RED_STEP(4)
                SDRGPU_RED_STEP(2)
                SDRGPU_RED_STEP(1)
#undef SDRGPU_RED_STEP
                const float2 y = w[0];
                const int j = BT * bt + kb * D + p;   // local output index
                const long long m = mseg + j;
                if constexpr (QUAD) {
                    // y[m - 1]: lane p - 1 of the group, or the group's last output of the previous block
                    const int srcl = (lane & ~(D - 1)) + ((p + D - 1) & (D - 1));
                    float2 prev = make_float2(__shfl(y.x, srcl), __shfl(y.y, srcl));
                    if (p == 0) prev = ylast;
                    const int lastl = (lane & ~(D - 1)) + D - 1;
                    ylast = make_float2(__shfl(y.x, lastl), __shfl(y.y, lastl));
                    if (m == 0) prev = a.din[0];
                    if (j >= QOFF && m >= 0 && m < a.M) {
                        const float br = prev.x, bi = -prev.y;
                        const float re = (y.x * br) - (y.y * bi);
                        const float im = (y.y * br) + (y.x * bi);
                        outf[m] = quad_atan2f(im, re) * a.invDev;
                        if (m == a.M - 1) a.dinNext[0] = y;
                    }
                } else {
                    if (m < a.M) out2[m] = y;
                }
            }
        }
    };
    if (interior) body(std::true_type{});
    else body(std::false_type{});
}

// A VFO's first stage (row kernel) run by the spectrum launches over the same device batch
// (fft.hip, sdrgpu_fft_execute_vfo_dev / _zoom_vfo_dev): vfo_stage1_prepare fills the launch
// arguments for a call of `count` samples at `in` without touching the VFO's state (1: fusable,
// 0: not -- the caller then runs the VFO on its own; < 0: error); the caller launches all M / (16 *
// RS) segment workgroups (16 segments of 128 outputs each) and the history workgroup; then
// vfo_stage1_finish commits the stage's state and runs the VFO's remaining stages into `out`.
struct VfoStage1 {
    FirArgs a;
    int M = 0, count = 0;
    void* out = nullptr;
};
int vfo_stage1_prepare(::sdrgpu_block* vfo, const void* in, int count, VfoStage1* st);
int vfo_stage1_finish(::sdrgpu_block* vfo, const VfoStage1& st, void* out, hipStream_t s);

}  // namespace sdrgpu
