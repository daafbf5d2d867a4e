// Radix-16 Stockham FFT building blocks shared by the spectrum kernels (fft.hip) and the
// polyphase channelizer (channelizer.hip): small DFTs in registers, padded LDS layout, and
// LDS -> LDS / LDS -> store stages. Forward transform (e^{-i}), unnormalised.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

namespace sdrgpu {

typedef float pk2 __attribute__((ext_vector_type(2)));

// a * b as two packed ops with the operand halves picked by op_sel, the same roundings as the
// contracted scalar form (re = fma(a.x, b.x, -(a.y b.y)), im = fma(a.x, b.y, a.y b.x)):
//   t = (a.y b.y, a.y b.x)                    v_pk_mul_f32, src0 (hi, hi), src1 (hi, lo)
//   r = (a.x b.x - t.x, a.x b.y + t.y)        v_pk_fma_f32, src0 (lo, lo), src2 lo negated
// Left to itself the compiler builds the broadcast / swapped operand pairs with v_mov_b32 (208
// moves in the 1M pass A's 1,559 VALU instructions, r3).
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
#ifdef SDRGPU_CMUL_C   // (A/B builds only)
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
#endif
    pk2 t, r;
    const pk2 x = {a.x, a.y}, y = {b.x, b.y};
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(x), "v"(y));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(x), "v"(y), "v"(t));
    return make_float2(r.x, r.y);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }   // a * (-i)

// a + (-i) b = (a.x + b.y, a.y - b.x) and a - (-i) b = (a.x - b.y, a.y + b.x) as ONE packed add
// each (src1 halves swapped by op_sel, one half negated). Left to itself the compiler forms both
// cross sums in two packed adds and assembles the results with four moves (r3: 439 v_mov_b32 in
// the 1M pass A's 1,900 VALU instructions).
__device__ __forceinline__ float2 add_negi(float2 a, float2 b) {
    pk2 r;
    const pk2 x = {a.x, a.y}, y = {b.x, b.y};
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    return make_float2(r.x, r.y);
}
__device__ __forceinline__ float2 sub_negi(float2 a, float2 b) {
    pk2 r;
    const pk2 x = {a.x, a.y}, y = {b.x, b.y};
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    return make_float2(r.x, r.y);
}

// ---- small forward DFTs in registers (e^{-i}) ------------------------------
__device__ __forceinline__ void dft2(float2* v) {
    float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}
__device__ __forceinline__ void dft4(float2& x0, float2& x1, float2& x2, float2& x3) {
    float2 a0 = cadd(x0, x2), a1 = csub(x0, x2), a2 = cadd(x1, x3), d13 = csub(x1, x3);
    x0 = cadd(a0, a2);
    x2 = csub(a0, a2);
    x1 = add_negi(a1, d13);   // a1 + (-i)(x1 - x3)
    x3 = sub_negi(a1, d13);
}
__device__ __forceinline__ void dft4v(float2* v) { dft4(v[0], v[1], v[2], v[3]); }

__device__ __forceinline__ void dft8(float2* v) {
    const float R2 = 0.70710678118654752440f;
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    o1 = make_float2(R2 * (o1.x + o1.y), R2 * (o1.y - o1.x));   // * W8^1 = (1-i)/sqrt2
    o3 = make_float2(R2 * (o3.y - o3.x), -R2 * (o3.x + o3.y));   // * W8^3 = (-1-i)/sqrt2
    v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
    v[1] = cadd(e1, o1); v[5] = csub(e1, o1);
    v[2] = add_negi(e2, o2); v[6] = sub_negi(e2, o2);            // o2 * W8^2 = o2 * (-i)
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
    y[2][3] = cmul(y[2][3], make_float2(-R2, -R2));
    y[3][1] = cmul(y[3][1], make_float2(S1, -C1));
    y[3][2] = cmul(y[3][2], make_float2(-R2, -R2));
    y[3][3] = cmul(y[3][3], make_float2(-C1, S1));
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        float2 a = y[0][k1], b = y[1][k1], c = y[2][k1], d = y[3][k1];
        if (k1 == 2) {   // c = y[2][2] * W16^4 = y[2][2] * (-i), folded into the first butterfly
            const float2 a0 = add_negi(a, c), a1 = sub_negi(a, c), a2 = cadd(b, d), d13 = csub(b, d);
            a = cadd(a0, a2);
            c = csub(a0, a2);
            b = add_negi(a1, d13);
            d = sub_negi(a1, d13);
        } else {
            dft4(a, b, c, d);
        }
        v[k1] = a; v[k1 + 4] = b; v[k1 + 8] = c; v[k1 + 12] = d;
    }
}

template <int R> __device__ __forceinline__ void dft(float2* v);
template <> __device__ __forceinline__ void dft<2>(float2* v) { dft2(v); }
template <> __device__ __forceinline__ void dft<4>(float2* v) { dft4v(v); }
template <> __device__ __forceinline__ void dft<8>(float2* v) { dft8(v); }
template <> __device__ __forceinline__ void dft<16>(float2* v) { dft16(v); }

__device__ __forceinline__ int pad16(int i) { return i + (i >> 4); }
// pad16(j + r S) for j >= 0: when S is a multiple of 16 the image moves by r (S + S / 16), a constant
// the unrolled loop folds into the LDS instruction's offset. (Written as pad16(j + r S) the compiler
// recomputed the shift per element: ~4 VALU per LDS access in the 1M pass A.)
// (SDRGPU_PAD16_PLAIN: the round-3 per-element form, an A/B build)
template <int S>
__device__ __forceinline__ int pad16s(int j, int r) {
#ifndef SDRGPU_PAD16_PLAIN
    if constexpr (S % 16 == 0) return pad16(j) + r * (S + S / 16);
#endif
    return pad16(j + r * S);
}
// pad16(16 t + r) for r < 16: 17 t + r
__device__ __forceinline__ int pad16lo(int t, int r) {
#ifndef SDRGPU_PAD16_PLAIN
    return 17 * t + r;
#else
    return pad16(t * 16 + r);
#endif
}
template <int L> struct Lds { static constexpr int LS = L + L / 16 + 1; };   // sequence stride (odd)

// tw16[16 r + jm] = tw[r jm (L / 256)] (r, jm < 16) for the T16 stages below; the caller's next
// barrier orders the writes
template <int L>
__device__ __forceinline__ void stage16_twiddles(float2* tw16, const float2* __restrict__ tw, int tid, int nthreads) {
    for (int i = tid; i < 256; i += nthreads) tw16[i] = tw[(i >> 4) * (i & 15) * (L / 256)];
}

// One Stockham radix-R stage, LDS -> LDS, for sequence s, thread t (T = L/16 threads per
// sequence, each owning butterflies j = t + b*T, b < 16/R). Caller provides the barriers.
// stage16_twiddles fills it (256 entries, once per workgroup)
// tw16 (optional, R = NS = 16): the stage's twiddles as tw16[16 r + jm] = tw[r jm (L / 256)], so
// the 16 lanes of different jm read 16 consecutive words for each r. Read from tw directly the
// stride r jm (L / 256) puts them in the same LDS banks for even r (16-way at r = 8 when tw is
// in LDS: the 1M pass B spent more cycles in bank conflicts than in LDS issue, r3 SQ counters).
template <int L, int R, int NS, bool T16 = false>
__device__ __forceinline__ void stage_lds(float2* seq, const float2* __restrict__ tw, int t, const float2* tw16 = nullptr) {
    constexpr int T = L / 16;
    constexpr int BPT = 16 / R;
    float2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T;
#pragma unroll
        for (int r = 0; r < R; r++) v[b][r] = seq[pad16s<L / R>(j, r)];
        const int jm = j % NS;
        if constexpr (T16 && R == 16 && NS == 16) {
#pragma unroll
            for (int r = 1; r < R; r++) v[b][r] = cmul(v[b][r], tw16[16 * r + jm]);
        } else {
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
        for (int r = 0; r < R; r++) seq[pad16s<NS>(idxD, r)] = v[b][r];
    }
    __syncthreads();
}

// Last stage: LDS -> registers -> store functor (output index k, value).
template <int L, int R, int NS, bool T16 = false, class Store>
__device__ __forceinline__ void stage_last(const float2* seq, const float2* __restrict__ tw, int t, Store&& st,
                                           const float2* tw16 = nullptr) {
    constexpr int T = L / 16;
    constexpr int BPT = 16 / R;
    float2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T;
#pragma unroll
        for (int r = 0; r < R; r++) v[b][r] = seq[pad16s<L / R>(j, r)];
        const int jm = j % NS;
        if constexpr (T16 && R == 16 && NS == 16) {   // (stage_lds's conflict-free layout)
#pragma unroll
            for (int r = 1; r < R; r++) v[b][r] = cmul(v[b][r], tw16[16 * r + jm]);
        } else {
#pragma unroll
            for (int r = 1; r < R; r++) v[b][r] = cmul(v[b][r], tw[r * jm * (L / (NS * R))]);
        }
        dft<R>(v[b]);
    }
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int j = t + b * T;
        const int idxD = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; r++) {
            // a store functor may also take the output's register slot (a compile-time constant
            // after unrolling), e.g. to keep the outputs in a register array
            if constexpr (std::is_invocable_v<Store&, int, float2, int>) st(idxD + r * NS, v[b][r], b * R + r);
            else st(idxD + r * NS, v[b][r]);
        }
    }
}

// Stage 1 of a length-L Stockham FFT on a thread's 16 register values (radix 16, NS = 1,
// no twiddles), written to the sequence's LDS image.
template <int L>
__device__ __forceinline__ void stage_first(float2* seq, float2 (&v)[16], int t) {
    dft16(v);
#pragma unroll
    for (int r = 0; r < 16; r++) seq[pad16lo(t, r)] = v[r];
}

// Stages after the first: LDS -> ... -> store functor. Expects stage_first's LDS writes
// to be complete (caller's barrier); leaves the LDS free for reuse on return. T16: the radix-16
// stage with NS = 16 (L >= 256) reads its twiddles from tw16 (stage_lds), staged by the caller.
// LS: the sequence stride of the caller's LDS image (stage_first wrote sequence s at lds + s LS).
template <int L, bool T16 = false, int LS = Lds<L>::LS, class Store>
__device__ __forceinline__ void stages_rest(float2* lds, const float2* __restrict__ tw, int sL, int tL, Store&& st,
                                            const float2* tw16 = nullptr) {
    const float2* seqL = lds + sL * LS;
    if constexpr (L == 64) {
        stage_last<L, 4, 16>(seqL, tw, tL, st);
    } else if constexpr (L == 128) {
        stage_last<L, 8, 16>(seqL, tw, tL, st);
    } else if constexpr (L == 256) {
        stage_last<L, 16, 16, T16>(seqL, tw, tL, st, tw16);
    } else {
        stage_lds<L, 16, 16, T16>(lds + sL * LS, tw, tL, tw16);   // middle stage (radix 16, NS = 16)
        if constexpr (L == 512) stage_last<L, 2, 256>(seqL, tw, tL, st);
        else if constexpr (L == 1024) stage_last<L, 4, 256>(seqL, tw, tL, st);
        else if constexpr (L == 2048) stage_last<L, 8, 256>(seqL, tw, tL, st);
        else stage_last<L, 16, 256>(seqL, tw, tL, st);
    }
}

}  // namespace sdrgpu
