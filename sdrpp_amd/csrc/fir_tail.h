// The FIR cascade tail (the VFO's stages behind the first one, short calls) shared by blocks.hip
// (fir_tail_kernel) and fft.hip (the front end's pass-B launch, which carries the tail workgroups).
#pragma once
#include "fir_rows.h"

namespace sdrgpu {

// ------------------------------------------------ FIR cascade tail (short calls)
// The FIR stages behind a chain's first stage -- the RxVFO's decimator stages 2.. and its channel
// low-pass: 9,600 -> 2,400 -> 1,200 -> 1,200 samples for a reference block -- in ONE launch
// instead of one 4.5-6 us launch each. Workgroup w owns outputs [w M / G, (w + 1) M / G) of the
// last stage and computes, stage by stage in LDS, exactly the outputs of the earlier stages its
// window needs (halos recomputed, so workgroups never exchange data). Each output is fir_kernel's
// fmaf chain -- phase p outer, padded tap q inner, the block's own [p][Q] tap table, the same
// register window -- so a stage's outputs are bit-identical to fir_kernel's. The last workgroup
// also writes every stage's next-call history (fir.h:80). Stage images use fir_kernel's
// phase-major, row-swizzled LDS layout (conflict-free window reads). The kernel runs once per
// call on a few CUs, so it is written for latency: one global round trip for all image loads,
// power-of-two decimations (shifts, not divisions), stage loops kept rolled (small code).
constexpr int TAIL_MAXS = 4;    // stages
// consecutive outputs per thread (register window), TailArgs::K. Short calls: each thread's chain of D *
// Q FMAs per output is the kernel's critical path (one or two waves per stage are busy), so fewer
// outputs per thread (more waves) measured faster: per-call trace 12.0 / 10.3 / 10.0 / 15.5 us at K =
// 4 / 2 / 1 / 8; prefetching the next tap chunk's LDS reads measured slower (13.8 us at K = 4, 12.0 at
// K = 2). Big calls (thousands of workgroups): K = 4, 3 us less per C5 step than 2 (r5o), 8 slower
// (75.2 vs 58.5 us, r5m); 512- and 128-thread workgroups slower (r5o)
constexpr int TAIL_K = 2;
constexpr int TAIL_NT = 256;    // threads per workgroup (short calls)
#ifndef SDRGPU_TAIL_KBIG
#define SDRGPU_TAIL_KBIG 4
#endif
#ifndef SDRGPU_TAIL_NTBIG
#define SDRGPU_TAIL_NTBIG 256
#endif
constexpr int TAIL_K_BIG = SDRGPU_TAIL_KBIG;     // big calls (A/B builds)
constexpr int TAIL_NT_BIG = SDRGPU_TAIL_NTBIG;
#ifndef SDRGPU_TAIL_PF
#define SDRGPU_TAIL_PF 16
#endif
#ifndef SDRGPU_TAIL_LDSMAX
#define SDRGPU_TAIL_LDSMAX 65536
#endif
constexpr int TAIL_PF = SDRGPU_TAIL_PF;     // image loads per thread issued together (A/B builds)
constexpr int TAIL_LDSMAX = SDRGPU_TAIL_LDSMAX;   // bytes of LDS a tail workgroup may take
struct TailStage {
    const float2* hist;   // H samples (newest last)
    float2* histNext;     // next call's history: [hist || in][n + k], k < H
    const float* taps;    // [D][Q] phase-major, zero past ntaps = H + 1
    int H, n, D, dsh, Q, off, M;   // dsh = log2 D
};
struct TailArgs {
    const float2* in;     // stage 0's input (n of stage 0 samples)
    float2* out;          // last stage's output
    int S, G;
    int K;                // outputs per thread (TAIL_K): the image layout depends on it
    int NT;               // threads per workgroup (TAIL_NT / TAIL_NT_BIG)
    int ldsEl;            // float2 elements of the largest workgroup's images (the taps follow)
    int tapTotal;         // floats of all stages' tap tables
    int tapOff[TAIL_MAXS];   // float offset of stage s's [D][Q] taps behind the images
    TailStage st[TAIL_MAXS];
};
// Per workgroup and stage: outputs [a, b), image of [hist || in] elements [B, E) (B = off + a D,
// so an image row is one output step), swizzle strides, LDS base. Returns the LDS elements.
struct TailGeom { int a, b, B, E, RSK, RSP, base, nel; };
__host__ __device__ inline int tail_geometry(const TailArgs& t, int w, TailGeom* g) {
    const bool last = w == t.G - 1;
    const int Ml = t.st[t.S - 1].M;
    int lo = (int)((long long)Ml * w / t.G), hi = (int)((long long)Ml * (w + 1) / t.G);
#pragma unroll
    for (int s = TAIL_MAXS - 1; s >= 0; s--) {   // (static indices: g stays in registers)
        if (s >= t.S) continue;
        const TailStage& st = t.st[s];
        TailGeom& q = g[s];
        const int len = st.H + st.n;
        q.a = lo;
        q.b = hi;
        if (lo < hi) {
            q.B = st.off + lo * st.D;
            q.E = st.off + (hi - 1) * st.D + st.H + 1;   // the last output's window end (<= len)
        } else {
            q.B = q.E = len;
        }
        if (last) {   // + the next call's history [n, len): off + (M - 1) D < n, so B stays aligned
            q.B = q.B < st.n ? q.B : st.n;
            q.E = len;
        }
        const int K = t.K;
        const int nthr = (hi - lo + K - 1) / K;
        int rows = nthr * K + st.Q + 2 * K;
        const int need = (q.E - q.B + st.D - 1) / st.D + 1;
        rows = rows > need ? rows : need;
        q.RSK = (rows + K - 1) / K;
        q.RSP = K * q.RSK + 1;
        q.nel = st.D * q.RSK * K;
        // the previous stage's outputs this image holds: in[] indices of [B, E)
        lo = q.B - st.H > 0 ? q.B - st.H : 0;
        hi = q.E - st.H < st.n ? q.E - st.H : st.n;
        if (lo >= hi) lo = hi = 0;
    }
    int base = 0;
#pragma unroll
    for (int s = 0; s < TAIL_MAXS; s++) {
        if (s >= t.S) break;
        g[s].base = base;
        base += t.st[s].D * g[s].RSP;
    }
    return base;
}
// Tail workgroup w (last: it also writes every stage's next-call history) on threads [0, NT) of the
// block, images in XS, geometry in gs (LDS). Threads past NT (the spectrum's 512-thread pass-B launch,
// fft.hip) take part in the barriers only. K == t.K, NT == t.NT.
template <int K, int NT>
__device__ __forceinline__ void fir_tail_block(const TailArgs& t, int w, bool last, float2* XS, TailGeom* gs) {
    const int tid = threadIdx.x;
    const bool act = tid < NT;
    // every global load of the launch is issued in one batch (one memory round trip; a dependent
    // round trip to HBM costs ~1-2 us, which is what this kernel is built to avoid): the stages'
    // tap tables, the histories of stages >= 1 (H <= NT, host-checked) and stage 0's image
    // (<= TAIL_PF * NT elements, host-checked). The geometry is wave-uniform (scalar).
    TailGeom g[TAIL_MAXS];
    tail_geometry(t, w, g);
    // image element sx (from B) of stage s -> LDS index (fir_kernel's layout)
    auto slot = [&](const TailGeom& q, int dsh, int sx) {
        const int r = sx >> dsh;
        return q.base + (sx & ((1 << dsh) - 1)) * q.RSP + (r & (K - 1)) * q.RSK + r / K;
    };
    float* TS = reinterpret_cast<float*>(XS + t.ldsEl);
    if (act) {
        constexpr int TAIL_TP = 2;   // tap loads per thread: <= 512 taps in all (host-checked)
        float tap[TAIL_TP];
#pragma unroll
        for (int u = 0; u < TAIL_TP; u++) {
            tap[u] = 0.f;
            const int j = tid + u * NT;
#pragma unroll
            for (int s = 0; s < TAIL_MAXS; s++) {
                if (s >= t.S) break;
                const int i = j - t.tapOff[s];
                if (i >= 0 && i < t.st[s].D * t.st[s].Q) tap[u] = t.st[s].taps[i];
            }
        }
        float2 hv[TAIL_MAXS];
#pragma unroll
        for (int s = 1; s < TAIL_MAXS; s++) {
            if (s >= t.S) break;
            const int e = g[s].B + tid;
            hv[s] = (e < t.st[s].H && e < g[s].E) ? t.st[s].hist[e] : make_float2(0.f, 0.f);
        }
        const TailStage& s0 = t.st[0];
        float2 v[TAIL_PF];
#pragma unroll
        for (int u = 0; u < TAIL_PF; u++) {
            const int e = g[0].B + tid + u * NT;
            const float2* src = (e < g[0].E) ? (e < s0.H ? s0.hist + e : t.in + (e - s0.H)) : nullptr;
            v[u] = src ? *src : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < TAIL_TP; u++)
            if (tid + u * NT < t.tapTotal) TS[tid + u * NT] = tap[u];
#pragma unroll
        for (int s = 0; s < TAIL_MAXS; s++)
            if (tid == s && s < t.S) gs[s] = g[s];
        {   // stage 0: D | NT, so a thread's slots advance by a constant (fixed phase and lane)
            int idx = slot(g[0], s0.dsh, tid);
            const int inc = (NT >> s0.dsh) / K;
#pragma unroll
            for (int u = 0; u < TAIL_PF; u++) {
                if (tid + u * NT < g[0].nel) XS[idx] = v[u];
                idx += inc;
            }
        }
        // stages >= 1: history part [B, min(H, E)) and zeros past E; [max(B, H), E) is written by the
        // stage before
#pragma unroll
        for (int s = 1; s < TAIL_MAXS; s++) {
            if (s >= t.S) break;
            const int H = t.st[s].H;
            if (g[s].B + tid < H && g[s].B + tid < g[s].E) XS[slot(g[s], t.st[s].dsh, tid)] = hv[s];
            for (int sx = (g[s].E - g[s].B) + tid; sx < g[s].nel; sx += NT) XS[slot(g[s], t.st[s].dsh, sx)] = make_float2(0.f, 0.f);
        }
    }
    __syncthreads();
#pragma unroll 1
    for (int s = 0; s < t.S; s++) {
        if (act) {
            const TailStage& st = t.st[s];
            const TailGeom q = gs[s];
            if (last)
                for (int k = tid; k < st.H; k += NT) st.histNext[k] = XS[slot(q, st.dsh, st.n + k - q.B)];
            const int nthr = (q.b - q.a + K - 1) / K;
            for (int l = tid; l < nthr; l += NT) {
                // (packed fp32: x h + acc per component is the fmaf of mac(), so the same bits)
                f2v acc[K];
#pragma unroll
                for (int i = 0; i < K; i++) acc[i] = f2v{0.f, 0.f};
                constexpr int QC = 8;   // st.Q is a multiple of 8 (FirBlock::upload_taps)
                static_assert(QC % K == 0, "tap chunks of whole register windows");
                for (int p = 0; p < st.D; p++) {
                    const float2* Xj[K];
#pragma unroll
                    for (int j = 0; j < K; j++) Xj[j] = XS + q.base + p * q.RSP + j * q.RSK + l;
                    const float* Hp = TS + t.tapOff[s] + p * st.Q;   // wave-uniform LDS broadcasts
                    f2v w[K];
#pragma unroll
                    for (int i = 0; i < K; i++) w[i] = to_v(Xj[i][0]);
                    for (int q0 = 0; q0 < st.Q; q0 += QC) {
                        float hv[QC];
                        f2v nx[QC];
#pragma unroll
                        for (int u = 0; u < QC; u++) hv[u] = Hp[q0 + u];
#pragma unroll
                        for (int u = 0; u < QC; u++) nx[u] = to_v(Xj[u % K][1 + (q0 + u) / K]);
#pragma unroll
                        for (int u = 0; u < QC; u++) {
#pragma unroll
                            for (int i = 0; i < K; i++) acc[i] = __builtin_elementwise_fma(w[(i + u) % K], f2v{hv[u], hv[u]}, acc[i]);
                            w[u % K] = nx[u];
                        }
                    }
                }
                const bool lastStage = s == t.S - 1;
                const TailGeom* qn = &gs[lastStage ? s : s + 1];
                const int dshN = t.st[lastStage ? s : s + 1].dsh, HN = t.st[lastStage ? s : s + 1].H;
#pragma unroll
                for (int i = 0; i < K; i++) {
                    const int m = q.a + l * K + i;
                    if (m < q.b) {
                        if (lastStage) t.out[m] = to_f2(acc[i]);
                        else XS[slot(*qn, dshN, HN + m - qn->B)] = to_f2(acc[i]);
                    }
                }
            }
        }
        __syncthreads();
    }
}

// the tail of a VFO whose first stage ran in the front end's pass-A launch, as the pass-B launch
// carries it (blocks.hip): 1 = t / lds filled, no state changed -- the caller launches the t.G tail
// workgroups, then calls vfo_tail_commit (stage 1 and the tail stages move on together); 0 = not
// applicable (nothing changed: the caller then calls vfo_stage1_finish)
int vfo_tail_prepare(::sdrgpu_block* vfo, const VfoStage1& st, void* out, TailArgs* t, size_t* lds);
int vfo_tail_commit(::sdrgpu_block* vfo, const VfoStage1& st, const TailArgs& t);

}  // namespace sdrgpu
