// Serial (data-dependent) loops of the demodulators and the blocks composed from them:
//   loop::AGC<T>           loop/agc.h:88-147
//   correction::DCBlocker  correction/dc_blocker.h:54-60
//   demod::AM<T>           demod/am.h:114-142     ([carrier AGC] -> |x| -> DC block -> [audio AGC] -> LPF)
//   demod::SSB<T>          demod/ssb.h:90-105     (xlate +-bw/2 -> Re -> AGC)
//
// The AGC and the DC blocker are first-order recurrences whose next state depends on the
// current sample (the AGC nonlinearly), so they run as ONE workgroup per stream: the block is
// walked in 1024-sample chunks; all 256 lanes stage the chunk (and, for the AGC, its
// amplitudes and the exact suffix maxima its clip look-ahead needs) in LDS, lane 0 runs the
// recurrence over the chunk from LDS, and all lanes write the chunk out. This file is compiled
// with -ffp-contract=off (sdrpp_amd/build.py: HIP contracts a*b+c into an FMA by default),
// every step is written in the
// reference's order, and division / square root are IEEE (correctly rounded), so the GPU
// result is bit-identical to the reference arithmetic (oracle/sdr_oracle.c orc_agc / orc_dcb).
//
// The AGC's clip look-ahead scans amplitudes from sample i to the end of the CURRENT block
// (agc.h:109-118; O(n^2) worst case in the reference). The suffix maximum over the block is
// precomputed in parallel (max is exact), so the serial loop is O(n) and the result is the
// same value. State (average amplitude, gain; DC offset) stays on the device between calls.
#include <algorithm>
#include <cmath>
#include <memory>
#include <vector>
#include "sdrgpu_internal.h"

namespace sdrgpu {

constexpr int LOOP_CHUNK = 1024;
constexpr int LOOP_NT = 256;

// |x| exactly as complex_t::amplitude() (types.h:79) / fabsf, no contraction
__device__ __forceinline__ float amp_of(float x) { return fabsf(x); }
// (sqrtf is correctly rounded under HIP's default -fhip-fp32-correctly-rounded-divide-sqrt;
// __fsqrt_rn is the native approximation unless OCML_BASIC_ROUNDED_OPERATIONS is defined)
__device__ __forceinline__ float amp_of(float2 x) { return sqrtf((x.x * x.x) + (x.y * x.y)); }
__device__ __forceinline__ float scale_of(float x, float g) { return x * g; }
__device__ __forceinline__ float2 scale_of(float2 x, float g) { return make_float2(x.x * g, x.y * g); }

struct AgcParams {
    float setPoint, attack, invAttack, decay, invDecay, maxGain, maxOutputAmp;
    int enabled;
};
struct AgcState {
    float amp, gain;
};

// per-chunk amplitude maxima (exact), one workgroup per chunk
template <typename DT>
__global__ __launch_bounds__(LOOP_NT) void chunk_max_kernel(const DT* __restrict__ in, int count, float* __restrict__ cm) {
    __shared__ float red[LOOP_NT];
    const int c = blockIdx.x;
    float m = 0.0f;
    for (int i = c * LOOP_CHUNK + threadIdx.x; i < min(count, (c + 1) * LOOP_CHUNK); i += LOOP_NT) m = fmaxf(m, amp_of(in[i]));
    red[threadIdx.x] = m;
    __syncthreads();
    for (int s = LOOP_NT / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) cm[c] = red[0];
}

// One workgroup: the whole block, chunk by chunk. `cm` holds the chunk maxima on entry.
template <typename DT>
__global__ __launch_bounds__(LOOP_NT) void agc_kernel(const DT* __restrict__ in, DT* __restrict__ out, int count,
                                                      AgcParams p, AgcState* __restrict__ st, float* __restrict__ cm,
                                                      const float* __restrict__ setGain) {
    __shared__ DT X[LOOP_CHUNK];
    __shared__ float A[LOOP_CHUNK], S[LOOP_CHUNK], G[LOOP_CHUNK];
    const int t = threadIdx.x;
    const int nchunks = (count + LOOP_CHUNK - 1) / LOOP_CHUNK;
    if (t == 0) {   // cm[c] <- max over chunks > c (the look-ahead beyond chunk c)
        float run = 0.0f;
        for (int c = nchunks - 1; c >= 0; c--) {
            const float v = cm[c];
            cm[c] = run;
            run = fmaxf(run, v);
        }
    }
    __syncthreads();
    float amp = st->amp, gain = st->gain;
    if (setGain) gain = *setGain;                          // AGC::setGain latched at this call
    for (int c = 0; c < nchunks; c++) {
        const int i0 = c * LOOP_CHUNK;
        const int n = min(LOOP_CHUNK, count - i0);
        for (int i = t; i < LOOP_CHUNK; i += LOOP_NT) {
            if (i < n) {
                const DT v = in[i0 + i];
                X[i] = v;
                A[i] = amp_of(v);
            } else {
                A[i] = 0.0f;
            }
        }
        __syncthreads();
        if (p.enabled) {
            // S[i] = max(A[i..n-1], beyond): Hillis-Steele suffix max, exact
            for (int i = t; i < LOOP_CHUNK; i += LOOP_NT) S[i] = (i == n - 1) ? fmaxf(A[i], cm[c]) : A[i];
            __syncthreads();
            for (int d = 1; d < LOOP_CHUNK; d <<= 1) {
                float v[LOOP_CHUNK / LOOP_NT];
#pragma unroll
                for (int k = 0; k < LOOP_CHUNK / LOOP_NT; k++) {
                    const int i = t + k * LOOP_NT;
                    v[k] = (i + d < n) ? fmaxf(S[i], S[i + d]) : S[i];
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < LOOP_CHUNK / LOOP_NT; k++) S[t + k * LOOP_NT] = v[k];
                __syncthreads();
            }
        }
        if (t == 0) {
            if (p.enabled) {
                for (int i = 0; i < n; i++) {
                    const float inAmp = A[i];
                    if (inAmp != 0.0f) {
                        amp = (inAmp > amp) ? ((amp * p.invAttack) + (inAmp * p.attack))
                                            : ((amp * p.invDecay) + (inAmp * p.decay));
                        const float q = p.setPoint / amp;
                        gain = (p.maxGain < q) ? p.maxGain : q;              // std::min<float>
                    } else {
                        gain = 1.0f;
                    }
                    if (inAmp * gain > p.maxOutputAmp) {                     // clip look-ahead
                        amp = S[i];
                        const float q = p.setPoint / amp;
                        gain = (p.maxGain < q) ? p.maxGain : q;
                    }
                    G[i] = gain;
                }
            } else {
                for (int i = 0; i < n; i++) {
                    const float inAmp = A[i];
                    G[i] = (inAmp * gain > p.maxOutputAmp) ? (p.maxOutputAmp / inAmp) : gain;
                }
            }
        }
        __syncthreads();
        for (int i = t; i < n; i += LOOP_NT) out[i0 + i] = scale_of(X[i], G[i]);
        __syncthreads();
    }
    if (t == 0) {
        st->amp = amp;
        st->gain = gain;
    }
}

// DC blocker (dc_blocker.h:54-60): out = in - off; off += out * rate, per component
template <typename DT>
__global__ __launch_bounds__(LOOP_NT) void dcb_kernel(const DT* __restrict__ in, DT* __restrict__ out, int count,
                                                      float rate, float2* __restrict__ st) {
    __shared__ DT X[LOOP_CHUNK];
    const int t = threadIdx.x;
    float2 off = *st;
    for (int i0 = 0; i0 < count; i0 += LOOP_CHUNK) {
        const int n = min(LOOP_CHUNK, count - i0);
        for (int i = t; i < n; i += LOOP_NT) X[i] = in[i0 + i];
        __syncthreads();
        if (t == 0) {
            for (int i = 0; i < n; i++) {
                if constexpr (sizeof(DT) == 4) {
                    const float o = X[i] - off.x;
                    off.x += o * rate;
                    X[i] = o;
                } else {
                    const float2 v = X[i];
                    const float ox = v.x - off.x, oy = v.y - off.y;
                    off.x += ox * rate;
                    off.y += oy * rate;
                    X[i] = make_float2(ox, oy);
                }
            }
        }
        __syncthreads();
        for (int i = t; i < n; i += LOOP_NT) out[i0 + i] = X[i];
        __syncthreads();
    }
    if (t == 0) *st = off;
}

// filter::Deemphasis<T> (filter/deephasis.h:57-77): out = alpha * in + (1 - alpha) * prev,
// per channel (float: 1, stereo_t: 2); prev carried on the device
template <int C>
__global__ __launch_bounds__(LOOP_NT) void deemp_kernel(const float* __restrict__ in, float* __restrict__ out, int count,
                                                        float alpha, float2* __restrict__ st) {
    __shared__ float X[LOOP_CHUNK * C];
    const int t = threadIdx.x;
    float last[2] = {st->x, st->y};
    const float beta = 1 - alpha;                               // (1 - alpha): int - float -> float
    for (int i0 = 0; i0 < count; i0 += LOOP_CHUNK) {
        const int n = min(LOOP_CHUNK, count - i0);
        for (int i = t; i < n * C; i += LOOP_NT) X[i] = in[(size_t)i0 * C + i];
        __syncthreads();
        if (t == 0) {
            for (int i = 0; i < n; i++)
#pragma unroll
                for (int c = 0; c < C; c++) {
                    const float y = (alpha * X[i * C + c]) + (beta * last[c]);
                    X[i * C + c] = y;
                    last[c] = y;
                }
        }
        __syncthreads();
        for (int i = t; i < n * C; i += LOOP_NT) out[(size_t)i0 * C + i] = X[i];
        __syncthreads();
    }
    if (t == 0) *st = make_float2(last[0], last[1]);
}

// volk_32fc_magnitude_32f (AM) / ComplexToReal (SSB) / MonoToStereo
__global__ void magnitude_kernel(const float2* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = amp_of(in[i]);
}
__global__ void real_part_kernel(const float2* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i].x;
}
__global__ void mono_to_stereo_kernel(const float* __restrict__ in, float2* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float2(in[i], in[i]);
}

// ------------------------------------------------------- BroadcastFM stereo
// demod/broadcast_fm.h:144-191 with loop/pll.h:64-70 + loop/phase_control_loop.h:59-66.
struct PllParams {
    float alpha, beta, minPhase, maxPhase, phaseDelta, minFreq, maxFreq;
};
__global__ void real_to_complex_kernel(const float* __restrict__ in, float2* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float2(in[i], 0.0f);           // convert::RealToComplex
}
__global__ void phase_kernel(const float2* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = atan2f(in[i].y, in[i].x);             // complex_t::phase() (types.h:57)
}
// The PLL recurrence (one workgroup): in place, th[i] = input phase -> the phase the VCO
// outputs for sample i (math::phasor(pcl.phase) BEFORE advance). State (phase, freq) on device.
__global__ __launch_bounds__(LOOP_NT) void pll_kernel(float* __restrict__ th, int count, PllParams p, float2* __restrict__ st) {
    __shared__ float T[LOOP_CHUNK];
    const int t = threadIdx.x;
    float phase = st->x, freq = st->y;
    const float PI = 3.1415926535f;                            // FL_M_PI (math/constants.h:4)
    for (int i0 = 0; i0 < count; i0 += LOOP_CHUNK) {
        const int n = min(LOOP_CHUNK, count - i0);
        for (int i = t; i < n; i += LOOP_NT) T[i] = th[i0 + i];
        __syncthreads();
        if (t == 0) {
            for (int i = 0; i < n; i++) {
                float diff = T[i] - phase;
                T[i] = phase;
                if (diff > PI) diff -= 2.0f * PI;               // math::normalizePhase
                else if (diff <= -PI) diff += 2.0f * PI;
                freq += p.beta * diff;                          // PhaseControlLoop::advance
                if (freq > p.maxFreq) freq = p.maxFreq;
                else if (freq < p.minFreq) freq = p.minFreq;
                phase += freq + (p.alpha * diff);
                while (phase > p.maxPhase) phase -= p.phaseDelta;
                while (phase < p.minPhase) phase += p.phaseDelta;
            }
        }
        __syncthreads();
        for (int i = t; i < n; i += LOOP_NT) th[i0 + i] = T[i];
        __syncthreads();
    }
    if (t == 0) *st = make_float2(phase, freq);
}
// Delays, conjugate, the two complex multiplies, x2, L = (L+R) + (L-R), R = (L+R) - (L-R),
// written (l, r) as a float2 pair for the audio FIR. lmrDelay's input is RealToComplex of
// the MPX, so its delayed imaginary part is exactly 0: the products are formed as the
// reference forms them (0 * x terms included) and round identically.
__global__ void stereo_matrix_kernel(const float* __restrict__ mpx, const float* __restrict__ hist, int delay,
                                     const float* __restrict__ vcoPhase, float2* __restrict__ lr, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float d = i < delay ? hist[i] : mpx[i - delay];       // Delay<float> / Delay<complex_t>.re
    const float vr = cosf(vcoPhase[i]), vi = -sinf(vcoPhase[i]);   // Conjugate(phasor)
    float ar = d, ai = 0.0f;
#pragma unroll
    for (int k = 0; k < 2; k++) {                              // Multiply<complex_t>, twice
        const float nr = (ar * vr) - (ai * vi);
        const float ni = (ai * vr) + (ar * vi);
        ar = nr;
        ai = ni;
    }
    const float lmr = ar * 2.0f;
    lr[i] = make_float2(d + lmr, d - lmr);
}
__global__ void delay_hist_kernel(const float* __restrict__ hist, const float* __restrict__ in, float* __restrict__ next,
                                  int delay, int count) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= delay) return;
    const long long b = (long long)count + k;                  // last `delay` of [hist || in]
    next[k] = b < delay ? hist[b] : in[b - delay];
}

// ---------------------------------------------------------------- blocks
struct AgcBlock : Block {
    AgcParams p{};
    float initGain = 1.0f;
    DevBuf state, cm, pend;
    bool pending = false;
    float pendingGain = 0.0f;
    int setup(int dev, int dtype, double setPoint, double attack, double decay, double maxGain, double maxOutputAmp,
              double initGain_) {
        device = dev;
        in_dtype = out_dtype = dtype;
        // AGC::init (agc.h:13-26): members are float
        p.setPoint = (float)setPoint;
        p.attack = (float)attack;
        p.invAttack = 1.0f - p.attack;
        p.decay = (float)decay;
        p.invDecay = 1.0f - p.decay;
        p.maxGain = (float)maxGain;
        p.maxOutputAmp = (float)maxOutputAmp;
        initGain = (float)initGain_;
        p.enabled = 1;
        SDRGPU_CHECK(init_stream());
        SDRGPU_CHECK(state.ensure(sizeof(AgcState)));
        SDRGPU_CHECK(pend.ensure(sizeof(float)));
        return reset();
    }
    int out_count(int count) override { return count; }
    int reset() override {   // agc.h:81-86
        SDRGPU_SET_DEVICE(device);
        AgcState s;
        s.amp = p.setPoint / initGain;
        s.gain = (p.maxGain < initGain) ? p.maxGain : initGain;
        SDRGPU_HIP(hipMemcpy(state.p, &s, sizeof(s), hipMemcpyHostToDevice));
        pending = false;
        return SDRGPU_OK;
    }
    int set_gain(float g) {   // agc.h:31-35, applied at the next process()
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemcpy(pend.p, &g, sizeof(g), hipMemcpyHostToDevice));
        pending = true;
        pendingGain = g;
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count < 0) { set_error("agc: negative count"); return SDRGPU_EARG; }
        SDRGPU_SET_DEVICE(device);
        const float* pg = pending ? pend.as<float>() : nullptr;
        pending = false;
        if (count == 0 && !pg) return 0;
        const int nchunks = std::max(1, (count + LOOP_CHUNK - 1) / LOOP_CHUNK);
        SDRGPU_CHECK(cm.ensure(sizeof(float) * nchunks));
        if (in_dtype == SDRGPU_C64) {
            if (count > 0 && p.enabled)
                hipLaunchKernelGGL(chunk_max_kernel<float2>, dim3(nchunks), dim3(LOOP_NT), 0, s, (const float2*)in, count, cm.as<float>());
            hipLaunchKernelGGL(agc_kernel<float2>, dim3(1), dim3(LOOP_NT), 0, s, (const float2*)in, (float2*)out, count, p,
                               state.as<AgcState>(), cm.as<float>(), pg);
        } else {
            if (count > 0 && p.enabled)
                hipLaunchKernelGGL(chunk_max_kernel<float>, dim3(nchunks), dim3(LOOP_NT), 0, s, (const float*)in, count, cm.as<float>());
            hipLaunchKernelGGL(agc_kernel<float>, dim3(1), dim3(LOOP_NT), 0, s, (const float*)in, (float*)out, count, p,
                               state.as<AgcState>(), cm.as<float>(), pg);
        }
        SDRGPU_HIP(hipGetLastError());
        return count;
    }
};

struct DcbBlock : Block {
    float rate = 0.0f;
    DevBuf state;
    int setup(int dev, int dtype, double r) {
        device = dev;
        in_dtype = out_dtype = dtype;
        rate = (float)r;
        SDRGPU_CHECK(init_stream());
        SDRGPU_CHECK(state.ensure(sizeof(float2)));
        return reset();
    }
    int out_count(int count) override { return count; }
    int reset() override {
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemset(state.p, 0, sizeof(float2)));
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count < 0) { set_error("dc_blocker: negative count"); return SDRGPU_EARG; }
        if (count == 0) return 0;
        SDRGPU_SET_DEVICE(device);
        if (in_dtype == SDRGPU_C64)
            hipLaunchKernelGGL(dcb_kernel<float2>, dim3(1), dim3(LOOP_NT), 0, s, (const float2*)in, (float2*)out, count, rate, state.as<float2>());
        else
            hipLaunchKernelGGL(dcb_kernel<float>, dim3(1), dim3(LOOP_NT), 0, s, (const float*)in, (float*)out, count, rate, state.as<float2>());
        SDRGPU_HIP(hipGetLastError());
        return count;
    }
};

struct DeempBlock : Block {
    float alpha = 1.0f;
    DevBuf state;
    int setup(int dev, int dtype, double tau, double samplerate) {
        device = dev;
        in_dtype = out_dtype = dtype;                 // F32 (float) or C64 (stereo_t)
        set_alpha(tau, samplerate);
        SDRGPU_CHECK(init_stream());
        SDRGPU_CHECK(state.ensure(sizeof(float2)));
        return reset();
    }
    void set_alpha(double tau, double samplerate) {   // updateAlpha (deephasis.h:90-93)
        const float dt = (float)(1.0f / samplerate);
        alpha = (float)((double)dt / (tau + (double)dt));
    }
    int out_count(int count) override { return count; }
    int reset() override {
        SDRGPU_SET_DEVICE(device);
        SDRGPU_HIP(hipMemset(state.p, 0, sizeof(float2)));
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count < 0) { set_error("deemphasis: negative count"); return SDRGPU_EARG; }
        if (count == 0) return 0;     // (the reference reads out[-1] for count == 0)
        SDRGPU_SET_DEVICE(device);
        if (in_dtype == SDRGPU_C64)
            hipLaunchKernelGGL(deemp_kernel<2>, dim3(1), dim3(LOOP_NT), 0, s, (const float*)in, (float*)out, count, alpha, state.as<float2>());
        else
            hipLaunchKernelGGL(deemp_kernel<1>, dim3(1), dim3(LOOP_NT), 0, s, (const float*)in, (float*)out, count, alpha, state.as<float2>());
        SDRGPU_HIP(hipGetLastError());
        return count;
    }
};

// elementwise converters used inside the demod chains
struct MapBlock : Block {
    int kind = 0;   // 0 magnitude (c64 -> f32), 1 real part (c64 -> f32), 2 mono -> stereo (f32 -> c64)
    int out_count(int count) override { return count; }
    int reset() override { return SDRGPU_OK; }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count <= 0) return count < 0 ? SDRGPU_EARG : 0;
        SDRGPU_SET_DEVICE(device);
        const dim3 g((count + 255) / 256), b(256);
        if (kind == 0) hipLaunchKernelGGL(magnitude_kernel, g, b, 0, s, (const float2*)in, (float*)out, count);
        else if (kind == 1) hipLaunchKernelGGL(real_part_kernel, g, b, 0, s, (const float2*)in, (float*)out, count);
        else hipLaunchKernelGGL(mono_to_stereo_kernel, g, b, 0, s, (const float*)in, (float2*)out, count);
        SDRGPU_HIP(hipGetLastError());
        return count;
    }
};

static std::unique_ptr<MapBlock> make_map(int dev, int kind) {
    auto m = std::make_unique<MapBlock>();
    m->device = dev;
    m->kind = kind;
    m->in_dtype = kind == 2 ? SDRGPU_F32 : SDRGPU_C64;
    m->out_dtype = kind == 2 ? SDRGPU_C64 : SDRGPU_F32;
    return m;
}

// A chain of blocks run back to back on one stream (defined in blocks.hip)
int chain_new(int dev, int in_dtype, int out_dtype, Block** out);
int chain_append(Block* chain, Block* kid);
int chain_size(Block* chain);
Block* chain_kid(Block* chain, int i);
Block* make_fir_block(int dev, int dtype, int ttype, const float* taps, int n, int decim, bool stereo, int* rc);
Block* make_xlator_block(int dev, double offsetRad, int* rc);


// BroadcastFM (demod/broadcast_fm.h:34-60, 144-215): quadrature -> [stereo: pilot band-pass
// (complex, 305 taps at 240 kS/s) -> PLL -> matrix] -> audio low-pass -> stereo_t
Block* make_quad_block(int dev, double deviationRad, int* rc);
Block* make_xlate_resample_block(int dev, double inSr, double outSr, double w, int* rc);
struct BroadcastFmBlock : Block {
    bool stereo = true, lowPass = true;
    std::unique_ptr<Block> quad, pilot, audio;
    // RDS branch (broadcast_fm.h:164-171, 193-203): MPX as complex -> FrequencyXlator(-57 kHz) ->
    // RationalResampler<complex_t>(fs -> 5 kHz); off unless set_rds(true) (setRDSOut)
    bool rds = false;
    double fs = 0.0;
    std::unique_ptr<Block> rdsChain;
    DevBuf rdsIn, rdsOut;
    int rdsN = 0;
    int set_rds(bool on) {
        rds = on;
        rdsN = 0;
        if (on && !rdsChain) {
            int rc;
            rdsChain.reset(make_xlate_resample_block(device, fs, 5000.0, hz_to_rads(-57000.0, fs), &rc));
            if (rc < 0) { rdsChain.reset(); rds = false; return rc; }
        }
        return SDRGPU_OK;
    }
    PllParams pp{};
    float initPhase = 0.0f, initFreq = 0.0f;
    int delay = 0;
    DevBuf mpx, cplx, pf, ph, lr, pllState, hist[2];
    int cur = 0;
    int setup(int dev, double deviation, double samplerate, bool st, bool lp) {
        device = dev;
        in_dtype = SDRGPU_C64;
        out_dtype = SDRGPU_C64;
        stereo = st;
        lowPass = lp;
        fs = samplerate;
        SDRGPU_CHECK(init_stream());
        int rc;
        quad.reset(make_quad_block(dev, hz_to_rads(deviation, samplerate), &rc));
        SDRGPU_CHECK(rc);
        const int np = taps_band_pass_c(18750.0, 19250.0, 3000.0, samplerate, 1, nullptr);
        if (np < 1) return np < 0 ? np : SDRGPU_EARG;
        std::vector<float> pt(2 * (size_t)np);
        taps_band_pass_c(18750.0, 19250.0, 3000.0, samplerate, 1, pt.data());
        pilot.reset(make_fir_block(dev, SDRGPU_C64, SDRGPU_C64, pt.data(), np, 1, false, &rc));
        SDRGPU_CHECK(rc);
        delay = ((np - 1) / 2) + 1;                                   // lprDelay / lmrDelay
        // PLL(25000 / fs, 0, 19 kHz, 18.75 kHz, 19.25 kHz) (broadcast_fm.h:47); criticallyDamped
        // evaluated as PhaseControlLoop<float> does (phase_control_loop.h:31-36)
        const float bw = (float)(25000.0 / samplerate);
        const float df = (float)(std::sqrt(2.0) / 2.0);
        const float den = (float)((1.0 + 2.0 * (double)df * (double)bw) + (double)(bw * bw));
        pp.alpha = ((float)4 * df * bw) / den;
        pp.beta = ((float)4 * bw * bw) / den;
        pp.minPhase = -3.1415926535f;
        pp.maxPhase = 3.1415926535f;
        pp.phaseDelta = pp.maxPhase - pp.minPhase;
        pp.minFreq = (float)hz_to_rads(18750.0, samplerate);
        pp.maxFreq = (float)hz_to_rads(19250.0, samplerate);
        initPhase = 0.0f;
        initFreq = (float)hz_to_rads(19000.0, samplerate);
        const int na = taps_low_pass(15000.0, 4000.0, samplerate, 0, nullptr);
        if (na < 1) return na < 0 ? na : SDRGPU_EARG;
        std::vector<float> at(na);
        taps_low_pass(15000.0, 4000.0, samplerate, 0, at.data());
        if (!lowPass) { at.assign(1, 1.0f); }                          // identity: raw L/R (or MPX) pairs
        // (l, r) pairs filtered as one complex stream with real taps = alFir / arFir
        audio.reset(make_fir_block(dev, SDRGPU_C64, SDRGPU_F32, at.data(), (int)at.size(), 1, false, &rc));
        SDRGPU_CHECK(rc);
        SDRGPU_CHECK(pllState.ensure(sizeof(float2)));
        for (int k = 0; k < 2; k++) SDRGPU_CHECK(hist[k].ensure(sizeof(float) * delay));
        return reset();
    }
    int out_count(int count) override { return count; }
    int reset() override {   // broadcast_fm.h:129-141
        SDRGPU_SET_DEVICE(device);
        SDRGPU_CHECK(quad->reset());
        SDRGPU_CHECK(pilot->reset());
        SDRGPU_CHECK(audio->reset());
        if (rdsChain) SDRGPU_CHECK(rdsChain->reset());
        const float2 st = make_float2(initPhase, initFreq);
        SDRGPU_HIP(hipMemcpy(pllState.p, &st, sizeof(st), hipMemcpyHostToDevice));
        SDRGPU_HIP(hipMemset(hist[cur].p, 0, sizeof(float) * delay));
        return SDRGPU_OK;
    }
    int run(const void* in, int count, void* out, hipStream_t s) override {
        if (count < 0) { set_error("broadcast_fm: negative count"); return SDRGPU_EARG; }
        rdsN = 0;
        if (count == 0) return 0;
        SDRGPU_SET_DEVICE(device);
        SDRGPU_CHECK(mpx.ensure(sizeof(float) * count));
        SDRGPU_CHECK(lr.ensure(sizeof(float2) * count));
        int m = quad->run(in, count, mpx.p, s);
        if (m < 0) return m;
        const dim3 g((count + 255) / 256), b(256);
        if (stereo) {
            SDRGPU_CHECK(cplx.ensure(sizeof(float2) * count));
            SDRGPU_CHECK(pf.ensure(sizeof(float2) * count));
            SDRGPU_CHECK(ph.ensure(sizeof(float) * count));
            hipLaunchKernelGGL(real_to_complex_kernel, g, b, 0, s, mpx.as<float>(), cplx.as<float2>(), count);
            m = pilot->run(cplx.p, count, pf.p, s);
            if (m < 0) return m;
            hipLaunchKernelGGL(phase_kernel, g, b, 0, s, pf.as<float2>(), ph.as<float>(), count);
            hipLaunchKernelGGL(pll_kernel, dim3(1), dim3(LOOP_NT), 0, s, ph.as<float>(), count, pp, pllState.as<float2>());
            hipLaunchKernelGGL(stereo_matrix_kernel, g, b, 0, s, mpx.as<float>(), hist[cur].as<float>(), delay,
                               ph.as<float>(), lr.as<float2>(), count);
            hipLaunchKernelGGL(delay_hist_kernel, dim3((delay + 255) / 256), dim3(256), 0, s, hist[cur].as<float>(),
                               mpx.as<float>(), hist[cur ^ 1].as<float>(), delay, count);
            cur ^= 1;
        } else {
            hipLaunchKernelGGL(mono_to_stereo_kernel, g, b, 0, s, mpx.as<float>(), lr.as<float2>(), count);
        }
        SDRGPU_HIP(hipGetLastError());
        if (rds && rdsChain) {
            // the undelayed MPX as complex (the stereo path already holds it in cplx)
            const float2* c = cplx.as<float2>();
            if (!stereo) {
                SDRGPU_CHECK(rdsIn.ensure(sizeof(float2) * count));
                hipLaunchKernelGGL(real_to_complex_kernel, g, b, 0, s, mpx.as<float>(), rdsIn.as<float2>(), count);
                SDRGPU_HIP(hipGetLastError());
                c = rdsIn.as<float2>();
            }
            const int want = rdsChain->out_count(count);
            if (want < 0) return want;
            SDRGPU_CHECK(rdsOut.ensure(sizeof(float2) * (size_t)std::max(want, 1)));
            rdsN = rdsChain->run(c, count, rdsOut.p, s);
            if (rdsN < 0) return rdsN;
        }
        return audio->run(lr.p, count, out, s);
    }
};
}  // namespace sdrgpu

using namespace sdrgpu;

namespace {
int wrap_block(sdrgpu_block** h, Block* b, int rc) {
    if (rc < 0) { delete b; return rc; }
    *h = new sdrgpu_block{b};
    return SDRGPU_OK;
}
}  // namespace

extern "C" int sdrgpu_agc_create(sdrgpu_block** h, int device, int dtype, double setPoint, double attack, double decay,
                                 double maxGain, double maxOutputAmp, double initGain) {
    if (!h || (dtype != SDRGPU_F32 && dtype != SDRGPU_C64)) { set_error("agc_create: bad argument"); return SDRGPU_EARG; }
    auto* a = new AgcBlock();
    return wrap_block(h, a, a->setup(device, dtype, setPoint, attack, decay, maxGain, maxOutputAmp, initGain));
}
// AGC setters (agc.h:44-79): parameters change, the running amplitude / gain are kept
extern "C" int sdrgpu_agc_set_params(sdrgpu_block* h, double setPoint, double attack, double decay, double maxGain,
                                     double maxOutputAmp, double initGain) {
    auto* a = h ? dynamic_cast<AgcBlock*>(h->impl) : nullptr;
    if (!a) { set_error("not an AGC"); return SDRGPU_EARG; }
    a->p.setPoint = (float)setPoint;
    a->p.attack = (float)attack;
    a->p.invAttack = 1.0f - a->p.attack;
    a->p.decay = (float)decay;
    a->p.invDecay = 1.0f - a->p.decay;
    a->p.maxGain = (float)maxGain;
    a->p.maxOutputAmp = (float)maxOutputAmp;
    a->initGain = (float)initGain;
    return SDRGPU_OK;
}
extern "C" int sdrgpu_agc_set_enabled(sdrgpu_block* h, int enabled) {
    auto* a = h ? dynamic_cast<AgcBlock*>(h->impl) : nullptr;
    if (!a) { set_error("not an AGC"); return SDRGPU_EARG; }
    a->p.enabled = enabled ? 1 : 0;
    return SDRGPU_OK;
}
extern "C" int sdrgpu_agc_set_gain(sdrgpu_block* h, float gain) {
    auto* a = h ? dynamic_cast<AgcBlock*>(h->impl) : nullptr;
    if (!a) { set_error("not an AGC"); return SDRGPU_EARG; }
    return a->set_gain(gain);
}
extern "C" int sdrgpu_agc_get_gain(sdrgpu_block* h, float* gain) {
    auto* a = h ? dynamic_cast<AgcBlock*>(h->impl) : nullptr;
    if (!a || !gain) { set_error("agc_get_gain: bad argument"); return SDRGPU_EARG; }
    if (a->pending) { *gain = a->pendingGain; return SDRGPU_OK; }
    SDRGPU_SET_DEVICE(a->device);
    AgcState s;
    SDRGPU_HIP(hipDeviceSynchronize());   // (UI-rate query: waits for the block's queued work)
    SDRGPU_HIP(hipMemcpy(&s, a->state.p, sizeof(s), hipMemcpyDeviceToHost));
    *gain = s.gain;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_dc_blocker_create(sdrgpu_block** h, int device, int dtype, double rate) {
    if (!h || (dtype != SDRGPU_F32 && dtype != SDRGPU_C64)) { set_error("dc_blocker_create: bad argument"); return SDRGPU_EARG; }
    auto* d = new DcbBlock();
    return wrap_block(h, d, d->setup(device, dtype, rate));
}

// demod::AM<T> (am.h:27-49, 114-142): agcMode 0 OFF, 1 CARRIER, 2 AUDIO; stereo -> stereo_t out
extern "C" int sdrgpu_am_create(sdrgpu_block** h, int device, int agcMode, double bandwidth, double agcAttack,
                                double agcDecay, double dcBlockRate, double samplerate, int stereo) {
    if (!h || agcMode < 0 || agcMode > 2) { set_error("am_create: bad argument"); return SDRGPU_EARG; }
    Block* c = nullptr;
    int rc = chain_new(device, SDRGPU_C64, stereo ? SDRGPU_C64 : SDRGPU_F32, &c);
    if (rc < 0) return rc;
    if (agcMode == 1) {
        auto* a = new AgcBlock();
        rc = a->setup(device, SDRGPU_C64, 1.0, agcAttack, agcDecay, 10e6, 10.0, INFINITY);
        if (rc >= 0) rc = chain_append(c, a); else delete a;
    }
    if (rc >= 0) rc = chain_append(c, make_map(device, 0).release());
    if (rc >= 0) {
        auto* d = new DcbBlock();
        rc = d->setup(device, SDRGPU_F32, dcBlockRate);
        if (rc >= 0) rc = chain_append(c, d); else delete d;
    }
    if (rc >= 0 && agcMode != 1) {   // audioAgc runs unless CARRIER; enabled only for AUDIO
        auto* a = new AgcBlock();
        rc = a->setup(device, SDRGPU_F32, 1.0, agcAttack, agcDecay, 10e6, 10.0, INFINITY);
        if (rc >= 0) { a->p.enabled = agcMode == 2; rc = chain_append(c, a); } else delete a;
    }
    if (rc >= 0) {
        const double fc = bandwidth / 2.0;
        const int n = taps_low_pass(fc, fc * 0.1, samplerate, 0, nullptr);
        rc = n < 1 ? (n < 0 ? n : SDRGPU_EARG) : SDRGPU_OK;
        if (rc >= 0) {
            std::vector<float> t(n);
            taps_low_pass(fc, fc * 0.1, samplerate, 0, t.data());
            Block* f = make_fir_block(device, SDRGPU_F32, SDRGPU_F32, t.data(), n, 1, stereo != 0, &rc);
            if (rc >= 0) rc = chain_append(c, f); else delete f;
        }
    }
    return wrap_block(h, c, rc);
}

// demod::SSB<T> (ssb.h:27-105): mode 0 USB, 1 LSB, 2 DSB
extern "C" int sdrgpu_ssb_create(sdrgpu_block** h, int device, int mode, double bandwidth, double samplerate,
                                 int agcEnabled, double agcAttack, double agcDecay, int stereo) {
    if (!h || mode < 0 || mode > 2) { set_error("ssb_create: bad argument"); return SDRGPU_EARG; }
    Block* c = nullptr;
    int rc = chain_new(device, SDRGPU_C64, stereo ? SDRGPU_C64 : SDRGPU_F32, &c);
    if (rc < 0) return rc;
    const double tr = mode == 0 ? bandwidth / 2.0 : (mode == 1 ? -bandwidth / 2.0 : 0.0);   // getTranslation
    Block* x = make_xlator_block(device, hz_to_rads(tr, samplerate), &rc);
    if (rc >= 0) rc = chain_append(c, x); else delete x;
    if (rc >= 0) rc = chain_append(c, make_map(device, 1).release());
    if (rc >= 0) {
        auto* a = new AgcBlock();
        rc = a->setup(device, SDRGPU_F32, 1.0, agcAttack, agcDecay, 10e6, 10.0, INFINITY);
        if (rc >= 0) { a->p.enabled = agcEnabled ? 1 : 0; rc = chain_append(c, a); } else delete a;
    }
    if (rc >= 0 && stereo) rc = chain_append(c, make_map(device, 2).release());
    return wrap_block(h, c, rc);
}

// AGC access inside the AM / SSB chains: `which` 0 = the first AGC of the chain (AM carrier
// AGC in CARRIER mode, the SSB AGC), 1 = the last (AM audio AGC)
static AgcBlock* demod_agc(sdrgpu_block* h, int which) {
    if (!h || !h->impl) return nullptr;
    const int n = chain_size(h->impl);
    AgcBlock* found = nullptr;
    for (int i = 0; i < n; i++) {
        auto* a = dynamic_cast<AgcBlock*>(chain_kid(h->impl, i));
        if (a) {
            found = a;
            if (which == 0) break;
        }
    }
    return found;
}
extern "C" int sdrgpu_demod_agc_set_gain(sdrgpu_block* h, int which, float gain) {
    AgcBlock* a = demod_agc(h, which);
    if (!a) { set_error("demod has no AGC"); return SDRGPU_ESTATE; }
    return a->set_gain(gain);
}
extern "C" int sdrgpu_demod_agc_get_gain(sdrgpu_block* h, int which, float* gain) {
    AgcBlock* a = demod_agc(h, which);
    if (!a) { set_error("demod has no AGC"); return SDRGPU_ESTATE; }
    sdrgpu_block tmp{a};
    return sdrgpu_agc_get_gain(&tmp, gain);
}
extern "C" int sdrgpu_demod_agc_set_enabled(sdrgpu_block* h, int which, int enabled) {
    AgcBlock* a = demod_agc(h, which);
    if (!a) { set_error("demod has no AGC"); return SDRGPU_ESTATE; }
    a->p.enabled = enabled ? 1 : 0;
    return SDRGPU_OK;
}
extern "C" int sdrgpu_demod_agc_set_attack_decay(sdrgpu_block* h, double attack, double decay) {
    if (!h || !h->impl) { set_error("null block handle"); return SDRGPU_EARG; }
    const int n = chain_size(h->impl);
    int found = 0;
    for (int i = 0; i < n; i++) {
        if (auto* a = dynamic_cast<AgcBlock*>(chain_kid(h->impl, i))) {
            a->p.attack = (float)attack;
            a->p.invAttack = 1.0f - a->p.attack;
            a->p.decay = (float)decay;
            a->p.invDecay = 1.0f - a->p.decay;
            found++;
        }
    }
    if (!found) { set_error("demod has no AGC"); return SDRGPU_ESTATE; }
    return SDRGPU_OK;
}
extern "C" int sdrgpu_dc_blocker_set_rate(sdrgpu_block* h, double rate) {
    DcbBlock* d = h ? dynamic_cast<DcbBlock*>(h->impl) : nullptr;
    if (!d && h && h->impl) {   // the AM chain's DC blocker
        for (int i = 0, n = chain_size(h->impl); i < n && !d; i++) d = dynamic_cast<DcbBlock*>(chain_kid(h->impl, i));
    }
    if (!d) { set_error("no DC blocker"); return SDRGPU_ESTATE; }
    d->rate = (float)rate;
    return SDRGPU_OK;
}

// demod::BroadcastFM (broadcast_fm.h), stereo decoder and RDS branch included
extern "C" int sdrgpu_broadcast_fm_create(sdrgpu_block** h, int device, double deviation, double samplerate, int stereo,
                                          int lowPass) {
    if (!h || !(samplerate > 0)) { set_error("broadcast_fm_create: bad argument"); return SDRGPU_EARG; }
    auto* w = new BroadcastFmBlock();
    return wrap_block(h, w, w->setup(device, deviation, samplerate, stereo != 0, lowPass != 0));
}
extern "C" int sdrgpu_broadcast_fm_set_rds(sdrgpu_block* h, int enabled) {   // setRDSOut (broadcast_fm.h:121-127)
    auto* w = h ? dynamic_cast<BroadcastFmBlock*>(h->impl) : nullptr;
    if (!w) { set_error("not a broadcast_fm block"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(w->device);
    return w->set_rds(enabled != 0);
}
// RDS samples (complex_t at 5 kS/s) of the last process call: device pointer and count
extern "C" int sdrgpu_broadcast_fm_rds_dev(sdrgpu_block* h, const void** out, int* n) {
    auto* w = h ? dynamic_cast<BroadcastFmBlock*>(h->impl) : nullptr;
    if (!w) { set_error("not a broadcast_fm block"); return SDRGPU_EARG; }
    if (out) *out = w->rdsOut.p;
    if (n) *n = w->rds ? w->rdsN : 0;
    return w->rds ? w->rdsN : 0;
}
extern "C" int sdrgpu_broadcast_fm_read_rds(sdrgpu_block* h, void* out, int max) {   // host copy (waits for the block)
    auto* w = h ? dynamic_cast<BroadcastFmBlock*>(h->impl) : nullptr;
    if (!w || (!out && max > 0)) { set_error("broadcast_fm_read_rds: bad argument"); return SDRGPU_EARG; }
    const int n = std::min(max, w->rds ? w->rdsN : 0);
    if (n <= 0) return 0;
    SDRGPU_SET_DEVICE(w->device);
    SDRGPU_HIP(hipDeviceSynchronize());
    SDRGPU_HIP(hipMemcpy(out, w->rdsOut.p, sizeof(float2) * (size_t)n, hipMemcpyDeviceToHost));
    return n;
}

// filter::Deemphasis<T> (deephasis.h): dtype F32 (float) or C64 (stereo_t)
extern "C" int sdrgpu_deemphasis_create(sdrgpu_block** h, int device, int dtype, double tau, double samplerate) {
    if (!h || (dtype != SDRGPU_F32 && dtype != SDRGPU_C64) || !(samplerate > 0)) { set_error("deemphasis_create: bad argument"); return SDRGPU_EARG; }
    auto* d = new DeempBlock();
    return wrap_block(h, d, d->setup(device, dtype, tau, samplerate));
}
extern "C" int sdrgpu_deemphasis_set(sdrgpu_block* h, double tau, double samplerate) {   // setTau / setSamplerate
    auto* d = h ? dynamic_cast<DeempBlock*>(h->impl) : nullptr;
    if (!d || !(samplerate > 0)) { set_error("not a deemphasis block"); return SDRGPU_EARG; }
    d->set_alpha(tau, samplerate);
    return SDRGPU_OK;
}
