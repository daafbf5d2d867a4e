// Internal declarations shared by the libsdrgpu translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include "../../include/sdrgpu.h"

namespace sdrgpu {
bool host_pinned(const void* p, size_t bytes);   // inside a sdrgpu_host_register range (capi.cpp)

void set_error(const char* fmt, ...);

// Kernel-selection / tile-shape overrides for A/B measurements (SDRGPU_FIR_*, SDRGPU_FFT_*,
// SDRGPU_CHAN_*). They are read only when SDRGPU_TUNING=1 is set as well, so a stray variable
// in a deployment cannot change the kernels that run. Every override selects another exact
// kernel or tile shape of the same transform (none of them trades correctness for speed).
const char* tuning_env(const char* name);

#define SDRGPU_HIP(call)                                                              \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            ::sdrgpu::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorName(e_),  \
                                __FILE__, __LINE__);                                  \
            return SDRGPU_EHIP;                                                       \
        }                                                                             \
    } while (0)

// Select a device, reporting SDRGPU_ENODEV (not a generic HIP error) when there is no
// GPU or the index is out of range.
#define SDRGPU_SET_DEVICE(dev)                                                        \
    do {                                                                              \
        int n_ = 0, d_ = (dev);                                                       \
        if (hipGetDeviceCount(&n_) != hipSuccess || d_ < 0 || d_ >= n_) {             \
            ::sdrgpu::set_error("HIP device %d not available (%d devices)", d_, n_);  \
            return SDRGPU_ENODEV;                                                     \
        }                                                                             \
        SDRGPU_HIP(hipSetDevice(d_));                                                 \
    } while (0)

#define SDRGPU_CHECK(call)                 \
    do {                                   \
        int r_ = (call);                   \
        if (r_ < 0) return r_;             \
    } while (0)

// Device buffer owned by a handle; grows on demand (never inside a capture).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want);
    void release();
    ~DevBuf() { release(); }
    template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};

// Pinned host staging for the host-pointer (drop-in) call style.
struct PinnedBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want);
    ~PinnedBuf();
    template <typename T> const T* as_const() const { return reinterpret_cast<const T*>(p); }
};

inline size_t esize(int dtype) { return dtype == SDRGPU_C64 ? 8 : 4; }

// A handle's device state is rewritten by every call (NCO coarse table, history / quadrature
// ping-pong buffers, FFT scratch), so calls must not overlap. Calls on one stream are ordered by
// the stream: a handle driven from one stream (the common case) pays nothing. The first call on
// another stream cannot know whether the previous stream still exists (a caller may destroy a
// stream after its call), so it waits with a device-wide synchronise -- the one ordering that
// needs no handle on that stream -- and the handle switches to multi-stream mode: from then on
// every entry point records `ev` on its own stream when it has enqueued its work (done), and a
// call on another stream waits for that event (follow). The event always belongs to a stream that
// was live when it was recorded, and the new stream waits for exactly the previous call's work.
// (Recording on every call costs ~2.7 us per entry point in a device-bound call sequence, which is
// why a single-stream handle does not.) Handles driven only through another handle (a front
// end's VFOs and FFT plan) skip this: the owner orders them.
struct StreamOrder {
    hipStream_t last = nullptr;   // stream of the previous call
    hipEvent_t ev = nullptr;      // multi-stream mode: recorded on `last` at the end of the previous call
    bool multi = false;
    int follow(hipStream_t s);
    int done(hipStream_t s);
    ~StreamOrder();
};
// follow() at the start of an entry point, done() when the scope ends
struct OrderScope {
    StreamOrder& o;
    hipStream_t s;
    OrderScope(StreamOrder& o_, hipStream_t s_) : o(o_), s(s_) {}
    ~OrderScope() { (void)o.done(s); }
};

// ---- host-side design (host_design.cpp) -----------------------------------
double window_value(int type, double n, double N);
int create_window(int type, float* buffer, int size, int centered);
int taps_windowed_sinc(int count, double omega, double norm, float* out);
int taps_low_pass(double cutoff, double tw, double fs, int odd, float* out);
int taps_high_pass(double cutoff, double tw, double fs, int odd, float* out);
int taps_band_pass_f(double start, double stop, double tw, double fs, int odd, float* out);
int taps_band_pass_c(double start, double stop, double tw, double fs, int odd, float* out);
int decim_plan(int ratio, int* decims, int* ntaps, const float** taps);
double hz_to_rads(double f, double fs);
double xlator_effective_omega(double offsetRad);

// Double-double phase accumulator: keeps (w * n) mod 2pi to ~1e-16 rad over
// arbitrarily long streams (the NCO origin of the next call).
struct PhaseAcc {
    double hi = 0.0, lo = 0.0;
    void reset() { hi = lo = 0.0; }
    void advance(double w, long long n);
    double value() const { return hi + lo; }
};

// ---- blocks ------------------------------------------------------------------
struct Block {
    int device = 0;
    int in_dtype = SDRGPU_C64, out_dtype = SDRGPU_C64;
    hipStream_t own = nullptr;
    PinnedBuf pin_in, pin_out;
    DevBuf dev_in, dev_out;
    StreamOrder order;   // entry points (process / process_dev) only; sub-blocks share the caller's stream
    virtual ~Block();
    int init_stream();
    // exact number of outputs the next process() of `count` inputs yields
    virtual int out_count(int count) = 0;
    // asynchronous device-side processing on `s`; returns the output count
    virtual int run(const void* in, int count, void* out, hipStream_t s) = 0;
    virtual int reset() = 0;
};

// kernels (fir.hip / fft.hip)
struct FirState;   // defined in fir.hip

}  // namespace sdrgpu

struct sdrgpu_block {
    sdrgpu::Block* impl;
};
struct sdrgpu_fft;

namespace sdrgpu {
// entry points without the cross-stream ordering, for a handle owned by another handle
int block_run_owned(sdrgpu_block* h, const void* in, int count, void* out, hipStream_t s);
int fft_execute_owned(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out, hipStream_t s);
// The 64k plan's transform: 1 = the one-pass kernel (the batch default), 0 = the two-pass launches
// (the front end's: its per-block calls hold a few frames, where two short launches of 8 workgroups
// per frame finish sooner than one launch of 2 long ones, and its split path reads the straddling
// frame in place). Returns SDRGPU_EARG for a null handle.
int fft_set_onepass(sdrgpu_fft* h, int onepass);
// Up to two device copies of complex samples done by spare workgroups of another launch.
struct SideCopy {
    float2* dst[2];
    const float2* src[2];
    int n[2];
    int count;
};
// Frames f = 0 .. frames - 1 of a stream split over two buffers: frame 0 is [head[0, nh) ||
// body[0, nz - nh)], frame f >= 1 starts at body + f * stride - nh. The pass-A launch reads frame 0
// from both buffers (no stitch copy) and runs `side` with spare workgroups. Returns frames, or
// SDRGPU_ESTATE when the plan has no such path (the caller then stitches and calls fft_execute_owned).
// vfo (non-null): a prepared VfoStage1 (fir_rows.h) of vfoBlock that the pass-A launch also runs
// (its segments, its history workgroup); the pass-B launch then carries the VFO's tail workgroups
// where its later stages have that form, else they run after it. The VFO's output count goes to
// *vfoN. Returns SDRGPU_ESTATE (nothing launched, the VFO untouched) where the plan has no split path.
struct VfoStage1;
int fft_execute_split(sdrgpu_fft* h, const float2* head, int nh, const float2* body, long long stride, int frames, float* out,
                      const SideCopy& side, hipStream_t s, const VfoStage1* vfo = nullptr, sdrgpu_block* vfoBlock = nullptr,
                      void* vfoOut = nullptr, int* vfoN = nullptr);
// fp64-interior spectrum (fft64.hip): the opt-in parity mode behind sdrgpu_fft_set_precision
struct Fft64Plan;
int fft64_create(Fft64Plan** out, int N);
void fft64_destroy(Fft64Plan* p);
int fft64_execute(Fft64Plan* p, const float2* in, long long stride, int frames, const float* win, int nz, float* out,
                  hipStream_t s);
}  // namespace sdrgpu
