// Device-resident IQ front end: the MI355X replacement of IQFrontEnd's data path
// (signal_path/iq_frontend.cpp:15-52, 115-249) and of the host fan-out it runs on
// (buffer/frame_buffer.h SampleFrameBuffer -> routing/splitter.h Splitter -> one memcpy per
// VFO + buffer/reshaper.h Reshaper -> FFT handler). SURVEY.md §8f rank 1.
//
// One push of a source block does, all on one HIP stream:
//   [H2D of the raw block] -> ingest conversion (u8/i16/i24/i32/f64/i8 or complex float,
//   file_source/src/main.cpp:361-542) -> [PowerDecimator] -> [DCBlocker<complex_t>]
//   -> [Conjugate] -> every VFO (RxVFO) reads the block in place, and the spectrum frames
//   whose samples are complete are transformed straight out of the block.
// Framing is the Reshaper's keep/skip (reshaper.h:100-127, keep = nz, skip from
// genReshapeParams, iq_frontend.h:56-60): frame j covers samples [j*(nz+skip), j*(nz+skip)+nz)
// of the preprocessed stream. Only the (at most one) frame straddling two pushes is
// stitched, from a device tail buffer of < nz samples; every other frame is read in place,
// so each sample crosses PCIe once and is read from HBM once per consumer (a push with a
// straddling frame and at most 4 more copies those behind it, so one transform launch pair
// covers the push).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <vector>
#include "sdrgpu_internal.h"
#include "fir_rows.h"

namespace sdrgpu {
__global__ void conjugate_kernel(float2* __restrict__ x, int n) {   // math/conjugate.h
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i].y = -x[i].y;
}
}  // namespace sdrgpu

using namespace sdrgpu;

namespace {
struct VfoSlot {
    sdrgpu_block* vfo = nullptr;
    DevBuf out;
    PinnedBuf pin;
    int n = 0;
    PinnedBuf res[2];   // pipelined call style: this VFO's output of the block in result slot k
    int resN[2] = {0, 0};
};
// One in-flight block of the pipelined host call style (sdrgpu_frontend_submit / collect).
struct PipeSlot {
    PinnedBuf stage;             // the host block, when the caller's buffer is not registered
    DevBuf raw;                  // its device copy
    PinnedBuf rows, iq;          // results: dB rows, preprocessed IQ
    int nrows = 0, niq = 0;
    long long ticket = -1;       // block in this slot (-1: free)
    bool collected = true;
    hipEvent_t h2d = nullptr;    // H2D done (staging reusable)
    hipEvent_t consumed = nullptr;   // the block's kernels have read `raw`
    hipEvent_t ready = nullptr;      // results are in the pinned buffers
};
const int kConvSize[] = {1, 2, 3, 4, 8, 1, 4};   // bytes per real value of SDRGPU_CONV_U8..F32
}  // namespace

struct sdrgpu_frontend {
    int device = 0;
    double sampleRate = 0, fftRate = 0, effSr = 0;
    int decim = 1, fftSize = 0, window = 0, nz = 0, skip = 0;
    bool dcBlocking = false, invertIQ = false;
    hipStream_t s = nullptr;
    StreamOrder order;        // tails, stitch and VFO state are per front end: serialise across streams
    const float2* lastIQ = nullptr;   // the last push's preprocessed block (device) and its length
    int lastIQn = 0;
    sdrgpu_block* decimB = nullptr;
    sdrgpu_block* dcb = nullptr;
    sdrgpu_fft* fft = nullptr;
    PinnedBuf pin, pinSpec;
    DevBuf raw, conv, pre, tail[2], stitch, spectra;
    int curTail = 0;
    long long total = 0;      // preprocessed samples seen before this push
    long long nextFrame = 0;  // absolute start of the next spectrum frame
    int tailLen = 0;          // device tail = samples [total - tailLen, total), all >= nextFrame
    int nSpec = 0;
    int nextVfoId = 1;
    std::map<int, VfoSlot> vfos;
    long long stride() const { return (long long)nz + skip; }
    // pipelined host call style: a copy stream for the H2D of block k + 1 while block k computes
    hipStream_t cs = nullptr;
    PipeSlot pipe[2];
    long long nextTicket = 0;
    int split = 1;   // fft_execute_split for pushes that complete frames (else stitch copies)
    // the first VFO's first stage inside that pass-A launch 
    int fuse = 1;
};

static void destroy_parts(sdrgpu_frontend* f) {
    if (f->decimB) sdrgpu_block_destroy(f->decimB);
    if (f->dcb) sdrgpu_block_destroy(f->dcb);
    if (f->fft) sdrgpu_fft_destroy(f->fft);
    f->decimB = f->dcb = nullptr;
    f->fft = nullptr;
}

// IQFrontEnd::updateFFTPath / updateFFTSize (iq_frontend.cpp:251-296): reshaper keep/skip and plan
static int fe_update_fft(sdrgpu_frontend* f) {
    int skip = 0, nz = 0;
    sdrgpu_gen_reshape_params(f->effSr, f->fftSize, f->fftRate, &skip, &nz);
    if (nz < 1 || skip < 0) { set_error("frontend: bad FFT framing (size %d, rate %g)", f->fftSize, f->fftRate); return SDRGPU_EARG; }
    if (f->fft) sdrgpu_fft_destroy(f->fft);
    f->fft = nullptr;
    SDRGPU_CHECK(sdrgpu_fft_create(&f->fft, f->device, f->fftSize, nz, f->window));
    SDRGPU_CHECK(fft_set_onepass(f->fft, 0));   // per-block calls: the two-pass launches (sdrgpu_internal.h)
    f->nz = nz;
    f->skip = skip;
    // the reshaper restarts on a path update: the next frame starts at the next sample
    f->nextFrame = f->total;
    f->tailLen = 0;
    return SDRGPU_OK;
}

// preproc chain of IQFrontEnd::init (iq_frontend.cpp:29-39)
static int fe_build_preproc(sdrgpu_frontend* f) {
    if (f->decimB) sdrgpu_block_destroy(f->decimB);
    if (f->dcb) sdrgpu_block_destroy(f->dcb);
    f->decimB = f->dcb = nullptr;
    f->effSr = f->sampleRate / f->decim;
    if (f->decim > 1) SDRGPU_CHECK(sdrgpu_power_decimator_create(&f->decimB, f->device, SDRGPU_C64, f->decim));
    if (f->dcBlocking) SDRGPU_CHECK(sdrgpu_dc_blocker_create(&f->dcb, f->device, SDRGPU_C64, 50.0 / f->effSr));   // genDCBlockRate
    return SDRGPU_OK;
}

extern "C" int sdrgpu_frontend_create(sdrgpu_frontend** out, int device, double sampleRate, int decimRatio, int dcBlocking,
                                      int fftSize, double fftRate, int windowType) {
    if (!out || !(sampleRate > 0) || decimRatio < 1 || !(fftRate > 0)) { set_error("frontend_create: bad argument"); return SDRGPU_EARG; }
    *out = nullptr;
    SDRGPU_SET_DEVICE(device);
    auto* f = new sdrgpu_frontend();
    f->device = device;
    f->sampleRate = sampleRate;
    f->decim = decimRatio;
    f->dcBlocking = dcBlocking != 0;
    f->fftSize = fftSize;
    f->fftRate = fftRate;
    f->window = windowType;
    int rc = hipStreamCreateWithFlags(&f->s, hipStreamNonBlocking) == hipSuccess ? SDRGPU_OK : SDRGPU_EHIP;
    if (rc < 0) set_error("frontend_create: hipStreamCreate failed");
    if (rc >= 0) rc = fe_build_preproc(f);
    if (rc >= 0) rc = fe_update_fft(f);
    if (rc < 0) {
        destroy_parts(f);
        if (f->s) (void)hipStreamDestroy(f->s);
        delete f;
        return rc;
    }
    *out = f;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_frontend_destroy(sdrgpu_frontend* f) {
    if (!f) return SDRGPU_OK;
    (void)hipSetDevice(f->device);
    if (f->cs) (void)hipStreamSynchronize(f->cs);
    if (f->s) (void)hipStreamSynchronize(f->s);
    for (auto& [id, v] : f->vfos) sdrgpu_block_destroy(v.vfo);
    destroy_parts(f);
    for (auto& ps : f->pipe)
        for (hipEvent_t e : {ps.h2d, ps.consumed, ps.ready})
            if (e) (void)hipEventDestroy(e);
    if (f->cs) (void)hipStreamDestroy(f->cs);
    if (f->s) (void)hipStreamDestroy(f->s);
    delete f;
    return SDRGPU_OK;
}

#define NEED_FE(f) do { if (!(f)) { set_error("null frontend"); return SDRGPU_EARG; } } while (0)

// setSampleRate / setDecimation / setDCBlocking (iq_frontend.cpp:54-106): VFOs follow the new rate
extern "C" int sdrgpu_frontend_configure(sdrgpu_frontend* f, double sampleRate, int decimRatio, int dcBlocking) {
    NEED_FE(f);
    if (!(sampleRate > 0) || decimRatio < 1) { set_error("frontend_configure: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(f->device);
    if (f->cs) SDRGPU_HIP(hipStreamSynchronize(f->cs));
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    f->sampleRate = sampleRate;
    f->decim = decimRatio;
    f->dcBlocking = dcBlocking != 0;
    SDRGPU_CHECK(fe_build_preproc(f));
    SDRGPU_CHECK(fe_update_fft(f));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_frontend_set_invert_iq(sdrgpu_frontend* f, int enabled) {
    NEED_FE(f);
    f->invertIQ = enabled != 0;
    return SDRGPU_OK;
}
// setFFTSize / setFFTRate / setFFTWindow (iq_frontend.cpp:173-186)
extern "C" int sdrgpu_frontend_set_fft(sdrgpu_frontend* f, int fftSize, double fftRate, int windowType) {
    NEED_FE(f);
    if (!(fftRate > 0)) { set_error("frontend_set_fft: bad rate"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(f->device);
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    f->fftSize = fftSize;
    f->fftRate = fftRate;
    f->window = windowType;
    return fe_update_fft(f);
}
extern "C" int sdrgpu_frontend_framing(sdrgpu_frontend* f, int* nz, int* skip, double* effectiveSampleRate) {
    NEED_FE(f);
    if (nz) *nz = f->nz;
    if (skip) *skip = f->skip;
    if (effectiveSampleRate) *effectiveSampleRate = f->effSr;
    return SDRGPU_OK;
}

// addVFO / removeVFO (iq_frontend.cpp:115-160): an RxVFO fed from the device block in place
extern "C" int sdrgpu_frontend_add_vfo(sdrgpu_frontend* f, int* id, double outSampleRate, double bandwidth, double offset) {
    NEED_FE(f);
    if (!id) { set_error("frontend_add_vfo: null id"); return SDRGPU_EARG; }
    VfoSlot v;
    SDRGPU_CHECK(sdrgpu_rxvfo_create(&v.vfo, f->device, f->effSr, outSampleRate, bandwidth, offset));
    *id = f->nextVfoId++;
    f->vfos[*id] = std::move(v);
    return SDRGPU_OK;
}
extern "C" int sdrgpu_frontend_remove_vfo(sdrgpu_frontend* f, int id) {
    NEED_FE(f);
    auto it = f->vfos.find(id);
    if (it == f->vfos.end()) { set_error("frontend: no VFO %d", id); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(f->device);
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    sdrgpu_block_destroy(it->second.vfo);
    f->vfos.erase(it);
    return SDRGPU_OK;
}
extern "C" int sdrgpu_frontend_set_vfo_offset(sdrgpu_frontend* f, int id, double offset) {
    NEED_FE(f);
    auto it = f->vfos.find(id);
    if (it == f->vfos.end()) { set_error("frontend: no VFO %d", id); return SDRGPU_EARG; }
    return sdrgpu_rxvfo_set_offset(it->second.vfo, offset);
}

// up to four device-to-device copies of complex samples in one launch (replaces as many
// hipMemcpyAsync calls, each of which is a copy-kernel launch of its own)
struct CopySegArgs {
    float2* dst[8];
    const float2* src[8];
    int n[8];
    int count;
};
__global__ void copy_segs_kernel(CopySegArgs a) {
    const int seg = blockIdx.y;
    if (seg >= a.count) return;
    const int n = a.n[seg];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a.dst[seg][i] = a.src[seg][i];
}
struct CopySegs {
    CopySegArgs a{};
    int maxN = 0;
    void add(float2* d, const float2* s, int n) {
        if (n <= 0) return;
        a.dst[a.count] = d; a.src[a.count] = s; a.n[a.count] = n;
        a.count++;
        maxN = std::max(maxN, n);
    }
    int launch(hipStream_t s) {
        if (!a.count) return SDRGPU_OK;
        const int bx = std::min((maxN + 255) / 256, 256);
        hipLaunchKernelGGL(copy_segs_kernel, dim3(bx, a.count), dim3(256), 0, s, a);
        SDRGPU_HIP(hipGetLastError());
        return SDRGPU_OK;
    }
};

// Core of a push: the preprocessed block `x` (m samples, device) -> VFOs + spectrum frames.
static int fe_consume(sdrgpu_frontend* f, const float2* x, int m, hipStream_t s) {
    // frames with start s_j = nextFrame + j*stride and s_j + nz <= total + m
    const long long T = f->total, st = f->stride();
    int nf = 0;
    if (T + m >= f->nextFrame + f->nz) nf = (int)((T + m - f->nextFrame - f->nz) / st) + 1;
    // The first VFO whose first stage is the row decimator runs that stage inside the spectrum's
    // pass-A launch below (one launch fewer per block, DESIGN.md §3 per call); the others, and that
    // one when the spectrum has no such launch, run on their own.
    VfoStage1 vst;
    VfoSlot* fused = nullptr;
    for (auto& [id, v] : f->vfos) {
        const int want = sdrgpu_block_out_count(v.vfo, m);
        if (want < 0) return want;
        SDRGPU_CHECK(v.out.ensure(sizeof(float2) * (size_t)std::max(want, 1)));
        if (!fused && f->fuse && f->split && nf > 0 && m > 0) {
            const int r = vfo_stage1_prepare(v.vfo, x, m, &vst);
            if (r < 0) return r;
            if (r) {
                fused = &v;
                continue;
            }
        }
        const int n = m > 0 ? block_run_owned(v.vfo, x, m, v.out.p, s) : 0;
        if (n < 0) return n;
        v.n = n;
    }
    auto run_unfused = [&]() -> int {   // the prepared VFO on its own (no split launch took it)
        if (!fused) return SDRGPU_OK;
        const int n = block_run_owned(fused->vfo, x, m, fused->out.p, s);
        if (n < 0) return n;
        fused->n = n;
        return SDRGPU_OK;
    };
    SDRGPU_CHECK(f->spectra.ensure(sizeof(float) * (size_t)std::max(nf, 1) * f->fftSize));
    float* spec = f->spectra.as<float>();
    if (nf > 0 && f->split) {
        // One launch pair and no copy launch: pass A reads the frame straddling the previous push
        // from the device tail and this block in place (fft_execute_split), and its spare
        // workgroups copy the new tail (samples after the last frame: all in this block, since a
        // frame completed) into the other tail buffer. 45 -> see DESIGN.md §3 per call.
        const long long nextAfterS = f->nextFrame + (long long)nf * st, endS = T + m;
        const int head = f->nextFrame < T ? (int)(T - f->nextFrame) : 0;
        const float2* body = head > 0 ? x : x + (f->nextFrame - T);
        SideCopy side{};
        int newLenS = 0, nbS = f->curTail;
        if (nextAfterS < endS) {
            newLenS = (int)(endS - nextAfterS);
            nbS = f->curTail ^ 1;
            SDRGPU_CHECK(f->tail[0].ensure(sizeof(float2) * f->nz));
            SDRGPU_CHECK(f->tail[1].ensure(sizeof(float2) * f->nz));
            side.dst[0] = f->tail[nbS].as<float2>();
            side.src[0] = x + (m - newLenS);
            side.n[0] = newLenS;
            side.count = 1;
        }
        int vn = 0;
        const int rc = fft_execute_split(f->fft, head > 0 ? f->tail[f->curTail].as<float2>() : nullptr, head, body, st, nf,
                                         spec, side, s, fused ? &vst : nullptr, fused ? fused->vfo : nullptr,
                                         fused ? fused->out.p : nullptr, &vn);
        if (rc >= 0) {
            if (fused) fused->n = vn;
            f->nSpec = nf;
            f->nextFrame = nextAfterS;
            f->curTail = nbS;
            f->tailLen = newLenS;
            f->total = endS;
            return nf;
        }
        if (rc != SDRGPU_ESTATE) return rc;   // (ESTATE: this plan has no split path; stitch below)
    }
    SDRGPU_CHECK(run_unfused());   // (no split launch: the prepared VFO runs on its own)
    int done = 0;
    // the stitched straddling frame and the new tail are built by one copy launch (up to four
    // device segments) before the spectrum: both read only the old tail and this block
    CopySegs cs;
    // with a straddling frame, up to kGatherFrames in-block frames are copied behind it in the
    // same copy launch, so one transform launch pair covers the call (a reference-size block
    // has 1-2 frames: one pass-A / pass-B pair instead of two, ~10 us per call)
    constexpr int kGatherFrames = 4;
    const bool straddle = nf > 0 && f->nextFrame < T;
    const int gathered = (straddle && nf - 1 <= kGatherFrames) ? nf - 1 : 0;
    if (straddle) {
        // the one frame straddling the previous push: [tail (tailLen) || x[0 : nz - tailLen])
        const int head = (int)(T - f->nextFrame);   // == tailLen
        SDRGPU_CHECK(f->stitch.ensure(sizeof(float2) * (size_t)f->nz * (1 + gathered)));
        cs.add(f->stitch.as<float2>(), f->tail[f->curTail].as<float2>(), head);
        cs.add(f->stitch.as<float2>() + head, x, f->nz - head);
        for (int j = 1; j <= gathered; j++)
            cs.add(f->stitch.as<float2>() + (size_t)j * f->nz, x + (f->nextFrame + j * st - T), f->nz);
    }
    const long long nextAfter = f->nextFrame + (long long)nf * st;
    // new tail: samples [nextAfter, T + m) (fewer than nz), from the old tail and/or this block
    const long long end = T + m;
    int newLen = 0, nb = f->curTail;
    if (nextAfter < end) {
        newLen = (int)(end - nextAfter);
        nb = f->curTail ^ 1;
        SDRGPU_CHECK(f->tail[0].ensure(sizeof(float2) * f->nz));
        SDRGPU_CHECK(f->tail[1].ensure(sizeof(float2) * f->nz));
        float2* dst = f->tail[nb].as<float2>();
        int fromOld = 0;
        if (nextAfter < T) {   // keep part of the old tail (no frame completed)
            fromOld = (int)(T - nextAfter);
            cs.add(dst, f->tail[f->curTail].as<float2>() + (f->tailLen - fromOld), fromOld);
        }
        const long long fromBlock = newLen - fromOld;
        if (fromBlock > 0) cs.add(dst + fromOld, x + (m - fromBlock), (int)fromBlock);
    }
    SDRGPU_CHECK(cs.launch(s));
    if (straddle) {
        SDRGPU_CHECK(fft_execute_owned(f->fft, f->stitch.p, f->nz, 1 + gathered, spec, s));
        done = 1 + gathered;
    }
    if (nf > done) {   // frames entirely inside this block, read in place with the reshaper's stride
        const long long first = f->nextFrame + done * st - T;
        SDRGPU_CHECK(fft_execute_owned(f->fft, x + first, st, nf - done, spec + (size_t)done * f->fftSize, s));
    }
    f->nSpec = nf;
    f->nextFrame = nextAfter;
    f->curTail = nb;
    f->tailLen = newLen;
    f->total = end;
    return nf;
}

// preprocessing of a converted full-rate block in `conv` (n samples) -> f->pre / returned pointer
static int fe_preproc(sdrgpu_frontend* f, const float2* in, int n, hipStream_t s, const float2** outp) {
    const float2* x = in;
    int m = n;
    if (f->decimB) {
        const int want = sdrgpu_block_out_count(f->decimB, n);
        if (want < 0) return want;
        SDRGPU_CHECK(f->pre.ensure(sizeof(float2) * (size_t)std::max(want, 1)));
        m = n > 0 ? block_run_owned(f->decimB, x, n, f->pre.p, s) : 0;
        if (m < 0) return m;
        x = f->pre.as<float2>();
    }
    if ((f->dcb || f->invertIQ) && x == in) {   // in-place stages need a private copy of the caller's block
        SDRGPU_CHECK(f->pre.ensure(sizeof(float2) * (size_t)std::max(m, 1)));
        SDRGPU_HIP(hipMemcpyAsync(f->pre.p, x, sizeof(float2) * m, hipMemcpyDeviceToDevice, s));
        x = f->pre.as<float2>();
    }
    if (f->dcb && m > 0) {
        const int r = block_run_owned(f->dcb, x, m, (void*)x, s);
        if (r < 0) return r;
    }
    if (f->invertIQ && m > 0) {
        hipLaunchKernelGGL(conjugate_kernel, dim3((m + 255) / 256), dim3(256), 0, s, (float2*)x, m);
        SDRGPU_HIP(hipGetLastError());
    }
    *outp = x;
    return m;
}

// Device-resident block (complex float, or raw `kind` samples), caller stream (NULL = own).
// Returns the number of spectrum rows produced; rows and VFO outputs stay on the device.
extern "C" int sdrgpu_frontend_push_dev(sdrgpu_frontend* f, const void* in, int count, int kind, void* stream) {
    NEED_FE(f);
    if (count < 0 || (count > 0 && !in) || kind < -1 || kind > SDRGPU_CONV_F32) { set_error("frontend_push: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(f->device);
    hipStream_t s = stream ? (hipStream_t)stream : f->s;
    SDRGPU_CHECK(f->order.follow(s));
    OrderScope od(f->order, s);
    const float2* x = (const float2*)in;
    if (kind >= 0 && count > 0) {
        SDRGPU_CHECK(f->conv.ensure(sizeof(float2) * count));
        SDRGPU_CHECK(sdrgpu_convert_dev(f->device, kind, in, 2LL * count, f->conv.as<float>(), s));
        x = f->conv.as<float2>();
    }
    const float2* p = nullptr;
    const int m = fe_preproc(f, x, count, s, &p);
    if (m < 0) return m;
    f->lastIQ = p;
    f->lastIQn = m;
    return fe_consume(f, p, m, s);
}

// Host block (the drop-in call style): one H2D of the raw bytes, then as push_dev on the
// frontend's stream; synchronises so the host can read the results.
extern "C" int sdrgpu_frontend_push(sdrgpu_frontend* f, const void* in, int count, int kind) {
    NEED_FE(f);
    if (count < 0 || (count > 0 && !in) || kind < -1 || kind > SDRGPU_CONV_F32) { set_error("frontend_push: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(f->device);
    const size_t bytes = (size_t)count * (kind < 0 ? sizeof(float2) : 2 * kConvSize[kind]);
    if (count > 0) {
        SDRGPU_CHECK(f->pin.ensure(bytes));
        SDRGPU_CHECK(f->raw.ensure(bytes));
        SDRGPU_HIP(hipStreamSynchronize(f->s));   // the staging buffer is reused
        std::memcpy(f->pin.p, in, bytes);
        SDRGPU_HIP(hipMemcpyAsync(f->raw.p, f->pin.p, bytes, hipMemcpyHostToDevice, f->s));
    }
    const int nf = sdrgpu_frontend_push_dev(f, count > 0 ? f->raw.p : nullptr, count, kind, f->s);
    if (nf < 0) return nf;
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    return nf;
}

// results of the last push: device pointers (push_dev) or host copies (drop-in)
extern "C" int sdrgpu_frontend_spectra_dev(sdrgpu_frontend* f, const float** rows, int* nrows) {
    NEED_FE(f);
    if (rows) *rows = f->spectra.as<float>();
    if (nrows) *nrows = f->nSpec;
    return f->fftSize;
}
extern "C" int sdrgpu_frontend_read_spectra(sdrgpu_frontend* f, float* out, int maxRows) {
    NEED_FE(f);
    const int n = std::min(maxRows, f->nSpec);
    if (n <= 0) return 0;
    SDRGPU_SET_DEVICE(f->device);
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    SDRGPU_HIP(hipMemcpy(out, f->spectra.p, sizeof(float) * (size_t)n * f->fftSize, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int sdrgpu_frontend_vfo_dev(sdrgpu_frontend* f, int id, const void** out, int* n) {
    NEED_FE(f);
    auto it = f->vfos.find(id);
    if (it == f->vfos.end()) { set_error("frontend: no VFO %d", id); return SDRGPU_EARG; }
    if (out) *out = it->second.out.p;
    if (n) *n = it->second.n;
    return it->second.n;
}
// the last push's preprocessed IQ (decimated / DC-blocked / conjugated as configured): what the
// reference's Splitter hands to bound IQ streams (iq_frontend.cpp:114-120, routing/splitter.h:46-60)
extern "C" int sdrgpu_frontend_read_iq(sdrgpu_frontend* f, void* out, int max) {
    NEED_FE(f);
    const int n = std::min(max, f->lastIQn);
    if (n <= 0 || !f->lastIQ) return 0;
    SDRGPU_SET_DEVICE(f->device);
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    SDRGPU_HIP(hipMemcpy(out, f->lastIQ, sizeof(float2) * (size_t)n, hipMemcpyDeviceToHost));
    return n;
}

extern "C" int sdrgpu_frontend_read_vfo(sdrgpu_frontend* f, int id, void* out, int max) {
    NEED_FE(f);
    auto it = f->vfos.find(id);
    if (it == f->vfos.end()) { set_error("frontend: no VFO %d", id); return SDRGPU_EARG; }
    const int n = std::min(max, it->second.n);
    if (n <= 0) return 0;
    SDRGPU_SET_DEVICE(f->device);
    SDRGPU_HIP(hipStreamSynchronize(f->s));
    SDRGPU_HIP(hipMemcpy(out, it->second.out.p, sizeof(float2) * (size_t)n, hipMemcpyDeviceToHost));
    return n;
}

// ---- pipelined host call style (the IQFrontEnd drop-in) ------------------------------------
// submit(k): [stage the host block in pinned memory unless it is registered] -> H2D on the copy
// stream into slot k % 2 -> (compute stream waits for it) push_dev -> D2H of the block's rows,
// VFO outputs and, with SDRGPU_FE_IQ, preprocessed IQ into the slot's pinned results -> event.
// Nothing waits for the device: block k + 1's H2D runs on the copy stream while block k's kernels
// and read-back run on the compute stream, and the host hands block k - 1's results on meanwhile.
// collect(k) waits for block k's results. Calls on one front end come from one thread at a time.
static int pipe_slot_init(sdrgpu_frontend* f, PipeSlot& ps) {
    if (!f->cs) SDRGPU_HIP(hipStreamCreateWithFlags(&f->cs, hipStreamNonBlocking));
    for (hipEvent_t* e : {&ps.h2d, &ps.consumed, &ps.ready})
        if (!*e) SDRGPU_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return SDRGPU_OK;
}

extern "C" int sdrgpu_frontend_submit(sdrgpu_frontend* f, const void* in, int count, int kind, int flags) {
    NEED_FE(f);
    if (count < 0 || (count > 0 && !in) || kind < -1 || kind > SDRGPU_CONV_F32) { set_error("frontend_submit: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(f->device);
    const long long t = f->nextTicket;
    PipeSlot& ps = f->pipe[t & 1];
    if (!ps.collected) { set_error("frontend_submit: ticket %lld not collected (at most 2 blocks in flight)", ps.ticket); return SDRGPU_ESTATE; }
    SDRGPU_CHECK(pipe_slot_init(f, ps));
    const size_t bytes = (size_t)count * (kind < 0 ? sizeof(float2) : 2 * kConvSize[kind]);
    const void* raw = nullptr;
    if (count > 0) {
        SDRGPU_CHECK(ps.raw.ensure(bytes));
        // the slot's last H2D finished (its staging is reusable), and its last block's kernels
        // have read `raw` (copy stream waits: device side)
        const void* src = in;
        if (!host_pinned(in, bytes)) {
            SDRGPU_HIP(hipEventSynchronize(ps.h2d));
            SDRGPU_CHECK(ps.stage.ensure(bytes));
            std::memcpy(ps.stage.p, in, bytes);
            src = ps.stage.p;
        }
        SDRGPU_HIP(hipStreamWaitEvent(f->cs, ps.consumed, 0));
        SDRGPU_HIP(hipMemcpyAsync(ps.raw.p, src, bytes, hipMemcpyHostToDevice, f->cs));
        SDRGPU_HIP(hipEventRecord(ps.h2d, f->cs));
        SDRGPU_HIP(hipStreamWaitEvent(f->s, ps.h2d, 0));
        raw = ps.raw.p;
    }
    const int nf = sdrgpu_frontend_push_dev(f, raw, count, kind, f->s);
    if (nf < 0) return nf;
    SDRGPU_HIP(hipEventRecord(ps.consumed, f->s));
    // read-back into the slot's pinned results (sizes are host-side state of this push)
    ps.nrows = nf;
    if (nf > 0) {
        const size_t rb = sizeof(float) * (size_t)nf * f->fftSize;
        SDRGPU_CHECK(ps.rows.ensure(rb));
        SDRGPU_HIP(hipMemcpyAsync(ps.rows.p, f->spectra.p, rb, hipMemcpyDeviceToHost, f->s));
    }
    for (auto& [id, v] : f->vfos) {
        const int k = (int)(t & 1);
        v.resN[k] = v.n;
        if (v.n > 0) {
            SDRGPU_CHECK(v.res[k].ensure(sizeof(float2) * (size_t)v.n));
            SDRGPU_HIP(hipMemcpyAsync(v.res[k].p, v.out.p, sizeof(float2) * (size_t)v.n, hipMemcpyDeviceToHost, f->s));
        }
    }
    ps.niq = 0;
    if ((flags & SDRGPU_FE_IQ) && f->lastIQn > 0 && f->lastIQ) {
        ps.niq = f->lastIQn;
        SDRGPU_CHECK(ps.iq.ensure(sizeof(float2) * (size_t)ps.niq));
        SDRGPU_HIP(hipMemcpyAsync(ps.iq.p, f->lastIQ, sizeof(float2) * (size_t)ps.niq, hipMemcpyDeviceToHost, f->s));
    }
    SDRGPU_HIP(hipEventRecord(ps.ready, f->s));
    ps.ticket = t;
    ps.collected = false;
    f->nextTicket = t + 1;
    return (int)(t & 0x7fffffff);
}

static PipeSlot* pipe_find(sdrgpu_frontend* f, int ticket) {
    PipeSlot& ps = f->pipe[ticket & 1];
    if (ps.ticket < 0 || (int)(ps.ticket & 0x7fffffff) != ticket) {
        set_error("frontend: ticket %d is not in flight", ticket);
        return nullptr;
    }
    return &ps;
}

extern "C" int sdrgpu_frontend_collect(sdrgpu_frontend* f, int ticket, const float** rows, const void** iq, int* niq) {
    NEED_FE(f);
    PipeSlot* ps = pipe_find(f, ticket);
    if (!ps) return SDRGPU_EARG;
    SDRGPU_SET_DEVICE(f->device);
    SDRGPU_HIP(hipEventSynchronize(ps->ready));
    if (rows) *rows = ps->nrows > 0 ? ps->rows.as_const<float>() : nullptr;
    if (iq) *iq = ps->niq > 0 ? ps->iq.p : nullptr;
    if (niq) *niq = ps->niq;
    return ps->nrows;
}

extern "C" int sdrgpu_frontend_collected_vfo(sdrgpu_frontend* f, int ticket, int id, const void** out, int* n) {
    NEED_FE(f);
    PipeSlot* ps = pipe_find(f, ticket);
    if (!ps) return SDRGPU_EARG;
    auto it = f->vfos.find(id);
    if (it == f->vfos.end()) { set_error("frontend: no VFO %d", id); return SDRGPU_EARG; }
    const int k = ticket & 1;
    if (out) *out = it->second.resN[k] > 0 ? it->second.res[k].p : nullptr;
    if (n) *n = it->second.resN[k];
    return it->second.resN[k];
}

// the host is done with the ticket's results: its slot may take a new block
extern "C" int sdrgpu_frontend_release(sdrgpu_frontend* f, int ticket) {
    NEED_FE(f);
    PipeSlot* ps = pipe_find(f, ticket);
    if (!ps) return SDRGPU_EARG;
    ps->collected = true;
    ps->ticket = -1;   // a released ticket is gone: a late collect / release gets SDRGPU_EARG
    return SDRGPU_OK;
}
