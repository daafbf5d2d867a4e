// Consumers on either side of the hot path:
//   * the waterfall's max-decimating zoom, fft_scaler::doZoom (gui/widgets/fft_scaler.h:27-64),
//     applied to device spectrum rows so only display-width rows leave the GPU;
//   * the IQ wire codec, SampleStreamCompressor / Decompressor
//     (dsp/compression/sample_stream_compressor.h:26-60, sample_stream_decompressor.h:13-33).
//   * the recorder's WAV sample encoders (utils/wav.cpp:296-336).
// All are bit-identical to the reference arithmetic: the zoom's bin ranges are the reference's
// own sequential double accumulation, evaluated on the host once per geometry; the codec
// reduces the SIGNED maximum (volk_32f_index_max_32u, first index on ties -- a quirk: not
// the magnitude) exactly and converts with the VOLK generic rounding (x * s, clamp, rintf).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include "sdrgpu_internal.h"

namespace sdrgpu {

// ------------------------------------------------------------------ zoom
// one output per thread: max over data[i0[o], i1[o]) (i1 = i0 + 1 when factor <= 1)
__global__ void zoom_kernel(const float* __restrict__ rows, int fftSize, int nrows, const int2* __restrict__ range,
                            int outSize, float* __restrict__ out) {
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (o >= outSize || r >= nrows) return;
    const float* d = rows + (size_t)r * fftSize;
    const int2 rg = range[o];
    float m = d[rg.x];
    for (int j = rg.x + 1; j < rg.y; j++) m = fmaxf(m, d[j]);   // std::max(maxVal, data[j])
    out[(size_t)r * outSize + o] = m;
}

// ----------------------------------------------- WaterFall::pushFFT consumers
// colormap (waterfall.cpp:903-910): one pixel per thread, IEEE division, no contraction
__global__ void colormap_kernel(const float* __restrict__ in, long long n, float wfMin, float wfMax,
                                const unsigned* __restrict__ pallet, int res, unsigned* __restrict__ out) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const float dataRange = wfMax - wfMin;
    float v = in[j];
    v = v < wfMin ? wfMin : (wfMax < v ? wfMax : v);   // std::clamp<float>
    const float pixel = (v - wfMin) / dataRange;
    out[j] = pallet[(int)(pixel * (res - 1))];
}

// FFT smoothing + hold (waterfall.cpp:918-925, 952-957): one column per thread, rows in order
__global__ void smooth_hold_kernel(float* __restrict__ rows, int nrows, int width, int smoothing, float alpha, float beta,
                                   float* __restrict__ smooth, int holdOn, float holdSpeed, float* __restrict__ hold) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= width) return;
    float sm = smoothing ? smooth[i] : 0.0f;
    float h = holdOn ? hold[i] : 0.0f;
    for (int r = 0; r < nrows; r++) {
        float v = rows[(size_t)r * width + i];
        if (smoothing) {
            const float a = v * alpha;   // volk_32f_s32f_multiply_32f (latest)
            const float b = sm * beta;   // volk_32f_s32f_multiply_32f (smoothingBuf)
            sm = b + a;                  // volk_32f_x2_add_32f(smoothingBuf, latest, smoothingBuf)
            v = sm;
            rows[(size_t)r * width + i] = v;
        }
        if (holdOn && i >= 1) {
            const float hs = h - holdSpeed;
            h = (v < hs) ? hs : v;       // std::max<float>(latestFFT[i], latestFFTHold[i] - fftHoldSpeed)
        }
    }
    if (smoothing) smooth[i] = sm;
    if (holdOn) hold[i] = h;
}

// WaterFall::calculateVFOSignalInfo (waterfall.cpp:563-601): one workgroup per raw dB row; the
// side-band mean is a double sum (exact, so order-free, while it fits 53 bits) and the in-band max
__global__ void vfo_info_kernel(const float* __restrict__ rows, int fftSize, int a0, int a1, int b0, int b1,
                                float* __restrict__ strength, float* __restrict__ snr) {
    __shared__ double ssum[256];
    __shared__ float smax[256];
    const float* line = rows + (size_t)blockIdx.x * fftSize;
    const int tid = threadIdx.x;
    double acc = 0.0;
    float mx = -INFINITY;
    for (int i = a0 + tid; i < a1; i += 256) acc += line[i];
    for (int i = b0 + 1 + tid; i < b1; i += 256) acc += line[i];
    for (int i = a1 + tid; i <= b0 && i < fftSize; i += 256) mx = line[i] > mx ? line[i] : mx;
    ssum[tid] = acc;
    smax[tid] = mx;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) {
            ssum[tid] += ssum[tid + o];
            smax[tid] = smax[tid + o] > smax[tid] ? smax[tid + o] : smax[tid];
        }
        __syncthreads();
    }
    if (tid == 0) {
        const int cnt = (a1 > a0 ? a1 - a0 : 0) + (b1 > b0 + 1 ? b1 - b0 - 1 : 0);
        const double avg = ssum[0] / (double)cnt;
        strength[blockIdx.x] = smax[0];
        snr[blockIdx.x] = smax[0] - avg;
    }
}

// ---------------------------------------------------------------- codec
__global__ void signed_max_kernel(const float* __restrict__ x, long long n, unsigned* __restrict__ bits) {
    // max over floats as an order-preserving unsigned key (exact; NaN-free input)
    float m = -INFINITY;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        m = fmaxf(m, x[i]);
    for (int s = 32; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
    if ((threadIdx.x & 63) == 0) {
        const unsigned u = __float_as_uint(m);
        const unsigned key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        atomicMax(bits, key);
    }
}
__device__ __forceinline__ float key_to_float(unsigned key) {
    return __uint_as_float((key & 0x80000000u) ? (key & 0x7fffffffu) : ~key);
}
template <typename IT>
__global__ void compress_kernel(const float* __restrict__ x, long long n, const unsigned* __restrict__ maxKey,
                                float full, float lo, float hi, unsigned char* __restrict__ out) {
    const float mv = key_to_float(*maxKey);
    const float sc = full / mv;                                   // 128.0f / maxVal, 32768.0f / maxVal
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i == 0) {                                                  // header: {u16 0, u16 type, f32 scaler}
        const unsigned short ct = 0, st = sizeof(IT) == 1 ? 0 : 1;
        memcpy(out, &ct, 2);
        memcpy(out + 2, &st, 2);
        memcpy(out + 4, &mv, 4);
    }
    if (i >= n) return;
    float r = x[i] * sc;                                           // volk_32f_s32f_convert_{8,16}i generic
    if (r > hi) r = hi;
    else if (r < lo) r = lo;
    reinterpret_cast<IT*>(out + 8)[i] = (IT)rintf(r);
}
__global__ void f32_header_kernel(unsigned char* __restrict__ out) {
    const unsigned short ct = 0, st = 2;
    const float z = 0.0f;
    memcpy(out, &ct, 2);
    memcpy(out + 2, &st, 2);
    memcpy(out + 4, &z, 4);
}
__global__ void decompress16_kernel(const short* __restrict__ in, long long n, float scaler, float* __restrict__ out) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const float sc = 32768.0f / scaler;
    if (i < n) out[i] = ((float)in[i]) / sc;                       // volk_16i_s32f_convert_32f generic
}
__global__ void decompress8_kernel(const signed char* __restrict__ in, long long n, float isc, float* __restrict__ out) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) out[i] = ((float)in[i]) * isc;                      // volk_8i_s32f_convert_32f generic
}

// ------------------------------------------------------- recorder encoders
// utils/wav.cpp:296-336: clamp to [-1, 1], scale, offset, lroundf (half away from zero); this
// file is compiled with -ffp-contract=off so the scale and offset round separately
__global__ void wav_encode_kernel(int kind, const float* __restrict__ in, long long n, unsigned char* __restrict__ out) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = in[i];
    const float c = (v < -1.0f) ? -1.0f : (1.0f < v) ? 1.0f : v;   // std::clamp
    switch (kind) {
    case 0: out[i] = (unsigned char)lroundf(c * (128.0f - 0.5f) - 0.5f + 128); break;
    case 1: reinterpret_cast<short*>(out)[i] = (short)lroundf(c * (32768.0f - 0.5f) - 0.5f); break;
    case 2: {
        const int q = (int)lroundf(c * (8388608.0f - 0.5f) - 0.5f);
        out[3 * i] = (unsigned char)q;
        out[3 * i + 1] = (unsigned char)(q >> 8);
        out[3 * i + 2] = (unsigned char)(q >> 16);
    } break;
    case 3: reinterpret_cast<int*>(out)[i] = (int)lroundf((float)((double)c * (2147483648.0 - 0.5) - 0.5)); break;
    default: reinterpret_cast<float*>(out)[i] = v; break;
    }
}

struct ZoomPlan {
    int device = 0, fftSize = 0, outSize = 0;
    DevBuf range;
};

}  // namespace sdrgpu

using namespace sdrgpu;

struct sdrgpu_zoom {
    ZoomPlan p;
};

// fft_scaler(viewOffset, viewBandwidth, wholeBandwidth, fftSize, outSize) + its doZoom index walk
extern "C" int sdrgpu_zoom_create(sdrgpu_zoom** out, int device, double viewOffset, double viewBandwidth,
                                  double wholeBandwidth, int fftSize, int outSize) {
    if (!out || fftSize < 1 || outSize < 1 || !(wholeBandwidth > 0)) { set_error("zoom_create: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    const double offsetRatio = viewOffset / (wholeBandwidth / 2.0);
    double width = (viewBandwidth / wholeBandwidth) * fftSize;
    double offset = (((double)fftSize / 2.0) * (offsetRatio + 1)) - (width / 2);
    if (offset < 0) offset = 0;
    if (width > fftSize - offset) width = fftSize - offset;
    const double factor = width / outSize;
    std::vector<int2> rg(outSize);
    double f0 = offset;
    if (factor <= 1.0) {
        for (int i = 0; i < outSize; i++) {
            const double f1 = f0 + factor;
            const int i0 = (int)roundf((float)f0);
            rg[i] = make_int2(i0, i0 + 1);
            f0 = f1;
        }
    } else {
        int i0 = (int)roundf((float)f0);
        for (int i = 0; i < outSize; i++) {
            const double f1 = f0 + factor;
            const int i1 = (int)roundf((float)f1);
            rg[i] = make_int2(i0, std::max(i1, i0 + 1));
            f0 = f1;
            i0 = i1;
        }
    }
    for (auto& r : rg)
        if (r.x < 0 || r.x >= fftSize || r.y > fftSize) {
            set_error("zoom_create: view outside the spectrum (bins %d..%d of %d)", r.x, r.y, fftSize);
            return SDRGPU_EARG;
        }
    auto* z = new sdrgpu_zoom();
    z->p.device = device;
    z->p.fftSize = fftSize;
    z->p.outSize = outSize;
    int rc = z->p.range.ensure(sizeof(int2) * outSize);
    if (rc >= 0 && hipMemcpy(z->p.range.p, rg.data(), sizeof(int2) * outSize, hipMemcpyHostToDevice) != hipSuccess) {
        set_error("zoom_create: upload failed");
        rc = SDRGPU_EHIP;
    }
    if (rc < 0) { delete z; return rc; }
    *out = z;
    return SDRGPU_OK;
}
extern "C" int sdrgpu_zoom_execute_dev(sdrgpu_zoom* z, const float* rows, int nrows, float* out, void* stream) {
    if (!z || nrows < 0 || (nrows > 0 && (!rows || !out))) { set_error("zoom_execute: bad argument"); return SDRGPU_EARG; }
    if (nrows == 0) return 0;
    SDRGPU_SET_DEVICE(z->p.device);
    hipLaunchKernelGGL(zoom_kernel, dim3((z->p.outSize + 255) / 256, nrows), dim3(256), 0, (hipStream_t)stream, rows,
                       z->p.fftSize, nrows, z->p.range.as<int2>(), z->p.outSize, out);
    SDRGPU_HIP(hipGetLastError());
    return nrows;
}
extern "C" int sdrgpu_zoom_destroy(sdrgpu_zoom* z) {
    delete z;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_colormap_dev(int device, const float* in, long long n, float wfMin, float wfMax, const unsigned* pallet,
                                   int res, unsigned* out, void* stream) {
    if (n < 0 || (n > 0 && (!in || !pallet || !out)) || res < 1) { set_error("colormap: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    if (n == 0) return 0;
    hipLaunchKernelGGL(colormap_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, in, n, wfMin, wfMax,
                       pallet, res, out);
    SDRGPU_HIP(hipGetLastError());
    return (int)std::min<long long>(n, 0x7fffffff);
}

extern "C" int sdrgpu_fft_smooth_hold_dev(int device, float* rows, int nrows, int width, int smoothing, float alpha, float beta,
                                          float* smooth, int holdOn, float holdSpeed, float* hold, void* stream) {
    if (nrows < 0 || width < 1 || (nrows > 0 && !rows) || (smoothing && !smooth) || (holdOn && !hold)) {
        set_error("fft_smooth_hold: bad argument");
        return SDRGPU_EARG;
    }
    SDRGPU_SET_DEVICE(device);
    if (nrows == 0) return 0;
    hipLaunchKernelGGL(smooth_hold_kernel, dim3((width + 255) / 256), dim3(256), 0, (hipStream_t)stream, rows, nrows, width,
                       smoothing, alpha, beta, smooth, holdOn, holdSpeed, hold);
    SDRGPU_HIP(hipGetLastError());
    return nrows;
}

extern "C" int sdrgpu_vfo_signal_info_dev(int device, const float* rows, int nrows, int fftSize, double wholeBandwidth,
                                          double centerOffset, double bandwidth, float* strength, float* snr, void* stream) {
    if (nrows < 0 || fftSize < 2 || !(wholeBandwidth > 0) || (nrows > 0 && (!rows || !strength || !snr))) {
        set_error("vfo_signal_info: bad argument");
        return SDRGPU_EARG;
    }
    SDRGPU_SET_DEVICE(device);
    if (nrows == 0) return 0;
    // the reference's bin offsets, in its double arithmetic (waterfall.cpp:567-574)
    auto ofs = [&](double f) {
        const int i = (int)(((f / (wholeBandwidth / 2.0)) * (double)(fftSize / 2)) + (fftSize / 2));
        return std::clamp<int>(i, 0, fftSize);
    };
    const int a0 = ofs(centerOffset - bandwidth), a1 = ofs(centerOffset - (bandwidth / 2.0));
    const int b0 = ofs(centerOffset + (bandwidth / 2.0)), b1 = ofs(centerOffset + bandwidth);
    hipLaunchKernelGGL(vfo_info_kernel, dim3(nrows), dim3(256), 0, (hipStream_t)stream, rows, fftSize, a0, a1, b0, b1,
                       strength, snr);
    SDRGPU_HIP(hipGetLastError());
    return nrows;
}

// SampleStreamCompressor::process on a device block of `count` complex samples. pcmType:
// 0 I8, 1 I16, 2 F32 (dsp/compression/pcm_type.h). Returns the byte count written to `out`.
extern "C" int sdrgpu_compress_dev(int device, int pcmType, const float* in, int count, unsigned char* out,
                                   unsigned* scratch, void* stream) {
    if (pcmType < 0 || pcmType > 2 || count < 1 || !in || !out || (pcmType != 2 && !scratch)) { set_error("compress: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    hipStream_t s = (hipStream_t)stream;
    const long long n = 2LL * count;
    if (pcmType == 2) {   // F32: no compression, scaler 0
        hipLaunchKernelGGL(f32_header_kernel, dim3(1), dim3(1), 0, s, out);
        SDRGPU_HIP(hipMemcpyAsync(out + 8, in, sizeof(float) * n, hipMemcpyDeviceToDevice, s));
        return 8 + count * 8;
    }
    SDRGPU_HIP(hipMemsetAsync(scratch, 0, sizeof(unsigned), s));
    const int g = (int)std::min<long long>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(signed_max_kernel, dim3(g), dim3(256), 0, s, in, n, scratch);
    const dim3 gc((unsigned)((n + 255) / 256)), b(256);
    if (pcmType == 0)
        hipLaunchKernelGGL((compress_kernel<signed char>), gc, b, 0, s, in, n, scratch, 128.0f, -128.0f, 127.0f, out);
    else
        hipLaunchKernelGGL((compress_kernel<short>), gc, b, 0, s, in, n, scratch, 32768.0f, -32768.0f, 32767.0f, out);
    SDRGPU_HIP(hipGetLastError());
    return (int)(8 + n * (pcmType == 0 ? 1 : 2));
}

// SampleStreamDecompressor::process: `hdr` is the 8-byte header (host copy: it decides the
// output count), `payload` the device bytes after it. Returns complex samples written.
extern "C" int sdrgpu_decompress_dev(int device, const unsigned char* hdr, const unsigned char* payload, int nbytes,
                                     float* out, void* stream) {
    if (!hdr || nbytes < 8 || (nbytes > 8 && (!payload || !out))) { set_error("decompress: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    hipStream_t s = (hipStream_t)stream;
    unsigned short st;
    float scaler;
    std::memcpy(&st, hdr + 2, 2);
    std::memcpy(&scaler, hdr + 4, 4);
    if (st == 2) {
        const int oc = (nbytes - 8) / 8;
        if (oc > 0) SDRGPU_HIP(hipMemcpyAsync(out, payload, (size_t)oc * 8, hipMemcpyDeviceToDevice, s));
        return oc;
    }
    if (st == 1) {
        const int oc = (nbytes - 8) / 4;
        const long long n = 2LL * oc;
        if (n > 0) hipLaunchKernelGGL(decompress16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                                      (const short*)payload, n, scaler, out);
        SDRGPU_HIP(hipGetLastError());
        return oc;
    }
    if (st == 0) {
        const int oc = (nbytes - 8) / 2;
        const long long n = 2LL * oc;
        const float sc = 128.0f / scaler;
        const float isc = (float)(1.0 / sc);                      // volk generic: iScalar = 1.0 / scalar
        if (n > 0) hipLaunchKernelGGL(decompress8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                                      (const signed char*)payload, n, isc, out);
        SDRGPU_HIP(hipGetLastError());
        return oc;
    }
    set_error("decompress: unknown sample type %u", (unsigned)st);
    return SDRGPU_EARG;
}

// recorder WAV encoders (utils/wav.cpp:296-336) of a device buffer of n sample values:
// kind 0 u8, 1 i16, 2 i24 (packed little-endian), 3 i32, 4 f32; returns bytes written
extern "C" int sdrgpu_wav_encode_dev(int device, int kind, const float* in, long long n, unsigned char* out, void* stream) {
    static const int sz[] = {1, 2, 3, 4, 4};
    if (kind < 0 || kind > 4 || n < 0 || (n > 0 && (!in || !out))) { set_error("wav_encode: bad argument"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    if (n == 0) return 0;
    hipLaunchKernelGGL(wav_encode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, kind, in, n, out);
    SDRGPU_HIP(hipGetLastError());
    return (int)std::min<long long>(n * sz[kind], 0x7fffffff);
}
