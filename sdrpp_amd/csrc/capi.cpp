// C ABI: runtime helpers and the host-side design entry points of libsdrgpu.
#include <cstdlib>
#include <map>
#include <mutex>
#include "sdrgpu_internal.h"

namespace sdrgpu { const char* last_error(); }
using namespace sdrgpu;

namespace sdrgpu {
const char* tuning_env(const char* name) {
    const char* t = std::getenv("SDRGPU_TUNING");
    if (!t || t[0] != '1' || t[1] != 0) return nullptr;
    return std::getenv(name);
}
}  // namespace sdrgpu

extern "C" int sdrgpu_version(void) { return SDRGPU_VERSION; }
extern "C" const char* sdrgpu_last_error(void) { return last_error(); }

extern "C" int sdrgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
extern "C" int sdrgpu_malloc(int device, void** dptr, size_t bytes) {
    if (!dptr) { set_error("malloc: null out pointer"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    SDRGPU_HIP(hipMalloc(dptr, bytes));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_free(void* dptr) {
    SDRGPU_HIP(hipFree(dptr));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    SDRGPU_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    SDRGPU_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    SDRGPU_HIP(hipStreamSynchronize((hipStream_t)stream));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_stream_create(int device, void** stream) {
    if (!stream) { set_error("stream_create: null out pointer"); return SDRGPU_EARG; }
    SDRGPU_SET_DEVICE(device);
    hipStream_t s;
    SDRGPU_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void*)s;
    return SDRGPU_OK;
}
extern "C" int sdrgpu_stream_destroy(void* stream) {
    SDRGPU_HIP(hipStreamDestroy((hipStream_t)stream));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_stream_synchronize(void* stream) {
    SDRGPU_HIP(hipStreamSynchronize((hipStream_t)stream));
    return SDRGPU_OK;
}
// Registered (page-locked) host ranges. The host-buffer process calls DMA straight from / to
// a registered buffer and stage through their own pinned buffers otherwise.
namespace {
std::mutex g_pinMtx;
struct PinnedRange {
    size_t bytes;
    bool allocated;   // hipHostMalloc'd (sdrgpu_host_alloc) vs registered (sdrgpu_host_register)
};
std::map<uintptr_t, PinnedRange> g_pinned;   // start -> range
// removes ptr's entry if it was pinned the given way; SDRGPU_EARG (entry kept) otherwise
int take_pinned(void* ptr, bool allocated, const char* what) {
    std::lock_guard<std::mutex> lk(g_pinMtx);
    auto it = g_pinned.find((uintptr_t)ptr);
    if (it == g_pinned.end() || it->second.allocated != allocated) {
        set_error("%s: %p was not %s by this library", what, ptr, allocated ? "allocated (sdrgpu_host_alloc)" : "registered (sdrgpu_host_register)");
        return SDRGPU_EARG;
    }
    g_pinned.erase(it);
    return SDRGPU_OK;
}
}  // namespace
namespace sdrgpu {
bool host_pinned(const void* p, size_t bytes) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_pinMtx);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return false;
    --it;
    return a >= it->first && a + bytes <= it->first + it->second.bytes;
}
}  // namespace sdrgpu
extern "C" int sdrgpu_host_register(void* ptr, size_t bytes) {
    if (!ptr || bytes == 0) { set_error("host_register: empty range"); return SDRGPU_EARG; }
    SDRGPU_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    std::lock_guard<std::mutex> lk(g_pinMtx);
    g_pinned[(uintptr_t)ptr] = {bytes, false};
    return SDRGPU_OK;
}
extern "C" int sdrgpu_host_alloc(void** ptr, size_t bytes) {
    if (!ptr || bytes == 0) { set_error("host_alloc: bad argument"); return SDRGPU_EARG; }
    *ptr = nullptr;
    SDRGPU_HIP(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
    std::lock_guard<std::mutex> lk(g_pinMtx);
    g_pinned[(uintptr_t)*ptr] = {bytes, true};
    return SDRGPU_OK;
}
extern "C" int sdrgpu_host_free(void* ptr) {
    if (!ptr) return SDRGPU_OK;
    SDRGPU_CHECK(take_pinned(ptr, true, "host_free"));
    SDRGPU_HIP(hipHostFree(ptr));
    return SDRGPU_OK;
}
extern "C" int sdrgpu_host_unregister(void* ptr) {
    SDRGPU_CHECK(take_pinned(ptr, false, "host_unregister"));
    SDRGPU_HIP(hipHostUnregister(ptr));
    return SDRGPU_OK;
}

extern "C" int sdrgpu_create_window(int type, float* buffer, int size, int centered) {
    return create_window(type, buffer, size, centered);
}
extern "C" void sdrgpu_gen_reshape_params(double sampleRate, int size, double rate, int* skip, int* nz) {
    // IQFrontEnd::genReshapeParams (signal_path/iq_frontend.h:56-60)
    int fftInterval = (int)std::round(sampleRate / rate);
    int n = fftInterval < size ? fftInterval : size;
    if (nz) *nz = n;
    if (skip) *skip = fftInterval - n;
}
extern "C" int sdrgpu_taps_estimate_count(double transWidth, double sampleRate) {
    return (int)(3.8 * sampleRate / transWidth);
}
extern "C" int sdrgpu_taps_windowed_sinc(int count, double omega, double norm, float* out) {
    return taps_windowed_sinc(count, omega, norm, out);
}
extern "C" int sdrgpu_taps_low_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out) {
    return taps_low_pass(cutoff, transWidth, sampleRate, odd, out);
}
extern "C" int sdrgpu_taps_high_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out) {
    return taps_high_pass(cutoff, transWidth, sampleRate, odd, out);
}
extern "C" int sdrgpu_taps_band_pass_f(double start, double stop, double transWidth, double sampleRate, int odd, float* out) {
    return taps_band_pass_f(start, stop, transWidth, sampleRate, odd, out);
}
extern "C" int sdrgpu_taps_band_pass_c(double start, double stop, double transWidth, double sampleRate, int odd, float* out) {
    return taps_band_pass_c(start, stop, transWidth, sampleRate, odd, out);
}
extern "C" int sdrgpu_decim_plan(int ratio, int* decims, int* ntaps, const float** taps) {
    return decim_plan(ratio, decims, ntaps, taps);
}
