// Shared plumbing of the GPU-backed drop-in blocks: RAII over an sdrgpu_block handle,
// device placement and error reporting. Errors are printed the way the reference's
// flog::error would report them and make run() return -1 (core/src/dsp/block.h:70-72 stops
// the worker on a negative return).
//
// Device placement (one process driving several GPUs). A block binds to a device when it is
// first created and keeps it across rebuilds (the setters that re-plan), so its state never
// moves behind its back. The device is, in order:
//   1. the innermost DeviceScope on the constructing thread:
//        { dsp::gpu::DeviceScope on(3); vfo.init(&iq, fs, 240e3, 200e3, offset); }
//   2. for the independent streams -- RxVFO, i.e. the VFOs IQFrontEnd::addVFO creates through
//      VFOManager::createVFO (iq_frontend.cpp:122-142, vfo_manager.cpp:95) -- with
//      SDRGPU_PLACEMENT=spread: the visible GPUs in turn (round-robin per created VFO);
//   3. SDRGPU_DEVICE=<n> (default 0).
// setDevice(n) on a block moves it to another GPU (its filter state restarts, as after reset()).
// A VFO's output is a host dsp::stream, so the demodulator behind it may sit on any device.
#pragma once
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sdrgpu.h>

namespace dsp::gpu {
inline thread_local int scope_device = -1;

class DeviceScope {
public:
    explicit DeviceScope(int dev) : _prev(scope_device) { scope_device = dev; }
    ~DeviceScope() { scope_device = _prev; }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
private:
    int _prev;
};

inline int device() {
    if (scope_device >= 0) return scope_device;
    const char* e = std::getenv("SDRGPU_DEVICE");
    return e ? std::atoi(e) : 0;
}
// device for a new independent stream (RxVFO): DeviceScope, else SDRGPU_PLACEMENT=spread
// round-robin over the visible GPUs, else device()
inline int stream_device() {
    if (scope_device >= 0) return scope_device;
    const char* p = std::getenv("SDRGPU_PLACEMENT");
    if (p && std::strcmp(p, "spread") == 0) {
        static std::atomic<unsigned> next{0};
        const int n = sdrgpu_device_count();
        if (n > 0) return (int)(next.fetch_add(1) % (unsigned)n);
    }
    return device();
}
inline bool ok(int rc, const char* what) {
    if (rc >= 0) return true;
    std::fprintf(stderr, "[sdrgpu] %s failed (%d): %s\n", what, rc, sdrgpu_last_error());
    return false;
}
struct Handle {
    sdrgpu_block* h = nullptr;
    int dev = -1;   // bound at the first creation; kept by rebuilds
    Handle() = default;
    Handle(const Handle&) = delete;
    Handle& operator=(const Handle&) = delete;
    ~Handle() { reset(nullptr); }
    void reset(sdrgpu_block* n) {
        if (h) sdrgpu_block_destroy(h);
        h = n;
    }
    // the block's device: the policy's choice at first use, then fixed
    int bind(int policyDevice) {
        if (dev < 0) dev = policyDevice;
        return dev;
    }
    // reference process(count, in, out) semantics on host buffers: returns outCount, -1 on error
    int process(const void* in, int count, void* out, const char* what) {
        int m = sdrgpu_block_process(h, in, count, out);
        return ok(m, what) ? m : -1;
    }
};
}  // namespace dsp::gpu
