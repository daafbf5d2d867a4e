// Shared plumbing of the GPU-backed drop-in blocks: RAII over an sdrgpu_block handle,
// device selection (SDRGPU_DEVICE, default 0) and error reporting. Errors are printed
// the way the reference's flog::error would report them and make run() return -1
// (core/src/dsp/block.h:70-72 stops the worker on a negative return).
#pragma once
#include <cstdio>
#include <cstdlib>
#include <sdrgpu.h>

namespace dsp::gpu {
inline int device() {
    const char* e = std::getenv("SDRGPU_DEVICE");
    return e ? std::atoi(e) : 0;
}
inline bool ok(int rc, const char* what) {
    if (rc >= 0) return true;
    std::fprintf(stderr, "[sdrgpu] %s failed (%d): %s\n", what, rc, sdrgpu_last_error());
    return false;
}
struct Handle {
    sdrgpu_block* h = nullptr;
    Handle() = default;
    Handle(const Handle&) = delete;
    Handle& operator=(const Handle&) = delete;
    ~Handle() { reset(nullptr); }
    void reset(sdrgpu_block* n) {
        if (h) sdrgpu_block_destroy(h);
        h = n;
    }
    // reference process(count, in, out) semantics on host buffers: returns outCount, -1 on error
    int process(const void* in, int count, void* out, const char* what) {
        int m = sdrgpu_block_process(h, in, count, out);
        return ok(m, what) ? m : -1;
    }
};
}  // namespace dsp::gpu
