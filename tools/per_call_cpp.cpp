// C5 at the reference block size from a native host (no Python): one 307,200-sample block per
// call through the C ABI -- sdrgpu_frontend_push_dev (spectrum frames + one RxVFO), then the
// mono WFM demodulator on the VFO output -- i.e. the per-block launch sequence an SDR++ build
// linking libsdrgpu would issue (file_source/src/main.cpp:296,440: fs / 200 per block).
// usage: tools/bin/per_call_cpp [calls]   (build: make -C tools per_call_cpp)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "sdrgpu.h"

#define OK(x) do { int rc_ = (x); if (rc_ < 0) { std::fprintf(stderr, "%s failed: %s\n", #x, sdrgpu_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    const int calls = argc > 1 ? std::atoi(argv[1]) : 1000;
    const int block = 307200;
    const double fs = 61.44e6;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    std::vector<float> h(2 * (size_t)block * 8);
    unsigned x = 7;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (float)(x >> 8) / 8388608.0f - 1.0f; }
    void* d = nullptr;
    void* audio = nullptr;
    if (hipMalloc(&d, sizeof(float) * h.size()) != hipSuccess || hipMalloc(&audio, 8 * 8192) != hipSuccess) return 1;
    if (hipMemcpy(d, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice) != hipSuccess) return 1;
    sdrgpu_frontend* fe = nullptr;
    OK(sdrgpu_frontend_create(&fe, 0, fs, 1, 0, 65536, fs / 65536, 6));
    int vid = 0;
    OK(sdrgpu_frontend_add_vfo(fe, &vid, 240000, 200000, 2.5e6));
    sdrgpu_block* wfm = nullptr;
    OK(sdrgpu_wfm_create(&wfm, 0, 100000, 240000, 1));
    auto one = [&](int k) -> int {
        const float* in = (const float*)d + 2 * (size_t)block * (k % 8);
        if (sdrgpu_frontend_push_dev(fe, in, block, -1, s) < 0) return -1;
        const void* p = nullptr;
        int n = 0;
        if (sdrgpu_frontend_vfo_dev(fe, vid, &p, &n) < 0) return -1;
        return sdrgpu_block_process_dev(wfm, p, n, audio, s);
    };
    for (int k = 0; k < 50; k++) OK(one(k));
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < calls; k++) OK(one(k));
    const auto t1 = std::chrono::steady_clock::now();   // host time to issue the calls
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    const auto t2 = std::chrono::steady_clock::now();
    const double issue = std::chrono::duration<double, std::micro>(t1 - t0).count() / calls;
    const double wall = std::chrono::duration<double, std::micro>(t2 - t0).count() / calls;
    std::printf("{\"block\": %d, \"calls\": %d, \"us_per_call_device\": %.1f, \"us_host_issue_per_call\": %.1f, "
                "\"MSps_device\": %.1f, \"host\": \"C++ (C ABI)\"}\n", block, calls, wall, issue, block / wall);
    sdrgpu_block_destroy(wfm);
    sdrgpu_frontend_destroy(fe);
    (void)hipFree(d);
    (void)hipFree(audio);
    (void)hipStreamDestroy(s);
    return 0;
}
