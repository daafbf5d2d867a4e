// Issue cost of the VALU instructions the 64k one-pass spectrum kernel spends its time in
// (fft_1p_kernel: fp32 packed butterflies, fp64 twiddle products and conversions, the dB
// epilogue's frexp / log): 8 independent chains per lane, 4 waves per SIMD on every CU, each
// instruction in inline asm so the compiler cannot change it. Prints wave-instructions per
// microsecond per SIMD and the ratio to v_fma_f32 (one full-rate wave64 instruction).
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_rates.hip -o tools/bin/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kChains = 8, kUnroll = 8;

#define CHAIN8(BODY)                                                                               \
    for (int i = 0; i < iters; i++) {                                                              \
        _Pragma("unroll") for (int u = 0; u < kUnroll; u++) {                                      \
            _Pragma("unroll") for (int c = 0; c < kChains; c++) { BODY; }                          \
        }                                                                                          \
    }

__global__ __launch_bounds__(256) void k_fma_f32(float* out, int iters) {
    float a[kChains], b = 1.0000001f, cc = 1e-8f;
    for (int c = 0; c < kChains; c++) a[c] = threadIdx.x + c;
    CHAIN8(asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(cc)))
    float s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pk_fma_f32(float* out, int iters) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[kChains], b = {1.0000001f, 1.0000001f}, cc = {1e-8f, 1e-8f};
    for (int c = 0; c < kChains; c++) a[c] = f2{(float)threadIdx.x, (float)c};
    CHAIN8(asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(cc)))
    float s = 0;
    for (int c = 0; c < kChains; c++) s += a[c].x + a[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fma_f64(float* out, int iters) {
    double a[kChains], b = 1.0000000001, cc = 1e-12;
    for (int c = 0; c < kChains; c++) a[c] = threadIdx.x + c;
    CHAIN8(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(cc)))
    double s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}
__global__ __launch_bounds__(256) void k_mul_f64(float* out, int iters) {
    double a[kChains], b = 1.0000000001;
    for (int c = 0; c < kChains; c++) a[c] = threadIdx.x + c;
    CHAIN8(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
    double s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}
__global__ __launch_bounds__(256) void k_cvt_f32_f64(float* out, int iters) {
    float a[kChains];
    double d = 1.0 + threadIdx.x;
    for (int c = 0; c < kChains; c++) a[c] = 0;
    CHAIN8(asm volatile("v_cvt_f32_f64 %0, %1" : "+v"(a[c]) : "v"(d)))
    float s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cvt_f64_f32(float* out, int iters) {
    double a[kChains];
    float f = 1.0f + threadIdx.x;
    for (int c = 0; c < kChains; c++) a[c] = 0;
    CHAIN8(asm volatile("v_cvt_f64_f32 %0, %1" : "+v"(a[c]) : "v"(f)))
    double s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}
__global__ __launch_bounds__(256) void k_log_f32(float* out, int iters) {
    float a[kChains];
    for (int c = 0; c < kChains; c++) a[c] = 2.0f + threadIdx.x + c;
    CHAIN8(asm volatile("v_log_f32 %0, %0" : "+v"(a[c])))
    float s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_frexp_mant(float* out, int iters) {
    float a[kChains];
    for (int c = 0; c < kChains; c++) a[c] = 3.0f + threadIdx.x + c;
    CHAIN8(asm volatile("v_frexp_mant_f32 %0, %0" : "+v"(a[c])))
    float s = 0;
    for (int c = 0; c < kChains; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pk_add_f32(float* out, int iters) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[kChains], b = {1e-8f, 1e-8f};
    for (int c = 0; c < kChains; c++) a[c] = f2{(float)threadIdx.x, (float)c};
    CHAIN8(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
    float s = 0;
    for (int c = 0; c < kChains; c++) s += a[c].x + a[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef void (*Kern)(float*, int);

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4, iters = 2000;   // 4 workgroups x 4 waves per CU = 4 waves per SIMD
    float* out = nullptr;
    if (hipMalloc(&out, sizeof(float) * blocks * 256) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct { const char* name; Kern k; } ks[] = {
        {"v_fma_f32", k_fma_f32},         {"v_pk_fma_f32", k_pk_fma_f32}, {"v_pk_add_f32", k_pk_add_f32},
        {"v_fma_f64", k_fma_f64},         {"v_mul_f64", k_mul_f64},       {"v_cvt_f32_f64", k_cvt_f32_f64},
        {"v_cvt_f64_f32", k_cvt_f64_f32}, {"v_log_f32", k_log_f32},       {"v_frexp_mant_f32", k_frexp_mant},
    };
    double base = 0;
    for (auto& e : ks) {
        double best = 0;
        for (int rep = 0; rep < 5; rep++) {
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(e.k, dim3(blocks), dim3(256), 0, 0, out, iters);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) return 1;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            // wave-instructions per microsecond per SIMD
            const double winst = (double)blocks * 4 * iters * kUnroll * kChains;
            const double r = winst / (ms * 1e3) / (cus * 4.0);
            if (r > best) best = r;
        }
        if (base == 0) base = best;
        std::printf("{\"instr\": \"%s\", \"winst_per_us_per_simd\": %.1f, \"cost_vs_v_fma_f32\": %.2f}\n", e.name, best,
                    base / best);
    }
    (void)hipFree(out);
    return 0;
}
