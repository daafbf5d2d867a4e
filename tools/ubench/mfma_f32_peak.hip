// Sustained f32 matrix-core rate on this device: back-to-back v_mfma_f32_32x32x2_f32 and
// v_mfma_f32_16x16x4_f32 with register operands, 4 independent accumulators per wave, 2 waves
// per SIMD on every CU. The C4 channelizer's dense-DFT-as-GEMM alternative (512 flop per
// sample) can run no faster than 2^28 x 512 flop at this rate.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/mfma_f32_peak.hip -o tools/bin/mfma_f32_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma32(float* out, int iters, float a0, float b0) {
    float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int k = 0; k < 16; k++) s += c0[k] + c1[k] + c2[k] + c3[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void mfma16(float* out, int iters, float a0, float b0) {
    float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int k = 0; k < 4; k++) s += c0[k] + c1[k] + c2[k] + c3[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 2, iters = 20000;   // 2 workgroups x 4 waves per CU = 2 waves per SIMD
    float* out = nullptr;
    if (hipMalloc(&out, sizeof(float) * blocks * 256) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int which = 0; which < 2; which++) {
        double best = 0;
        for (int rep = 0; rep < 5; rep++) {
            (void)hipEventRecord(e0, 0);
            if (which == 0) hipLaunchKernelGGL(mfma32, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f, 0.25f);
            else hipLaunchKernelGGL(mfma16, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f, 0.25f);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) return 1;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double flop_per_mfma = which == 0 ? 32.0 * 32 * 2 * 2 : 16.0 * 16 * 4 * 2;
            const double tf = (double)blocks * 4 * iters * 4 * flop_per_mfma / (ms * 1e-3) / 1e12;
            if (tf > best) best = tf;
        }
        std::printf("{\"mfma\": \"%s\", \"cus\": %d, \"tflops_f32\": %.1f}\n",
                    which == 0 ? "v_mfma_f32_32x32x2_f32" : "v_mfma_f32_16x16x4_f32", cus, best);
    }
    (void)hipFree(out);
    return 0;
}
