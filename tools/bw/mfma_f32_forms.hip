// Issue rate of the f32-input MFMA forms on gfx950: v_mfma_f32_16x16x4_f32 (the C3 FIR's form) against
// v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4 blocks: a Toeplitz FIR block of N = 4 columns pads its
// k range to Q + 3 instead of Q + 15). Every SIMD runs W waves of independent accumulator chains with
// operands in registers; reports MACs per cycle per CU from the kernel time and the shader clock
// (s_memtime ticks over the same loop).
//   hipcc --offload-arch=gfx950 -O3 tools/bw/mfma_f32_forms.hip -o gpurun_out/mfma_forms && gpurun_out/mfma_forms
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

template <int FORM>
__global__ __launch_bounds__(256) void mfma_loop(float* out, float a0, float b0, long long* ticks) {
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    float a = a0 + threadIdx.x * 1e-7f, b = b0;
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < ITERS; i++) {
        if constexpr (FORM == 0) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
        } else {
            c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, b, c3, 0, 0, 0);
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    const f4 s = c0 + c1 + c2 + c3;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w;
    if (threadIdx.x == 0 && blockIdx.x == 0) ticks[0] = t1 - t0;
}

// operand / result layout probe of v_mfma_f32_4x4x1_16b_f32: D = A x B with A = lane id, B = 1 (which
// lane's A lands in result register v of lane l), then A = 1, B = lane id
__global__ void layout_probe(float* out) {
    const float lane = (float)threadIdx.x;
    f4 z = {0, 0, 0, 0};
    const f4 da = __builtin_amdgcn_mfma_f32_4x4x1f32(lane, 1.0f, z, 0, 0, 0);
    const f4 db = __builtin_amdgcn_mfma_f32_4x4x1f32(1.0f, lane, z, 0, 0, 0);
    for (int v = 0; v < 4; v++) {
        out[v * 64 + threadIdx.x] = da[v];
        out[256 + v * 64 + threadIdx.x] = db[v];
    }
}

int main() {
    float* out;
    long long* ticks;
    hipMalloc(&out, 4096 * 256 * 4);
    hipMalloc(&ticks, 8);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"rows\": [", cus);
    for (int form = 0; form < 2; form++) {
        for (int wpc = 4; wpc <= 8; wpc += 4) {   // waves per CU (1 or 2 per SIMD): 256-thread workgroups
            const int grid = cus * wpc / 4;
            auto k = form ? mfma_loop<1> : mfma_loop<0>;
            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.0f, 2.0f, ticks);
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.0f, 2.0f, ticks);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            long long tk = 0;
            hipMemcpy(&tk, ticks, 8, hipMemcpyDeviceToHost);
            const double macs_per_instr = form ? 256.0 : 1024.0;   // 16 x 4x4x1 or 16x16x4, per wave
            const double waves = (double)grid * 4;
            const double macs = waves * ITERS * 4 * macs_per_instr;
            const double cyc_per_instr_per_wave = (double)tk / (ITERS * 4.0);
            printf("%s{\"form\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.4f, \"TMACs\": %.1f, \"ticks_per_mfma_one_wave\": %.2f}",
                   (form || wpc > 4) ? ", " : "", form ? "4x4x1_16b" : "16x16x4", wpc, ms, macs / (ms * 1e-3) / 1e12,
                   cyc_per_instr_per_wave);
        }
    }
    printf("], \"layout\": {");
    hipLaunchKernelGGL(layout_probe, dim3(1), dim3(64), 0, 0, out);
    float h[512];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    for (int w = 0; w < 2; w++) {
        printf("%s\"%s\": [", w ? ", " : "", w ? "A1_Blane" : "Alane_B1");
        for (int v = 0; v < 4; v++)
            for (int l = 0; l < 64; l++) printf("%s%d", (v || l) ? "," : "", (int)h[w * 256 + v * 64 + l]);
        printf("]");
    }
    printf("}}\n");
    return 0;
}
