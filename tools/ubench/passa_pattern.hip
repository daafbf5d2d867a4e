// Micro-benchmark: the 64k pass-A access pattern (16 columns x 256 rows per workgroup, 8-B
// lanes, 2-KB row stride) as a plain copy, over one 64 MB chunk (128 frames) and over 1024
// frames, with and without the 35 KB of LDS the real kernel allocates (4 workgroups/CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int S, int V>   // V = 1: 8-B lanes; V = 2: 16-B lanes (two adjacent columns)
__global__ void copy_cols(const float2* __restrict__ a, float2* __restrict__ b, int N1, int N2, int contigStore) {

    const long long base = (long long)blockIdx.y * N1 * N2 + blockIdx.x * S;
    constexpr int P = S / V;
    const int c = threadIdx.x % P, t = threadIdx.x / P, T = blockDim.x / P;
    if (V == 1) {
        float2 v[16];
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = a[base + (long long)(t + r * T) * N2 + c];
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const long long o = contigStore ? (long long)blockIdx.y * N1 * N2 + (long long)blockIdx.x * S * N1 + (long long)r * blockDim.x + threadIdx.x
                                            : base + (long long)(t + r * T) * N2 + c;
            b[o] = v[r];
        }
    } else {
        float4 v[16];
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = *reinterpret_cast<const float4*>(a + base + (long long)(t + r * T) * N2 + 2 * c);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const long long o = contigStore ? (long long)blockIdx.y * N1 * N2 + (long long)blockIdx.x * S * N1 + 2 * ((long long)r * blockDim.x + threadIdx.x)
                                            : base + (long long)(t + r * T) * N2 + 2 * c;
            *reinterpret_cast<float4*>(b + o) = v[r];
        }
    }
}
__global__ void copy_contig(const float4* __restrict__ a, float4* __restrict__ b, long long n4) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n4) b[i] = a[i];
}

template <int S, int V>
float run(const float2* a, float2* b, int frames, size_t lds, int cs, int reps) {
    const int N1 = 256, N2 = 256;
    dim3 grid(N2 / S, frames);
    auto k = copy_cols<S, V>;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const long long fsz = (long long)N1 * N2;
    const int chunks = 1024 / frames;
    for (int w = 0; w < 2; w++) for (int c = 0; c < chunks; c++) hipLaunchKernelGGL(k, grid, dim3(S / V * N1 / 16), lds, 0, a + c * frames * fsz, b + c * frames * fsz, N1, N2, cs);
    hipEventRecord(e0);
    for (int w = 0; w < reps; w++) for (int c = 0; c < chunks; c++) hipLaunchKernelGGL(k, grid, dim3(S / V * N1 / 16), lds, 0, a + c * frames * fsz, b + c * frames * fsz, N1, N2, cs);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / reps / chunks;   // per launch
}
int main() {
    const long long n = 256LL * 256 * 1024;   // 1024 frames of 64k, 512 MB per buffer
    float2 *a, *b;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8));
    const int reps = 5;
    for (int frames : {128, 1024}) {
        const double bytes = 2.0 * frames * 65536 * 8;
        {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            const long long n4 = frames * 65536LL / 2;
            const int chunks = 1024 / frames;
            hipEventRecord(e0);
            for (int w = 0; w < reps; w++) for (int c = 0; c < chunks; c++)
                hipLaunchKernelGGL(copy_contig, dim3((n4 + 255) / 256), dim3(256), 0, 0, (const float4*)(a + c * frames * 65536LL), (float4*)(b + c * frames * 65536LL), n4);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ms /= reps * chunks;
            printf("frames %4d contig float4 copy           : %8.1f us  %6.0f GB/s\n", frames, ms * 1e3, bytes / ms / 1e6);
        }
        for (int cs : {0, 1}) for (size_t lds : {(size_t)0, (size_t)35 * 1024, (size_t)70 * 1024}) {
            float t = run<16, 1>(a, b, frames, lds, cs, reps);
            printf("frames %4d S16 8B  lds %3zuK store %s: %8.1f us  %6.0f GB/s\n", frames, lds / 1024, cs ? "tile " : "cols ", t * 1e3, bytes / t / 1e6);
            t = run<32, 2>(a, b, frames, lds, cs, reps);
            printf("frames %4d S32 16B lds %3zuK store %s: %8.1f us  %6.0f GB/s\n", frames, lds / 1024, cs ? "tile " : "cols ", t * 1e3, bytes / t / 1e6);
            t = run<16, 2>(a, b, frames, lds, cs, reps);
            printf("frames %4d S16 16B lds %3zuK store %s: %8.1f us  %6.0f GB/s\n", frames, lds / 1024, cs ? "tile " : "cols ", t * 1e3, bytes / t / 1e6);
            t = run<64, 2>(a, b, frames, lds, cs, reps);
            printf("frames %4d S64 16B lds %3zuK store %s: %8.1f us  %6.0f GB/s\n", frames, lds / 1024, cs ? "tile " : "cols ", t * 1e3, bytes / t / 1e6);
        }
    }
    return 0;
}
