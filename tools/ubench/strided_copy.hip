// Micro-benchmark: achievable HBM bandwidth of the four-step access patterns on MI355X.
// Copies frames of N = N1 x N2 complex floats with (a) contiguous rows, (b) pass-A style
// column blocks of S columns (S*8-byte segments, stride N2*8 bytes), reading and writing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void copy_contig(const float4* __restrict__ a, float4* __restrict__ b, long long n4) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n4; i += stride) b[i] = a[i];
}
// one WG per (column block, frame): S columns x N1 rows; each lane moves 8 B
template <int S>
__global__ void copy_cols(const float2* __restrict__ a, float2* __restrict__ b, int N1, int N2) {
    const long long base = (long long)blockIdx.y * N1 * N2 + blockIdx.x * S;
    const int c = threadIdx.x % S, t = threadIdx.x / S, T = blockDim.x / S;
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = a[base + (long long)(t + r * T) * N2 + c];
#pragma unroll
    for (int r = 0; r < 16; r++) b[base + (long long)(t + r * T) * N2 + c] = v[r];
}
template <int S>
float run_cols(const float2* a, float2* b, int N1, int N2, int frames) {
    dim3 grid(N2 / S, frames);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(copy_cols<S>, grid, dim3(S * N1 / 16), 0, 0, a, b, N1, N2);
    hipEventRecord(e0);
    for (int w = 0; w < 10; w++) hipLaunchKernelGGL(copy_cols<S>, grid, dim3(S * N1 / 16), 0, 0, a, b, N1, N2);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}
int main() {
    const int N1 = 256, N2 = 256, frames = 1024;   // 64k frames, 512 MB per buffer
    const long long n = (long long)N1 * N2 * frames;
    float2 *a, *b;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(copy_contig, dim3(4096), dim3(256), 0, 0, (const float4*)a, (float4*)b, n / 2);
    hipEventRecord(e0);
    for (int w = 0; w < 10; w++) hipLaunchKernelGGL(copy_contig, dim3(4096), dim3(256), 0, 0, (const float4*)a, (float4*)b, n / 2);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 10;
    printf("contig copy      : %.3f ms  %.0f GB/s (r+w)\n", ms, 2.0 * n * 8 / ms / 1e6);
    float t;
    t = run_cols<8>(a, b, N1, N2, frames);  printf("cols S=8  (64B)  : %.3f ms  %.0f GB/s\n", t, 2.0 * n * 8 / t / 1e6);
    t = run_cols<16>(a, b, N1, N2, frames); printf("cols S=16 (128B) : %.3f ms  %.0f GB/s\n", t, 2.0 * n * 8 / t / 1e6);
    t = run_cols<32>(a, b, N1, N2, frames); printf("cols S=32 (256B) : %.3f ms  %.0f GB/s\n", t, 2.0 * n * 8 / t / 1e6);
    t = run_cols<64>(a, b, N1, N2, frames); printf("cols S=64 (512B) : %.3f ms  %.0f GB/s\n", t, 2.0 * n * 8 / t / 1e6);
    return 0;
}
