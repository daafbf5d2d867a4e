// Copy / read bandwidth against working-set size: where the Infinity Cache (256 MB) serves a
// two-pass FFT's intermediate, and at what rate. For each buffer size S: dst = src (16-B loads and
// stores, grid-stride, 8192 x 256 threads), and a read-only pass (sum kept live). Reports the median
// of 20 launches after 3 warm-ups, in GB/s of bytes moved (copy: 2 S, read: S).
//   hipcc --offload-arch=gfx950 -O3 tools/bw/mall_copy.hip -o gpurun_out/mall_copy && gpurun_out/mall_copy
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void copy_k(const float4* __restrict__ s, float4* __restrict__ d, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) d[i] = s[i];
}
__global__ __launch_bounds__(256) void read_k(const float4* __restrict__ s, long long n, float* __restrict__ sink) {
    float a = 0.f;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const float4 v = s[i];
        a += v.x + v.y + v.z + v.w;
    }
    if (a == 123.456f) sink[0] = a;   // keeps the loads live; never true for the zero-filled buffer
}

int main() {
    const long long sizes_mb[] = {16, 32, 64, 96, 128, 192, 256, 512, 2048};
    const long long maxb = 2048LL << 20;
    float4 *a, *b;
    float* sink;
    CK(hipMalloc(&a, maxb));
    CK(hipMalloc(&b, maxb));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(a, 0, maxb));
    CK(hipMemset(b, 0, maxb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"rows\": [");
    for (int k = 0; k < (int)(sizeof(sizes_mb) / sizeof(sizes_mb[0])); k++) {
        const long long bytes = sizes_mb[k] << 20, n = bytes / 16;
        double res[2];
        for (int mode = 0; mode < 2; mode++) {
            std::vector<float> t;
            for (int r = 0; r < 23; r++) {
                CK(hipEventRecord(e0, 0));
                if (mode == 0) hipLaunchKernelGGL(copy_k, dim3(8192), dim3(256), 0, 0, a, b, n);
                else hipLaunchKernelGGL(read_k, dim3(8192), dim3(256), 0, 0, a, n, sink);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 3) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double ms = t[t.size() / 2];
            res[mode] = (mode == 0 ? 2.0 : 1.0) * bytes / (ms * 1e-3) / 1e9;
        }
        printf("%s{\"MB\": %lld, \"copy_GBs\": %.0f, \"read_GBs\": %.0f}", k ? ", " : "", sizes_mb[k], res[0], res[1]);
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}
