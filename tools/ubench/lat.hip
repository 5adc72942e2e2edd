// Single-wave latency microbenchmarks for the local-solver step (gfx950).
// Each test runs N dependent iterations in one wave and reports cycles/iter.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../cocoa_amd/csrc/wave.h"
using namespace cocoa;

#define N 4096
__global__ __launch_bounds__(64) void k_lds_chain(uint64_t* out, int seed) {
    __shared__ int32_t t[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) t[i] = (i * 97 + 13 + seed) & 4095;
    __syncthreads();
    int p = threadIdx.x;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) p = t[p];
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = p; }
}
__global__ __launch_bounds__(64) void k_lds_uniform_chain(uint64_t* out, int seed) {
    __shared__ int32_t t[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) t[i] = (i * 97 + 13 + seed) & 4095;
    __syncthreads();
    int p = 0;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) p = uni(t[p]);
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = p; }
}
__global__ __launch_bounds__(64) void k_wavesum(uint64_t* out, double seed) {
    double x = seed + threadIdx.x;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) x = wave_sum(x) * 1e-3 + (double)threadIdx.x;
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = (uint64_t)x; }
}
__global__ __launch_bounds__(64) void k_div(uint64_t* out, double seed) {
    double x = seed + threadIdx.x, q = 1.7 + seed;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) x = (x / q) + 1.0;
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = (uint64_t)x; }
}
__global__ __launch_bounds__(64) void k_fma(uint64_t* out, double seed) {
    double x = seed + threadIdx.x;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) x = x * 0.999 + 1.0;
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = (uint64_t)x; }
}
__global__ __launch_bounds__(64) void k_readfirst(uint64_t* out, double seed) {
    double x = seed + threadIdx.x;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) x = uni(x) * 0.999 + (double)threadIdx.x;
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = (uint64_t)x; }
}
// LDS write then dependent read of the same address (store->load through LDS)
__global__ __launch_bounds__(64) void k_lds_wr_rd(uint64_t* out, int seed) {
    __shared__ double t[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) t[i] = i;
    __syncthreads();
    double x = seed;
    int p = threadIdx.x * 7;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) {
        double v = t[p & 4095];
        x = v + 1.0;
        t[p & 4095] = x;
        p = (int)x;
    }
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = (uint64_t)x; }
}
// global store each iteration + LDS-only chain (does a store stall the chain?)
__global__ __launch_bounds__(64) void k_store_lds(uint64_t* out, double* g, int seed) {
    __shared__ int32_t t[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) t[i] = (i * 97 + 13 + seed) & 4095;
    __syncthreads();
    int p = threadIdx.x;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) {
        p = t[p];
        g[(p * 131 + i * 64 + threadIdx.x) & ((1 << 20) - 1)] = (double)p;
    }
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = p; }
}
// scalar load chain from global (s_load)
__global__ __launch_bounds__(64) void k_sload(uint64_t* out, const int32_t* g) {
    int p = 0;
    uint64_t c0 = clock64();
    for (int i = 0; i < N; ++i) p = __builtin_amdgcn_readfirstlane(g[p]);
    uint64_t c1 = clock64();
    if (threadIdx.x == 0) { out[0] = (c1 - c0); out[1] = p; }
}

int main() {
    uint64_t* d; hipMalloc(&d, 64); double* g; hipMalloc(&g, (1 << 20) * 8);
    int32_t* gi; hipMalloc(&gi, 4096 * 4);
    int32_t h[4096]; for (int i = 0; i < 4096; ++i) h[i] = (i * 97 + 13) & 4095;
    hipMemcpy(gi, h, sizeof h, hipMemcpyHostToDevice);
    uint64_t r[2];
    auto rep = [&](const char* name) { hipDeviceSynchronize(); hipMemcpy(r, d, 16, hipMemcpyDeviceToHost);
        printf("%-22s %8.1f cyc/iter\n", name, (double)r[0] / N); };
    for (int rep_ = 0; rep_ < 2; ++rep_) {
    k_lds_chain<<<1, 64>>>(d, 0); rep("lds_chain");
    k_lds_uniform_chain<<<1, 64>>>(d, 0); rep("lds_uniform_chain");
    k_wavesum<<<1, 64>>>(d, 0.5); rep("wave_sum+fma");
    k_div<<<1, 64>>>(d, 0.5); rep("div+add");
    k_fma<<<1, 64>>>(d, 0.5); rep("fma");
    k_readfirst<<<1, 64>>>(d, 0.5); rep("readfirstlane+fma");
    k_lds_wr_rd<<<1, 64>>>(d, 1); rep("lds wr->rd chain");
    k_store_lds<<<1, 64>>>(d, g, 0); rep("global store+lds chain");
    k_sload<<<1, 64>>>(d, gi); rep("global load chain(uni)");
    }
    return 0;
}
