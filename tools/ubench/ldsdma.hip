// Does LDS-DMA traffic of other waves slow one wave's LDS reads? (gfx950)
//
// One workgroup per CU on every CU.  Wave 0 times a dependent chain of LDS
// reads (cycles per read); waves 1..W stream a large buffer into LDS while it
// runs, by one of:
//   mode 0  nothing (idle partner waves)
//   mode 1  global_load_lds_dword   (4 B per lane, three per "unit", as the Gram
//                                    solver's fetch waves do)
//   mode 2  global_load_lds_dwordx3 (12 B per lane: one per unit)
//   mode 3  global_load_dword x3 into registers + ds_write_b32 x3
// The partner waves stop when wave 0 sets an LDS flag.  Printed: the chain's
// cycles per read, and the partner bytes moved per chain cycle.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHAIN 4096
typedef __attribute__((address_space(3))) void lvoid;

#define DMA(g, l, sz) __builtin_amdgcn_global_load_lds((g), (lvoid*)(l), sz, 0, 0)

template <int MODE>
__global__ __launch_bounds__(384) void k(const uint32_t* buf, int64_t nwords, uint64_t* out) {
    __shared__ int32_t t[4096];
    __shared__ __attribute__((aligned(16))) uint8_t ring[5][64 * 12 * 4];
    __shared__ int stop;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 4096; i += blockDim.x) t[i] = (i * 97 + 13) & 4095;
    if (tid == 0) stop = 0;
    __syncthreads();
    if (wv == 0) {
        int p = lane;
        const uint64_t c0 = __builtin_readcyclecounter();
        for (int i = 0; i < CHAIN; ++i) p = t[p];
        const uint64_t c1 = __builtin_readcyclecounter();
        __hip_atomic_store(&stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane == 0) {
            out[blockIdx.x * 4 + 0] = c1 - c0;
            out[blockIdx.x * 4 + 1] = p;
        }
    } else {
        uint64_t moved = 0;
        const int64_t per = (nwords / gridDim.x) & ~(int64_t)1023;
        const uint32_t* my = buf + (int64_t)blockIdx.x * per;
        int64_t off = (int64_t)(wv - 1) * 768 * 7;
        uint8_t* r = ring[wv - 1];
        for (int it = 0; MODE != 0; ++it) {
            if (__hip_atomic_load(&stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
            if (off + 768 > per) off = 0;
            const uint32_t* g = my + off;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (MODE == 1) {
                    DMA(g + u * 192 + lane, r + u * 768, 4);
                    DMA(g + u * 192 + 64 + lane, r + u * 768 + 256, 4);
                    DMA(g + u * 192 + 128 + lane, r + u * 768 + 512, 4);
                } else if (MODE == 2) {
                    DMA(g + u * 192 + 3 * lane, r + u * 768, 12);
                } else if (MODE == 3) {
                    const uint32_t a = g[u * 192 + lane], b = g[u * 192 + 64 + lane], c = g[u * 192 + 128 + lane];
                    ((uint32_t*)(r + u * 768))[lane] = a;
                    ((uint32_t*)(r + u * 768 + 256))[lane] = b;
                    ((uint32_t*)(r + u * 768 + 512))[lane] = c;
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            moved += 4 * 768;
            off += 768 * 5;
        }
        if (lane == 0) atomicAdd((unsigned long long*)&out[blockIdx.x * 4 + 2], (unsigned long long)moved);
    }
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int64_t nwords = (int64_t)1 << 28;  // 1 GiB streamed
    uint32_t* buf;
    uint64_t* out;
    hipMalloc(&buf, nwords * 4);
    hipMemset(buf, 1, nwords * 4);
    hipMalloc(&out, (size_t)ncu * 4 * sizeof(uint64_t));
    const char* names[4] = {"idle", "dma 3x dword", "dma dwordx3", "load+ds_write"};
    for (int waves : {1, 5}) {
        for (int mode = 0; mode < 4; ++mode) {
            for (int rep = 0; rep < 2; ++rep) {
                hipMemset(out, 0, (size_t)ncu * 4 * sizeof(uint64_t));
                const int thr = 64 * (1 + waves);
                if (mode == 0) k<0><<<ncu, thr>>>(buf, nwords, out);
                if (mode == 1) k<1><<<ncu, thr>>>(buf, nwords, out);
                if (mode == 2) k<2><<<ncu, thr>>>(buf, nwords, out);
                if (mode == 3) k<3><<<ncu, thr>>>(buf, nwords, out);
                hipDeviceSynchronize();
            }
            uint64_t h[4 * 512];
            hipMemcpy(h, out, (size_t)ncu * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost);
            double cyc = 0, bytes = 0;
            for (int b = 0; b < ncu; ++b) {
                cyc += (double)h[b * 4];
                bytes += (double)h[b * 4 + 2];
            }
            cyc /= ncu;
            bytes /= ncu;
            printf("partner waves %d  %-14s  chain %6.1f cyc/read   partner %6.1f B/cyc per CU\n", waves, names[mode],
                   cyc / CHAIN, bytes / cyc);
        }
    }
    hipFree(buf);
    hipFree(out);
    return 0;
}
