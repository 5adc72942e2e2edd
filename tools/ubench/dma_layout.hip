// Where does one LDS-DMA wave instruction of 12 / 16 bytes per lane put each
// lane's bytes?  Lane l reads 16-byte-spaced source words (value = dword index)
// and the LDS image is dumped.  All addresses are fixed and in bounds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int SIZE>
__global__ void probe(const uint32_t* src, uint32_t* out, int shift) {
    src += shift;  // shift 2: 8-byte- but not 16-byte-aligned sources
    __shared__ uint32_t lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xEEEEEEEEu;
    __syncthreads();
    if (SIZE == 12)
        __builtin_amdgcn_global_load_lds(src + 4 * threadIdx.x, (__attribute__((address_space(3))) void*)lds, 12, 0, 0);
    else
        __builtin_amdgcn_global_load_lds(src + 4 * threadIdx.x, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}

int main() {
    uint32_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (uint32_t)i;
    uint32_t *src, *out;
    hipMalloc(&src, sizeof(h));
    hipMalloc(&out, 4096);
    hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
    uint32_t o[1024];
    probe<12><<<1, 64>>>(src, out, 0);
    hipMemcpy(o, out, 4096, hipMemcpyDeviceToHost);
    printf("size 12: first 24 dwords:");
    for (int i = 0; i < 24; ++i) printf(" %x", o[i]);
    int last = 0;
    for (int i = 0; i < 1024; ++i) if (o[i] != 0xEEEEEEEEu) last = i;
    printf("\nsize 12: last written dword %d (packed lane*12 -> 191; lane*16 -> 255)\n", last);
    for (int shift = 0; shift <= 2; shift += 2) {
        probe<16><<<1, 64>>>(src, out, shift);
        hipMemcpy(o, out, 4096, hipMemcpyDeviceToHost);
        last = 0;
        int bad = 0;
        for (int i = 0; i < 1024; ++i) if (o[i] != 0xEEEEEEEEu) last = i;
        for (int l = 0; l < 64; ++l)
            for (int w = 0; w < 4; ++w) bad += o[4 * l + w] != (uint32_t)(shift + 4 * l + w);
        printf("size 16, source shift %d dwords: first 8 dwords: %x %x %x %x %x %x %x %x; last written %d; wrong %d\n",
               shift, o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], last, bad);
    }
    return 0;
}
