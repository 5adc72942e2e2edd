// Which CUs a CU-masked stream's workgroups land on (hipExtStreamCreateWithCUMask):
// every workgroup records its XCC id and its CU / SE ids (HW_REG_HW_ID); the
// host prints, for an unmasked stream and for a stream whose mask clears the
// first 64 bits, how many distinct CUs each XCC used.  Decides whether
// clearing mask bits 0..63 leaves 8 CUs free on every XCD (the Gram solver's
// 64 workgroups land 8 per XCD) for a side stream that must not take them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

__global__ void where_kernel(uint32_t* out, int spin) {
    if (threadIdx.x == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    // keep the CU busy a little so later workgroups spread out
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(10);
}

static void report(const char* name, const std::vector<uint32_t>& h, int nb) {
    std::vector<std::set<uint32_t>> cus(16);
    for (int b = 0; b < nb; ++b) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
        const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        cus[xcc].insert((se << 5) | (sh << 4) | cu);
    }
    std::printf("%s:", name);
    for (int x = 0; x < 16; ++x)
        if (!cus[x].empty()) std::printf(" xcc%d=%zu", x, cus[x].size());
    std::printf("\n");
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nb = 4096;
    uint32_t* d = nullptr;
    CK(hipMalloc(&d, sizeof(uint32_t) * 2 * nb));
    std::vector<uint32_t> h(2 * nb);
    std::printf("CUs: %d\n", ncu);
    hipStream_t s0;
    CK(hipStreamCreate(&s0));
    where_kernel<<<nb, 64, 0, s0>>>(d, 200);
    CK(hipStreamSynchronize(s0));
    CK(hipMemcpy(h.data(), d, sizeof(uint32_t) * 2 * nb, hipMemcpyDeviceToHost));
    report("unmasked", h, nb);
    const int words = (ncu + 31) / 32;
    for (int variant = 0; variant < 2; ++variant) {
        std::vector<uint32_t> mask(words, 0xFFFFFFFFu);
        if (variant == 0) {
            mask[0] = mask[1] = 0;  // clear bits 0..63
        } else {
            for (int i = 0; i < ncu; ++i)  // clear every 4th bit
                if (i % 4 == 0) mask[i / 32] &= ~(1u << (i % 32));
        }
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()));
        CK(hipMemset(d, 0, sizeof(uint32_t) * 2 * nb));
        where_kernel<<<nb, 64, 0, s>>>(d, 200);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d, sizeof(uint32_t) * 2 * nb, hipMemcpyDeviceToHost));
        report(variant == 0 ? "mask without bits 0..63" : "mask without every 4th bit", h, nb);
        CK(hipStreamDestroy(s));
    }
    return 0;
}
