// java.util.Random (the JDK's 48-bit LCG) for host and device, as drawn by
// scala.util.Random(seed) in CoCoA.scala:144,151 (and MinibatchCD.scala:91,98,
// SGD.scala:99,109).  The device sampler uses the affine jump-ahead
//   s_{m+k} = A_k * s_m + C_k  (mod 2^48)
// so that 256 threads draw consecutive raw values in parallel.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define COCOA_HD __host__ __device__
#else
#define COCOA_HD
#endif

namespace cocoa {

constexpr uint64_t kJrMult = 0x5DEECE66DULL;
constexpr uint64_t kJrAdd = 0xBULL;
constexpr uint64_t kJrMask = (1ULL << 48) - 1;

COCOA_HD inline uint64_t jr_scramble(int64_t seed) { return ((uint64_t)seed ^ kJrMult) & kJrMask; }
COCOA_HD inline uint64_t jr_step(uint64_t s) { return (s * kJrMult + kJrAdd) & kJrMask; }
// next(31) of the state *after* the step
COCOA_HD inline int32_t jr_bits31(uint64_t s) { return (int32_t)(s >> 17); }

// Random.nextInt(bound) acceptance for a raw next(31) value: returns true and
// the value when accepted (power-of-two bounds always accept).
COCOA_HD inline bool jr_accept(int32_t bits, int32_t bound, int32_t* out) {
    const int32_t m = bound - 1;
    if ((bound & m) == 0) {
        *out = (int32_t)(((int64_t)bound * (int64_t)bits) >> 31);
        return true;
    }
    const int32_t v = bits % bound;
    *out = v;
    // Java int arithmetic: bits - v + m overflows negative => reject
    return (int32_t)((uint32_t)bits - (uint32_t)v + (uint32_t)m) >= 0;
}

// compose affine maps: apply (a1,c1) then (a2,c2)
COCOA_HD inline void jr_compose(uint64_t a1, uint64_t c1, uint64_t a2, uint64_t c2, uint64_t* a, uint64_t* c) {
    *a = (a2 * a1) & kJrMask;
    *c = (a2 * c1 + c2) & kJrMask;
}

// (A_k, C_k) for k steps
COCOA_HD inline void jr_jump(uint64_t k, uint64_t* A, uint64_t* C) {
    uint64_t ra = 1, rc = 0, ba = kJrMult, bc = kJrAdd;
    while (k) {
        if (k & 1) jr_compose(ra, rc, ba, bc, &ra, &rc);
        jr_compose(ba, bc, ba, bc, &ba, &bc);
        k >>= 1;
    }
    *A = ra;
    *C = rc;
}

struct JRandom {
    uint64_t s;
    COCOA_HD explicit JRandom(int64_t seed) : s(jr_scramble(seed)) {}
    COCOA_HD int32_t next(int bits) {
        s = jr_step(s);
        return (int32_t)(uint32_t)(s >> (48 - bits));
    }
    COCOA_HD int32_t next_int(int32_t bound) {
        for (;;) {
            int32_t v;
            if (jr_accept(next(31), bound, &v)) return v;
        }
    }
};

}  // namespace cocoa
