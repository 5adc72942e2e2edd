// Wave-level (64-lane) helpers for gfx950: DPP reductions for fp64, uniform
// broadcasts, Java Math.min/max semantics, LDS ordering inside one wave.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cocoa {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Broadcast lane 0 (first active lane) -> SGPR: marks values wave-uniform.
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double uni(double x) { return __longlong_as_double(uni((int64_t)__double_as_longlong(x))); }

__device__ __forceinline__ double readlane_d(double x, int l) {
    const int64_t b = __double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)((uint64_t)b >> 32), l);
    return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ int64_t readlane_i64(int64_t x, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)x, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)((uint64_t)x >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Move a double through DPP (both 32-bit halves with the same control).
// Lanes whose source is disabled / out of row receive +0.0.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ double dpp_d(double x) {
    const int64_t b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, BANK_MASK, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)b >> 32), CTRL, ROW_MASK, BANK_MASK, false);
    return __longlong_as_double((int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// In-row DPP move with every source lane valid (quad_perm / row_ror): no
// "old" operand, so no zero-initialising moves are emitted.
template <int CTRL>
__device__ __forceinline__ double dpp_row_d(double x) {
    const int64_t b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double((int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// Sum within each DPP row of 16 lanes; every lane of the row ends with the sum.
__device__ __forceinline__ double row16_sum(double x) {
    x += dpp_row_d<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_row_d<0x4E>(x);   // quad_perm [2,3,0,1]
    x += dpp_row_d<0x124>(x);  // row_ror:4
    x += dpp_row_d<0x128>(x);  // row_ror:8
    return x;
}

// Full 64-lane sum, returned wave-uniform (all lanes identical).
__device__ __forceinline__ double wave_sum(double x) {
    x = row16_sum(x);
    x += dpp_d<0x142, 0xA>(x);  // row_bcast:15 -> rows 1,3
    x += dpp_d<0x143, 0xC>(x);  // row_bcast:31 -> rows 2,3
    return readlane_d(x, 63);
}

// Inclusive prefix max of an int over the wave in lane order (all lanes
// active; values >= -1): row_shr steps inside each 16-lane row, then the
// row_bcast:15 / row_bcast:31 carries between rows.  DPP only, no LDS.
__device__ __forceinline__ int32_t wave_incl_max(int32_t x) {
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));  // row_shr:1
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));  // row_shr:2
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));  // row_shr:4
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));  // row_shr:8
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false));  // row_bcast:15 -> rows 1, 3
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false));  // row_bcast:31 -> rows 2, 3
    return x;
}

// Inclusive prefix sum of an int within each DPP row of 16 lanes (four
// independent scans, DPP only: four VALU moves, no LDS round trip).
__device__ __forceinline__ int32_t row16_incl_scan(int32_t x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
    return x;
}

// Inclusive prefix sum of an int over the wave (all lanes active): the row
// scans, then the row_bcast:15 / row_bcast:31 carries as in wave_incl_max.
// DPP only (the __shfl_up form took six LDS round trips).
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x) {
    x = row16_incl_scan(x);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Order LDS writes of some lanes before LDS reads of other lanes in the SAME
// wave (LDS executes one wave's operations in order; this only stops the
// compiler from reordering across the point).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// java.lang.Math.max / min on doubles: NaN-propagating, -0.0 < +0.0.
__device__ __forceinline__ double jmax(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0) return signbit(a) ? b : a;
    return a >= b ? a : b;
}
__device__ __forceinline__ double jmin(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0) return signbit(a) ? a : b;
    return a <= b ? a : b;
}

}  // namespace cocoa
