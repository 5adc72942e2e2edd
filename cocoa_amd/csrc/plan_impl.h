// Per-round step plan, shared by the strict and fast translation units.
//
// For every step (k, s) of the round: the sampled row's entry offset, nnz,
// label, ||x||^2 and x.w (w is read-only within a round for CoCoA+ and MbCD,
// CoCoA.scala:159 / MinibatchCD.scala:104).  One chip-wide pass, so the local
// solvers' loader waves read one coalesced record per step instead of the
// samples -> row_ptr -> (col, val) -> w chain.
// STRICT: one lane per step, x.w summed sequentially in stored order (the
// reference's SparseVector.dot); fast: 16 lanes per step, DPP row sum, FMA.
// One thread per step when no dot is formed here (strict, x.w reused from the
// eval, or CoCoA), 16 otherwise; plan_threads_per_step is the shared rule.
#pragma once
#include "kernels.h"
#include "wave.h"

namespace cocoa {

__host__ __device__ __forceinline__ int plan_threads_per_step(bool strict, const PlanArgs& a) {
    return (strict || !a.need_xw || a.xw_cache) ? 1 : 16;
}

// Look-back of the Gram-window solver's alpha forwarding (solver_gram.h): for
// step j of a partition, the latest earlier step j' of the same partition with
// the same sampled row inside j's window [16 floor(j/16) - win, j), or -1.  The
// step whose alpha update a later step must see before the deltaW it reads
// (CoCoA.scala:151, 186): the loader marks j' to forward its new alpha to j.
// Formed here, chip-wide and beside the previous round, instead of by the
// loader wave's 16-step ballot search (3,500 of its ~10,400 cycles per batch
// on C2, r08c).  The block's samples and the 63 before them are staged in LDS.
constexpr int kPlanLook = 79;  // >= win + 15 for every window the solver takes (kGW <= 64)

template <bool STRICT>
__global__ __launch_bounds__(256) void plan_kernel(PlanArgs a) {
    const int tid = threadIdx.x;
    const int per = plan_threads_per_step(STRICT, a);
    const int64_t g = (int64_t)blockIdx.x * (256 / per) + tid / per;
    const int sub = tid % per;
    const bool valid = g < a.steps;
    const int64_t gg = valid ? g : 0;
    __shared__ int32_t sw[256 + kPlanLook];  // samples of steps [gb - kPlanLook, gb + 256 / per)
    const int64_t gb = (int64_t)blockIdx.x * (256 / per);
    if (a.win > 0) {
        for (int i = tid; i < 256 / per + kPlanLook; i += 256) {
            const int64_t q = gb - kPlanLook + i;
            sw[i] = (q >= 0 && q < a.steps) ? a.samples[q] : -1;
        }
        __syncthreads();
    }
    const int32_t k = (int32_t)(gg / a.H);
    const int64_t gr = a.part_ptr[k] + a.samples[gg];
    const int64_t b = a.row_ptr[gr], e = a.row_ptr[gr + 1];
    double xw = 0.0;
    if (a.need_xw && a.xw_cache) {
        xw = valid ? a.xw_cache[gr] : 0.0;  // the last eval pass already formed x.w for this w
    } else if (a.need_xw) {
        if (STRICT) {
            for (int64_t q = b; q < e; ++q) xw += a.val[q] * a.w[a.col[q]];
        } else {
            double acc = 0.0;
            for (int64_t q = b + sub; q < e; q += 16) acc += a.val[q] * a.w[a.col[q]];
            xw = row16_sum(acc);
        }
    }
    if (valid && sub == 0) {  // read once by the solver's loader: nontemporal, like its reads
        __builtin_nontemporal_store(b, a.beg + g);
        __builtin_nontemporal_store(a.row_zs ? a.row_zs[gr] : (int32_t)(e - b), a.z + g);
        __builtin_nontemporal_store(a.y[gr], a.py + g);
        __builtin_nontemporal_store(a.sqn[gr], a.pq + g);
        if (a.xw) __builtin_nontemporal_store(xw, a.xw + g);  // (null: xw_produce_kernel forms x.w)
        if (a.zc) {
            // the ends of the row's column runs 0 .. R-2 (all of it in run 0 without
            // row_zc), and the step's look-back (above) in the last word (the row's
            // length there is plan z's)
            typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
            const int32_t zz = (int32_t)(e - b);
            if (kGramRuns == 8) {
                const i32x4 lo = a.row_zc ? *(const i32x4*)(a.row_zc + kGramRuns * gr) : i32x4{zz, zz, zz, zz};
                __builtin_nontemporal_store(lo, (i32x4*)(a.zc + kGramRuns * g));
            }
            i32x4 z4 = a.row_zc ? *(const i32x4*)(a.row_zc + kGramRuns * gr + kGramRuns - 4) : i32x4{zz, zz, zz, zz};
            int32_t prev = -1;
            if (a.win > 0) {
                const int32_t j = (int32_t)(g - (int64_t)k * a.H);
                const int32_t lo = max((j / 16) * 16 - a.win, 0);
                const int32_t me = a.samples[g];
                const int iw = (int)(g - gb) + kPlanLook;
                for (int32_t jp = j - 1; jp >= lo; --jp)
                    if (sw[iw - (j - jp)] == me) {
                        prev = jp;
                        break;
                    }
            }
            z4.w = prev;
            __builtin_nontemporal_store(z4, (i32x4*)(a.zc + kGramRuns * g + kGramRuns - 4));
        }
    }
}

template <bool STRICT>
void launch_plan_impl(const PlanArgs& a, hipStream_t s) {
    const int per = plan_threads_per_step(STRICT, a);
    const int64_t blocks = (a.steps * per + 255) / 256;
    if (blocks > 0) plan_kernel<STRICT><<<(unsigned)blocks, 256, 0, s>>>(a);
}

}  // namespace cocoa
