// Fast translation unit (-ffp-contract=fast): wave-tree dot products and
// fused multiply-adds.  Results agree with the strict path within the 1e-9
// relative tolerance of BASELINE.json's north_star.
#include "kernels.h"
#include "solver_impl.h"
#include "wave.h"

namespace cocoa {

void launch_solver_fast(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                        hipStream_t s) {
    launch_solver_impl<false>(mode, vec_lds, alpha_lds, a, grid, lds, s);
}

// ----------------------------------------------------------- fused eval --
// One pass over train + test CSR (OptUtils.scala:57-98): 16-lane groups per
// row (one DPP row), 4 entries per lane in flight, w gathered from L2; the
// same launch sums alpha and ||w||^2.  Block partials -> fixed-order final
// reduction (deterministic run to run).
constexpr int kEvalBlock = 256;
constexpr int kEvalMaxBlocks = 2048;

__global__ __launch_bounds__(kEvalBlock) void eval_fast_kernel(EvalArgs a) {
    __shared__ double red[4][kEvalBlock / 64];
    const int tid = threadIdx.x;
    const int sub = tid & 15;
    const int64_t ngroups = (int64_t)gridDim.x * (kEvalBlock / 16);
    const int64_t g0 = (int64_t)blockIdx.x * (kEvalBlock / 16) + (tid >> 4);
    const int64_t rows = a.n + a.n_test;
    double hinge = 0.0, err = 0.0;
    for (int64_t r = g0; r < rows; r += ngroups) {
        const bool test = r >= a.n;
        const int64_t rr = test ? r - a.n : r;
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const int32_t* cl = test ? a.t_col : a.col;
        const double* vl = test ? a.t_val : a.val;
        const int64_t b = rp[rr], e = rp[rr + 1];
        double acc0 = 0.0, acc1 = 0.0;
        int64_t q = b + sub;
        for (; q + 48 < e; q += 64) {
            const int32_t c0 = cl[q], c1 = cl[q + 16], c2 = cl[q + 32], c3 = cl[q + 48];
            const double v0 = vl[q], v1 = vl[q + 16], v2 = vl[q + 32], v3 = vl[q + 48];
            acc0 += v0 * a.w[c0];
            acc1 += v1 * a.w[c1];
            acc0 += v2 * a.w[c2];
            acc1 += v3 * a.w[c3];
        }
        for (; q < e; q += 16) acc0 += vl[q] * a.w[cl[q]];
        const double dot = row16_sum(acc0 + acc1);
        if (sub == 0) {
            if (!test)
                hinge += jmax(1 - a.y[rr] * dot, 0.0);
            else
                err += (dot * a.t_y[rr] > 0) ? 0.0 : 1.0;
        }
    }
    const int64_t gt = (int64_t)blockIdx.x * kEvalBlock + tid;
    const int64_t gs = (int64_t)gridDim.x * kEvalBlock;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    const double v[4] = {wave_sum(hinge), wave_sum(al), wave_sum(w2), wave_sum(err)};
    if ((tid & 63) == 0)
        for (int i = 0; i < 4; ++i) red[i][tid >> 6] = v[i];
    __syncthreads();
    if (tid < 4) {
        double s = 0.0;
        for (int wv = 0; wv < kEvalBlock / 64; ++wv) s += red[tid][wv];
        a.partials[(size_t)blockIdx.x * 4 + tid] = s;
    }
}

__global__ __launch_bounds__(256) void eval_final_kernel(const double* partials, int blocks, double* out) {
    __shared__ double red[4][4];
    const int tid = threadIdx.x;
    double v[4] = {0, 0, 0, 0};
    for (int b = tid; b < blocks; b += 256)
        for (int i = 0; i < 4; ++i) v[i] += partials[(size_t)b * 4 + i];
    for (int i = 0; i < 4; ++i) {
        const double s = wave_sum(v[i]);
        if ((tid & 63) == 0) red[i][tid >> 6] = s;
    }
    __syncthreads();
    if (tid < 4) out[tid] = ((red[tid][0] + red[tid][1]) + red[tid][2]) + red[tid][3];
}

int eval_fast_blocks(int64_t n, int64_t n_test) {
    const int64_t rows = n + n_test;
    int64_t b = (rows + (kEvalBlock / 16) - 1) / (kEvalBlock / 16);
    if (b > kEvalMaxBlocks) b = kEvalMaxBlocks;
    if (b < 1) b = 1;
    return (int)b;
}

void launch_eval_fast(const EvalArgs& a, int blocks, hipStream_t s) {
    eval_fast_kernel<<<blocks, kEvalBlock, 0, s>>>(a);
    eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
}

}  // namespace cocoa
