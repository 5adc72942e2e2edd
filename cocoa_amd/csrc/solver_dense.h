// Dense rows (config C3, epsilon-shaped: every row stores all d features in
// index order), fast mode.  The CSR value array of such data IS the row-major
// matrix X[n][d], so these kernels read 8 B per entry instead of 12 and no
// column indices at all.
//
// dense_solver_kernel -- CoCoA.localSDCA (CoCoA.scala:148-188) and the MbCD
// local solver (MinibatchCD.scala:95-125), one 256-thread workgroup per
// partition.  deltaW and w never touch memory during the round: thread t owns
// the 16-byte column chunks t, t + 256, ... of the row and keeps w and deltaW
// for those columns in registers.  Per step:
//   1. the thread's partial of x.w (+ sigma x.deltaW for CoCoA+, + x.deltaW
//      for CoCoA, whose task-local w is w + deltaW) over its chunks (FMA);
//   2. a DPP wave sum, one LDS slot per wave, ONE workgroup barrier, and every
//      thread adds the 4 wave sums in the same order (so every thread holds the
//      same dot and evaluates the same update rule: no broadcast round trip);
//   3. deltaW += c x on the thread's chunks, in registers; lane 0 of every
//      wave stores the new alpha (alpha of the partition lives in LDS; each
//      wave reads it before the barrier, after its own earlier stores).
// The rows are streamed P steps ahead of the chain into a register ring
// (nontemporal 16-byte loads; each row is read about once per round), and the
// per-step records (sampled row, y, ||x||^2 from the plan kernel) one and two
// groups of P steps ahead, lane j of a record register holding step
// group*P + j, read with v_readlane: no load on the chain depends on another.
//
// eval_dense_kernel -- OptUtils.scala:57-98 over dense train + test rows: one
// wave per row (two rows in flight per wave), w in registers, DPP row sum.
#pragma once
#include "kernels.h"
#include "wave.h"

namespace cocoa {

typedef double f64x2v __attribute__((ext_vector_type(2)));

// threads of a dense-solver workgroup: one wave per SIMD.  The chain is issue
// bound -- every wave runs the whole per-step sequence (DPP reduction, update
// rule, address arithmetic, ~100 instructions around its FMAs), so two waves
// per SIMD (512 threads) took twice the cycles per step of one (C3: 2.70 ms
// per round with 512 threads)
constexpr int kDT = 256;

__device__ __forceinline__ f64x2v ld_nt2(const double* p) { return __builtin_nontemporal_load((const f64x2v*)p); }


template <int MODE, int CPT, int P, int NTH, bool PROJ>
__global__ __launch_bounds__(NTH) void dense_solver_kernel(DenseArgs a) {
    constexpr int NWV = NTH / 64;
    extern __shared__ double al[];  // alpha of the partition (rows [p0, p0 + nl))
    __shared__ double red[2][NWV];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = blockIdx.x;
    const int64_t p0 = a.part_ptr[k];
    const int32_t nl = (int32_t)(a.part_ptr[k + 1] - p0);
    const int32_t H = a.H;
    const int64_t d = a.d, nch = d >> 1;
    for (int i = tid; i < nl; i += NTH) al[i] = a.alpha[p0 + i];

    int64_t cof[CPT];
    bool okc[CPT];
    f64x2v wr[CPT], dr[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int64_t ci = tid + (int64_t)NTH * c;
        const bool ok = ci < nch;
        okc[c] = ok;
        cof[c] = 2 * (ok ? ci : nch - 1);  // past the row: an in-row address, w = deltaW = 0 (kept 0)
        wr[c] = ok ? *(const f64x2v*)(a.w + 2 * ci) : f64x2v{0.0, 0.0};
        dr[c] = f64x2v{0.0, 0.0};
    }
    const double* X = a.X + p0 * d;
    const size_t sb = (size_t)k * (size_t)H;
    const int jl = lane & (P - 1);
    // records of group g: lane j -> step g*P + j (clamped to the last step)
    auto rec_r = [&](int64_t g) { return a.samples[sb + (size_t)min<int64_t>(g * P + jl, H - 1)]; };
    auto rec_y = [&](int64_t g) { return a.plan_y[sb + (size_t)min<int64_t>(g * P + jl, H - 1)]; };
    auto rec_q = [&](int64_t g) { return a.plan_q[sb + (size_t)min<int64_t>(g * P + jl, H - 1)]; };

    int32_t r0 = rec_r(0), r1 = rec_r(1);
    double y0 = rec_y(0), y1 = rec_y(1), q0 = rec_q(0), q1 = rec_q(1);
    f64x2v xs[P][CPT];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const double* xr = X + (int64_t)__builtin_amdgcn_readlane(r0, j) * d;
#pragma unroll
        for (int c = 0; c < CPT; ++c) xs[j][c] = ld_nt2(xr + cof[c]);
    }
    __syncthreads();  // alpha staged

    const int64_t G = ((int64_t)H + P - 1) / P;
    for (int64_t g = 0; g < G; ++g) {
        // records two groups ahead (their loads have a whole group to land)
        const int32_t r2 = rec_r(g + 2);
        const double y2 = rec_y(g + 2), q2 = rec_q(g + 2);
        // this group's 1 / qii (off the chain); -1 marks qii == 0 (alpha -> 1)
        const double qii = MODE == MODE_PLUS ? q0 * a.sigma : q0;
        const double rq0 = qii != 0.0 ? 1.0 / qii : -1.0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t s = g * P + j;
            if (s < H) {
                double t0 = 0.0, t1 = 0.0;
#pragma unroll
                for (int c = 0; c < CPT; ++c) {
                    const f64x2v x = xs[j][c];
                    t0 = fma(x.x, wr[c].x, t0);
                    t0 = fma(x.y, wr[c].y, t0);
                    if (MODE != MODE_MBCD) {
                        t1 = fma(x.x, dr[c].x, t1);
                        t1 = fma(x.y, dr[c].y, t1);
                    }
                }
                // alpha before the barrier: every wave stores the new alpha itself
                // (the same value in all waves), so its own stores of earlier steps
                // precede this read in program order, and no wave stores this
                // step's value before all waves have passed the barrier
                const int32_t r = __builtin_amdgcn_readlane(r0, j);
                const double aa = al[r];
                const double t = MODE == MODE_PLUS ? fma(a.sigma, t1, t0) : (MODE == MODE_COCOA ? t0 + t1 : t0);
                const double ws = wave_sum(t);
                if (lane == 0) red[s & 1][wv] = ws;
                __syncthreads();
                double tot = red[s & 1][0];
#pragma unroll
                for (int i = 1; i < NWV; ++i) tot += red[s & 1][i];
                const double yv = readlane_d(y0, j), rq = readlane_d(rq0, j);
                const double grad = (yv * tot - 1.0) * a.lam_n;  // CoCoA.scala:157-163
                // projection + skip (CoCoA.scala:166-172) fold into the clamp while aa
                // lies in [0, 1]: a vanishing projected gradient returns aa, so c = 0.
                // PROJ (alpha possibly outside [0, 1]): the explicit skip test.
                double nt = rq < 0.0 ? 1.0 : fmin(fmax(aa - grad * rq, 0.0), 1.0);
                if (PROJ) {
                    const double pg = aa <= 0.0 ? fmin(grad, 0.0) : (aa >= 1.0 ? fmax(grad, 0.0) : grad);
                    if (pg == 0.0) nt = aa;
                }
                const double cc = yv * (nt - aa) * a.inv_lam_n;  // CoCoA.scala:181
                if (lane == 0) al[r] = nt;
#pragma unroll
                for (int c = 0; c < CPT; ++c) {
                    const double cm = okc[c] ? cc : 0.0;
                    dr[c].x = fma(cm, xs[j][c].x, dr[c].x);
                    dr[c].y = fma(cm, xs[j][c].y, dr[c].y);
                }
            }
            // refill slot j with step (g + 1) P + j
            const double* xr = X + (int64_t)__builtin_amdgcn_readlane(r1, j) * d;
#pragma unroll
            for (int c = 0; c < CPT; ++c) xs[j][c] = ld_nt2(xr + cof[c]);
        }
        r0 = r1;
        y0 = y1;
        q0 = q1;
        r1 = r2;
        y1 = y2;
        q1 = q2;
    }
    // deltaW slice of the partition (all d entries: the slice needs no zeroing)
    double* dk = a.dw + (size_t)k * (size_t)d;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int64_t ci = tid + (int64_t)NTH * c;
        if (ci < nch) *(f64x2v*)(dk + 2 * ci) = dr[c];
    }
    __syncthreads();
    // alpha <- alphaOld + (alpha - alphaOld) * scaling (CoCoA.scala:101)
    for (int i = tid; i < nl; i += NTH) {
        const double old = a.alpha[p0 + i];
        a.alpha[p0 + i] = old + (al[i] - old) * a.scaling;
    }
}

// ------------------------------------------------------------------ eval --
template <int CE, int R>
__global__ __launch_bounds__(256) void eval_dense_kernel(EvalArgs a) {
    __shared__ double red[4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t d = a.d, nch = d >> 1;
    int64_t cof[CE];
    f64x2v wr[CE];
#pragma unroll
    for (int c = 0; c < CE; ++c) {
        const int64_t ci = lane + 64 * (int64_t)c;
        const bool ok = ci < nch;
        cof[c] = 2 * (ok ? ci : nch - 1);
        wr[c] = ok ? *(const f64x2v*)(a.w + 2 * ci) : f64x2v{0.0, 0.0};
    }
    const int64_t rows = a.n + a.n_test;
    const int64_t gw = (int64_t)blockIdx.x * 4 + wv, nw = (int64_t)gridDim.x * 4;
    double hinge = 0.0, err = 0.0;
    for (int64_t r = gw * R; r < rows; r += nw * R) {
        f64x2v x[R][CE];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int64_t rr = min<int64_t>(r + i, rows - 1);
            const double* xr = rr < a.n ? a.val + rr * d : a.t_val + (rr - a.n) * d;
#pragma unroll
            for (int c = 0; c < CE; ++c) x[i][c] = ld_nt2(xr + cof[c]);
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
            double t0 = 0.0, t1 = 0.0;
#pragma unroll
            for (int c = 0; c < CE; ++c) {
                t0 = fma(x[i][c].x, wr[c].x, t0);
                t1 = fma(x[i][c].y, wr[c].y, t1);
            }
            const double dot = wave_sum(t0 + t1);
            const int64_t rr = r + i;
            if (lane == 0 && rr < rows) {
                if (rr < a.n) {
                    hinge += fmax(1.0 - a.y[rr] * dot, 0.0);  // OptUtils.scala:57-60
                    if (a.row_xw) a.row_xw[rr] = dot;
                } else {
                    err += (dot * a.t_y[rr - a.n] > 0) ? 0.0 : 1.0;  // OptUtils.scala:95-98
                }
            }
        }
    }
    const int64_t gt = (int64_t)blockIdx.x * 256 + tid, gs = (int64_t)gridDim.x * 256;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    double v[4] = {hinge, al, w2, err};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double s = wave_sum(v[i]);
        __syncthreads();
        if (lane == 0) red[wv] = s;
        __syncthreads();
        if (tid == 0) a.partials[(size_t)blockIdx.x * 4 + i] = ((red[0] + red[1]) + red[2]) + red[3];
    }
}

}  // namespace cocoa
