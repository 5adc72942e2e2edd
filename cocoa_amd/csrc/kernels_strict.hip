// Strict translation unit: compiled with -ffp-contract=off so that every
// multiply and add rounds exactly like the JVM reference (no FMA).  Holds the
// bit-exact local solver instantiations and every kernel whose result feeds
// the shared state (sampler, deltaW fold, w apply, strict evaluation, SGD).
#include "jrandom.h"
#include "kernels.h"
#include "plan_impl.h"
#include "solver_impl.h"
#include "wave.h"

namespace cocoa {

void launch_solver_strict(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                          hipStream_t s) {
    launch_solver_impl<true>(mode, vec_lds, alpha_lds, a, grid, lds, s);
}

void launch_plan_strict(const PlanArgs& a, hipStream_t s) { launch_plan_impl<true>(a, s); }

// ---------------------------------------------------------------- sampler --
// Partition k draws java.util.Random(seed).nextInt(n_k) H times
// (CoCoA.scala:144,151).  Thread t of the block produces raw draw number
// 256*c + t + 1 through the affine jump table; accepted draws are compacted
// in order (a rejected raw value is skipped exactly as nextInt's loop does).
// jt[2*(j-1)], jt[2*(j-1)+1] = (A_j, C_j) for j = 1..256.
__global__ __launch_bounds__(256) void sampler_kernel(const int64_t* part_ptr, int32_t seed, int32_t H,
                                                      int32_t* samples, const uint64_t* jt) {
    __shared__ int32_t wtot[4];
    const int k = blockIdx.x;
    const int t = threadIdx.x;
    const int lane = t & 63, wv = t >> 6;
    const int32_t bound = (int32_t)(part_ptr[k + 1] - part_ptr[k]);
    int32_t* out = samples + (size_t)k * H;
    if (bound <= 0) return;
    const uint64_t s0 = jr_scramble((int64_t)seed);
    uint64_t st = (jt[2 * t] * s0 + jt[2 * t + 1]) & kJrMask;
    const uint64_t A256 = jt[2 * 255], C256 = jt[2 * 255 + 1];
    int32_t base = 0;
    while (base < H) {
        int32_t v;
        const bool acc = jr_accept(jr_bits31(st), bound, &v);
        const uint64_t bal = __ballot(acc);
        const int32_t pre = (int32_t)__popcll(bal & ((1ULL << lane) - 1ULL));
        if (lane == 0) wtot[wv] = (int32_t)__popcll(bal);
        __syncthreads();
        int32_t off = 0, tot = 0;
        for (int i = 0; i < 4; ++i) {
            if (i < wv) off += wtot[i];
            tot += wtot[i];
        }
        const int32_t pos = base + off + pre;
        if (acc && pos < H) out[pos] = v;
        base += tot;
        st = (A256 * st + C256) & kJrMask;
        __syncthreads();
    }
}

void launch_sampler(const int64_t* part_ptr, int32_t K, int32_t seed, int32_t H, int32_t* samples,
                    const uint64_t* jump_tab, hipStream_t s) {
    sampler_kernel<<<K, 256, 0, s>>>(part_ptr, seed, H, samples, jump_tab);
}

// ------------------------------------------------------- deltaW fold/apply --
// sum = ((dW_0 + dW_1) + dW_2) + ... in partition order (the reference's
// reduce(_ + _), CoCoA.scala:47), zeroing each private slice for the next
// round; then w += sum * mult (CoCoA.scala:48) or the sum is stored for the
// exchange between ranks.  init (original feature order, or null): the fold
// of the previous ranks' partitions, which this rank's fold continues (the
// strict-mode chain across ranks keeps the single-process fold order).
__global__ __launch_bounds__(256) void fold_kernel(double* dw, int32_t K, int64_t d, double* dw_sum, double* w,
                                                   double mult, int apply, const int32_t* inv, int zero,
                                                   const double* init) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t jo = inv ? inv[j] : j;
        double s = init ? init[jo] + dw[j] : dw[j];
        if (zero) dw[j] = 0.0;
        int32_t k = 1;
        // eight slices' loads in flight at a time (the zero stores, which may
        // alias as far as the compiler knows, go after them); partition order kept
        for (; k + 8 <= K; k += 8) {
            double v[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] = dw[(size_t)(k + t) * d + j];
#pragma unroll
            for (int t = 0; t < 8; ++t) s = s + v[t];
            if (zero) {
#pragma unroll
                for (int t = 0; t < 8; ++t) dw[(size_t)(k + t) * d + j] = 0.0;
            }
        }
        for (; k < K; ++k) {
            const size_t o = (size_t)k * d + j;
            s = s + dw[o];
            if (zero) dw[o] = 0.0;
        }
        if (apply)
            w[j] = w[j] + (s * mult);
        else
            dw_sum[jo] = s;
    }
}

__global__ void status_slot_kernel(const int* status, double* slot) { *slot = status[0] != 0 ? 1.0 : 0.0; }

void launch_status_slot(const int* status, double* slot, hipStream_t s) { status_slot_kernel<<<1, 1, 0, s>>>(status, slot); }

void launch_fold(const double* dw, int32_t K, int64_t d, double* dw_sum, double* w, double mult, bool apply,
                 const int32_t* inv, bool zero, hipStream_t s, const double* init) {
    int blocks = (int)std::min<int64_t>((d + 255) / 256, 2048);
    if (blocks < 1) blocks = 1;
    fold_kernel<<<blocks, 256, 0, s>>>(const_cast<double*>(dw), K, d, dw_sum, w, mult, apply ? 1 : 0, inv,
                                       zero ? 1 : 0, init);
}

// Fold of compact deltaW slices (C4 layout, cocoa_ctx::compact_ready): one
// thread per device column j sums the slice entries that hold j in partition
// order -- the dense fold's order with its zero terms dropped -- and, with a
// single slice set, zeroes them for the next round (double-buffered sets are
// re-zeroed by a streaming memset beside the next round's solver instead:
// the scattered 8-byte zero stores cost a partial-line write each).  Device order puts the columns every partition
// touches first, and a partition's slice lists its columns in device order,
// so the threads of a wave read neighbouring positions of each slice.
__global__ __launch_bounds__(256) void fold_compact_kernel(double* dw, const int64_t* fptr, const uint32_t* fpos,
                                                           int64_t d, double* dw_sum, double* w, double mult,
                                                           int apply, const int32_t* inv, const double* init, int zero) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t jo = inv ? inv[j] : j;
        const int64_t b = fptr[j], e = fptr[j + 1];
        double s = 0.0;
        int64_t q = b;
        if (q < e) {
            const uint32_t p = fpos[q++];
            s = init ? init[jo] + dw[p] : dw[p];
            if (zero) dw[p] = 0.0;
        } else if (init) {
            s = init[jo];
        }
        for (; q + 4 <= e; q += 4) {  // four independent gathers in flight
            const uint32_t p0 = fpos[q], p1 = fpos[q + 1], p2 = fpos[q + 2], p3 = fpos[q + 3];
            const double v0 = dw[p0], v1 = dw[p1], v2 = dw[p2], v3 = dw[p3];
            s = s + v0;
            s = s + v1;
            s = s + v2;
            s = s + v3;
            if (zero) {
                dw[p0] = 0.0;
                dw[p1] = 0.0;
                dw[p2] = 0.0;
                dw[p3] = 0.0;
            }
        }
        for (; q < e; ++q) {
            const uint32_t p = fpos[q];
            s = s + dw[p];
            if (zero) dw[p] = 0.0;
        }
        if (apply)
            w[j] = w[j] + (s * mult);
        else
            dw_sum[jo] = s;
    }
}

void launch_fold_compact(double* dw, const int64_t* fptr, const uint32_t* fpos, int64_t d, double* dw_sum, double* w,
                         double mult, bool apply, const int32_t* inv, bool zero, hipStream_t s, const double* init) {
    int blocks = (int)std::min<int64_t>((d + 255) / 256, 8192);
    if (blocks < 1) blocks = 1;
    fold_compact_kernel<<<blocks, 256, 0, s>>>(dw, fptr, fpos, d, dw_sum, w, mult, apply ? 1 : 0, inv, init,
                                               zero ? 1 : 0);
}

// Background re-zeroing of a folded deltaW set (double-buffered slices): a
// narrow grid of 16-byte non-temporal stores, so it drains at a bounded rate
// beside the latency-bound local solver instead of competing for all of HBM.
__global__ __launch_bounds__(256) void zero_kernel(double* p, int64_t n2) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    f64x2* q = (f64x2*)p;
    const f64x2 z = {0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
        __builtin_nontemporal_store(z, q + i);
}

void launch_zero(double* p, int64_t n, int blocks, hipStream_t s) {
    if (n & 1) (void)hipMemsetAsync(p + n - 1, 0, sizeof(double), s);
    if (n >= 2) zero_kernel<<<blocks < 1 ? 1 : blocks, 256, 0, s>>>(p, n / 2);
}

// column indices of dense rows (entry q of row-major X[n][d] is column q mod d),
// built on the device only when a CSR kernel needs them (strict mode, the
// chain / SGD solvers): cocoa_set_train_dense keeps no column array
__global__ __launch_bounds__(256) void dense_cols_kernel(int32_t* col, uint16_t* col16, int64_t nnz, int32_t d) {
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nnz; q += (int64_t)gridDim.x * 256) {
        const int32_t c = (int32_t)(q % d);
        col[q] = c;
        if (col16) col16[q] = (uint16_t)c;
    }
}

// The multi-device context's fast exchange, member r's part of the
// reduce-scatter: own[j] = ((x_0[j] + x_1[j]) + x_2[j]) + ... over the n
// members in member order, where x_r is own itself and the others' pieces sit
// in stage[0 .. n-2] (member q at q, or q-1 past r), len doubles each.
__global__ __launch_bounds__(256) void sum_slices_kernel(double* own, const double* stage, int32_t n, int32_t r,
                                                         int64_t len) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < len; j += (int64_t)gridDim.x * 256) {
        double acc = 0.0;
        for (int32_t q = 0; q < n; ++q) {
            const double v = q == r ? own[j] : stage[(size_t)(q < r ? q : q - 1) * (size_t)len + (size_t)j];
            acc = q == 0 ? v : acc + v;
        }
        own[j] = acc;
    }
}

void launch_sum_slices(double* own, const double* stage, int32_t n, int32_t r, int64_t len, hipStream_t s) {
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((len + 255) / 256, 2048));
    if (n > 1 && len > 0) sum_slices_kernel<<<blocks, 256, 0, s>>>(own, stage, n, r, len);
}

void launch_dense_cols(int32_t* col, uint16_t* col16, int64_t nnz, int32_t d, hipStream_t s) {
    if (nnz > 0) dense_cols_kernel<<<2048, 256, 0, s>>>(col, col16, nnz, d);
}

__global__ __launch_bounds__(256) void apply_kernel(double* w, const double* dw_sum, int64_t d, double mult,
                                                    const int32_t* inv) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
        w[j] = w[j] + (dw_sum[inv ? inv[j] : j] * mult);
}

void launch_apply(double* w, const double* dw_sum, int64_t d, double mult, const int32_t* inv, hipStream_t s) {
    int blocks = (int)std::min<int64_t>((d + 255) / 256, 2048);
    apply_kernel<<<blocks < 1 ? 1 : blocks, 256, 0, s>>>(w, dw_sum, d, mult, inv);
}

__global__ __launch_bounds__(256) void scale_kernel(double* w, int64_t d, double scale) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
        w[j] = w[j] * scale;  // w :*= scale (SGD.scala:49)
}

void launch_scale(double* w, int64_t d, double scale, hipStream_t s) {
    int blocks = (int)std::min<int64_t>((d + 255) / 256, 2048);
    scale_kernel<<<blocks < 1 ? 1 : blocks, 256, 0, s>>>(w, d, scale);
}

// ------------------------------------------------------------ strict eval --
// Pass 1: one lane per row, dot in stored order; train rows store their hinge
// loss, test rows store 1.0 for a misclassification (OptUtils.scala:57-61,95-98).
__global__ __launch_bounds__(256) void eval_rows_strict(EvalArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) {
        const int64_t b = a.row_ptr[i], e = a.row_ptr[i + 1];
        double s = 0.0;
        for (int64_t q = b; q < e; ++q) s += a.val[q] * a.w[a.col[q]];
        a.row_scratch[i] = jmax(1 - a.y[i] * (s), 0.0);
    } else if (i < a.n + a.n_test) {
        const int64_t r = i - a.n;
        const int64_t b = a.t_row_ptr[r], e = a.t_row_ptr[r + 1];
        double s = 0.0;
        for (int64_t q = b; q < e; ++q) s += a.t_val[q] * a.w[a.t_col[q]];
        a.row_scratch[i] = ((s) * (a.t_y[r]) > 0) ? 0.0 : 1.0;
    }
}

// Pass 2: per-partition reduceLeft of the hinge losses and DenseVector.sum of
// alpha (thread k), merged in partition order; ||w||^2 summed in index order.
__global__ __launch_bounds__(1024) void eval_fold_strict(EvalArgs a) {
    double* part = a.partials;  // [K][2]
    for (int k = threadIdx.x; k < a.K; k += blockDim.x) {
        const int64_t r0 = a.part_ptr[k], r1 = a.part_ptr[k + 1];
        double h = 0.0, al = 0.0;
        for (int64_t r = r0; r < r1; ++r) {
            h = (r == r0) ? a.row_scratch[r] : h + a.row_scratch[r];
            al += a.alpha[r];
        }
        part[2 * k] = h;
        part[2 * k + 1] = al;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double h = 0.0, al = 0.0;
        bool have = false;
        for (int32_t q = 0; q < a.K; ++q) {
            al = (q == 0) ? part[2 * q + 1] : al + part[2 * q + 1];
            if (a.part_ptr[q + 1] > a.part_ptr[q]) {
                h = have ? h + part[2 * q] : part[2 * q];
                have = true;
            }
        }
        double w2 = 0.0;
        for (int64_t j = 0; j < a.d; ++j) {  // index order of the original features
            const double wj = a.w[a.perm ? a.perm[j] : j];
            w2 += wj * wj;
        }
        double err = 0.0;
        for (int64_t r = 0; r < a.n_test; ++r) err += a.row_scratch[a.n + r];
        a.out[0] = h;
        a.out[1] = al;
        a.out[2] = w2;
        a.out[3] = err;
    }
}

void launch_eval_strict(const EvalArgs& a, hipStream_t s) {
    const int64_t rows = a.n + a.n_test;
    const int blocks = (int)((rows + 255) / 256);
    if (blocks > 0) eval_rows_strict<<<blocks, 256, 0, s>>>(a);
    eval_fold_strict<<<1, 1024, 0, s>>>(a);
}

// -------------------------------------------------------------- SGD (C5) --
// SGD.partitionUpdate (SGD.scala:87-139), one workgroup per partition.
// mb-SGD: w is the driver's (already shrunk) w, read-only; deltaW accumulates
// x*y over violators.  local-SGD: the task's copy w_loc is shrunk by
// (1 - step*lambda) every step (O(d), as the reference does) and moved by
// x*y*step; the returned deltaW is w_loc - wInit.
template <bool LOCAL>
__global__ __launch_bounds__(256) void sgd_kernel(SolverArgs a, double lambda, double t0) {
    __shared__ double red[4];
    __shared__ double sh_eval;
    const int k = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t p0 = a.part_ptr[k];
    const int64_t d = a.d;
    double* dwk = a.dw + (size_t)k * d;
    double* wl = LOCAL ? a.wloc + (size_t)k * d : const_cast<double*>(a.w);
    if (LOCAL) {
        for (int64_t j = tid; j < d; j += 256) wl[j] = a.w[j];
        __syncthreads();
    }
    for (int32_t i = 1; i <= a.H; ++i) {
        const double step = 1.0 / (lambda * (t0 + (double)i));         // SGD.scala:106
        const int32_t idx = a.samples[(size_t)k * a.H + (i - 1)];
        const int64_t gr = p0 + idx;
        const int64_t b = a.row_ptr[gr], e = a.row_ptr[gr + 1];
        const double yv = a.y[gr];
        if (wv == 0) {
            // x.dot(w) in stored order (strict: lane 0 sequential)
            double s = 0.0;
            if (lane == 0)
                for (int64_t q = b; q < e; ++q) s += a.val[q] * wl[a.col[q]];
            if (lane == 0) sh_eval = 1.0 - (yv * (s));                    // SGD.scala:115
        }
        __syncthreads();
        const double ev = sh_eval;
        if (LOCAL) {
            const double scale = 1.0 - (step * lambda);                  // SGD.scala:119-120
            for (int64_t j = tid; j < d; j += 256) wl[j] = wl[j] * scale;
            __syncthreads();
        }
        if (ev > 0) {                                                    // SGD.scala:124-130
            if (tid == 0) {
                for (int64_t q = b; q < e; ++q) {
                    const double u = a.val[q] * yv;
                    if (!LOCAL) dwk[a.col[q]] = dwk[a.col[q]] + u;
                    if (LOCAL) wl[a.col[q]] = wl[a.col[q]] + (u * step);
                }
            }
        }
        __syncthreads();
    }
    if (LOCAL)
        for (int64_t j = tid; j < d; j += 256) dwk[j] = wl[j] - a.w[j];  // deltaW = w - wInit (SGD.scala:133)
    (void)red;
}

void launch_sgd(bool local, const SolverArgs& a, double lambda, double t0, int grid, hipStream_t s) {
    if (local)
        sgd_kernel<true><<<grid, 256, 0, s>>>(a, lambda, t0);
    else
        sgd_kernel<false><<<grid, 256, 0, s>>>(a, lambda, t0);
}

}  // namespace cocoa
