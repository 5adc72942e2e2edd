// Fast translation unit (-ffp-contract=fast): wave-tree dot products and
// fused multiply-adds.  Results agree with the strict path within the 1e-9
// relative tolerance of BASELINE.json's north_star.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"
#include "plan_impl.h"
#include "solver_dense.h"
#include "solver_gram.h"
#include "solver_impl.h"
#include "wave.h"

namespace cocoa {

void launch_solver_fast(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                        hipStream_t s) {
    launch_solver_impl<false>(mode, vec_lds, alpha_lds, a, grid, lds, s);
}

void launch_plan_fast(const PlanArgs& a, hipStream_t s) { launch_plan_impl<false>(a, s); }

// ------------------------------------------------- Gram-window solver --
size_t gram_solver_lds(int64_t d, int32_t* hot, bool mirror) {
    constexpr size_t kLds = 160 * 1024;
    const size_t st = mirror ? sizeof(GramSolverLdsT<kGramRuns / 2>) : sizeof(GramSolverLdsT<kGramClasses>);
    const size_t base = (st + 15) & ~(size_t)15;
    // the most frequent columns (device order) of deltaW in the remaining LDS
    const int64_t h = std::max<int64_t>(0, std::min<int64_t>(d, (int64_t)((kLds - base) / sizeof(double)) & ~(int64_t)63));
    if (hot) *hot = (int32_t)h;
    return base + sizeof(double) * (size_t)h;
}

// Gram rows of a round.  a.chunks > 0: gram_seq_kernel (K * chunks workgroups,
// each a run of one partition's batches), then gram_list_kernel over the
// windows its pool could not hold (usually none: the blocks read a zero count
// and exit).  a.chunks == 0: gram_kernel, one workgroup per window.
void launch_gram(const GramArgs& a, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)gram_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sizeof(GramLds));
        (void)hipFuncSetAttribute((const void*)gram_list_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sizeof(GramLds));
        (void)hipFuncSetAttribute((const void*)gram_seq_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sizeof(GramSeqLds));
        attr = true;
    }
    const int64_t grid = (int64_t)a.K * a.nbatch;
    if (grid <= 0) return;
    if (a.chunks > 0) {
        (void)hipMemsetAsync(a.fb_n, 0, sizeof(int32_t), s);
        gram_seq_kernel<<<(unsigned)((int64_t)a.K * a.chunks), kGsThreads, sizeof(GramSeqLds), s>>>(a);
        gram_list_kernel<<<(unsigned)std::min<int64_t>(grid, 256), kGramThreads, sizeof(GramLds), s>>>(a);
    } else {
        gram_kernel<<<(unsigned)grid, kGramThreads, sizeof(GramLds), s>>>(a);
    }
}
size_t gram_seq_lds() { return sizeof(GramSeqLds); }

// x.w of the round's sampled rows beside the Gram solver, so that no evaluation
// pass has to form them in line before the round (plan_impl.h forms the same
// sums, 16 lanes per step, when it runs in line).  Block (b, k) of the
// batch-major grid takes batch b of partition k, one step per 16 lanes; the
// early batches of every partition land first, on the XCD of the partition's
// solver workgroup (both grids deal k round robin).  Publication
// (MI355X_MICROARCH.md, inter-workgroup visibility, the write-through form):
// sc1 (agent-scope relaxed) stores, every wave's vmcnt(0), a barrier, then one
// lane's sc1 flag store; the loader polls the flags, takes one agent acquire per
// 16 batches (these blocks run several per CU, outside the guide's one-per-CU
// sc1-load row) and loads the values with sc1 loads (solver_gram.h).  Every
// value is stored sc1 and drained before its flag, so the flag store needs no
// release fence either (the guide's sc1 producer form).  An L2 write-back per block
// (buffer_wbl2) also flushed the solver's freshly dirtied deltaW lines and took
// the producer to 2.0-2.4 ms and the solver beside it to 4.7 ms (r04m).
__global__ __launch_bounds__(256) void xw_produce_kernel(XwArgs a) {
    const int k = (int)(blockIdx.x % (unsigned)a.K), b = (int)(blockIdx.x / (unsigned)a.K);
    const int tid = threadIdx.x, sub = tid & 15;
    const int32_t j = b * kGB + (tid >> 4);
    if (j < a.H) {  // whole 16-lane rows: the row sum's DPP stays inside active rows
        const int64_t r = a.part_ptr[k] + a.samples[(size_t)k * a.H + j];
        const int64_t q0 = a.row_ptr[r], q1 = a.row_ptr[r + 1];
        double acc = 0.0;
        for (int64_t q = q0 + sub; q < q1; q += 16) acc += a.val[q] * a.w[a.col[q]];
        const double xw = row16_sum(acc);
        if (sub == 0) __hip_atomic_store(a.xw + (size_t)k * a.stride + j, xw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    vm_drain();
    __syncthreads();
    if (tid == 0)
        __hip_atomic_store(a.flag + (size_t)k * a.nbatch + b, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int gram_window_batches() { return kGNB; }
bool gram_seq_supported() { return kGsWindowOK; }

void launch_xw_produce(const XwArgs& a, hipStream_t s) {
    // 4 KB of (unused) LDS: a block then never fits beside a Gram-solver
    // workgroup (~159 KB), whose issue-bound memory waves it would slow
    const int64_t grid = (int64_t)a.K * a.nbatch;
    if (grid > 0) xw_produce_kernel<<<(unsigned)grid, 256, 4096, s>>>(a);
}

template <int MODE, bool HOTLDS, bool PROJ, int XWM>
static void launch_sg4(const GramSolverArgs& a, int grid, size_t lds, hipStream_t s) {
    // the mirrored form (two workgroups per partition): hot columns in LDS; the
    // caller sets a.mirror only then
    constexpr bool MIR_OK = HOTLDS;
    if (MIR_OK && a.mirror) {
        (void)hipFuncSetAttribute((const void*)solver_gram_kernel<MODE, HOTLDS, PROJ, XWM, MIR_OK>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        solver_gram_kernel<MODE, HOTLDS, PROJ, XWM, MIR_OK>
            <<<2 * grid, GCfg<kGramRuns / 2>::kThreads + 64, lds, s>>>(a);
        return;
    }
    (void)hipFuncSetAttribute((const void*)solver_gram_kernel<MODE, HOTLDS, PROJ, XWM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    solver_gram_kernel<MODE, HOTLDS, PROJ, XWM><<<grid, GCfg<kGramClasses>::kThreads, lds, s>>>(a);
}
// the loader's x.w: xw_produce_kernel's flags or the plan's (MbCD has no Gram
// rows, hence no side stream and no producer: always the plan's).  Measured and
// not kept (r04s): the loader gathering x.w from the evaluation's per-row cache
// itself, the sample loaded a batch ahead: solver 2.56 -> 2.90 ms (16 scattered
// lines per batch on the loader instead of one).
template <int MODE, bool HOTLDS, bool PROJ>
static void launch_sg3(const GramSolverArgs& a, int grid, size_t lds, hipStream_t s) {
    if (MODE != MODE_MBCD && a.xw_flag)
        launch_sg4<MODE, HOTLDS, PROJ, MODE != MODE_MBCD ? kXwProducer : kXwPlan>(a, grid, lds, s);
    else
        launch_sg4<MODE, HOTLDS, PROJ, kXwPlan>(a, grid, lds, s);
}

// plan_xw[g] = row_xw[part_ptr[k] + samples[g]]: the step plan's x.w from the
// evaluation's per-row cache, when the rest of the plan was formed beside the
// previous round
__global__ __launch_bounds__(256) void xw_gather_kernel(const int64_t* part_ptr, const int32_t* samples, int32_t H,
                                                        int64_t steps, const double* row_xw, double* xw) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= steps) return;
    const int64_t r = part_ptr[g / H] + samples[g];
    __builtin_nontemporal_store(row_xw[r], xw + g);
}

void launch_xw_gather(const int64_t* part_ptr, const int32_t* samples, int32_t H, int64_t steps,
                      const double* row_xw, double* xw, hipStream_t s) {
    if (steps > 0 && H > 0)
        xw_gather_kernel<<<(unsigned)((steps + 255) / 256), 256, 0, s>>>(part_ptr, samples, H, steps, row_xw, xw);
}
template <int MODE, bool HOTLDS>
static void launch_sg(const GramSolverArgs& a, int grid, size_t lds, hipStream_t s) {
    if (a.proj) launch_sg3<MODE, HOTLDS, true>(a, grid, lds, s);
    else launch_sg3<MODE, HOTLDS, false>(a, grid, lds, s);
}

// The most frequent deltaW columns (device order) in LDS (HOTLDS) or every
// column in the L2-resident slice.  Round 2 measured the LDS path 9% slower
// with one memory wave (a select and an LDS read per gathered entry on an
// issue-bound wave); with two memory waves and the scatter reads ahead of the
// drain (round 3) the hot columns' atomics and gathers leaving the TA pay:
// 1,088 columns (64% of C2's entries, the LDS the rings leave) took the solver
// 2.90 -> 2.74 ms (r03 A/B).
static bool gram_hot_lds() {
#ifdef COCOA_DIAG
    if (const char* e = getenv("COCOA_GRAM_HOTLDS")) return atoi(e) != 0;  // diagnostic A/B only
#endif
    return true;
}

void launch_solver_gram(int mode, const GramSolverArgs& a, int grid, hipStream_t s) {
    GramSolverArgs g = a;
    size_t lds = gram_solver_lds(a.d, &g.hot, a.mirror != 0);
#ifdef COCOA_DIAG
    // diagnostic builds only (make diag): timing experiments, results invalid with DIAG
    if (const char* e = getenv("COCOA_GRAM_HOT")) {  // cap the LDS-resident columns
        const int32_t h = std::min<int32_t>(g.hot, (int32_t)atoi(e) & ~63);
        lds -= sizeof(double) * (size_t)(g.hot - h);
        g.hot = h;
    }
    if (const char* e = getenv("COCOA_GRAM_DIAG")) g.diag = atoi(e);
#endif
    g.hot_split = 0;
    if (!gram_hot_lds() || g.hot == 0) {
        g.mirror = 0;  // (the mirrored form keeps the hot columns in LDS)
        lds = (sizeof(GramSolverLdsT<kGramClasses>) + 15) & ~(size_t)15;
        g.hot = 0;
        if (mode == MODE_PLUS) launch_sg<MODE_PLUS, false>(g, grid, lds, s);
        else if (mode == MODE_COCOA) launch_sg<MODE_COCOA, false>(g, grid, lds, s);
        else if (mode == MODE_LSGD) launch_sg3<MODE_LSGD, false, false>(g, grid, lds, s);
        else launch_sg<MODE_MBCD, false>(g, grid, lds, s);
        return;
    }
    if (mode == MODE_PLUS) launch_sg<MODE_PLUS, true>(g, grid, lds, s);
    else if (mode == MODE_COCOA) launch_sg<MODE_COCOA, true>(g, grid, lds, s);
    else if (mode == MODE_LSGD) launch_sg3<MODE_LSGD, true, false>(g, grid, lds, s);
    else launch_sg<MODE_MBCD, true>(g, grid, lds, s);
}

// ----------------------------------------------------------- fused eval --
// One pass over train + test CSR (OptUtils.scala:57-98) as a CSR stream.
// Each block takes a tile of whole rows holding <= TILE entries and reads it
// from the 4-entry-aligned base e0 & ~3, so each thread moves 4 consecutive
// entries per unit with one 16-B col load and two 16-B val loads
// (nontemporal: the stream must not evict the solver's deltaW slices from
// L2).  It gathers w (L1/L2-resident, frequency-ordered), parks the products
// in LDS, then 16-lane groups (one DPP row each) sum the rows; row offsets
// inside a tile are 16-bit.  A row longer than a tile is summed by the whole
// block.  The same launch sums alpha and ||w||^2 and stores every train row's
// x.w (the next round's step plan reuses it).  Block partials -> fixed-order
// final reduction (deterministic run to run).  The CSR entry arrays carry 64
// zero bytes of tail padding so the last unit stays in bounds.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int BLOCK>
__device__ __forceinline__ double block_sum_n(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < BLOCK / 64; ++i) s += red[i];
    return s;
}

typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

// 4 column indices at entry offset k: int32 (16 B) or, when d <= 65,536, the
// uint16 copy (8 B: the stream drops from 12 to 10 B per entry)
template <bool C16>
__device__ __forceinline__ i32x4 load_cols(const int32_t* c32, const uint16_t* c16, int64_t k) {
    if (C16) {
        const u16x4 v = __builtin_nontemporal_load((const u16x4*)(c16 + k));
        return i32x4{(int32_t)v.x, (int32_t)v.y, (int32_t)v.z, (int32_t)v.w};
    }
    return __builtin_nontemporal_load((const i32x4*)(c32 + k));
}

// w gather of the fast eval: columns below HOT (device order: the most
// frequent) from the block's LDS copy, the rest from global memory.  The two
// are exclusive per lane (a branch, not a select), so the global gather
// instruction only carries the cold lanes: the texture addresser processes a
// gather lane by lane, and it -- not HBM -- bounds the pass (C2 PMC: TA busy
// 80% of the kernel with every gather global).
// (address-space-qualified accesses: with plain pointers the compiler merges
// the two branches into one FLAT load on a selected pointer)
typedef __attribute__((address_space(1))) const double gdouble;
typedef __attribute__((address_space(3))) const double ldouble;
template <int HOT>
__device__ __forceinline__ double w_at(const double* w, const double* whot, int32_t c) {
    double x;
    if (HOT > 0 && c < HOT)
        x = ((ldouble*)whot)[c];
    else
        x = ((gdouble*)w)[c];
    return x;
}

// The block partials' sum in a fixed order (threads [0, 256) of the calling
// block; every thread of the block calls it): out[0..3], and out_host (system
// scope) when set.  sc1: the partials were handed over write-through.
__device__ __forceinline__ void eval_reduce(const double* partials, int blocks, double* out, double* out_host,
                                            double (*red)[4], bool sc1) {
    const int tid = threadIdx.x;
    double v[4] = {0, 0, 0, 0};
    if (tid < 256)
        for (int b = tid; b < blocks; b += 256)
            for (int i = 0; i < 4; ++i) {
                double* q = const_cast<double*>(partials) + (size_t)b * 4 + i;
                v[i] += sc1 ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
            }
    for (int i = 0; i < 4; ++i) {
        const double s = wave_sum(v[i]);
        if ((tid & 63) == 0 && tid < 256) red[i][tid >> 6] = s;
    }
    __syncthreads();
    if (tid < 4) {
        const double r = ((red[tid][0] + red[tid][1]) + red[tid][2]) + red[tid][3];
        out[tid] = r;
        if (out_host) __hip_atomic_store(out_host + tid, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// BASE: the train rows' dot starts from row_base[r] (the hot pass below: the
// pass then streams the cold part of a hot / cold split, cocoa_ctx::split_ready)
template <int TILE, int BLOCK, bool C16, int DIAGW = 0, int HOT = 0, bool BASE = false>
__global__ __launch_bounds__(BLOCK) void eval_stream_kernel(EvalArgs a) {
    constexpr int UNITS = TILE / (4 * BLOCK);  // 4-entry units per thread (base alignment adds one)
    __shared__ double prod[TILE + 4];
    __shared__ uint16_t roff[TILE + 2];
    __shared__ double red[BLOCK / 64];
    __shared__ double whot[HOT > 0 ? HOT : 1];
    // the tile's labels (and hot-pass dots) loaded with its row offsets, up front:
    // read per row after its LDS sum, each was a dependent global round trip per
    // row a 16-lane group takes (C2's cold pass: ~8 rows per group and tile)
    __shared__ double yl[kEvalRows];
    __shared__ double bl[BASE ? kEvalRows : 1];
    const int tid = threadIdx.x;
    if (HOT > 0) {
        const int32_t h = (int32_t)min<int64_t>(HOT, a.d);
        for (int32_t j = tid; j < h; j += BLOCK) whot[j] = a.w[j];
        __syncthreads();
    }
    const int sub = tid & 15, grp = tid >> 4;
    double hinge = 0.0, err = 0.0;
    const int64_t ntiles = a.n_tiles + a.n_t_tiles;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const bool test = t >= a.n_tiles;
        const int64_t tt = test ? t - a.n_tiles : t;
        const int64_t* tl = test ? a.t_tiles : a.tiles;
        const int64_t* te = tl + (test ? a.n_t_tiles : a.n_tiles) + 1;
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const int32_t* cl = test ? a.t_col : a.col;
        const uint16_t* cl16 = test ? a.t_col16 : a.col16;
        const double* vl = test ? a.t_val : a.val;
        const double* yy = test ? a.t_y : a.y;
        const int64_t r0 = tl[tt], r1 = tl[tt + 1];
        const int64_t e0 = te[tt], e1 = te[tt + 1];
        const int64_t T = e1 - e0;
        // the row's hot-pass dot: train rows at row_base[r], split test rows at [n + r]
        const bool has_base = BASE && (!test || a.n_th_tiles > 0);
        const double* rb = test ? a.row_base + a.n : a.row_base;
        if (T > TILE) {
            double acc = 0.0;
            for (int64_t q = e0 + tid; q < e1; q += BLOCK) acc += vl[q] * a.w[cl[q]];
            const double dot = block_sum_n<BLOCK>(acc, red) + (has_base ? rb[r0] : 0.0);
            if (tid == 0) {
                if (!test) {
                    hinge += jmax(1 - yy[r0] * dot, 0.0);
                    if (a.row_xw) a.row_xw[r0] = dot;
                } else {
                    err += (dot * yy[r0] > 0) ? 0.0 : 1.0;
                }
            }
            continue;
        }
        const int nr = (int)(r1 - r0);
        for (int i = tid; i <= nr; i += BLOCK) {
            roff[i] = (uint16_t)(rp[r0 + i] - e0);
            if (i < nr) {
                yl[i] = yy[r0 + i];
                if (has_base) bl[i] = rb[r0 + i];
            }
        }
        const int64_t base = e0 & ~(int64_t)3;
        const int sh = (int)(e0 - base);  // prod[k] holds entry base + k; rows index from sh
        const int64_t span = e1 - base;
        i32x4 c[UNITS + 1];
        f64x2 v0[UNITS + 1], v1[UNITS + 1];
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            c[u] = i32x4{0, 0, 0, 0};
            v0[u] = f64x2{0.0, 0.0};
            v1[u] = v0[u];
            if (k < span) {
                c[u] = load_cols<C16>(cl, cl16, base + k);
                if (DIAGW == 1) c[u] &= 4095;  // timing diagnostic only: every gather in a 32 KB window
                if (DIAGW == 2) c[u] &= 0;     // timing diagnostic only: one address
                v0[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k));
                v1[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k + 2));
            }
        }
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            if (k < span) {
                // entries past e1 inside the last unit are never summed (roff bounds rows)
                *(f64x2*)(prod + k) = f64x2{v0[u].x * w_at<HOT>(a.w, whot, c[u].x), v0[u].y * w_at<HOT>(a.w, whot, c[u].y)};
                *(f64x2*)(prod + k + 2) = f64x2{v1[u].x * w_at<HOT>(a.w, whot, c[u].z), v1[u].y * w_at<HOT>(a.w, whot, c[u].w)};
            }
        }
        __syncthreads();
        for (int r = grp; r < nr; r += BLOCK / 16) {
            const int b = roff[r] + sh, e = roff[r + 1] + sh;
            double acc = 0.0;
            for (int q = b + sub; q < e; q += 16) acc += prod[q];
            double dot = row16_sum(acc);
            if (sub == 0) {
                if (has_base) dot += bl[r];
                if (!test) {
                    hinge += jmax(1 - yl[r] * dot, 0.0);
                    if (a.row_xw) a.row_xw[r0 + r] = dot;
                } else {
                    err += (dot * yl[r] > 0) ? 0.0 : 1.0;
                }
            }
        }
        __syncthreads();
    }
    const int64_t gt = (int64_t)blockIdx.x * BLOCK + tid;
    const int64_t gs = (int64_t)gridDim.x * BLOCK;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    const double s0 = block_sum_n<BLOCK>(hinge, red);
    const double s1 = block_sum_n<BLOCK>(al, red);
    const double s2 = block_sum_n<BLOCK>(w2, red);
    const double s3 = block_sum_n<BLOCK>(err, red);
    double* p = a.partials + (size_t)blockIdx.x * 4;
    if (!a.counter) {
        if (tid == 0) {
            p[0] = s0;
            p[1] = s1;
            p[2] = s2;
            p[3] = s3;
        }
        return;
    }
    // the last block to finish sums the partials (MI355X_MICROARCH.md's
    // write-through hand-off: sc1 partials, the storing lane's vmcnt(0), one
    // agent-scope add per block, sc1 loads by the block whose add came last)
    __shared__ int last;
    if (tid == 0) {
        __hip_atomic_store(p + 0, s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 1, s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 2, s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 3, s3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vm_drain();
        last = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __shared__ double red4[4][4];
    eval_reduce(a.partials, (int)gridDim.x, a.out, a.out_host, red4, true);
    if (tid == 0) __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    if (tid == 4 && a.status_host)
        __hip_atomic_store(a.status_host, a.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifdef COCOA_DIAG
// Row-parallel variant: one 16-lane group per row, straight from global memory
// (no LDS staging, no barriers), U loads per lane in flight per row chunk,
// rows walked grid-stride so every wave always has rows of its own in flight.
// Every load stays in bounds (a lane past the row reloads the row's last
// entry and drops it), so the compiler issues a chunk's loads back to back.
template <int U, bool C16>
__global__ __launch_bounds__(256) void eval_rows_kernel(EvalArgs a) {
    constexpr int G = 16;
    __shared__ double red[4];
    const int tid = threadIdx.x, lane = tid & 63, sub = lane & (G - 1);
    const int64_t rows = a.n + a.n_test;
    const int64_t ng = (int64_t)gridDim.x * (256 / G);
    double hinge = 0.0, err = 0.0;
    for (int64_t r = ((int64_t)blockIdx.x * 256 + tid) / G; r < rows; r += ng) {
        const bool test = r >= a.n;
        const int64_t rr = test ? r - a.n : r;
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const int32_t* cl = test ? a.t_col : a.col;
        const uint16_t* cl16 = test ? a.t_col16 : a.col16;
        const double* vl = test ? a.t_val : a.val;
        const int64_t b = rp[rr], e = rp[rr + 1];
        double acc = 0.0;
        for (int64_t q0 = b; q0 < e; q0 += G * U) {
            int32_t c[U];
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t q = min(q0 + u * G + sub, e - 1);
                c[u] = C16 ? (int32_t)__builtin_nontemporal_load(cl16 + q) : __builtin_nontemporal_load(cl + q);
                v[u] = __builtin_nontemporal_load(vl + q);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double x = a.w[c[u]];
                acc = fma(q0 + u * G + sub < e ? v[u] : 0.0, x, acc);
            }
        }
        const double dot = row16_sum(acc);
        if (sub == 0) {
            if (!test) {
                hinge += jmax(1 - a.y[rr] * dot, 0.0);          // OptUtils.scala:57-61
                if (a.row_xw) a.row_xw[rr] = dot;
            } else {
                err += (dot * a.t_y[rr] > 0) ? 0.0 : 1.0;        // OptUtils.scala:95-98
            }
        }
    }
    const int64_t gt = (int64_t)blockIdx.x * 256 + tid, gs = (int64_t)gridDim.x * 256;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    const double s0 = block_sum_n<256>(hinge, red);
    const double s1 = block_sum_n<256>(al, red);
    const double s2 = block_sum_n<256>(w2, red);
    const double s3 = block_sum_n<256>(err, red);
    if (tid == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
        p[3] = s3;
    }
}

#endif

__global__ __launch_bounds__(256) void eval_final_kernel(const double* partials, int blocks, double* out) {
    __shared__ double red[4][4];
    eval_reduce(partials, blocks, out, nullptr, red, false);
}

// 4,096-entry tiles, 512 threads, 3 blocks per CU (41 KB of LDS per block).
// Measured on C2 (r01): 0.211-0.227 ms, 38-40% of HBM peak.
int eval_fast_blocks(int64_t n_tiles, int64_t n_t_tiles) {
    int64_t b = n_tiles + n_t_tiles;
    if (b > 256 * 3) b = 256 * 3;
    return (int)(b < 1 ? 1 : b);
}

#ifdef COCOA_DIAG
// diagnostic builds only (make diag): A/B variants of the pass (DESIGN.md
// section 3.3 lists what each measured; results of 3 and 4 are invalid)
static int eval_variant() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("COCOA_EVAL_VARIANT");
        v = e ? atoi(e) : 0;
    }
    return v;
}
int eval_tile_entries(int64_t d) {
    if (const char* e = getenv("COCOA_EVAL_TILE")) return atoi(e) == 2048 ? 2048 : kEvalTile;
    if (eval_variant() >= 6 && eval_variant() <= 9) return 2048;
    return d > kEvalWideD ? 2048 : kEvalTile;
}

static bool launch_eval_diag(const EvalArgs& a, bool c16, hipStream_t s) {
    const int v = eval_variant();
    if (v == 8 || v == 9) {  // 2,048-entry tiles, more blocks per CU
        const int64_t nt = a.n_tiles + a.n_t_tiles;
        if (v == 8) {  // 512 threads, 4 blocks per CU
            const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(nt, 1024));
            if (c16) eval_stream_kernel<2048, 512, true><<<nb, 512, 0, s>>>(a);
            else eval_stream_kernel<2048, 512, false><<<nb, 512, 0, s>>>(a);
            eval_final_kernel<<<1, 256, 0, s>>>(a.partials, nb, a.out);
        } else {  // 256 threads, 8 blocks per CU
            const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(nt, 2048));
            if (c16) eval_stream_kernel<2048, 256, true><<<nb, 256, 0, s>>>(a);
            else eval_stream_kernel<2048, 256, false><<<nb, 256, 0, s>>>(a);
            eval_final_kernel<<<1, 256, 0, s>>>(a.partials, nb, a.out);
        }
        return true;
    }
    // hot w columns in LDS, and the timing diagnostics, for either column width
#define COCOA_EVAL_C16(...)                          \
    do {                                             \
        if (c16) {                                   \
            constexpr bool C = true;                 \
            __VA_ARGS__;                             \
        } else {                                     \
            constexpr bool C = false;                \
            __VA_ARGS__;                             \
        }                                            \
    } while (0)
    if (v >= 5) {
        const int nb = eval_fast_blocks(a.n_tiles, a.n_t_tiles);
        if (v == 5) {  // 4,096-entry tiles, 32 KB of w: 2 blocks per CU
            const int n2 = (int)std::min<int64_t>(a.n_tiles + a.n_t_tiles, 512);
            COCOA_EVAL_C16((eval_stream_kernel<kEvalTile, 512, C, 0, 4096><<<n2, 512, 0, s>>>(a)));
            eval_final_kernel<<<1, 256, 0, s>>>(a.partials, n2, a.out);
        } else if (v == 6) {  // 2,048-entry tiles, 32 KB of w: 3 blocks per CU
            COCOA_EVAL_C16((eval_stream_kernel<2048, 512, C, 0, 4096><<<nb, 512, 0, s>>>(a)));
            eval_final_kernel<<<1, 256, 0, s>>>(a.partials, nb, a.out);
        } else {  // 2,048-entry tiles, 64 KB of w (8,192 columns): 2 blocks per CU
            const int n2 = (int)std::min<int64_t>(a.n_tiles + a.n_t_tiles, 512);
            COCOA_EVAL_C16((eval_stream_kernel<2048, 512, C, 0, 8192><<<n2, 512, 0, s>>>(a)));
            eval_final_kernel<<<1, 256, 0, s>>>(a.partials, n2, a.out);
        }
        return true;
    }
    if (v == 3 || v == 4) {  // timing diagnostics (results invalid)
        const int nb = eval_fast_blocks(a.n_tiles, a.n_t_tiles);
        if (v == 3) COCOA_EVAL_C16((eval_stream_kernel<kEvalTile, 512, C, 1><<<nb, 512, 0, s>>>(a)));
        else COCOA_EVAL_C16((eval_stream_kernel<kEvalTile, 512, C, 2><<<nb, 512, 0, s>>>(a)));
        eval_final_kernel<<<1, 256, 0, s>>>(a.partials, nb, a.out);
        return true;
    }
#undef COCOA_EVAL_C16
    if (v == 1 || v == 2) {  // one 16-lane group per row, 8 / 4 loads per lane in flight
        const int nb = 2048;
        if (v == 1) {
            if (c16) eval_rows_kernel<8, true><<<nb, 256, 0, s>>>(a);
            else eval_rows_kernel<8, false><<<nb, 256, 0, s>>>(a);
        } else {
            if (c16) eval_rows_kernel<4, true><<<nb, 256, 0, s>>>(a);
            else eval_rows_kernel<4, false><<<nb, 256, 0, s>>>(a);
        }
        eval_final_kernel<<<1, 256, 0, s>>>(a.partials, nb, a.out);
        return true;
    }
    return false;
}
#else
int eval_tile_entries(int64_t d) { return d > kEvalWideD ? 2048 : kEvalTile; }
#endif

// Hot pass of the split evaluation (cocoa_ctx::split_ready): the train rows'
// entries in device columns < HOT -- the most frequent: C2 78%, C4 72% of the
// entries at 4,096 -- as their own CSR with 16-bit columns, w's first HOT
// columns in LDS, so the pass issues no global gather at all (the texture
// addresser's per-instruction cost bounds the one-pass kernel, DESIGN.md section
// 3.3); each row's partial dot goes to row_base.  The cold pass
// (eval_stream_kernel<..., BASE>) then streams the remaining entries with global
// gathers, adds row_base and does the hinge / error / alpha / ||w|| sums.  Tiles
// and loads as in eval_stream_kernel.
// WARM: the warm pass over the third CSR (EvalArgs::m_*): w gathered from global
// memory at kEvalHot + the 16-bit offset (a 0.5 MB slice, L2-resident), each
// row's dot added to the hot pass's row_base (staged per tile, like the labels
// of eval_stream_kernel)
template <int TILE, int BLOCK, int HOT, bool WARM = false>
__global__ __launch_bounds__(BLOCK) void eval_hot_kernel(EvalArgs a) {
    constexpr int UNITS = TILE / (4 * BLOCK);
    __shared__ double prod[TILE + 4];
    __shared__ uint16_t roff[TILE + 2];
    __shared__ double red[BLOCK / 64];
    __shared__ double whot[WARM ? 1 : HOT];
    __shared__ double bl[WARM ? kEvalRows : 1];
    const int tid = threadIdx.x;
    if (!WARM) {
        const int32_t h = (int32_t)min<int64_t>(HOT, a.d);
        for (int32_t j = tid; j < HOT; j += BLOCK) whot[j] = j < h ? a.w[j] : 0.0;
        __syncthreads();
    }
    const gdouble* wm = (const gdouble*)(a.w + kEvalHot);
    auto w_of = [&](int32_t c) -> double { return WARM ? wm[c] : whot[c]; };
    const int sub = tid & 15, grp = tid >> 4;
    const int64_t nt = WARM ? a.n_m_tiles : a.n_h_tiles;
    // (the hot pass also takes the split test rows' tiles, after the train ones)
    const int64_t ntt = WARM ? 0 : a.n_th_tiles;
    for (int64_t t = blockIdx.x; t < nt + ntt; t += gridDim.x) {
        const bool test = t >= nt;
        const int64_t tt = test ? t - nt : t;
        const int64_t* tl = test ? a.th_tiles : WARM ? a.m_tiles : a.h_tiles;
        const int64_t* te = tl + (test ? ntt : nt) + 1;
        const int64_t* rp = test ? a.th_row_ptr : WARM ? a.m_row_ptr : a.h_row_ptr;
        const uint16_t* cl = test ? a.th_col16 : WARM ? a.m_col16 : a.h_col16;
        const double* vl = test ? a.th_val : WARM ? a.m_val : a.h_val;
        double* rb = test ? a.row_base + a.n : a.row_base;
        const int64_t r0 = tl[tt], r1 = tl[tt + 1];
        const int64_t e0 = te[tt], e1 = te[tt + 1];
        const int64_t T = e1 - e0;
        if (T > TILE) {
            double acc = 0.0;
            for (int64_t q = e0 + tid; q < e1; q += BLOCK) acc += vl[q] * w_of(cl[q]);
            const double dot = block_sum_n<BLOCK>(acc, red);
            if (tid == 0) rb[r0] = WARM ? rb[r0] + dot : dot;
            continue;
        }
        const int nr = (int)(r1 - r0);
        for (int i = tid; i <= nr; i += BLOCK) {
            roff[i] = (uint16_t)(rp[r0 + i] - e0);
            if (WARM && i < nr) bl[i] = rb[r0 + i];
        }
        const int64_t base = e0 & ~(int64_t)3;
        const int sh = (int)(e0 - base);
        const int64_t span = e1 - base;
        i32x4 c[UNITS + 1];
        f64x2 v0[UNITS + 1], v1[UNITS + 1];
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            c[u] = i32x4{0, 0, 0, 0};
            v0[u] = f64x2{0.0, 0.0};
            v1[u] = v0[u];
            if (k < span) {
                c[u] = load_cols<true>(nullptr, cl, base + k);
                v0[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k));
                v1[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k + 2));
            }
        }
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            if (k < span) {
                *(f64x2*)(prod + k) = f64x2{v0[u].x * w_of(c[u].x), v0[u].y * w_of(c[u].y)};
                *(f64x2*)(prod + k + 2) = f64x2{v1[u].x * w_of(c[u].z), v1[u].y * w_of(c[u].w)};
            }
        }
        __syncthreads();
        for (int r = grp; r < nr; r += BLOCK / 16) {
            const int b = roff[r] + sh, e = roff[r + 1] + sh;
            double acc = 0.0;
            for (int q = b + sub; q < e; q += 16) acc += prod[q];
            const double dot = row16_sum(acc);
            if (sub == 0) rb[r0 + r] = WARM ? bl[r] + dot : dot;
        }
        __syncthreads();
    }
}

// tile entries and block threads of the two passes (A/B knobs: make variant DEFS=...)
#ifndef COCOA_HOT_TILE
#define COCOA_HOT_TILE 4096
#endif
#ifndef COCOA_HOT_BLOCK
#define COCOA_HOT_BLOCK 1024  // (C2, one box: 512 threads 0.213 ms for both passes, 1,024 0.205; 2,048-entry tiles 0.216 / 0.233)
#endif
#ifndef COCOA_HOT_WGS
#define COCOA_HOT_WGS 2  // workgroups per CU the hot pass launches
#endif
#ifndef COCOA_COLD_TILE
#define COCOA_COLD_TILE 4096
#endif
#ifndef COCOA_COLD_BLOCK
#define COCOA_COLD_BLOCK 512
#endif
void eval_split_tiles(int* hot_cap, int* cold_cap) {
    *hot_cap = COCOA_HOT_TILE;
    *cold_cap = COCOA_COLD_TILE;
}

// A grid-stride pass with more blocks than fit the device at once runs its
// last ones as a second wave over the same number of tiles each: cap the grid at
// the kernel's resident blocks (its LDS sets how many share a CU).
template <typename F>
static int resident_grid(F kernel, int threads, int want) {
    int per_cu = 0, dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) {
        (void)hipGetLastError();
        return want;
    }
    return std::max(1, std::min(want, per_cu * cus));
}

// the split evaluation: hot pass, then the cold pass over a's (cold) train CSR
// and the test rows (their cold entries when n_th_tiles > 0, else whole)
static bool launch_eval_split(const EvalArgs& a, int blocks, hipStream_t s) {
    const bool c16 = a.col16 && (a.n_test == 0 || a.t_col16);
    const int hb = (int)std::max<int64_t>(1, std::min<int64_t>(a.n_h_tiles + a.n_th_tiles, 256 * COCOA_HOT_WGS));
    eval_hot_kernel<COCOA_HOT_TILE, COCOA_HOT_BLOCK, kEvalHot><<<hb, COCOA_HOT_BLOCK, 0, s>>>(a);
    if (a.n_m_tiles > 0) {
        const int mb = resident_grid(eval_hot_kernel<COCOA_HOT_TILE, COCOA_HOT_BLOCK, kEvalHot, true>, COCOA_HOT_BLOCK,
                                     (int)std::max<int64_t>(1, std::min<int64_t>(a.n_m_tiles, 256 * 8)));
        eval_hot_kernel<COCOA_HOT_TILE, COCOA_HOT_BLOCK, kEvalHot, true><<<mb, COCOA_HOT_BLOCK, 0, s>>>(a);
    }
    if (c16) {
        blocks = resident_grid(eval_stream_kernel<COCOA_COLD_TILE, COCOA_COLD_BLOCK, true, 0, 0, true>, COCOA_COLD_BLOCK,
                               blocks);
        eval_stream_kernel<COCOA_COLD_TILE, COCOA_COLD_BLOCK, true, 0, 0, true><<<blocks, COCOA_COLD_BLOCK, 0, s>>>(a);
    } else {
        blocks = resident_grid(eval_stream_kernel<COCOA_COLD_TILE, COCOA_COLD_BLOCK, false, 0, 0, true>,
                               COCOA_COLD_BLOCK, blocks);
        eval_stream_kernel<COCOA_COLD_TILE, COCOA_COLD_BLOCK, false, 0, 0, true><<<blocks, COCOA_COLD_BLOCK, 0, s>>>(a);
    }
    if (!a.counter) eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
    return a.counter && a.out_host;
}

bool launch_eval_fast(const EvalArgs& a, int blocks, hipStream_t s) {
    if (a.row_base) return launch_eval_split(a, blocks, s);
    const bool c16 = a.col16 && (a.n_test == 0 || a.t_col16);
#ifdef COCOA_DIAG
    EvalArgs u = a;
    u.counter = nullptr;  // the variants end with eval_final_kernel
    if (launch_eval_diag(u, c16, s)) return false;
#endif
    if (c16) {
        blocks = resident_grid(eval_stream_kernel<kEvalTile, 512, true>, 512, blocks);
        eval_stream_kernel<kEvalTile, 512, true><<<blocks, 512, 0, s>>>(a);
    } else if (a.d > kEvalWideD) {
        blocks = resident_grid(eval_stream_kernel<2048, 512, false, 0, 4096>, 512, blocks);
        eval_stream_kernel<2048, 512, false, 0, 4096><<<blocks, 512, 0, s>>>(a);
    } else {
        blocks = resident_grid(eval_stream_kernel<kEvalTile, 512, false>, 512, blocks);
        eval_stream_kernel<kEvalTile, 512, false><<<blocks, 512, 0, s>>>(a);
    }
    if (!a.counter) eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
    return a.counter && a.out_host;
}

// --------------------------------------------- compact fold by blocks --
// Fast-mode fold of compact deltaW slices (C4: 1,024 slices of up to 64,847
// positions, 62 M live entries).  The per-column gather fold
// (fold_compact_kernel) reads slice k at position i_k(j) for column j: for a
// column held by a few hundred partitions the lanes of a wave land in
// different slices, so almost every 8-byte read costs a whole line (1.65 ms
// per C4 round, r03).  Here a work item takes one block of kFoldJ device
// columns over a range of partitions: since every slice lists its columns in
// device order, the block's entries of slice k are the contiguous run
// [fbnd[b][k], fbnd[b+1][k]), read with consecutive lanes and added into an
// LDS accumulator of the block's columns.  The block takes 64 partitions at a
// time: lane l holds run l's bounds, a prefix sum packs the 64 runs, and each
// lane finds the run of its packed position by a 6-step search over the
// lanes, so short runs (the cold blocks: a few entries per slice) cost no
// per-partition loop, and long ones (the hot blocks: thousands per slice) are
// shared by all four waves, four 64-entry pieces per wave in flight.  The block's sums then go to tmp (a plain store when the
// item is the block's only one, else an fp64 atomic add), and fold_finish
// moves tmp into the rank's sum (original order) or into w, re-zeroing tmp.
// Sums are reassociated and atomic: fast mode.
// TAIL: the private columns' tail (FoldTail) after the slices' runs, with the
// same packing: entry (row, c, v) adds v * rowcoef[row] to column c.  (Measured
// on C4, same box: 0.57 ms per fold against 0.21 without the tail; a separate
// pass forming the tail's deltaW first, partition-major so its rowcoef reads
// stay in one partition's rows, took 0.32 ms and the fold 0.25 after it; the
// solver's epilogue forming them, 46 k dependent gathers per workgroup behind
// its chain, +0.9 ms on the solver.)
template <bool TAIL>
__global__ __launch_bounds__(256) void fold_blocks_kernel(const double* dw, const uint16_t* fcol16,
                                                          const uint32_t* fbnd, const int32_t* items, int32_t K,
                                                          int64_t max_u, int64_t d, double* tmp, FoldTail tl) {
    constexpr int kUn = 4;  // 64-entry pieces per wave in flight
    __shared__ double acc[kFoldJ];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int32_t* it = items + 4 * (size_t)blockIdx.x;
    const int32_t b = it[0], k0 = it[1], k1 = it[2], sole = it[3];
    for (int i = tid; i < kFoldJ; i += 256) acc[i] = 0.0;
    __syncthreads();
    // the whole block walks the partitions 64 at a time; the 4 waves share each
    // group's packed entries, kUn pieces of 64 per wave in flight
    for (int part = 0; part < (TAIL ? 2 : 1); ++part) {
        const uint32_t* bnd = part ? tl.tbnd : fbnd;
        for (int32_t kk = k0; kk < k1; kk += 64) {
            const int32_t k = kk + lane;
            const bool ok = k < k1;
            const int32_t lo = ok ? (int32_t)bnd[(size_t)b * K + k] : 0;
            const int32_t n = ok ? (int32_t)bnd[(size_t)(b + 1) * K + k] - lo : 0;
            const int32_t incl = wave_incl_scan(n);
            const int32_t T = __shfl(incl, 63, 64);
            const int32_t excl = incl - n;
            for (int32_t q0 = 64 * kUn * wv; q0 < T; q0 += 64 * kUn * 4) {
                size_t pos[kUn];
                bool val[kUn];
#pragma unroll
                for (int u = 0; u < kUn; ++u) {
                    const int32_t q = q0 + 64 * u + lane;
                    // largest lane j with excl_j <= q (every lane active in the shuffles)
                    int j = 0;
#pragma unroll
                    for (int st = 32; st >= 1; st >>= 1) {
                        const int32_t e = __shfl(excl, j + st, 64);
                        if (e <= q) j += st;
                    }
                    const int32_t lj = __shfl(lo, j, 64), ej = __shfl(excl, j, 64);
                    val[u] = q < T;
                    const size_t in = (size_t)(lj + (q - ej));
                    pos[u] = !val[u] ? 0 : part ? in : (size_t)(kk + j) * (size_t)max_u + in;
                }
                uint16_t c[kUn];
                double v[kUn];
                if (part) {
                    int32_t r[kUn];
#pragma unroll
                    for (int u = 0; u < kUn; ++u) {
                        c[u] = tl.tcol16[pos[u]];
                        v[u] = tl.tval[pos[u]];
                        r[u] = tl.trow[pos[u]];
                    }
#pragma unroll
                    for (int u = 0; u < kUn; ++u) v[u] *= tl.rowcoef[r[u]];
                } else {
#pragma unroll
                    for (int u = 0; u < kUn; ++u) {
                        c[u] = fcol16[pos[u]];
                        v[u] = dw[pos[u]];
                    }
                }
#pragma unroll
                for (int u = 0; u < kUn; ++u)
                    if (val[u]) atomicAdd(&acc[c[u]], v[u]);
            }
        }
    }
    __syncthreads();
    const int64_t j0 = (int64_t)b * kFoldJ;
    for (int i = tid; i < kFoldJ && j0 + i < d; i += 256) {
        const double x = acc[i];
        if (sole)
            tmp[j0 + i] = x;
        else if (x != 0.0)
            unsafeAtomicAdd(tmp + j0 + i, x);
    }
}

__global__ __launch_bounds__(256) void fold_finish_kernel(double* tmp, int64_t d, double* dw_sum, double* w,
                                                          double mult, int apply, const int32_t* inv) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < d; j += (int64_t)gridDim.x * 256) {
        const double v = tmp[j];
        tmp[j] = 0.0;
        if (apply)
            w[j] = w[j] + v * mult;
        else
            dw_sum[inv ? inv[j] : j] = v;
    }
}

void launch_fold_blocks(const double* dw, const uint16_t* fcol16, const uint32_t* fbnd, const int32_t* items,
                        int32_t n_items, int32_t K, int64_t max_u, int64_t d, double* tmp, double* dw_sum, double* w,
                        double mult, bool apply, const int32_t* inv, hipStream_t s, const FoldTail* tail) {
    if (n_items > 0) {
        if (tail)
            fold_blocks_kernel<true><<<n_items, 256, 0, s>>>(dw, fcol16, fbnd, items, K, max_u, d, tmp, *tail);
        else
            fold_blocks_kernel<false><<<n_items, 256, 0, s>>>(dw, fcol16, fbnd, items, K, max_u, d, tmp, FoldTail{});
    }
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((d + 255) / 256, 4096));
    fold_finish_kernel<<<blocks, 256, 0, s>>>(tmp, d, dw_sum, w, mult, apply ? 1 : 0, inv);
}

// ------------------------------------------------------------ dense rows --
// 16-byte column chunks per thread: CPT * kDT * 2 >= d
static int dense_cpt(int64_t d) { return d <= 512 ? 1 : d <= 1024 ? 2 : d <= 2048 ? 4 : d <= 4096 ? 8 : 0; }

bool dense_solver_fits(int64_t d, int64_t max_nl) {
    return d >= 2 && (d & 1) == 0 && dense_cpt(d) > 0 && max_nl >= 1 && max_nl * 8 <= 150 * 1024;
}
bool dense_eval_fits(int64_t d) { return d >= 2 && (d & 1) == 0 && d <= 4096; }

template <int MODE, int CPT, int P, bool PROJ>
static void launch_ds3(const DenseArgs& a, int grid, size_t lds, hipStream_t s) {
    (void)hipFuncSetAttribute((const void*)dense_solver_kernel<MODE, CPT, P, kDT, PROJ>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dense_solver_kernel<MODE, CPT, P, kDT, PROJ><<<grid, kDT, lds, s>>>(a);
}
template <int MODE, int CPT, int P>
static void launch_ds(const DenseArgs& a, int grid, size_t lds, hipStream_t s) {
    if (a.proj) launch_ds3<MODE, CPT, P, true>(a, grid, lds, s);
    else launch_ds3<MODE, CPT, P, false>(a, grid, lds, s);
}

template <int MODE>
static void launch_ds_mode(const DenseArgs& a, int grid, size_t lds, hipStream_t s) {
    // P = rows in flight per workgroup (16 KB each at d = 2,000); the ring is
    // P * CPT * 4 VGPRs
    switch (dense_cpt(a.d)) {
        case 1: launch_ds<MODE, 1, 16>(a, grid, lds, s); break;
        case 2: launch_ds<MODE, 2, 16>(a, grid, lds, s); break;
        case 4: launch_ds<MODE, 4, 8>(a, grid, lds, s); break;
        default: launch_ds<MODE, 8, 4>(a, grid, lds, s); break;
    }
}

void launch_solver_dense(int mode, const DenseArgs& a, int grid, int64_t max_nl, hipStream_t s) {
    const size_t lds = sizeof(double) * (size_t)max_nl;
    if (mode == MODE_PLUS) launch_ds_mode<MODE_PLUS>(a, grid, lds, s);
    else if (mode == MODE_COCOA) launch_ds_mode<MODE_COCOA>(a, grid, lds, s);
    else launch_ds_mode<MODE_MBCD>(a, grid, lds, s);
}

void launch_eval_dense(const EvalArgs& a, hipStream_t s) {
    constexpr int kBlocks = 1024;  // 4 per CU, one row per wave-iteration pair
    const int64_t nch = a.d >> 1;
    if (nch <= 256) eval_dense_kernel<4, 2><<<kBlocks, 256, 0, s>>>(a);
    else if (nch <= 512) eval_dense_kernel<8, 2><<<kBlocks, 256, 0, s>>>(a);
    else if (nch <= 1024) eval_dense_kernel<16, 2><<<kBlocks, 256, 0, s>>>(a);
    else eval_dense_kernel<32, 1><<<kBlocks, 256, 0, s>>>(a);
    eval_final_kernel<<<1, 256, 0, s>>>(a.partials, kBlocks, a.out);
}

}  // namespace cocoa


namespace cocoa {

// ------------------------------------------------------- fast SGD (C5) --
// mb-SGD (SGD.scala:87-139 with local = false): within a round every sampled
// row is tested against the same driver w, so the H steps of a partition are
// independent.  One wave per coordinate step over all K_loc * H steps of the
// launch: wave-tree x.w, and a violator (1 - y x.w > 0, SGD.scala:115,124)
// adds x*y into its partition's private deltaW slice with fire-and-forget
// atomics (sum order differs from the reference's sequential adds: fast mode).
__global__ __launch_bounds__(256) void mbsgd_fast_kernel(SolverArgs a, int32_t K) {
    const int lane = threadIdx.x & 63;
    const int64_t total = (int64_t)K * a.H;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < total; g += nw) {
        const int32_t k = (int32_t)(g / a.H);
        const int64_t gr = a.part_ptr[k] + a.samples[g];
        const int64_t b = a.row_ptr[gr], e = a.row_ptr[gr + 1];
        const double yv = a.y[gr];
        double acc = 0.0;
        for (int64_t q = b + lane; q < e; q += 64) acc = fma(a.val[q], a.w[a.col[q]], acc);
        const double dot = wave_sum(acc);
        if (1.0 - yv * dot > 0) {
            double* dwk = a.dw + (size_t)k * a.d;
            for (int64_t q = b + lane; q < e; q += 64) unsafeAtomicAdd(dwk + a.col[q], a.val[q] * yv);
        }
    }
}

// local SGD (SGD.scala:87-139 with local = true): one wave per partition runs
// the sequential chain.  The reference shrinks its whole w copy by
// (1 - step*lambda) every step (O(d), SGD.scala:119-120); here w = s * v with
// the shrink folded into the scalar s, so a step costs O(z):
//   x.w = s (x.v);  s *= 1 - step*lambda;  v += x*y*step / s  (if violator).
// A shrink factor of exactly 0 (the first step of round 1) zeroes v and
// resets s; a tiny s is folded back into v.  deltaW = s v - wInit.
__device__ void localsgd_rescale(double* v, int64_t d, double f) {
    for (int64_t j = lane_id(); j < d; j += 64) v[j] = v[j] * f;
}

__global__ __launch_bounds__(64) void localsgd_fast_kernel(SolverArgs a, double lambda, double t0) {
    const int k = blockIdx.x;
    const int lane = lane_id();
    const int64_t p0 = a.part_ptr[k];
    const int64_t d = a.d;
    double* v = a.wloc + (size_t)k * d;
    double* dwk = a.dw + (size_t)k * d;
    for (int64_t j = lane; j < d; j += 64) v[j] = a.w[j];
    double s = 1.0;
    for (int32_t i = 1; i <= a.H; ++i) {
        const double step = 1.0 / (lambda * (t0 + (double)i));          // SGD.scala:106
        const int64_t gr = p0 + a.samples[(size_t)k * a.H + (i - 1)];
        const int64_t b = a.row_ptr[gr], e = a.row_ptr[gr + 1];
        const double yv = a.y[gr];
        double acc = 0.0;
        for (int64_t q = b + lane; q < e; q += 64) acc = fma(a.val[q], v[a.col[q]], acc);
        const double ev = 1.0 - yv * (s * wave_sum(acc));                // SGD.scala:115
        const double scale = 1.0 - step * lambda;                        // SGD.scala:119-120
        if (scale == 0.0) {
            localsgd_rescale(v, d, 0.0);
            s = 1.0;
        } else {
            s *= scale;
        }
        if (ev > 0) {                                                    // SGD.scala:124-130
            const double u = (yv * step) / s;
            if (a.any_dup && a.rowflags && (a.rowflags[gr] & 1)) {
                if (lane == 0)
                    for (int64_t q = b; q < e; ++q) v[a.col[q]] = v[a.col[q]] + a.val[q] * u;
            } else {
                for (int64_t q = b + lane; q < e; q += 64) v[a.col[q]] = fma(a.val[q], u, v[a.col[q]]);
            }
        }
        if (fabs(s) < 1e-150) {
            localsgd_rescale(v, d, s);
            s = 1.0;
        }
    }
    for (int64_t j = lane; j < d; j += 64) dwk[j] = s * v[j] - a.w[j];  // SGD.scala:133
}

// ---------------------------------------------- mb-SGD, pull form (C5) --
// SGD.scala:108-129 with local = false: every sampled step tests its row against
// the same w (the driver's, scaled by 1 - step lambda at SGD.scala:48-49), and a
// violator adds x y to deltaW.  Summed over the round, deltaW = sum_r cnt_r y_r
// [1 - y_r x_r.w > 0] x_r = X^T c.  mbsgd_fast_kernel scatters it with fp64
// atomics, one per entry of every violating step; atomics execute at the memory
// side, ~17x slower scattered than streamed (MI355X_MICROARCH.md, global float
// atomics), and bound that kernel.  Here: the round's sample counts per row,
// c_r, then every device column's sum of val * c[row] over a CSC copy (built
// once, cocoa_init), tile by tile: a tile of whole short columns is summed by
// 16-lane groups from LDS products and stored; a slice of a long column (the
// frequency order puts them first) is summed by the block and added atomically
// (a few per long column).  Same terms, another order: fast mode.

// CSC fill: entries of row r to their column's next slot (cursor: csc_ptr copy)
__global__ __launch_bounds__(256) void csc_fill_kernel(const int64_t* row_ptr, const int32_t* col, const double* val,
                                                       int64_t n_rows, int64_t* cursor, int32_t* csc_row,
                                                       double* csc_val) {
    const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int sub = threadIdx.x & 15;
    if (r >= n_rows) return;
    for (int64_t q = row_ptr[r] + sub; q < row_ptr[r + 1]; q += 16) {
        const unsigned long long pos = atomicAdd((unsigned long long*)(cursor + col[q]), 1ull);
        csc_row[pos] = (int32_t)r;
        csc_val[pos] = val[q];
    }
}

void launch_csc_fill(const int64_t* row_ptr, const int32_t* col, const double* val, int64_t n_rows, int64_t* cursor,
                     int32_t* csc_row, double* csc_val, hipStream_t s) {
    if (n_rows > 0)
        csc_fill_kernel<<<(unsigned)((n_rows * 16 + 255) / 256), 256, 0, s>>>(row_ptr, col, val, n_rows, cursor, csc_row,
                                                                           csc_val);
}

__global__ __launch_bounds__(256) void mbsgd_count_kernel(const int64_t* part_ptr, const int32_t* samples, int32_t H,
                                                          int64_t steps, int32_t* cnt) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= steps) return;
    atomicAdd(cnt + part_ptr[g / H] + samples[g], 1);
}

// c_r = cnt_r y_r if 1 - y_r x_r.w > 0 (SGD.scala:115, 124), 16 lanes per row;
// x_r.w = scale * cached (the last evaluation's x.w of the unscaled w) or the
// dot with the scaled w; cnt_r reset for the next round
__global__ __launch_bounds__(256) void mbsgd_coef_kernel(const int64_t* row_ptr, const int32_t* col, const double* val,
                                                         const double* y, const double* w, const double* xw_cache,
                                                         double scale, int64_t n_rows, int32_t* cnt, double* c) {
    const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int sub = threadIdx.x & 15;
    const bool ok = r < n_rows;
    const int32_t k = ok ? cnt[r] : 0;
    double xw = 0.0;
    if (k > 0 && !xw_cache) {
        double acc = 0.0;
        for (int64_t q = row_ptr[r] + sub; q < row_ptr[r + 1]; q += 16) acc = fma(val[q], w[col[q]], acc);
        xw = acc;
    }
    if (!xw_cache) xw = row16_sum(xw);  // (whole 16-lane rows: the row sum stays inside them)
    if (ok && sub == 0) {
        double cv = 0.0;
        if (k > 0) {
            const double yv = y[r];
            const double d = xw_cache ? scale * xw_cache[r] : xw;
            if (1.0 - yv * d > 0) cv = (double)k * yv;
        }
        c[r] = cv;
        if (k) cnt[r] = 0;
    }
}

// tile t = tiles[4 t .. 4 t + 3] = (e0, e1, j0, j1): entries [e0, e1) holding
// the whole columns [j0, j1), or with j1 = -1 a slice of column j0 alone, added
// atomically (its column's out word is zero on entry); <= kPullTile entries
__global__ __launch_bounds__(256) void mbsgd_pull_kernel(MbsgdPull p, double* out) {
    __shared__ double prod[kPullTile];
    __shared__ double red[4];
    const int tid = threadIdx.x, sub = tid & 15, grp = tid >> 4;
    for (int64_t t = blockIdx.x; t < p.n_tiles; t += gridDim.x) {
        const int64_t e0 = p.tiles[4 * t], e1 = p.tiles[4 * t + 1];
        const int64_t j0 = p.tiles[4 * t + 2], j1 = p.tiles[4 * t + 3];
        const int n = (int)(e1 - e0);
        if (j1 < 0) {  // a slice of column j0
            double acc = 0.0;
            for (int i = tid; i < n; i += 256) acc = fma(p.csc_val[e0 + i], p.row_c[p.csc_row[e0 + i]], acc);
            const double s = block_sum_n<256>(acc, red);
            if (tid == 0) unsafeAtomicAdd(out + j0, s);
            __syncthreads();
            continue;
        }
        for (int i = tid; i < n; i += 256) prod[i] = p.csc_val[e0 + i] * p.row_c[p.csc_row[e0 + i]];
        __syncthreads();
        for (int64_t j = j0 + grp; j < j1; j += 16) {
            const int b = (int)(p.csc_ptr[j] - e0), e = (int)(p.csc_ptr[j + 1] - e0);
            double acc = 0.0;
            for (int q = b + sub; q < e; q += 16) acc += prod[q];
            const double s = row16_sum(acc);
            if (sub == 0) out[j] = s;
        }
        __syncthreads();
    }
}

void launch_mbsgd_pull(const SolverArgs& a, const MbsgdPull& p, int32_t K, int64_t n_rows, const double* xw_cache,
                       double scale, double* out, hipStream_t s) {
    const int64_t steps = (int64_t)K * a.H;
    if (steps > 0)
        mbsgd_count_kernel<<<(unsigned)((steps + 255) / 256), 256, 0, s>>>(a.part_ptr, a.samples, a.H, steps, p.row_cnt);
    if (n_rows > 0)
        mbsgd_coef_kernel<<<(unsigned)((n_rows * 16 + 255) / 256), 256, 0, s>>>(a.row_ptr, a.col, a.val, a.y, a.w, xw_cache,
                                                                              scale, n_rows, p.row_cnt, p.row_c);
    if (p.n_tiles > 0)
        mbsgd_pull_kernel<<<(unsigned)std::min<int64_t>(p.n_tiles, 2048), 256, 0, s>>>(p, out);
}

void launch_sgd_fast(bool local, const SolverArgs& a, double lambda, double t0, int K, hipStream_t s) {
    if (local) {
        localsgd_fast_kernel<<<K, 64, 0, s>>>(a, lambda, t0);
    } else {
        const int64_t waves = (int64_t)K * a.H;
        const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, 256 * 8));
        mbsgd_fast_kernel<<<blocks, 256, 0, s>>>(a, K);
    }
}

}  // namespace cocoa
