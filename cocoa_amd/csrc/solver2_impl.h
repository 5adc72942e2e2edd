// Local solver v2 for CoCoA+ and MbCD (CoCoA.scala:148-188, MinibatchCD.scala:95-125).
//
// Per step, the only mutable data the chain reads is deltaW at the row's
// columns (CoCoA+: the dot x.deltaW and the scatter deltaW += update; MbCD:
// the scatter).  x.w is read-only within a round and comes from the step plan
// (plan_kernel: one pass over the sampled rows on the whole chip).
//
// deltaW of the partition is split by device feature index (features are
// relabelled by descending frequency, engine.hip):
//   hot  [0, hot)  -- lives in LDS for the whole round: gathers and scatters
//                     are LDS operations;
//   cold [hot, d)  -- lives in the partition's private HBM slice.  The loader
//                     prefetches the cold entries of a batch into LDS next to
//                     the row's (col, val).  The prefetch runs one batch ahead,
//                     concurrently with the solver's writes, so a prefetched
//                     value may be stale if the solver wrote that feature in the
//                     previous or the current batch: the solver marks every cold
//                     write in a per-batch-parity dirty bitmap and re-reads a
//                     flagged entry from memory (its own stores are ordered
//                     before its own loads).  alpha_work[r] is prefetched and
//                     guarded the same way, with a row bitmap.
// Cross-wave reads of global data that the solver wave writes use agent-scope
// (L1-bypassing) loads; the solver drains its stores (vmcnt(0)) before every
// batch barrier.  Nothing here changes an arithmetic operation or its order,
// so the strict instantiation stays bit-exact.
//
// Workgroup: wave 0 = solver, waves 1.. = loaders (all loader waves load the
// batch's metadata; the entry stream is split between them).
#pragma once
#include "kernels.h"
#include "solver_impl.h"
#include "wave.h"

namespace cocoa {

constexpr int kLoaders2 = 2;                 // loader waves per workgroup
constexpr int kThreads2 = 64 * (1 + kLoaders2);
constexpr int kLoadUnroll2 = 8;

__device__ __forceinline__ double aload(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// s_waitcnt vmcnt(0) (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15), issued
// through the builtin so the compiler's wait-count pass sees it: after it the
// pass knows no vector-memory result is pending and inserts no wait of its own
// into the (LDS-only) solver loop.
__device__ __forceinline__ void drain_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ bool bit_set(const uint32_t* a, const uint32_t* b, uint32_t i) {
    return ((a[i >> 5] | b[i >> 5]) >> (i & 31)) & 1u;
}

// Loader: stage the next batch (up to 64 steps whose entries fit `cap`).
// `lw` = index of this loader wave (0..kLoaders2-1).
template <int MODE>
__device__ void load_batch2(const Solver2Args& a, int k, int64_t p0, int lw, int32_t& cursor, Batch2* mb,
                            int32_t* scol, double* sval, double* scold, const double* dwk) {
    const int lane = lane_id();
    const int32_t H = a.H;
    const int32_t C = a.cap;
    if (cursor >= H) {
        if (lw == 0 && lane == 0) mb->m = 0;
        return;
    }
    const int32_t s = cursor + lane;
    const bool valid = s < H;
    const size_t g = (size_t)k * H + s;
    int32_t r = 0, z = 0, fl = 0;
    int64_t beg = 0;
    double yv = 0.0, qv = 0.0, xw = 0.0, ap = 0.0;
    if (valid) {
        r = a.samples[g];
        beg = a.plan_beg[g];
        z = a.plan_z[g];
        yv = a.plan_y[g];
        qv = a.plan_q[g];
        if (MODE != MODE_COCOA) xw = a.plan_xw[g];
        if (a.any_dup) fl = a.rowflags[p0 + r];
    }
    if (lw == 0 && valid) ap = aload(a.alpha_work + p0 + r);
    const bool staged = z <= C;
    const int32_t zz = (valid && staged) ? z : 0;
    const int32_t incl = wave_incl_scan(zz);
    const bool fits = valid && incl <= C;
    const uint64_t mask = __ballot(fits);
    const int m = (~mask == 0ULL) ? 64 : __builtin_ctzll(~mask);  // >= 1
    const int32_t excl = incl - zz;
    if (lw == 0 && lane < m) {
        StepMeta& st = mb->st[lane];
        st.r = r;
        st.off = staged ? excl : -1;
        st.z = z;
        st.fl = fl;
        st.beg = beg;
        st.y = yv;
        st.q = qv;
        st.xw = xw;
        st.ap = ap;
    }
    const int32_t T = __shfl(incl, m - 1, 64);
    const int32_t hot = a.hot;
    const bool has_cold = scold != nullptr;
    // entry stream: 64-entry units, unit u of the batch handled by loader wave u % kLoaders2
    const int32_t units = (T + 63) >> 6;
    for (int32_t u0 = lw; u0 < units; u0 += kLoaders2 * kLoadUnroll2) {
        int32_t pc[kLoadUnroll2];
        double pv[kLoadUnroll2], pd[kLoadUnroll2];
#pragma unroll
        for (int u = 0; u < kLoadUnroll2; ++u) {
            const int32_t p = (u0 + u * kLoaders2) * 64 + lane;
            const int32_t pq = p < T ? p : T - 1;
            const int j = find_step(pq, excl, m);
            const int64_t bj = __shfl(beg, j, 64);
            const int32_t ej = __shfl(excl, j, 64);
            pc[u] = 0;
            pv[u] = 0.0;
            if (p < T) {
                const int64_t e = bj + (pq - ej);
                pc[u] = a.col[e];
                pv[u] = a.val[e];
            }
        }
        if (has_cold) {
#pragma unroll
            for (int u = 0; u < kLoadUnroll2; ++u) {
                const int32_t p = (u0 + u * kLoaders2) * 64 + lane;
                pd[u] = (p < T && pc[u] >= hot) ? aload(dwk + pc[u]) : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < kLoadUnroll2; ++u) {
            const int32_t p = (u0 + u * kLoaders2) * 64 + lane;
            if (p < T) {
                scol[p] = pc[u];
                sval[p] = pv[u];
                if (has_cold && pc[u] >= hot) scold[p] = pd[u];
            }
        }
    }
    if (lw == 0 && lane == 0) mb->m = m;
    cursor += m;
}

// deltaW value of feature c for the non-register paths: LDS for hot features,
// memory (this wave's own latest store) for cold ones.
__device__ __forceinline__ double dw_at(const double* hotv, int32_t hot, const double* dwk, int32_t c) {
    return c < hot ? hotv[c] : aload(dwk + c);
}

// Uniform (wave-wide) per-step values, read from the batch metadata.
struct StepU {
    int32_t r, off, z, fl;
    int64_t beg;
    double y, q, xw, ap;
};

__device__ __forceinline__ StepU read_step(const StepMeta& st) {
    StepU u;
    u.r = uni(st.r);
    u.off = uni(st.off);
    u.z = uni(st.z);
    u.fl = uni(st.fl);
    u.beg = uni(st.beg);
    u.y = uni(st.y);
    u.q = uni(st.q);
    u.xw = uni(st.xw);
    u.ap = uni(st.ap);
    return u;
}

// Per-step update rule shared by all paths (CoCoA.scala:157-186,
// MinibatchCD.scala:104-123).  Returns false when the step is skipped
// (projected gradient exactly 0); otherwise na / coef.
template <int MODE>
__device__ __forceinline__ bool sdca_rule(const StepU& st, double aa, double sdot, double sigma, double lam_n,
                                          double& na, double& coef) {
    double grad;
    if (MODE == MODE_PLUS)
        grad = (st.y * (st.xw + (sigma * sdot)) - 1.0) * lam_n;  // CoCoA.scala:159
    else
        grad = (st.y * (st.xw) - 1.0) * lam_n;                   // MinibatchCD.scala:104
    double proj = grad;                                          // CoCoA.scala:166-170
    if (aa <= 0.0)
        proj = jmin(grad, 0.0);
    else if (aa >= 1.0)
        proj = jmax(grad, 0.0);
    if (!(fabs(proj) != 0.0)) return false;                      // CoCoA.scala:172
    const double qii = MODE == MODE_PLUS ? st.q * sigma : st.q;  // CoCoA.scala:173-174
    na = 1.0;
    if (qii != 0.0) na = jmin(jmax((aa - (grad / qii)), 0.0), 1.0);  // CoCoA.scala:175-178
    coef = (st.y * (na - aa)) / lam_n;                           // CoCoA.scala:181
    return true;
}

struct SolverLds {
    const int32_t* scol;
    const double* sval;
    const double* scold;     // null when every feature is hot
    double* hotv;
    double* sink;            // 64 doubles: target of masked-off LDS writes
    uint32_t* dw_cur;
    const uint32_t* dw_prev;
    uint32_t* da_cur;
    const uint32_t* da_prev;
    double* scratch;
};

// Register path for a staged row of at most 64*NCH entries without duplicate
// columns.  Branch-free per entry: hot and cold candidates are both read and
// selected; masked-off lanes write to a private sink.
template <int MODE, bool STRICT, int NCH>
__device__ __forceinline__ void step_regs(const Solver2Args& a, const SolverLds& L, const StepU& st, double aa,
                                          double* dwk, int64_t p0, uint64_t (&sp)[6]) {
    const int lane = lane_id();
    const int32_t hot = a.hot;
    const uint32_t wmask = (uint32_t)a.wmask;
#ifdef COCOA_STEP_PROF
    uint64_t last_ = clock64();
#endif
    (void)sp;
    int32_t pc[NCH];
    double pv[NCH], pd[NCH];
    bool in[NCH], cold[NCH];
    uint32_t ci[NCH];
    uint32_t dirty = 0;
    const bool has_cold = L.scold != nullptr;
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
        const int32_t p = lane + 64 * u;
        in[u] = p < st.z;
        pc[u] = L.scol[st.off + p];
        const double v = L.sval[st.off + p];
        pv[u] = in[u] ? v : 0.0;
        const uint32_t hidx = min((uint32_t)pc[u], (uint32_t)(hot - 1));
        const double ph = L.hotv[hidx];
        cold[u] = has_cold && in[u] && pc[u] >= hot;
        ci[u] = (uint32_t)(pc[u] - hot) & wmask;
        if (has_cold) {
            const double pcv = L.scold[st.off + p];
            pd[u] = cold[u] ? pcv : ph;
            const uint32_t w = L.dw_cur[ci[u] >> 5] | L.dw_prev[ci[u] >> 5];
            if (cold[u] && ((w >> (ci[u] & 31)) & 1u)) dirty |= 1u << u;
        } else {
            pd[u] = ph;
        }
    }
    if (has_cold && __any(dirty != 0)) {
        // a staged cold value may predate a write of this or the previous batch
        double g[NCH];
#pragma unroll
        for (int u = 0; u < NCH; ++u) g[u] = ((dirty >> u) & 1) ? aload(dwk + pc[u]) : 0.0;
        drain_vm();  // retire the loads inside the rare branch
#pragma unroll
        for (int u = 0; u < NCH; ++u)
            if ((dirty >> u) & 1) pd[u] = g[u];
    }
    STEP_STAMP(1);
    double sdot = 0.0;
    if (MODE == MODE_PLUS) {
        if (STRICT) {
            double prod[kRegChunks];
#pragma unroll
            for (int u = 0; u < kRegChunks; ++u) prod[u] = u < NCH ? pv[u] * pd[u] : 0.0;
            sdot = dot_regs<true>(prod, st.z, L.scratch);
        } else {
            double acc = pv[0] * pd[0];
#pragma unroll
            for (int u = 1; u < NCH; ++u) acc += pv[u] * pd[u];
            sdot = wave_sum(acc);
        }
    }
    STEP_STAMP(2);
    double na, coef;
    if (!sdca_rule<MODE>(st, aa, sdot, a.sigma, a.lam_n, na, coef)) return;
    STEP_STAMP(3);
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
        const double nv = pd[u] + pv[u] * coef;                 // deltaW += update (CoCoA.scala:185)
        const bool hw = in[u] && !cold[u];
        double* dst = hw ? L.hotv + pc[u] : L.sink + lane;
        *dst = nv;
        if (has_cold) {
            atomicOr(L.dw_cur + (ci[u] >> 5), cold[u] ? (1u << (ci[u] & 31)) : 0u);
            if (cold[u]) dwk[pc[u]] = nv;
        }
    }
    if (lane == 0) {
        a.alpha_work[p0 + st.r] = na;                           // CoCoA.scala:186
        const uint32_t ri = (uint32_t)st.r & (uint32_t)a.amask;
        atomicOr(L.da_cur + (ri >> 5), 1u << (ri & 31));
    }
}

// Everything else: long / unstaged / duplicate-column rows (rare).  Cold
// values are always read from memory here (this wave's own stores are ordered
// before its own loads).
template <int MODE, bool STRICT>
__device__ void step_generic(const Solver2Args& a, const SolverLds& L, const StepU& st, double aa, double* dwk,
                             int64_t p0) {
    const int lane = lane_id();
    const int32_t hot = a.hot;
    const uint32_t wmask = (uint32_t)a.wmask;
    const int32_t z = st.z, off = st.off;
    auto col_at = [&](int32_t p) { return off >= 0 ? L.scol[off + p] : a.col[st.beg + p]; };
    auto val_at = [&](int32_t p) { return off >= 0 ? L.sval[off + p] : a.val[st.beg + p]; };
    double sdot = 0.0;
    if (MODE == MODE_PLUS) {
        if (STRICT) {
            double t = 0.0;
            for (int32_t c0 = 0; c0 < z; c0 += 64) {
                const int32_t p = c0 + lane;
                if (p < z) L.scratch[lane] = val_at(p) * dw_at(L.hotv, hot, dwk, col_at(p));
                wave_lds_sync();
                const int32_t cnt = z - c0 < 64 ? z - c0 : 64;
                if (lane == 0)
                    for (int32_t q = 0; q < cnt; ++q) t += L.scratch[q];
                wave_lds_sync();
            }
            sdot = uni(t);
        } else {
            double acc = 0.0;
            for (int32_t p = lane; p < z; p += 64) acc += val_at(p) * dw_at(L.hotv, hot, dwk, col_at(p));
            sdot = wave_sum(acc);
        }
    }
    double na, coef;
    if (sdca_rule<MODE>(st, aa, sdot, a.sigma, a.lam_n, na, coef)) {
        auto put = [&](int32_t c, double v) {
            const double nv = dw_at(L.hotv, hot, dwk, c) + v * coef;
            if (c < hot) {
                L.hotv[c] = nv;
            } else {
                dwk[c] = nv;
                const uint32_t ci = (uint32_t)(c - hot) & wmask;
                atomicOr(L.dw_cur + (ci >> 5), 1u << (ci & 31));
            }
        };
        if (st.fl & 1) {
            // duplicate column indices: the reference's sequential scatter
            if (lane == 0)
                for (int32_t q = 0; q < z; ++q) put(col_at(q), val_at(q));
        } else {
            for (int32_t p = lane; p < z; p += 64) put(col_at(p), val_at(p));
        }
        if (lane == 0) {
            a.alpha_work[p0 + st.r] = na;                       // CoCoA.scala:186
            const uint32_t ri = (uint32_t)st.r & (uint32_t)a.amask;
            atomicOr(L.da_cur + (ri >> 5), 1u << (ri & 31));
        }
    }
    drain_vm();
}

template <int MODE, bool STRICT>
__device__ void compute_batch2(const Solver2Args& a, const Batch2* mb, const SolverLds& L, double* dwk, int64_t p0,
                               uint64_t (&sp)[6]) {
    const int m = uni(mb->m);
    const uint32_t amask = (uint32_t)a.amask;
#ifdef COCOA_STEP_PROF
    uint64_t last_ = clock64();
#endif
    (void)sp;
    for (int s = 0; s < m; ++s) {
        const StepU st = read_step(mb->st[s]);
        double aa = st.ap;
        if (bit_set(L.da_cur, L.da_prev, (uint32_t)st.r & amask)) {
            aa = uni(aload(a.alpha_work + p0 + st.r));
            drain_vm();
        }
        STEP_STAMP(0);
        const int nch = (st.z + 63) >> 6;
        if (st.off >= 0 && (st.fl & 1) == 0 && nch <= 4) {
            switch (nch) {
                case 0:
                case 1: step_regs<MODE, STRICT, 1>(a, L, st, aa, dwk, p0, sp); break;
                case 2: step_regs<MODE, STRICT, 2>(a, L, st, aa, dwk, p0, sp); break;
                case 3: step_regs<MODE, STRICT, 3>(a, L, st, aa, dwk, p0, sp); break;
                default: step_regs<MODE, STRICT, 4>(a, L, st, aa, dwk, p0, sp); break;
            }
        } else {
            step_generic<MODE, STRICT>(a, L, st, aa, dwk, p0);
        }
        STEP_STAMP(4);
    }
}

template <int MODE, bool STRICT>
__global__ __launch_bounds__(kThreads2, 1) void solver2_kernel(Solver2Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int k = blockIdx.x;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int64_t p0 = a.part_ptr[k], p1 = a.part_ptr[k + 1];
    const int32_t nl = (int32_t)(p1 - p0);
    const int64_t d = a.d;
    const int32_t hot = a.hot;
    double* dwk = a.dw + (size_t)k * d;
    double* hotv = (double*)(lds + a.lds_hot);
    double* scratch = (double*)(lds + a.lds_scratch);
    const int nww = ((a.wmask + 1) + 31) >> 5, naw = ((a.amask + 1) + 31) >> 5;

    // prologue: working alpha = alphaOld; hot deltaW = 0; bitmaps clear
    for (int32_t i = tid; i < nl; i += kThreads2) a.alpha_work[p0 + i] = a.alpha[p0 + i];
    for (int32_t j = tid; j < hot; j += kThreads2) hotv[j] = 0.0;
    for (int b = 0; b < 2; ++b) {
        uint32_t* dwb = (uint32_t*)(lds + a.lds_dirty_w[b]);
        uint32_t* dab = (uint32_t*)(lds + a.lds_dirty_a[b]);
        for (int i = tid; i < nww; i += kThreads2) dwb[i] = 0u;
        for (int i = tid; i < naw; i += kThreads2) dab[i] = 0u;
    }
    drain_vm();
    __syncthreads();
    int32_t cursor = 0;
    auto buf_col = [&](int b) { return (int32_t*)(lds + a.lds_col[b]); };
    auto buf_val = [&](int b) { return (double*)(lds + a.lds_val[b]); };
    auto buf_cold = [&](int b) { return a.lds_cold[b] >= 0 ? (double*)(lds + a.lds_cold[b]) : (double*)nullptr; };
    auto buf_meta = [&](int b) { return (Batch2*)(lds + a.lds_batch[b]); };
    if (wave >= 1) load_batch2<MODE>(a, k, p0, wave - 1, cursor, buf_meta(0), buf_col(0), buf_val(0), buf_cold(0), dwk);
    __syncthreads();
    uint64_t t_busy = 0, t_wait = 0, n_batch = 0;
    uint64_t step_prof[6] = {0, 0, 0, 0, 0, 0};
    for (int b = 0;; ++b) {
        const int cur = b & 1;
        const Batch2* mb = buf_meta(cur);
        if (mb->m == 0) break;
        const uint64_t c0 = a.prof ? clock64() : 0;
        uint64_t c0x = 0;
        if (a.dbg_serial) {
            // diagnostics only: the loader stages the next batch while the solver
            // waits, so the solver's cycles below are free of LDS contention
            if (wave >= 1)
                load_batch2<MODE>(a, k, p0, wave - 1, cursor, buf_meta(cur ^ 1), buf_col(cur ^ 1),
                                  buf_val(cur ^ 1), buf_cold(cur ^ 1), dwk);
            __syncthreads();
        }
        if (wave >= 1) {
            if (!a.dbg_serial)
                load_batch2<MODE>(a, k, p0, wave - 1, cursor, buf_meta(cur ^ 1), buf_col(cur ^ 1),
                                  buf_val(cur ^ 1), buf_cold(cur ^ 1), dwk);
        } else {
            drain_vm();
            if (a.dbg_serial && a.prof) c0x = clock64();
            uint32_t* dw_cur = (uint32_t*)(lds + a.lds_dirty_w[cur]);
            uint32_t* da_cur = (uint32_t*)(lds + a.lds_dirty_a[cur]);
            // this parity held the bits of batch b-2, whose writes every
            // prefetch of batch b (and later) already sees
            for (int i = tid; i < nww; i += 64) dw_cur[i] = 0u;
            for (int i = tid; i < naw; i += 64) da_cur[i] = 0u;
            wave_lds_sync();
            SolverLds L;
            L.scol = buf_col(cur);
            L.sval = buf_val(cur);
            L.scold = buf_cold(cur);
            L.hotv = hotv;
            L.sink = (double*)(lds + a.lds_sink);
            L.dw_cur = dw_cur;
            L.dw_prev = (const uint32_t*)(lds + a.lds_dirty_w[cur ^ 1]);
            L.da_cur = da_cur;
            L.da_prev = (const uint32_t*)(lds + a.lds_dirty_a[cur ^ 1]);
            L.scratch = scratch;
            compute_batch2<MODE, STRICT>(a, mb, L, dwk, p0, step_prof);
            drain_vm();
        }
        const uint64_t c1 = a.prof ? clock64() : 0;
        __syncthreads();
        if (a.prof) {
            t_busy += c1 - (c0x ? c0x : c0);
            t_wait += clock64() - c1;
            n_batch += 1;
        }
    }
    if (a.prof && (tid & 63) == 0 && wave < 2) {
        uint64_t* pr = a.prof + ((size_t)k * 2 + wave) * 16;
        pr[0] = t_busy;
        pr[1] = t_wait;
        pr[2] = n_batch;
        for (int i = 0; i < 6; ++i) pr[3 + i] = step_prof[i];
    }
    // epilogue: hot slice back to the private deltaW; alpha = alphaOld +
    // (alpha - alphaOld) * scaling (CoCoA.scala:101, MinibatchCD.scala:127-128)
    for (int32_t j = tid; j < hot; j += kThreads2) dwk[j] = hotv[j];
    if (a.raw_alpha) {
        for (int32_t i = tid; i < nl; i += kThreads2) a.alpha[p0 + i] = aload(a.alpha_work + p0 + i);
    } else {
        for (int32_t i = tid; i < nl; i += kThreads2) {
            const double old = a.alpha[p0 + i];
            a.alpha[p0 + i] = old + ((aload(a.alpha_work + p0 + i) - old) * a.scaling);
        }
    }
}

template <bool STRICT>
void launch_solver2_impl(int mode, const Solver2Args& a, int grid, size_t lds, hipStream_t s) {
#define COCOA_LAUNCH2(M)                                                                             \
    do {                                                                                             \
        auto kern = solver2_kernel<M, STRICT>;                                                       \
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        kern<<<grid, kThreads2, lds, s>>>(a);                                                        \
    } while (0)
    if (mode == MODE_PLUS)
        COCOA_LAUNCH2(MODE_PLUS);
    else
        COCOA_LAUNCH2(MODE_MBCD);
#undef COCOA_LAUNCH2
}

// ---------------------------------------------------------------- step plan --
// For every step (k, s) of the round: the sampled row's entry offset, nnz,
// label, ||x||^2 and x.w (w is read-only within a round for CoCoA+ and MbCD).
// STRICT: one lane per step, x.w summed sequentially in stored order (the
// reference's SparseVector.dot); fast: 16 lanes per step, DPP row sum, FMA.
// One thread per step when no dot is formed here (strict, x.w reused from the
// eval, or CoCoA), 16 otherwise; plan_threads_per_step is the shared rule.
__host__ __device__ __forceinline__ int plan_threads_per_step(bool strict, const PlanArgs& a) {
    return (strict || !a.need_xw || a.xw_cache) ? 1 : 16;
}

template <bool STRICT>
__global__ __launch_bounds__(256) void plan_kernel(PlanArgs a) {
    const int tid = threadIdx.x;
    const int per = plan_threads_per_step(STRICT, a);
    const int64_t g = (int64_t)blockIdx.x * (256 / per) + tid / per;
    const int sub = tid % per;
    const bool valid = g < a.steps;
    const int64_t gg = valid ? g : 0;
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
        __builtin_nontemporal_store((int32_t)(e - b), a.z + g);
        __builtin_nontemporal_store(a.y[gr], a.py + g);
        __builtin_nontemporal_store(a.sqn[gr], a.pq + g);
        __builtin_nontemporal_store(xw, a.xw + g);
    }
}

template <bool STRICT>
void launch_plan_impl(const PlanArgs& a, hipStream_t s) {
    const int per = plan_threads_per_step(STRICT, a);
    const int64_t blocks = (a.steps * per + 255) / 256;
    if (blocks > 0) plan_kernel<STRICT><<<(unsigned)blocks, 256, 0, s>>>(a);
}

}  // namespace cocoa
