// Local-solver kernel template: one workgroup per partition, two waves.
//
//   wave 1 = loader: runs one batch ahead.  For up to 64 upcoming coordinate
//            steps it reads the sample indices, the rows' metadata and their
//            (col,val) entries from HBM into an LDS stream buffer, and -- when
//            w is read-only during the round (CoCoA+, MbCD) -- also the dot
//            x_i.w in stored-entry order.
//   wave 0 = solver: the strictly sequential chain of H coordinate steps of
//            CoCoA.localSDCA (CoCoA.scala:148-188) / MinibatchCD
//            (MinibatchCD.scala:95-125), reading its rows from LDS.  The only
//            memory it waits on per step is the gather of the mutable vector
//            (deltaW for CoCoA+, the task's w copy for CoCoA), which lives in
//            LDS when d fits, else in a private HBM/L2 slice.
//
// Double-buffered batches, one workgroup barrier per batch.  STRICT selects
// the bit-exact arithmetic (sequential dot sums in stored order by lane 0, no
// FMA: this header is compiled with -ffp-contract=off in kernels_strict.hip);
// otherwise wave-tree (DPP) sums and fused multiply-adds.
#pragma once
#include "kernels.h"
#include "wave.h"

namespace cocoa {

constexpr int kLoadUnroll = 32;  // 64-entry units each loader iteration keeps in flight (a whole 2,048-entry batch)

__device__ __forceinline__ int find_step(int32_t p, int32_t excl, int m) {
    // largest j < m with excl_j <= p (excl held by lane j); all lanes active
    int lo = 0;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
        const int c = lo + st;
        const int32_t e = __shfl(excl, c < 64 ? c : 63, 64);
        if (c < m && e <= p) lo = c;
    }
    return lo;
}

// The loader streams every sampled row's (col, val) once per round (614 MB on
// C2).  Nontemporal loads keep that stream from evicting the partitions'
// private deltaW slices, which the step chain gathers from L2.
#ifndef COCOA_LOADER_NT
#define COCOA_LOADER_NT 1
#endif
template <class T>
__device__ __forceinline__ T stream_ld(const T* p) {
    if (COCOA_LOADER_NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <int MODE, bool STRICT>
__device__ void load_batch(const SolverArgs& a, int k, int64_t p0, int32_t& cursor, BatchMeta* mb, int32_t* scol,
                           double* sval, double* prod) {
    const int lane = lane_id();
    const int32_t H = a.H;
    const int32_t C = a.stream_cap;
    if (cursor >= H) {
        if (lane == 0) mb->m = 0;
        return;
    }
    const int32_t s = cursor + lane;
    const bool valid = s < H;
    int32_t idx = 0;
    int64_t beg = 0, z = 0;
    double yv = 0.0, qv = 0.0;
    int32_t fl = 0;
    double pxw = 0.0, ppq = 0.0;
    const bool planned = a.plan_beg != nullptr;
    if (valid) {
        const size_t g = (size_t)k * H + s;
        idx = stream_ld(a.samples + g);
        const int64_t gr = p0 + idx;
        if (planned) {
            beg = stream_ld(a.plan_beg + g);
            z = stream_ld(a.plan_z + g);
            yv = stream_ld(a.plan_y + g);
            qv = stream_ld(a.plan_q + g);
            if (MODE != MODE_COCOA) pxw = stream_ld(a.plan_xw + g);
            if (MODE == MODE_PLUS && !STRICT && a.row_qp) {
                // private columns: the row's dot with them is pq (alpha - alpha^0),
                // alpha^0 folded into x.w here (off the chain)
                const double qp = a.row_qp[gr];
                if (qp != 0.0) {
                    ppq = (yv * qp) * (1.0 / a.lam_n);
                    pxw -= (a.sigma * ppq) * a.alpha[gr];
                }
            }
        } else {
            beg = a.row_ptr[gr];
            z = a.row_ptr[gr + 1] - beg;
            yv = a.y[gr];
            qv = a.sqn[gr];
        }
        if (a.any_dup) fl = a.rowflags[gr];
    }
    const bool staged = z <= C;
    const int32_t zz = (valid && staged) ? (int32_t)z : 0;
    const int32_t incl = wave_incl_scan(zz);
    const bool fits = valid && incl <= C;
    const uint64_t mask = __ballot(fits);
    const int m = (~mask == 0ULL) ? 64 : __builtin_ctzll(~mask);  // >= 1: step `cursor` always fits
    const int32_t excl = incl - zz;
    if (lane < m) {
        mb->r[lane] = idx;
        mb->off[lane] = staged ? excl : -1;
        mb->z[lane] = (int32_t)z;
        mb->flags[lane] = fl;
        mb->beg[lane] = beg;
        mb->y[lane] = yv;
        mb->q[lane] = qv;
        if (!STRICT) {
            const double qii = MODE == MODE_PLUS ? qv * a.sigma : qv;
            mb->rq[lane] = qii != 0.0 ? 1.0 / qii : 0.0;
            mb->pq[lane] = ppq;
        }
    }
    const int32_t T = __shfl(incl, m - 1, 64);
    // Owner step of every staged position: step j marks the start of its row
    // (scol[excl_j] = j), and a DPP prefix-max over each 64-position unit (plus
    // the previous unit's last owner) spreads the marks; the marks are then
    // overwritten by the entries.  No per-position search.
    for (int32_t q = lane; q < T; q += 64) scol[q] = -1;
    wave_lds_sync();
    if (lane < m && zz > 0) scol[excl] = lane;
    wave_lds_sync();
    int32_t carry = 0;
    // stream the batch's entries: 64 consecutive packed positions per unit
    for (int32_t base = 0; base < T; base += 64 * kLoadUnroll) {
        int32_t pc[kLoadUnroll];
        double pv[kLoadUnroll], pw[kLoadUnroll];
        int32_t own[kLoadUnroll];
#pragma unroll
        for (int u = 0; u < kLoadUnroll; ++u) {
            const int32_t p = base + 64 * u + lane;
            own[u] = p < T ? scol[p] : -1;
        }
#pragma unroll
        for (int u = 0; u < kLoadUnroll; ++u) {
            if (base + 64 * u < T) {
                own[u] = wave_incl_max(max(own[u], carry));
                carry = __builtin_amdgcn_readlane(own[u], 63);
            }
        }
#pragma unroll
        for (int u = 0; u < kLoadUnroll; ++u) {
            const int32_t p = base + 64 * u + lane;
            pc[u] = 0;
            pv[u] = 0.0;
            if (p < T) {
                const int j = own[u];
                const int64_t e = mb->beg[j] + (p - mb->off[j]);
                pc[u] = stream_ld(a.col + e);
                pv[u] = stream_ld(a.val + e);
            }
        }
        if (MODE != MODE_COCOA && !planned) {
#pragma unroll
            for (int u = 0; u < kLoadUnroll; ++u) {
                const int32_t p = base + 64 * u + lane;
                pw[u] = p < T ? a.w[pc[u]] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < kLoadUnroll; ++u) {
            const int32_t p = base + 64 * u + lane;
            if (p < T) {
                scol[p] = pc[u];
                sval[p] = pv[u];
                if (MODE != MODE_COCOA && !planned) prod[p] = pv[u] * pw[u];
            }
        }
    }
    if (MODE != MODE_COCOA && planned) {
        if (lane < m) mb->xw[lane] = pxw;
    } else if (MODE != MODE_COCOA) {
        wave_lds_sync();
        // x.w for each step, one lane per step, summed in stored-entry order
        double xw = 0.0;
        if (STRICT) {
            if (lane < m) {
                if (staged) {
                    for (int32_t q = 0; q < (int32_t)z; ++q) xw += prod[excl + q];
                } else {
                    for (int64_t q = 0; q < z; ++q) xw += a.val[beg + q] * a.w[a.col[beg + q]];
                }
            }
        } else {
            // fast: short staged rows one lane per step; long or unstaged rows
            // (dense data: 2,000 entries) by the whole wave, tree-summed
            const bool wide = !staged || z > 64;
            if (lane < m && !wide)
                for (int32_t q = 0; q < (int32_t)z; ++q) xw += prod[excl + q];
            uint64_t lm = __ballot(lane < m && wide);
            while (lm) {
                const int j = __builtin_ctzll(lm);
                lm &= lm - 1;
                const int64_t zj = __shfl(z, j, 64), bj = __shfl(beg, j, 64);
                const int32_t ej = __shfl(excl, j, 64);
                const bool sj = __shfl((int32_t)staged, j, 64) != 0;
                double acc = 0.0;
                if (sj)
                    for (int32_t q = lane; q < (int32_t)zj; q += 64) acc += prod[ej + q];
                else
                    for (int64_t q = lane; q < zj; q += 64) acc = fma(a.val[bj + q], a.w[a.col[bj + q]], acc);
                const double t = wave_sum(acc);
                if (lane == j) xw = t;
            }
        }
        if (lane < m) mb->xw[lane] = xw;
    }
    if (lane == 0) mb->m = m;
    cursor += m;
}

// Sequential (strict) or tree (fast) sum of the products held in registers.
template <bool STRICT>
__device__ __forceinline__ double dot_regs(const double (&prod)[kRegChunks], int32_t z, double* scratch) {
    const int lane = lane_id();
    if (STRICT) {
#pragma unroll
        for (int u = 0; u < kRegChunks; ++u)
            if (lane + 64 * u < z) scratch[lane + 64 * u] = prod[u];
        wave_lds_sync();
        double t = 0.0;
        if (lane == 0)
            for (int32_t q = 0; q < z; ++q) t += scratch[q];
        t = uni(t);
        wave_lds_sync();
        return t;
    } else {
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < kRegChunks; ++u) acc += prod[u];
        return wave_sum(acc);
    }
}

#ifdef COCOA_STEP_PROF
// diagnostic build only: per-step phase stamps (shares, not absolute times)
#define STEP_STAMP(i)                \
    do {                             \
        const uint64_t c_ = clock64(); \
        sp[i] += c_ - last_;         \
        last_ = c_;                  \
    } while (0)
#define STEP_KEEP(x) asm volatile("" ::"v"(x))
#else
#define STEP_STAMP(i) \
    do {              \
    } while (0)
#define STEP_KEEP(x) \
    do {             \
    } while (0)
#endif

template <int MODE, bool STRICT, bool VEC_LDS, bool ALPHA_LDS>
__device__ void compute_batch(const SolverArgs& a, const BatchMeta* mb, const int32_t* scol, const double* sval,
                              double* scratch, double* vec, double* dwk, double* alv, uint64_t (&sp)[6]) {
    const int lane = lane_id();
    const int m = uni(mb->m);
    const double lam_n = a.lam_n;
    const double inv_lam_n = 1.0 / a.lam_n;
    const double sigma = a.sigma;
#ifdef COCOA_STEP_PROF
    uint64_t last_ = clock64();
#endif
    (void)sp;
    for (int s = 0; s < m; ++s) {
        const int32_t r = uni(mb->r[s]);
        const int32_t off = uni(mb->off[s]);
        const int32_t z = uni(mb->z[s]);
        const int32_t fl = uni(mb->flags[s]);
        const double yv = uni(mb->y[s]);
        const double qv = uni(mb->q[s]);
        const double xw = MODE != MODE_COCOA ? uni(mb->xw[s]) : 0.0;
        const double aa = uni(alv[r]);  // after the previous step's write (in order)
        STEP_STAMP(0);

        const bool fast_path = off >= 0 && z <= 64 * kRegChunks && (fl & 1) == 0;
        int32_t pc[kRegChunks];
        double pv[kRegChunks], pd[kRegChunks];
        double sdot = 0.0;
        if (fast_path) {
#pragma unroll
            for (int u = 0; u < kRegChunks; ++u) {
                const int32_t p = lane + 64 * u;
                pc[u] = 0;
                pv[u] = 0.0;
                pd[u] = 0.0;
                if (p < z) {
                    pc[u] = scol[off + p];
                    pv[u] = sval[off + p];
                    if (MODE != MODE_MBCD) pd[u] = vec[pc[u]];
                }
            }
            if (MODE != MODE_MBCD) {
#pragma unroll
                for (int u = 0; u < kRegChunks; ++u) STEP_KEEP(pd[u]);
                STEP_STAMP(1);
                double prod[kRegChunks];
#pragma unroll
                for (int u = 0; u < kRegChunks; ++u) prod[u] = pv[u] * pd[u];
                sdot = dot_regs<STRICT>(prod, z, scratch);
                STEP_STAMP(2);
            }
        } else if (MODE != MODE_MBCD) {
            // generic path: long / unstaged / duplicate-column rows
            const int32_t* sc = off >= 0 ? scol + off : a.col + uni(mb->beg[s]);
            const double* sv = off >= 0 ? sval + off : a.val + uni(mb->beg[s]);
            if (STRICT) {
                double t = 0.0;
                for (int32_t c0 = 0; c0 < z; c0 += 64) {
                    const int32_t p = c0 + lane;
                    if (p < z) scratch[lane] = sv[p] * vec[sc[p]];
                    wave_lds_sync();
                    const int32_t cnt = z - c0 < 64 ? z - c0 : 64;
                    if (lane == 0)
                        for (int32_t q = 0; q < cnt; ++q) t += scratch[q];
                    wave_lds_sync();
                }
                sdot = uni(t);
            } else {
                double acc = 0.0;
                for (int32_t p = lane; p < z; p += 64) acc += sv[p] * vec[sc[p]];
                sdot = wave_sum(acc);
            }
        }

        double grad;
        if (MODE == MODE_PLUS)
            grad = (yv * (xw + (sigma * sdot)) - 1.0) * lam_n;   // CoCoA.scala:159
        else if (MODE == MODE_COCOA)
            grad = (yv * (sdot) - 1.0) * lam_n;                  // CoCoA.scala:161
        else
            grad = (yv * (xw) - 1.0) * lam_n;                    // MinibatchCD.scala:104
        double proj = grad;                                      // CoCoA.scala:166-170
        if (aa <= 0.0)
            proj = jmin(grad, 0.0);
        else if (aa >= 1.0)
            proj = jmax(grad, 0.0);
        if (fabs(proj) != 0.0) {                                 // CoCoA.scala:172
            const double qii = MODE == MODE_PLUS ? qv * sigma : qv;
            double na = 1.0;
            // fast mode multiplies by reciprocals staged off the chain (<= 1 ulp
            // per operation; strict keeps the reference's two divisions)
            if (qii != 0.0) na = jmin(jmax((aa - (STRICT ? grad / qii : grad * uni(mb->rq[s]))), 0.0), 1.0);
            const double coef = STRICT ? (yv * (na - aa)) / lam_n : (yv * (na - aa)) * inv_lam_n;  // CoCoA.scala:181
            STEP_KEEP(coef);
            STEP_STAMP(3);
            if (fast_path) {
#pragma unroll
                for (int u = 0; u < kRegChunks; ++u) {
                    if (lane + 64 * u < z) {
                        const double upd = pv[u] * coef;
                        if (MODE == MODE_PLUS) {
                            vec[pc[u]] = pd[u] + upd;                  // deltaW += update
                        } else if (MODE == MODE_COCOA) {
                            vec[pc[u]] = pd[u] + upd;                  // w += update
                            if (STRICT) dwk[pc[u]] = dwk[pc[u]] + upd; // deltaW += update
                            else unsafeAtomicAdd(dwk + pc[u], upd);
                        } else {
                            if (STRICT) vec[pc[u]] = vec[pc[u]] + upd;
                            else if (VEC_LDS) atomicAdd(vec + pc[u], upd);
                            else unsafeAtomicAdd(vec + pc[u], upd);
                        }
                    }
                }
            } else {
                const int32_t* sc = off >= 0 ? scol + off : a.col + uni(mb->beg[s]);
                const double* sv = off >= 0 ? sval + off : a.val + uni(mb->beg[s]);
                if (fl & 1) {
                    // duplicate column indices: the reference's sequential scatter
                    if (lane == 0) {
                        for (int32_t q = 0; q < z; ++q) {
                            const int32_t c = sc[q];
                            const double upd = sv[q] * coef;
                            vec[c] = vec[c] + upd;
                            if (MODE == MODE_COCOA) dwk[c] = dwk[c] + upd;
                        }
                    }
                } else {
                    for (int32_t p = lane; p < z; p += 64) {
                        const int32_t c = sc[p];
                        const double upd = sv[p] * coef;
                        vec[c] = vec[c] + upd;
                        if (MODE == MODE_COCOA) {
                            if (STRICT) dwk[c] = dwk[c] + upd;
                            else unsafeAtomicAdd(dwk + c, upd);
                        }
                    }
                }
            }
            if (lane == 0) alv[r] = na;                          // CoCoA.scala:186
        }
        STEP_STAMP(4);
    }
}

// ---------------------------------------------------------- chain v3 --
// Fast-mode CoCoA+ / MbCD step chain.  Same staged batches as v1, but the
// per-step work off the dependency chain is taken out of it:
//   * the next step's metadata and (col, val) chunks are read from the LDS
//     stream while the current step runs (they never change in a round);
//   * the only dependent access per step is the gather of deltaW at the row's
//     columns (LDS or the private HBM slice), issued for all chunks at once;
//   * the update rule is branch-free: reciprocals staged by the loader replace
//     the two divisions, fmin/fmax replace Java's Math.min/max (identical for
//     the finite values reachable here; +-0 and NaN differ only in the sign of
//     zero), and a skipped step (projected gradient 0) is coef = 0, na = aa.
// Agrees with the strict path within the north_star tolerance (fast mode).
template <int RC>
struct Chunks3 {
    int32_t c[RC];
    double v[RC];
};

struct Meta3 {
    int32_t r, off, z, fl;    // wave-uniform (SGPRs): control flow and addressing
    double y, q, rq, xw, aa, pq;  // broadcast LDS reads kept in VGPRs (no readfirstlane wait)
};

// Step metadata and alpha of the sampled row.  alpha is read before the
// current step writes its own row; compute_batch3 forwards the new value when
// the next step samples the same row.
__device__ __forceinline__ Meta3 read_meta3(const BatchMeta* mb, int s, const double* alv) {
    Meta3 m;
    m.r = uni(mb->r[s]);
    m.off = uni(mb->off[s]);
    m.z = uni(mb->z[s]);
    m.fl = uni(mb->flags[s]);
    m.y = mb->y[s];
    m.q = mb->q[s];
    m.rq = mb->rq[s];
    m.xw = mb->xw[s];
    m.pq = mb->pq[s];
    m.aa = alv[m.r];
    return m;
}

// (col, val) of a staged row, branch-free: lanes past z read the row's last
// entry (a valid column) with value 0.
template <int RC>
__device__ __forceinline__ void read_chunks3(const int32_t* scol, const double* sval, const Meta3& m, Chunks3<RC>& ch) {
    const int lane = lane_id();
    const bool ok = m.off >= 0 && m.z > 0;
    const int32_t last = ok ? m.off + m.z - 1 : 0;
#pragma unroll
    for (int u = 0; u < RC; ++u) {
        const int32_t p = lane + 64 * u;
        const int32_t q = min(m.off + p, last);
        ch.c[u] = scol[q];
        const double v = sval[q];
        ch.v[u] = (ok && p < m.z) ? v : 0.0;
    }
}

// RC: register chunks per row (rows with z <= 64 * RC take the register path);
// SolverArgs::reg_chunks picks 3 or 4 from the data's mean row length.
template <int MODE, bool VEC_LDS, int RC, bool HOT = false>
__device__ void compute_batch3(const SolverArgs& a, const BatchMeta* mb, const int32_t* scol, const double* sval,
                               double* vec, double* alv, double* hl = nullptr) {
    const int lane = lane_id();
    // HOT: slice positions below a.hot in LDS (hl); a hot lane's global load goes
    // to position 0 (one line for the wave, never written in HBM by this launch)
    const int32_t hot = HOT ? a.hot : 0;
    auto get = [&](int32_t c) -> double {
        if (!HOT) return vec[c];
        const bool h = c < hot;
        const double lv = hl[h ? c : 0];
        const double gv = vec[h ? 0 : c];
        return h ? lv : gv;
    };
    auto put = [&](int32_t c, double v) {
        if (HOT && c < hot)
            hl[c] = v;
        else
            vec[c] = v;
    };
    const int m = uni(mb->m);
    const double lam_n = a.lam_n;
    const double inv_lam_n = 1.0 / a.lam_n;
    const double sigma = a.sigma;
    Meta3 nm = read_meta3(mb, 0, alv);
    Chunks3<RC> nc;
    read_chunks3(scol, sval, nm, nc);
    // CoCoA.scala:159-186 / MinibatchCD.scala:104-123, branch-free
    auto rule = [&](const Meta3& st, double sdot, double& na, double& coef) -> bool {
        const double aa = st.aa;
        // (CoCoA+: the private columns' share of x.deltaW is pq aa, st.xw already
        // holds -sigma pq alpha^0; pq = 0 without private columns)
        const double grad = MODE == MODE_PLUS ? (st.y * (st.xw + sigma * fma(st.pq, aa, sdot)) - 1.0) * lam_n
                                              : (st.y * st.xw - 1.0) * lam_n;
        const double proj = aa <= 0.0 ? fmin(grad, 0.0) : (aa >= 1.0 ? fmax(grad, 0.0) : grad);
        const bool go = proj != 0.0;
        const double qii = MODE == MODE_PLUS ? st.q * sigma : st.q;
        const double nt = fmin(fmax(aa - grad * st.rq, 0.0), 1.0);
        na = go ? (qii != 0.0 ? nt : 1.0) : aa;
        coef = (st.y * (na - aa)) * inv_lam_n;
        return go;
    };
    auto next = [&](int s) {
        // the last step re-reads its own inputs (unused) instead of branching
        nm = read_meta3(mb, s + 1 < m ? s + 1 : s, alv);
        read_chunks3(scol, sval, nm, nc);
    };
    for (int s = 0; s < m; ++s) {
        const Meta3 st = nm;
        const Chunks3<RC> ch = nc;
        const int nch = (st.z + 63) >> 6;
        const bool regs = st.off >= 0 && nch <= RC && (st.fl & 1) == 0;
        double na, coef;
        if (MODE == MODE_PLUS && regs) {
            // CoCoA+ register path, one uniform branch per step: the dependent
            // gather goes out first (chunks past z hit the row's last column,
            // v = 0), then the next step's staged inputs
            double pd[RC];
#pragma unroll
            for (int u = 0; u < RC; ++u) pd[u] = get(ch.c[u]);
            next(s);
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < RC; ++u) acc = fma(ch.v[u], pd[u], acc);
            const bool go = rule(st, wave_sum(acc), na, coef);
            if (s + 1 < m && nm.r == st.r) nm.aa = na;           // same row sampled twice in a row
            if (uni((int32_t)go)) {
#pragma unroll
                for (int u = 0; u < RC; ++u)
                    if (u < nch && lane + 64 * u < st.z) put(ch.c[u], fma(ch.v[u], coef, pd[u]));  // deltaW += update
                if (lane == 0) alv[st.r] = na;                   // CoCoA.scala:186
            }
            continue;
        }
        next(s);
        double sdot = 0.0;
        if (MODE == MODE_PLUS) {
            // long row: 4 x 64 entries per pass, all gathers of a pass in flight
            const int32_t* sc = st.off >= 0 ? scol + st.off : a.col + uni(mb->beg[s]);
            const double* sv = st.off >= 0 ? sval + st.off : a.val + uni(mb->beg[s]);
            double acc = 0.0;
            for (int32_t p0 = 0; p0 < st.z; p0 += 256) {
                int32_t c4[4];
                double v4[4], g4[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int32_t p = p0 + lane + 64 * u;
                    c4[u] = p < st.z ? sc[p] : 0;
                    v4[u] = p < st.z ? sv[p] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) g4[u] = get(c4[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u) acc = fma(v4[u], g4[u], acc);
            }
            sdot = wave_sum(acc);
        }
        const bool go = rule(st, sdot, na, coef);
        if (s + 1 < m && nm.r == st.r) nm.aa = na;               // same row sampled twice in a row
        if (uni((int32_t)go)) {
            if (regs) {
                // MbCD register path: atomic adds into deltaW
#pragma unroll
                for (int u = 0; u < RC; ++u) {
                    if (u < nch && lane + 64 * u < st.z) {
                        if (VEC_LDS)
                            atomicAdd(vec + ch.c[u], ch.v[u] * coef);
                        else
                            unsafeAtomicAdd(vec + ch.c[u], ch.v[u] * coef);
                    }
                }
            } else {
                const int32_t* sc = st.off >= 0 ? scol + st.off : a.col + uni(mb->beg[s]);
                const double* sv = st.off >= 0 ? sval + st.off : a.val + uni(mb->beg[s]);
                if (st.fl & 1) {
                    if (lane == 0)
                        for (int32_t q = 0; q < st.z; ++q) put(sc[q], get(sc[q]) + sv[q] * coef);
                } else {
                    // distinct columns: a pass's reads all go out before its writes
                    for (int32_t p0 = 0; p0 < st.z; p0 += 256) {
                        int32_t c4[4];
                        double v4[4], g4[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int32_t p = p0 + lane + 64 * u;
                            c4[u] = p < st.z ? sc[p] : -1;
                            v4[u] = p < st.z ? sv[p] : 0.0;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) g4[u] = c4[u] >= 0 ? get(c4[u]) : 0.0;
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (c4[u] >= 0) put(c4[u], fma(v4[u], coef, g4[u]));
                    }
                }
            }
            if (lane == 0) alv[st.r] = na;                       // CoCoA.scala:186
        }
    }
}

// RC: chain v3 register chunks, a separate instantiation per count (one kernel
// holding both paths measured slower: its register allocation covers both).
template <int MODE, bool STRICT, bool VEC_LDS, bool ALPHA_LDS, int RC = kRegChunks, bool HOT = false>
__global__ __launch_bounds__(128, 1) void solver_kernel(SolverArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int k = blockIdx.x;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int64_t p0 = a.part_ptr[k], p1 = a.part_ptr[k + 1];
    const int32_t nl = (int32_t)(p1 - p0);
    const int64_t d = a.d;
    double* dwk = a.dw + (size_t)k * d;
    double* vec;
    if (VEC_LDS)
        vec = (double*)(lds + a.lds_vec);
    else
        vec = MODE == MODE_COCOA ? a.wloc + (size_t)k * d : dwk;
    double* alv = ALPHA_LDS ? (double*)(lds + a.lds_alpha) : a.alpha_work + p0;
    double* scratch = (double*)(lds + a.lds_scratch);
    double* prod = (double*)(lds + a.lds_prod);
    double* hl = HOT ? (double*)(lds + a.lds_hot) : nullptr;
    if (HOT)
        for (int32_t j = tid; j < a.hot; j += 128) hl[j] = 0.0;  // (the slice is zero on entry)

    // prologue: alphaOld stays in a.alpha; the working copy is alv
    for (int32_t i = tid; i < nl; i += 128) alv[i] = a.alpha[p0 + i];
    if (VEC_LDS) {
        for (int64_t j = tid; j < d; j += 128) vec[j] = MODE == MODE_COCOA ? a.w[j] : 0.0;
    } else if (MODE == MODE_COCOA) {
        for (int64_t j = tid; j < d; j += 128) vec[j] = a.w[j];  // the task's private copy of w
    }
    int32_t cursor = 0;
    if (wave == 1)
        load_batch<MODE, STRICT>(a, k, p0, cursor, (BatchMeta*)(lds + a.lds_meta[0]), (int32_t*)(lds + a.lds_stream_col[0]),
                                 (double*)(lds + a.lds_stream_val[0]), prod);
    __syncthreads();
    uint64_t t_busy = 0, t_wait = 0, n_batch = 0;
    uint64_t step_prof[6] = {0, 0, 0, 0, 0, 0};
    for (int b = 0;; ++b) {
        const int cur = b & 1;
        const BatchMeta* mb = (const BatchMeta*)(lds + a.lds_meta[cur]);
        if (mb->m == 0) break;
        const uint64_t c0 = a.prof ? clock64() : 0;
        if (wave == 1) {
            load_batch<MODE, STRICT>(a, k, p0, cursor, (BatchMeta*)(lds + a.lds_meta[cur ^ 1]),
                                     (int32_t*)(lds + a.lds_stream_col[cur ^ 1]), (double*)(lds + a.lds_stream_val[cur ^ 1]),
                                     prod);
        } else if (!STRICT && MODE != MODE_COCOA) {
            compute_batch3<MODE, VEC_LDS, RC, HOT>(a, mb, (const int32_t*)(lds + a.lds_stream_col[cur]),
                                                   (const double*)(lds + a.lds_stream_val[cur]), vec, alv, hl);
        } else {
            compute_batch<MODE, STRICT, VEC_LDS, ALPHA_LDS>(a, mb, (const int32_t*)(lds + a.lds_stream_col[cur]),
                                                            (const double*)(lds + a.lds_stream_val[cur]), scratch, vec,
                                                            dwk, alv, step_prof);
        }
        const uint64_t c1 = a.prof ? clock64() : 0;
        __syncthreads();
        if (a.prof) {
            t_busy += c1 - c0;
            t_wait += clock64() - c1;
            n_batch += 1;
        }
    }
    if (a.prof && (tid & 63) == 0) {
        // [block][wave][busy, wait, batches, step stamps x6]  (16 per wave)
        uint64_t* pr = a.prof + ((size_t)k * 2 + wave) * 16;
        pr[0] = t_busy;
        pr[1] = t_wait;
        pr[2] = n_batch;
        for (int i = 0; i < 6; ++i) pr[3 + i] = step_prof[i];
    }
    // epilogue: alpha = alphaOld + (alpha - alphaOld) * scaling (CoCoA.scala:101,
    // MinibatchCD.scala:127-128)
    if (a.raw_alpha) {
        for (int32_t i = tid; i < nl; i += 128) a.alpha[p0 + i] = alv[i];
        if (VEC_LDS && MODE == MODE_COCOA)
            for (int64_t j = tid; j < d; j += 128) a.wloc[(size_t)k * d + j] = vec[j];
    } else {
        for (int32_t i = tid; i < nl; i += 128) {
            const double old = a.alpha[p0 + i];
            // private columns: the row's deltaW per unit of x, y_r (alpha_r - alpha_r^0) /
            // (lambda n) -- the sum of its updates (CoCoA.scala:181-184) -- for the tail
            if (!STRICT && MODE == MODE_PLUS && a.rowcoef)
                a.rowcoef[p0 + i] = (a.y[p0 + i] * (alv[i] - old)) * (1.0 / a.lam_n);
            a.alpha[p0 + i] = old + ((alv[i] - old) * a.scaling);
        }
    }
    if (VEC_LDS && MODE != MODE_COCOA)
        for (int64_t j = tid; j < d; j += 128) dwk[j] = vec[j];
    if (HOT)
        for (int32_t j = tid; j < a.hot; j += 128) dwk[j] = hl[j];
}

template <bool STRICT>
void launch_solver_impl(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                        hipStream_t s) {
#define COCOA_LAUNCH(M, V, A)                                                                        \
    do {                                                                                             \
        constexpr int RCS = short_row_chunks(M, STRICT);                                           \
        auto kern = a.reg_chunks == RCS ? solver_kernel<M, STRICT, V, A, RCS> : solver_kernel<M, STRICT, V, A>; \
        if constexpr (M == MODE_PLUS && !STRICT && !V)                                               \
            if (a.hot > 0) kern = a.reg_chunks == RCS ? solver_kernel<M, STRICT, V, A, RCS, true>       \
                                                      : solver_kernel<M, STRICT, V, A, kRegChunks, true>; \
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        kern<<<grid, 128, lds, s>>>(a);                                                              \
    } while (0)
#define COCOA_LAUNCH_M(M)                           \
    do {                                            \
        if (vec_lds && alpha_lds) COCOA_LAUNCH(M, true, true);   \
        else if (vec_lds) COCOA_LAUNCH(M, true, false);          \
        else if (alpha_lds) COCOA_LAUNCH(M, false, true);        \
        else COCOA_LAUNCH(M, false, false);                      \
    } while (0)
    if (mode == MODE_PLUS)
        COCOA_LAUNCH_M(MODE_PLUS);
    else if (mode == MODE_COCOA)
        COCOA_LAUNCH_M(MODE_COCOA);
    else
        COCOA_LAUNCH_M(MODE_MBCD);
#undef COCOA_LAUNCH_M
#undef COCOA_LAUNCH
}

}  // namespace cocoa
