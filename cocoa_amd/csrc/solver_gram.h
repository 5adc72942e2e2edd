// Fast-mode local SDCA with a Gram window (CoCoA+, CoCoA, MbCD).
//
// CoCoA.localSDCA (CoCoA.scala:148-188) is a chain of H dependent coordinate
// steps per partition; step s needs x_s . deltaW with every earlier step's
// update in it.  The r01 solver formed that dot directly, so each step paid a
// dependent gather, a 64-lane reduction and the update rule (~1,600 cycles).
// Here the dot is split:
//
//   x_s . deltaW_s = base_s + sum_{j in window, j < s} c_j * G(s, j)
//
//   base_s  = x_s . deltaW as of a batch boundary four batches back, gathered
//             off the chain by a helper wave;
//   G(s, j) = x_s . x_j, the Gram entries of nearby steps, computed before the
//             round by gram_kernel (the sampled rows are known in advance:
//             java.util.Random does not depend on the data);
//   c_j     = y_j (alpha_new - alpha_old) / (lambda n), the scatter
//             coefficient of step j (CoCoA.scala:181).
//
// The chain wave keeps one accumulator per lane: lane l holds the pending
// correction of the step in window slot l (slot = step mod 64, four batches
// of 16).  Step j reads its own accumulator (v_readlane), applies the update
// rule, and adds c_j * G(., j) to every pending lane -- one FMA, no memory
// access and no reduction on the dependent path.
//
// Roles (one 256-thread workgroup per partition, one wave each):
//   wave 0  chain  -- the H sequential steps (update rule, alpha in LDS);
//   wave 1  memory -- per batch b: deltaW += c_j x_j for the steps of batch b
//                     (fp64 atomics into the partition's private slice), then
//                     the gathers of x_s . deltaW for batch b+4, software-
//                     pipelined one batch deep (issued now, summed next time);
//   wave 2  loader -- per-step records (constants of the update rule, the
//                     next occurrence of the same row in the window).
// The waves hand off through counters in LDS (release / acquire, s_sleep
// while waiting), not workgroup barriers, so the chain never waits on a
// helper that is merely busy with a later batch.
//
// Ordering of the deltaW slice: base(b) must contain exactly the updates of
// batches <= b-4.  The memory wave issues, in this order, the atomics of
// batch b-4 and then the gathers of base(b), and the atomics of batch b-3
// only after those gathers: one wave, one address stream, so the gathers see
// batch b-4 and nothing later.  Batches b-3 .. b reach the steps of batch b
// through the Gram corrections (window of 64 steps = 4 batches of 16).
//
// Numerics: fast mode (fused multiply-adds, reassociated dots, atomics); the
// results agree with the strict path / oracle within the north_star
// tolerance.  MbCD reads the stale w only (MinibatchCD.scala:104): no base,
// no Gram term, the chain is the update rule alone.
#pragma once
#include "kernels.h"
#include "wave.h"

namespace cocoa {

constexpr int kGB = 16;                  // steps per batch
constexpr int kGSlots = 64;              // window slots = lanes
constexpr int kGNB = kGSlots / kGB;      // batches in the window
constexpr int kGRing = 8;                // record / coefficient ring (batches)
constexpr int kGHot = 64;                // dense hot columns of gram_kernel (device order: most frequent first)
constexpr int kGMU = 24;                 // 64-entry units per batch the memory wave keeps in registers
constexpr int kGStage = kGMU * 64;       // staged gather values / products (one batch)

// ----------------------------------------------------------- LDS handoff --
__device__ __forceinline__ int lds_acquire(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Spin (s_sleep) until *p >= v.  Bounded: a wait that outlasts ~2^24 sleeps
// (far beyond any legitimate hand-off) raises the workgroup's abort flag and
// the kernel's status word, and every role then drains out of its loop, so a
// logic error ends the launch with an error instead of hanging the GPU.
__device__ __forceinline__ bool wait_ge(const int* p, int v, int* abort_flag, int* status, uint64_t* waited = nullptr) {
    if (lds_acquire(p) >= v) return true;
    const uint64_t t0 = waited ? __builtin_readcyclecounter() : 0;
    for (uint32_t it = 0;; ++it) {
        if (lds_acquire(p) >= v) {
            if (waited) *waited += __builtin_readcyclecounter() - t0;
            return true;
        }
        if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        if (it > (1u << 24)) {
            __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (status) __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// L1-bypassing read of the deltaW slice (the scatter wave's atomics land in L2)
__device__ __forceinline__ double dw_load(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// ================================================================ Gram ==
// Gt[k][j][slot] = x_{s} . x_j for the step s of window slot `slot` in j's
// window [16 floor(j/16), +64) with s > j; 0 otherwise.
// One workgroup per (partition, batch of 16 updaters): partners are the 64
// steps of the window.  Hot columns (device index < kGHot) go through a dense
// LDS image of the partners (lanes = partners, one LDS read per hot entry of
// the updater); the other columns through an LDS hash of the partners' cold
// entries (lanes = the updater's entries, a probe each).
constexpr int kGramTable = 8192;     // hash slots (power of two, >= 2 x kGramCap: probes stay short)
constexpr int kGramCap = 4096;       // packed partner positions per pass (their cold entries are inserted)

struct GramLds {
    double X[kGSlots][kGHot + 1];    // +1: partner rows start on different banks
    double acc[kGB][kGSlots];        // G of the block's updaters
    int32_t tkey[kGramTable];
    int32_t thead[kGramTable];
    double eval[kGramCap];
    int16_t enext[kGramCap];
    int8_t epart[kGramCap];
    int64_t pbeg[kGSlots];
    int32_t pz[kGSlots];
    int32_t pcum[kGSlots + 1];
};
static_assert(sizeof(GramLds) <= 160 * 1024, "gram_kernel LDS");

__device__ __forceinline__ uint32_t gram_hash(int32_t c) { return ((uint32_t)c * 2654435761u) >> 19; }  // 13 bits

constexpr int kGramGU = 8;    // 256-position units each thread keeps in flight while staging
constexpr int kGramUC = 2;    // register chunks (64 entries) per updater row; longer rows loop

__global__ __launch_bounds__(256, 1) void gram_kernel(GramArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramLds& L = *(GramLds*)lds_raw;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = blockIdx.x % a.K;
    const int g = blockIdx.x / a.K;
    const int32_t H = a.H;
    const int32_t j0 = g * kGB;
    const int32_t P = min(kGSlots, H - j0);     // partners [j0, j0 + P)
    const int32_t U = min(kGB, H - j0);          // updaters [j0, j0 + U) = partners [0, U)
    const int64_t p0 = a.part_ptr[k];
    const int32_t* smp = a.samples + (size_t)k * H;
    // partner rows
    if (tid < kGSlots) {
        int64_t b = 0;
        int32_t z = 0;
        if (tid < P) {
            const int64_t r = p0 + smp[j0 + tid];
            b = a.row_ptr[r];
            z = (int32_t)(a.row_ptr[r + 1] - b);
        }
        L.pbeg[tid] = b;
        L.pz[tid] = z;
    }
    for (int i = tid; i < kGSlots * (kGHot + 1); i += 256) (&L.X[0][0])[i] = 0.0;
    for (int i = tid; i < kGB * kGSlots; i += 256) (&L.acc[0][0])[i] = 0.0;
    __syncthreads();
    if (wv == 0) {
        const int32_t inc = wave_incl_scan(L.pz[lane]);
        L.pcum[lane + 1] = inc;
        if (lane == 0) L.pcum[0] = 0;
    }
    __syncthreads();
    const int32_t T = L.pcum[kGSlots];
    auto owner = [&](int32_t q) {  // partner whose entries hold packed position q: largest p, pcum[p] <= q
        int lo = 0;
#pragma unroll
        for (int st = kGSlots / 2; st >= 1; st >>= 1)
            if (L.pcum[lo + st] <= q) lo += st;
        return lo;
    };
    // this wave's updaters (u = wv + 4 i): first kGramUC chunks in registers,
    // loads issued now so they land while the partner structures are built
    constexpr int NU = kGB / 4;
    int32_t uc[NU][kGramUC];
    double uv[NU][kGramUC];
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        const int u = wv + 4 * i;
        const int64_t b = L.pbeg[u];
        const int32_t z = u < U ? L.pz[u] : 0;
#pragma unroll
        for (int c = 0; c < kGramUC; ++c) {
            const int32_t e = 64 * c + lane;
            uc[i][c] = e < z ? a.col[b + e] : -1;
            uv[i][c] = e < z ? a.val[b + e] : 0.0;
        }
    }
    // cold probe of one updater entry (col c >= kGHot, value v) against the table
    auto probe = [&](int u, int32_t c, double v) {
        uint32_t h = gram_hash(c) & (kGramTable - 1);
        for (;;) {
            const int32_t key = L.tkey[h];
            if (key == c) {
                for (int32_t i = L.thead[h]; i >= 0; i = L.enext[i]) {
                    const int p = L.epart[i];
                    if (p > u) atomicAdd(&L.acc[u][p], v * L.eval[i]);
                }
                return;
            }
            if (key == -1) return;
            h = (h + 1) & (kGramTable - 1);
        }
    };
    // passes of kGramCap packed partner positions: dense hot image of all
    // positions, hashed cold entries of the pass, cold probes of the updaters
    for (int32_t qa = 0; qa < T; qa += kGramCap) {
        if (qa > 0) __syncthreads();  // the previous pass's probes are done with the table
        for (int i = tid; i < kGramTable; i += 256) {
            L.tkey[i] = -1;
            L.thead[i] = -1;
        }
        __syncthreads();
        const int32_t qb = min(T, qa + kGramCap);
        for (int32_t q0 = qa; q0 < qb; q0 += 256 * kGramGU) {
            int32_t cc[kGramGU];
            double vv[kGramGU];
            int pp[kGramGU];
#pragma unroll
            for (int u = 0; u < kGramGU; ++u) {
                const int32_t q = q0 + 256 * u + tid;
                cc[u] = -1;
                vv[u] = 0.0;
                pp[u] = 0;
                if (q < qb) {
                    const int p = owner(q);
                    const int64_t e = L.pbeg[p] + (q - L.pcum[p]);
                    pp[u] = p;
                    cc[u] = a.col[e];
                    vv[u] = a.val[e];
                }
            }
#pragma unroll
            for (int u = 0; u < kGramGU; ++u) {
                const int32_t c = cc[u];
                if (c < 0) continue;
                if (c < kGHot) {  // duplicate columns of a row add up, as in the dot
                    atomicAdd(&L.X[pp[u]][c], vv[u]);
                    continue;
                }
                const int32_t i = q0 + 256 * u + tid - qa;
                L.epart[i] = (int8_t)pp[u];
                L.eval[i] = vv[u];
                uint32_t h = gram_hash(c) & (kGramTable - 1);
                for (;;) {
                    const int32_t old = atomicCAS(&L.tkey[h], -1, c);
                    if (old == -1 || old == c) break;
                    h = (h + 1) & (kGramTable - 1);
                }
                L.enext[i] = (int16_t)atomicExch(&L.thead[h], i);
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int u = wv + 4 * i;
            if (u >= U) continue;
#pragma unroll
            for (int c = 0; c < kGramUC; ++c)
                if (uc[i][c] >= kGHot) probe(u, uc[i][c], uv[i][c]);
            const int64_t b = L.pbeg[u];
            const int32_t z = L.pz[u];
            for (int32_t e = 64 * kGramUC + lane; e < z; e += 64) {  // rows past the register chunks
                const int32_t c = a.col[b + e];
                if (c >= kGHot) probe(u, c, a.val[b + e]);
            }
        }
    }
    __syncthreads();  // X complete, cold contributions in acc
    // hot part: lanes = partners, one LDS read per hot entry of the updater
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        const int u = wv + 4 * i;
        if (u >= U) continue;
        double acc = 0.0;
        auto hot = [&](int32_t c, double v) {
            uint64_t m = __ballot(c >= 0 && c < kGHot);
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1;
                const int32_t cc = __builtin_amdgcn_readlane(c, src);
                acc = fma(readlane_d(v, src), L.X[lane][cc], acc);
            }
        };
#pragma unroll
        for (int c = 0; c < kGramUC; ++c) hot(uc[i][c], uv[i][c]);
        const int64_t b = L.pbeg[u];
        const int32_t z = L.pz[u];
        for (int32_t e0 = 64 * kGramUC; e0 < z; e0 += 64) {
            const int32_t e = e0 + lane;
            hot(e < z ? a.col[b + e] : -1, e < z ? a.val[b + e] : 0.0);
        }
        L.acc[u][lane] += acc;  // this wave owns row u; its cold atomics are done (barrier above)
    }
    // Gt rows of the block's updaters: slot of partner p = (j0 + p) & 63
    double* out = a.gt + ((size_t)k * a.nbatch * kGB + j0) * kGSlots;
    for (int u = wv; u < kGB; u += 4) {
        const double v = (u < U && lane > u && lane < P) ? L.acc[u][lane] : 0.0;
        __builtin_nontemporal_store(v, out + (size_t)u * kGSlots + ((j0 + lane) & (kGSlots - 1)));
    }
}

// ============================================================== solver ==
// Per-step constants.  With sdot = x.deltaW (base + Gram corrections) the
// update rule of CoCoA.scala:159-186 is
//     grad = A sdot + Kx            A = y sigma' lambda n (CoCoA: y lambda n)
//     nt   = clamp(aa - grad / qii, 0, 1)
//          = clamp(AE - B sdot)     B = A / qii, E = Kx / qii, AE = aa - E
//     c    = y (nt - aa) / (lambda n) = Y nt - YA,   YA = Y aa
// and nt is the new alpha whether or not the projected gradient vanishes:
// with aa = 0 and grad >= 0, or aa = 1 and grad <= 0, the clamp returns aa.
// An empty row (qii = 0) always gets alpha = 1 (grad = -lambda n < 0):
// B = 0, E = -1.  MbCD (MinibatchCD.scala:104): A = 0, so B = 0.
struct GRec {                          // one step (64 B)
    double B, Y, AE, YA;               // AE, YA: set by the chain when the step's slot is filled
    double E;
    int32_t r;                         // sampled row (partition-local); padding steps: the alpha sink
    int32_t fw;                        // slot of the next step of the window with the same row, -1
    int32_t pad[4];
};

struct GramSolverLds {
    int cnt[8];                        // 0 chain_done, 1 scat_done, 2 base_done, 3 load_done, 4 abort
    GRec rec[kGRing * kGB];            // ring: (b % kGRing) * kGB + i
    double coef[kGRing * kGB];         // c_j, same ring (chain -> memory wave)
    double base[kGSlots];              // base_s per slot
    int32_t smpwin[kGSlots];           // loader: sampled rows of its window
    int32_t pdw[kGB];                  // loader: previous occurrence (window position) of its steps
    double stage[2][kGStage];          // memory wave: staged gather values, then products (by parity)
    int32_t mx[3][kGB + 1];            // memory wave: packed row offsets (0 scatter, 1 issue, 2 process)
    int64_t mb[3][kGB];                //   and row starts
    int32_t mu[3][kGMU];               //   units (row | chunk << 8), first kGMU of each batch
    int32_t mp[3][kGB + 1];            //   units before row i
};

template <int MODE>
__device__ __forceinline__ void gram_row_consts(const GramSolverArgs& a, double y, double q, double xw, double& B,
                                                double& E, double& Y) {
    const double A = MODE == MODE_PLUS ? y * a.sigma * a.lam_n : (MODE == MODE_COCOA ? y * a.lam_n : 0.0);
    const double Kx = (y * xw - 1.0) * a.lam_n;
    const double qii = MODE == MODE_PLUS ? q * a.sigma : q;
    if (qii != 0.0) {
        const double rq = 1.0 / qii;
        B = A * rq;
        E = Kx * rq;
    } else {
        B = 0.0;
        E = -1.0;
    }
    Y = y * a.inv_lam_n;
}

// packed position q of a batch's rows -> row: largest i with excl[i] <= q
__device__ __forceinline__ int gram_owner(const int32_t* excl, int32_t q) {
    int lo = 0;
#pragma unroll
    for (int st = kGB / 2; st >= 1; st >>= 1)
        if (excl[lo + st] <= q) lo += st;
    return lo;
}

// Layout of batch b's rows for the memory wave: packed offsets sx (row i at
// [sx[i], sx[i+1])), row starts sb, and the 64-entry units (row, chunk) of
// the first kGMU chunks (lanes of a unit = consecutive entries of one row, so
// a unit's address is a row start plus the lane).  Returns the entry count;
// up[i] = units before row i (up[kGB] = all units, may exceed kGMU).
__device__ __forceinline__ int32_t gram_pack(const GramSolverArgs& a, size_t g0, int32_t b, int32_t* sx, int64_t* sb,
                                             int32_t* units, int32_t* up) {
    const int lane = lane_id();
    const int32_t j = b * kGB + lane;
    int64_t beg = 0;
    int32_t z = 0;
    if (lane < kGB && j < a.H) {
        beg = a.plan_beg[g0 + j];
        z = a.plan_z[g0 + j];
    }
    const int32_t inc = wave_incl_scan(lane < kGB ? z : 0);
    const int32_t nc = lane < kGB ? (z + 63) >> 6 : 0;
    const int32_t uinc = wave_incl_scan(nc);
    if (lane < kGB) {
        sx[lane + 1] = inc;
        sb[lane] = beg;
        up[lane + 1] = uinc;
        for (int32_t c = 0, u = uinc - nc; c < nc && u < kGMU; ++c, ++u) units[u] = lane | (c << 8);
    }
    if (lane == 0) {
        sx[0] = 0;
        up[0] = 0;
    }
    wave_lds_sync();
    return __shfl(inc, kGB - 1, 64);
}

// scatter side: the first min(nunits, NU) units into registers
template <int NU>
__device__ __forceinline__ void gram_fetch(const GramSolverArgs& a, const int32_t* sx, const int64_t* sb,
                                           const int32_t* units, int32_t nunits, int32_t (&cc)[NU],
                                           double (&vv)[NU]) {
    const int lane = lane_id();
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        cc[u] = -1;
        vv[u] = 0.0;
        if (u < nunits) {
            const int32_t ut = units[u];
            const int i = ut & 0xFF;
            const int32_t e = ((ut >> 8) << 6) + lane;
            if (e < sx[i + 1] - sx[i]) {
                cc[u] = a.col[sb[i] + e];
                vv[u] = a.val[sb[i] + e];
            }
        }
    }
}

// gather side: columns in registers, values straight into the stage buffer
template <int NU>
__device__ __forceinline__ void gram_fetch_g(const GramSolverArgs& a, const int32_t* sx, const int64_t* sb,
                                             const int32_t* units, int32_t nunits, int32_t (&cc)[NU],
                                             double* stage) {
    const int lane = lane_id();
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        cc[u] = -1;
        if (u < nunits) {
            const int32_t ut = units[u];
            const int i = ut & 0xFF;
            const int32_t e = ((ut >> 8) << 6) + lane;
            if (e < sx[i + 1] - sx[i]) {
                cc[u] = a.col[sb[i] + e];
                stage[sx[i] + e] = a.val[sb[i] + e];
            }
        }
    }
}

// row sums of staged products [0, T) laid out by (sx): lanes < kGB take the
// rows of <= 64 entries in stored order, the whole wave the longer ones
__device__ __forceinline__ void gram_row_sums(const int32_t* sx, const double* stage, int32_t T, double* out) {
    const int lane = lane_id();
    const int32_t rb = lane < kGB ? sx[lane] : 0, re = lane < kGB ? sx[lane + 1] : 0;
    double sum = 0.0;
    if (lane < kGB && re - rb <= 64)
        for (int32_t q = rb; q < re; ++q) sum += stage[q];
    uint64_t lm = __ballot(lane < kGB && re - rb > 64);
    while (lm) {
        const int i = __builtin_ctzll(lm);
        lm &= lm - 1;
        const int32_t b0 = sx[i], b1 = sx[i + 1];
        double acc = 0.0;
        for (int32_t q = b0 + lane; q < b1; q += 64) acc += stage[q];
        const double t = wave_sum(acc);
        if (lane == i) sum = t;
    }
    if (lane < kGB) out[lane] = sum;
    (void)T;
}

template <int MODE, bool ALV_LDS>
__global__ __launch_bounds__(256, 1) void solver_gram_kernel(GramSolverArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramSolverLds& S = *(GramSolverLds*)lds_raw;
    // LDS after the hand-off state: deltaW of the hot columns [0, a.hot), then alpha
    double* hotl = (double*)(lds_raw + ((sizeof(GramSolverLds) + 15) & ~(size_t)15));
    double* alv_l = hotl + a.hot;
    const int32_t hot = a.hot;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = blockIdx.x;
    const int32_t H = a.H, NB = (H + kGB - 1) / kGB;
    const int64_t p0 = a.part_ptr[k];
    const int32_t nl = (int32_t)(a.part_ptr[k + 1] - p0);
    const size_t g0 = (size_t)k * H;
    double* dwk = a.dw + (size_t)k * a.d;
    // alpha of the partition, plus a sink at [nl] for the padding steps
    double* alv = ALV_LDS ? alv_l : a.alpha_work + p0 + k;
    const double* gt = a.gt + (size_t)k * a.nbatch * kGB * kGSlots;

    for (int32_t i = tid; i < nl; i += 256) alv[i] = a.alpha[p0 + i];
    if (tid == 0) alv[nl] = 0.0;  // sink of the padding steps
    for (int i = tid; i < kGSlots; i += 256) S.base[i] = 0.0;  // batches 0 .. kGNB-1: deltaW is still zero
    for (int32_t i = tid; i < hot; i += 256) hotl[i] = 0.0;
    if (tid < 8) S.cnt[tid] = 0;
    __syncthreads();
    if (tid == 0) S.cnt[2] = kGNB;  // base_done
    __syncthreads();
    // diagnostics (a.prof): per wave, cycles spent waiting on hand-offs and in total
    uint64_t wait_cycles = 0;
    uint64_t* pw = a.prof ? &wait_cycles : nullptr;
    const uint64_t t_start = a.prof ? __builtin_readcyclecounter() : 0;

    if (wv == 2) {
        // ------------------------------------------------------- loader --
        for (int32_t b = 0; b < NB; ++b) {
            // ring slot b % kGRing last held batch b - kGRing
            if (!wait_ge(&S.cnt[0], b - kGRing + 1, &S.cnt[4], a.status, pw)) break;
            // window of this batch's steps: batches b-3 .. b (positions 0..63)
            const int32_t w0 = (b - kGNB + 1) * kGB;
            const int32_t jw = w0 + lane;
            S.smpwin[lane] = (jw >= 0 && jw < H) ? a.samples[g0 + jw] : -2;
            const int32_t j = b * kGB + (lane & (kGB - 1));
            const bool valid = lane < kGB && j < H;
            int32_t r = nl;  // padding step: alpha sink
            double y = 0.0, q = 0.0, xw = 0.0;
            if (valid) {
                r = a.samples[g0 + j];
                y = a.plan_y[g0 + j];
                q = a.plan_q[g0 + j];
                xw = a.plan_xw[g0 + j];
            }
            wave_lds_sync();
            // previous occurrence of the same row in the window before this step
            int32_t pd = -1;
            const int32_t myw = (kGNB - 1) * kGB + (lane & (kGB - 1));
#pragma unroll 8
            for (int t = 0; t < kGSlots; ++t) {
                const int32_t rt = S.smpwin[t];
                if (valid && t < myw && rt == r) pd = t;
            }
            if (lane < kGB) {
                GRec& R = S.rec[(b % kGRing) * kGB + lane];
                double B = 0.0, E = 0.0, Y = 0.0;
                if (valid) gram_row_consts<MODE>(a, y, q, xw, B, E, Y);
                R.B = B;
                R.E = E;
                R.Y = Y;
                R.r = r;
                R.fw = -1;
                S.pdw[lane] = pd;
            }
            wave_lds_sync();
            // mark the earlier occurrences: step (w0 + pd) forwards its new alpha
            // to this step's slot (pd < myw, so in batches b-3 .. b)
            if (lane < kGB && pd >= 0) {
                const int32_t js = w0 + pd;
                S.rec[((js / kGB) % kGRing) * kGB + (js % kGB)].fw = j & (kGSlots - 1);
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[3], b + 1);
        }
    } else if (wv == 1) {
        // ------------------------------------------------------- memory --
        // layout slots: 0 = scatter batch, 1 = prefetched gather batch,
        // 2 = gather batch in flight (its products are formed next time)
        constexpr int NU = kGMU;
        int32_t cs[NU], cg[NU];
        double vs[NU], dw[NU];
        int32_t Ti = 0, Tp = 0;           // entries of the prefetched / in-flight gather batches
        bool piped = false;               // the in-flight gathers went out (else: gathered synchronously)
        const bool bases = MODE != MODE_MBCD;
        // deltaW: hot columns in LDS (no same-line L2 atomics), the rest in the slice
        auto dw_add = [&](int32_t c, double v) {
            if (c < hot) __hip_atomic_fetch_add(hotl + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else unsafeAtomicAdd(dwk + c, v);
        };
        auto dw_get = [&](int32_t c) { return c < hot ? hotl[c] : dw_load(dwk + c); };
        auto copy_layout = [&](int from, int to) {
            for (int i = lane; i <= kGB; i += 64) {
                S.mx[to][i] = S.mx[from][i];
                S.mp[to][i] = S.mp[from][i];
                if (i < kGB) S.mb[to][i] = S.mb[from][i];
            }
            for (int i = lane; i < NU; i += 64) S.mu[to][i] = S.mu[from][i];
            wave_lds_sync();
        };
        // prologue: data of step 0 (gather values of batch kGNB staged by parity)
        (void)gram_pack(a, g0, 0, S.mx[0], S.mb[0], S.mu[0], S.mp[0]);
        gram_fetch<NU>(a, S.mx[0], S.mb[0], S.mu[0], S.mp[0][kGB], cs, vs);
        if (bases && kGNB < NB) {
            Ti = gram_pack(a, g0, kGNB, S.mx[1], S.mb[1], S.mu[1], S.mp[1]);
            if (S.mp[1][kGB] <= NU) gram_fetch_g<NU>(a, S.mx[1], S.mb[1], S.mu[1], S.mp[1][kGB], cg, S.stage[kGNB & 1]);
        }
        for (int32_t b = 0; b < NB; ++b) {
            if (!wait_ge(&S.cnt[0], b + 1, &S.cnt[4], a.status, pw)) break;  // the chain finished batch b
            // 1. the gathers in flight (batch b-1+kGNB): products, row sums
            const int32_t bp = b - 1 + kGNB;
            if (bases && b >= 1 && bp < NB) {
                double* st = S.stage[bp & 1];
                if (piped) {
                    const int32_t nu = S.mp[2][kGB];
#pragma unroll
                    for (int u = 0; u < NU; ++u) {
                        // cg already holds the next prefetch: validity from the layout
                        if (u < nu) {
                            const int32_t ut = S.mu[2][u];
                            const int i = ut & 0xFF;
                            const int32_t e = ((ut >> 8) << 6) + lane;
                            if (e < S.mx[2][i + 1] - S.mx[2][i]) {
                                const int32_t qq = S.mx[2][i] + e;
                                st[qq] = st[qq] * dw[u];
                            }
                        }
                    }
                    wave_lds_sync();
                    gram_row_sums(S.mx[2], st, Tp, S.base + (bp % kGNB) * kGB);
                } else {
                    // a batch longer than the registers: gathered and summed here, in passes
                    double sum = 0.0;
                    for (int32_t qa = 0; qa < Tp; qa += kGStage) {
                        const int32_t qb = min(Tp, qa + kGStage);
                        for (int32_t q0 = qa; q0 < qb; q0 += 64) {
                            const int32_t qq = q0 + lane;
                            if (qq < qb) {
                                const int o = gram_owner(S.mx[2], qq);
                                const int64_t e = S.mb[2][o] + (qq - S.mx[2][o]);
                                st[qq - qa] = a.val[e] * dw_get(a.col[e]);
                            }
                        }
                        wave_lds_sync();
                        if (lane < kGB) {
                            const int32_t rb = max(S.mx[2][lane], qa), re = min(S.mx[2][lane + 1], qb);
                            for (int32_t q = rb; q < re; ++q) sum += st[q - qa];
                        }
                        wave_lds_sync();
                    }
                    if (lane < kGB) S.base[(bp % kGNB) * kGB + lane] = sum;
                }
                wave_lds_sync();
                if (lane == 0) lds_release(&S.cnt[2], bp + 1);
            }
            // 2. deltaW += c_j x_j for the steps of batch b (CoCoA.scala:181-185)
            {
                const double* cf = S.coef + (b % kGRing) * kGB;
                const int32_t nus = S.mp[0][kGB];
                // the batch's entries are in registers before the first atomic: without
                // this the compiler waits for every outstanding access (the previous
                // atomic included) before each one -- an L2 round trip per unit
                vm_drain();
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    if (u < nus && cs[u] >= 0) {
                        const double c = cf[S.mu[0][u] & 0xFF];
                        if (c != 0.0) dw_add(cs[u], vs[u] * c);
                    }
                }
                // units past the registers (long rows): row by row
                for (int i = 0; nus > NU && i < kGB; ++i) {
                    const int32_t u0 = S.mp[0][i], u1 = S.mp[0][i + 1];
                    if (u1 <= NU) continue;
                    const double c = cf[i];
                    if (c == 0.0) continue;
                    const int32_t z = S.mx[0][i + 1] - S.mx[0][i];
                    const int64_t rb = S.mb[0][i];
                    for (int32_t e = 64 * (u0 < NU ? NU - u0 : 0) + lane; e < z; e += 64)
                        dw_add(a.col[rb + e], a.val[rb + e] * c);
                }
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[1], b + 1);  // coefficient ring slot consumed
            // 3. issue the gathers of batch b+kGNB (they see batch b's atomics and
            //    nothing later: the next atomics go out after them)
            Tp = 0;
            if (bases && b + kGNB < NB) {
                copy_layout(1, 2);
                Tp = Ti;
                piped = S.mp[2][kGB] <= NU;
                if (piped) {
#pragma unroll
                    for (int u = 0; u < NU; ++u) dw[u] = cg[u] >= 0 ? dw_get(cg[u]) : 0.0;
                }
            }
            // 4. prefetch the data of step b+1
            if (b + 1 < NB) {
                (void)gram_pack(a, g0, b + 1, S.mx[0], S.mb[0], S.mu[0], S.mp[0]);
                gram_fetch<NU>(a, S.mx[0], S.mb[0], S.mu[0], S.mp[0][kGB], cs, vs);
                const int32_t bn = b + 1 + kGNB;
                if (bases && bn < NB) {
                    Ti = gram_pack(a, g0, bn, S.mx[1], S.mb[1], S.mu[1], S.mp[1]);
                    if (S.mp[1][kGB] <= NU) gram_fetch_g<NU>(a, S.mx[1], S.mb[1], S.mu[1], S.mp[1][kGB], cg, S.stage[bn & 1]);
                }
            }
        }
        vm_drain();  // the last atomics land before the kernel ends
    } else if (wv == 0) {
        // -------------------------------------------------------- chain --
        // lane = window slot (step mod 64): sdot = base + Gram corrections
        bool ok = wait_ge(&S.cnt[3], min(kGNB, NB), &S.cnt[4], a.status, pw);
        double acc = 0.0;
        // fill: this lane's slot takes the step (lane & 15) of batch b
        auto fill = [&](int32_t b) {
            GRec& R = S.rec[(b % kGRing) * kGB + (lane & (kGB - 1))];
            const double aa = alv[R.r];
            R.AE = aa - R.E;
            R.YA = R.Y * aa;
            acc = 0.0;
        };
        if (ok && lane / kGB < NB) fill(lane / kGB);
        wave_lds_sync();
        double gcur[kGB], gnxt[kGB];
#pragma unroll
        for (int i = 0; i < kGB; ++i) {
            gnxt[i] = 0.0;
            gcur[i] = (MODE != MODE_MBCD && i < H) ? __builtin_nontemporal_load(gt + (size_t)i * kGSlots + lane) : 0.0;
        }
        for (int32_t g = 0; ok && g < NB; ++g) {
            const int q4 = g % kGNB;          // this batch's quarter of the lanes
            const bool mine = lane / kGB == q4;
            if (MODE != MODE_MBCD && !wait_ge(&S.cnt[2], g + 1, &S.cnt[4], a.status, pw)) break;
            // coefficient ring slot g % kGRing held batch g - kGRing: consumed?
            if (!wait_ge(&S.cnt[1], g - kGRing + 1, &S.cnt[4], a.status, pw)) break;
            if (mine) acc += S.base[lane];
            const int32_t m = min(kGB, H - g * kGB);
            // next batch's Gram rows into registers while this one runs
            if (MODE != MODE_MBCD) {
#pragma unroll
                for (int i = 0; i < kGB; ++i) {
                    const int32_t jn = (g + 1) * kGB + i;
                    gnxt[i] = jn < H ? __builtin_nontemporal_load(gt + (size_t)jn * kGSlots + lane) : 0.0;
                }
            }
            GRec* rg = S.rec + (g % kGRing) * kGB;
            double* cfo = S.coef + (g % kGRing) * kGB;
            const int slot0 = q4 * kGB;
            // records one step ahead (uniform LDS reads)
            double nB = rg[0].B, nY = rg[0].Y, nAE = rg[0].AE, nYA = rg[0].YA, nE = rg[0].E;
            int32_t nR = rg[0].r, nF = rg[0].fw;
#pragma unroll
            for (int i = 0; i < kGB; ++i) {
                if (i < m) {
                    const double sB = nB, sY = nY, sAE = nAE, sYA = nYA;
                    const int32_t sr = nR, sf = uni(nF);
                    const int in = i + 1 < m ? i + 1 : i;
                    nB = rg[in].B;
                    nY = rg[in].Y;
                    nAE = rg[in].AE;
                    nYA = rg[in].YA;
                    nE = rg[in].E;
                    nR = rg[in].r;
                    nF = rg[in].fw;
                    const double sdot = readlane_d(acc, slot0 + i);
                    // CoCoA.scala:159-186 / MinibatchCD.scala:104-123 (see above)
                    const double nt = fmin(fmax(fma(-sB, sdot, sAE), 0.0), 1.0);
                    const double cf = fma(sY, nt, -sYA);
                    if (MODE != MODE_MBCD) acc = fma(cf, gcur[i], acc);
                    alv[sr] = nt;          // every lane: same address, same value
                    cfo[i] = cf;
                    if (sf >= 0) {
                        // a later step of the window samples the same row: its aa is nt
                        const int32_t sp = g * kGB + ((sf - g * kGB) & (kGSlots - 1));
                        GRec& T = S.rec[((sp / kGB) % kGRing) * kGB + (sp % kGB)];
                        const double tE = T.E, tY = T.Y;
                        T.AE = nt - tE;
                        T.YA = tY * nt;
                        if (sp == g * kGB + i + 1) {
                            nAE = nt - nE;
                            nYA = nY * nt;
                        }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < kGB; ++i) gcur[i] = gnxt[i];
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[0], g + 1);
            // refill this quarter with batch g + kGNB
            if (g + kGNB < NB) {
                if (!wait_ge(&S.cnt[3], g + kGNB + 1, &S.cnt[4], a.status, pw)) break;
                if (mine) fill(g + kGNB);
                wave_lds_sync();
            }
        }
    }
    if (a.prof && lane == 0) {
        uint64_t* pr = a.prof + ((size_t)k * 4 + wv) * 4;
        pr[0] = wait_cycles;
        pr[1] = __builtin_readcyclecounter() - t_start;
    }
    __syncthreads();
    for (int32_t i = tid; i < hot; i += 256) dwk[i] = hotl[i];  // the slice is zero there: plain stores
    // alpha = alphaOld + (alpha - alphaOld) * scaling (CoCoA.scala:101, MinibatchCD.scala:127-128)
    if (a.raw_alpha) {
        for (int32_t i = tid; i < nl; i += 256) a.alpha[p0 + i] = alv[i];
    } else {
        for (int32_t i = tid; i < nl; i += 256) {
            const double old = a.alpha[p0 + i];
            a.alpha[p0 + i] = old + ((alv[i] - old) * a.scaling);
        }
    }
}

}  // namespace cocoa
