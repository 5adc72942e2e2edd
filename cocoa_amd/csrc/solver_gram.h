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
//   base_s  = x_s . deltaW as of a batch boundary two batches back, gathered
//             off the chain by a helper wave;
//   G(s, j) = x_s . x_j, the Gram entries of nearby steps, computed before the
//             round by gram_kernel (the sampled rows are known in advance:
//             java.util.Random does not depend on the data);
//   c_j     = y_j (alpha_new - alpha_old) / (lambda n), the scatter
//             coefficient of step j (CoCoA.scala:181).
//
// The chain wave keeps one accumulator per lane: lane l holds the pending
// correction of the step in window slot l (slot = step mod 64, two batches of
// 32).  Step j reads its own accumulator (v_readlane), applies the update
// rule, and adds c_j * G(., j) to every pending lane -- one FMA, no memory
// access and no reduction on the dependent path.
//
// Roles (one 256-thread workgroup per partition, one wave each):
//   wave 0  chain   -- the H sequential steps (update rule, alpha in LDS);
//   wave 1  scatter -- deltaW += c_j x_j for finished batches (fp64 atomics
//                      into the partition's private slice), then waits for
//                      the acks;
//   wave 2  base    -- x_s . deltaW for the batch two ahead, between the
//                      scatters it must and must not see;
//   wave 3  loader  -- per-step records (label, x.w, ||x||^2, the previous
//                      occurrence of the same row in the window) for the
//                      slots being refilled.
// The waves hand off through counters in LDS (release / acquire, s_sleep
// while waiting), not workgroup barriers, so the chain never waits on a
// helper that is merely busy with a later batch.
//
// Ordering of the deltaW slice: base(b) must contain exactly the updates of
// batches <= b-2.  scatter(b) therefore waits until base(b+1) is gathered,
// and base(b) waits until scatter(b-2) is acknowledged.  Updates of batches
// b-1 and b reach step s of batch b through the Gram corrections.
//
// Numerics: fast mode (fused multiply-adds, reassociated dots, atomics); the
// results agree with the strict path / oracle within the north_star
// tolerance.  MbCD reads the stale w only (MinibatchCD.scala:104): no base,
// no Gram term, the chain is the update rule alone.
#pragma once
#include "kernels.h"
#include "wave.h"

namespace cocoa {

constexpr int kGB = 32;          // steps per batch
constexpr int kGSlots = 64;      // window slots = lanes (2 batches)
constexpr int kGHot = 64;        // dense hot columns of gram_kernel (device order: most frequent first)
constexpr int kGStage = 4096;    // entries per pass staged by the base wave
constexpr int kGSU = 24;         // 64-entry units per lane a helper keeps in flight

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
__device__ __forceinline__ bool wait_ge(const int* p, int v, int* abort_flag, int* status) {
    for (uint32_t it = 0;; ++it) {
        if (lds_acquire(p) >= v) return true;
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
// window [32 floor(j/32), +64) with s > j; 0 otherwise.
// One workgroup per (partition, batch of 32 updaters): partners are the 64
// steps of the window.  Hot columns (device index < kGHot) go through a dense
// LDS image of the partners (lanes = partners, one LDS read per hot entry of
// the updater); the other columns through an LDS hash of the partners' cold
// entries (lanes = the updater's entries, a probe each).
constexpr int kGramTable = 8192;     // hash slots (power of two, >= 2 x kGramCap: probes stay short)
constexpr int kGramCap = 4096;       // packed partner positions per pass (their cold entries are inserted)

struct GramLds {
    double X[kGSlots][kGHot + 1];    // +1: partner rows start on different banks
    double acc[kGB][kGSlots];        // G of the block's 32 updaters
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

__global__ __launch_bounds__(256, 1) void gram_kernel(GramArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramLds& L = *(GramLds*)lds_raw;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = blockIdx.x % a.K;
    const int g = blockIdx.x / a.K;
    const int32_t H = a.H;
    const int32_t j0 = g * kGB;
    const int32_t P = min(kGSlots, H - j0);     // partners [j0, j0 + P)
    const int32_t U = min(kGB, H - j0);          // updaters [j0, j0 + U)
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
        const int32_t z = L.pz[lane];
        const int32_t inc = wave_incl_scan(z);
        L.pcum[lane + 1] = inc;
        if (lane == 0) L.pcum[0] = 0;
    }
    __syncthreads();
    const int32_t T = L.pcum[kGSlots];
    auto owner = [&](int32_t q) {  // partner whose entries hold packed position q
        int lo = 0, hi = kGSlots;   // pcum[lo] <= q < pcum[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (L.pcum[mid] <= q) lo = mid; else hi = mid;
        }
        return lo;
    };
    // dense hot image (duplicate columns of a row add up, as in the dot)
    for (int32_t q = tid; q < T; q += 256) {
        const int p = owner(q);
        const int64_t e = L.pbeg[p] + (q - L.pcum[p]);
        const int32_t c = a.col[e];
        if (c < kGHot) atomicAdd(&L.X[p][c], a.val[e]);
    }
    __syncthreads();
    // hot part: lanes = partners; wave wv takes updaters wv, wv+4, ...
    for (int u = wv; u < U; u += 4) {
        const int64_t b = L.pbeg[u];
        const int32_t z = L.pz[u];
        double acc = 0.0;
        for (int32_t c0 = 0; c0 < z; c0 += 64) {
            const int32_t e = c0 + lane;
            const int32_t c = e < z ? a.col[b + e] : kGHot;
            const double v = e < z ? a.val[b + e] : 0.0;
            uint64_t m = __ballot(c < kGHot);
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1;
                const int32_t cc = __builtin_amdgcn_readlane(c, src);
                const double vv = readlane_d(v, src);
                acc = fma(vv, L.X[lane][cc], acc);
            }
        }
        L.acc[u][lane] = acc;  // this wave owns row u
    }
    // cold part, in passes of kGramCap packed partner positions
    for (int32_t qa = 0; qa < T; qa += kGramCap) {
        __syncthreads();
        for (int i = tid; i < kGramTable; i += 256) {
            L.tkey[i] = -1;
            L.thead[i] = -1;
        }
        __syncthreads();
        const int32_t qb = min(T, qa + kGramCap);
        for (int32_t q = qa + tid; q < qb; q += 256) {
            const int p = owner(q);
            const int64_t e = L.pbeg[p] + (q - L.pcum[p]);
            const int32_t c = a.col[e];
            if (c < kGHot) continue;
            const int32_t i = q - qa;
            L.epart[i] = (int8_t)p;
            L.eval[i] = a.val[e];
            uint32_t h = gram_hash(c) & (kGramTable - 1);
            for (;;) {
                const int32_t old = atomicCAS(&L.tkey[h], -1, c);
                if (old == -1 || old == c) break;
                h = (h + 1) & (kGramTable - 1);
            }
            L.enext[i] = (int16_t)atomicExch(&L.thead[h], i);
        }
        __syncthreads();
        for (int u = wv; u < U; u += 4) {
            const int64_t b = L.pbeg[u];
            const int32_t z = L.pz[u];
            for (int32_t c0 = 0; c0 < z; c0 += 64) {
                const int32_t e = c0 + lane;
                if (e >= z) continue;
                const int32_t c = a.col[b + e];
                if (c < kGHot) continue;
                const double v = a.val[b + e];
                uint32_t h = gram_hash(c) & (kGramTable - 1);
                for (;;) {
                    const int32_t key = L.tkey[h];
                    if (key == c) {
                        for (int32_t i = L.thead[h]; i >= 0; i = L.enext[i]) {
                            const int p = L.epart[i];
                            if (p > u) atomicAdd(&L.acc[u][p], v * L.eval[i]);
                        }
                        break;
                    }
                    if (key == -1) break;
                    h = (h + 1) & (kGramTable - 1);
                }
            }
        }
    }
    __syncthreads();
    // Gt rows of the block's updaters: slot of partner p = (j0 + p) & 63
    double* out = a.gt + ((size_t)k * a.nbatch * kGB + j0) * kGSlots;
    for (int u = wv; u < kGB; u += 4) {
        const double v = (u < U && lane > u && lane < P) ? L.acc[u][lane] : 0.0;
        __builtin_nontemporal_store(v, out + (size_t)u * kGSlots + ((j0 + lane) & (kGSlots - 1)));
    }
}

// ============================================================== solver ==
struct GramSolverLds {
    int cnt[8];                        // 0 chain_done, 1 scat_done, 2 base_done, 3 load_done, 4 abort
    // per-step records, ring of 4 batches (index (b & 3) * 32 + i)
    double rA[4 * kGB];                // y sigma' lambda n (CoCoA+), y lambda n (CoCoA), 0 (MbCD)
    double rKx[4 * kGB];               // (y x.w - 1) lambda n
    double rRq[4 * kGB];               // 1 / qii (0 when qii == 0)
    double rY[4 * kGB];                // y / (lambda n)
    double rCb[4 * kGB];               // rA * base + rKx, set by the chain at batch start
    int32_t rR[4 * kGB];               // sampled row (partition-local), -1 = padding step
    int32_t rPd[4 * kGB];              // slot of the previous step in the window with the same row, -1
    int32_t rF[4 * kGB];               // bit0: qii != 0
    double base[kGSlots];              // base_s per slot
    double coef[kGSlots];              // c_j per slot (chain -> scatter wave)
    int32_t smpwin[kGSlots];           // sampled rows of the loader's window
    double stage[kGStage];             // base wave: products x_e * deltaW[c_e]
    int32_t sexcl[kGB + 1];            // base wave: packed row offsets of its batch
    int64_t sbeg[kGB];
    int32_t cexcl[kGB + 1];            // scatter wave: the same for its batch
    int64_t cbeg[kGB];
};

template <int MODE>
__device__ __forceinline__ void gram_row_consts(const GramSolverArgs& a, double y, double q, double xw, double& A,
                                                double& Kx, double& rq, double& Y, int32_t& fl) {
    A = MODE == MODE_PLUS ? y * a.sigma * a.lam_n : (MODE == MODE_COCOA ? y * a.lam_n : 0.0);
    Kx = (y * xw - 1.0) * a.lam_n;
    const double qii = MODE == MODE_PLUS ? q * a.sigma : q;
    rq = qii != 0.0 ? 1.0 / qii : 0.0;
    Y = y * a.inv_lam_n;
    fl = qii != 0.0 ? 1 : 0;
}

// packed positions of a batch's rows -> (row, entry); rows [0, 32) of the batch
__device__ __forceinline__ int gram_owner(const int32_t* excl, int32_t q) {
    int lo = 0, hi = kGB;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (excl[mid] <= q) lo = mid; else hi = mid;
    }
    return lo;
}

template <int MODE, bool ALV_LDS>
__global__ __launch_bounds__(256, 1) void solver_gram_kernel(GramSolverArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramSolverLds& S = *(GramSolverLds*)lds_raw;
    double* alv_l = (double*)(lds_raw + sizeof(GramSolverLds));
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = blockIdx.x;
    const int32_t H = a.H, NB = (H + kGB - 1) / kGB;
    const int64_t p0 = a.part_ptr[k];
    const int32_t nl = (int32_t)(a.part_ptr[k + 1] - p0);
    const size_t g0 = (size_t)k * H;
    double* dwk = a.dw + (size_t)k * a.d;
    double* alv = ALV_LDS ? alv_l : a.alpha_work + p0;
    const double* gt = a.gt + (size_t)k * a.nbatch * kGB * kGSlots;

    for (int32_t i = tid; i < nl; i += 256) alv[i] = a.alpha[p0 + i];
    for (int i = tid; i < kGSlots; i += 256) {
        S.base[i] = 0.0;   // batches 0 and 1: deltaW is still zero
        S.coef[i] = 0.0;
    }
    if (tid < 8) S.cnt[tid] = 0;
    __syncthreads();
    if (tid == 0) S.cnt[2] = 2;  // base_done: bases of batches 0, 1
    __syncthreads();

    if (wv == 3) {
        // ------------------------------------------------------- loader --
        for (int32_t b = 0; b < NB; ++b) {
            if (!wait_ge(&S.cnt[0], b - 2, &S.cnt[4], a.status)) break;  // ring slot (b & 3) was last read when batch b-4's lanes were filled
            const int32_t j = b * kGB + (lane & 31);
            const bool valid = lane < kGB && j < H;
            // the window of this batch's steps: batches b-1 and b
            const int32_t jw = (b - 1) * kGB + lane;
            const int32_t rw = (jw >= 0 && jw < H) ? a.samples[g0 + jw] : -2;
            S.smpwin[lane] = rw;
            int32_t r = -1;
            double y = 0.0, q = 0.0, xw = 0.0;
            if (valid) {
                r = a.samples[g0 + j];
                y = a.plan_y[g0 + j];
                q = a.plan_q[g0 + j];
                xw = a.plan_xw[g0 + j];
            }
            wave_lds_sync();
            // previous occurrence of the same row in [32 (b-1), j): its slot, or -1
            int32_t pd = -1;
            const int32_t myw = kGB + (lane & 31);  // own position in the window
#pragma unroll 8
            for (int t = 0; t < kGSlots; ++t) {
                const int32_t rt = S.smpwin[t];
                if (valid && t < myw && rt == r) pd = ((b - 1) * kGB + t) & (kGSlots - 1);
            }
            if (lane < kGB) {
                const int ri = (b & 3) * kGB + lane;
                double A = 0.0, Kx = 0.0, rq = 0.0, Y = 0.0;
                int32_t fl = 0;
                if (valid) gram_row_consts<MODE>(a, y, q, xw, A, Kx, rq, Y, fl);
                S.rA[ri] = A;
                S.rKx[ri] = Kx;
                S.rRq[ri] = rq;
                S.rY[ri] = Y;
                S.rR[ri] = valid ? r : -1;
                S.rPd[ri] = pd;
                S.rF[ri] = fl;
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[3], b + 1);
        }
    } else if (wv == 2) {
        // --------------------------------------------------------- base --
        if (MODE != MODE_MBCD) {
            for (int32_t b = 2; b < NB; ++b) {
                // row extents of the batch (static: read before the handoff)
                const int32_t j = b * kGB + lane;
                int64_t beg = 0;
                int32_t z = 0;
                if (lane < kGB && j < H) {
                    beg = a.plan_beg[g0 + j];
                    z = a.plan_z[g0 + j];
                }
                const int32_t inc = wave_incl_scan(lane < kGB ? z : 0);
                if (lane < kGB) {
                    S.sexcl[lane + 1] = inc;
                    S.sbeg[lane] = beg;
                }
                if (lane == 0) S.sexcl[0] = 0;
                const int32_t T = __shfl(inc, kGB - 1, 64);
                wave_lds_sync();
                if (!wait_ge(&S.cnt[1], b - 1, &S.cnt[4], a.status)) break;  // scatter of batches <= b-2 acknowledged
                double sum = 0.0;
                for (int32_t qa = 0; qa < T; qa += kGStage) {
                    const int32_t qb = min(T, qa + kGStage);
                    // all gathers of a pass in flight: 16 entries per lane per round
                    for (int32_t q0 = qa; q0 < qb; q0 += 64 * 16) {
                        int32_t cc[16];
                        double vv[16];
#pragma unroll
                        for (int u = 0; u < 16; ++u) {
                            const int32_t q = q0 + 64 * u + lane;
                            cc[u] = -1;
                            vv[u] = 0.0;
                            if (q < qb) {
                                const int o = gram_owner(S.sexcl, q);
                                const int64_t e = S.sbeg[o] + (q - S.sexcl[o]);
                                cc[u] = a.col[e];
                                vv[u] = a.val[e];
                            }
                        }
                        double ww[16];
#pragma unroll
                        for (int u = 0; u < 16; ++u) ww[u] = cc[u] >= 0 ? dw_load(dwk + cc[u]) : 0.0;
#pragma unroll
                        for (int u = 0; u < 16; ++u) {
                            const int32_t q = q0 + 64 * u + lane;
                            if (q < qb) S.stage[q - qa] = vv[u] * ww[u];
                        }
                    }
                    wave_lds_sync();
                    // row sums over this pass (one lane per row; stored order)
                    if (lane < kGB) {
                        const int32_t rb = max(S.sexcl[lane], qa), re = min(S.sexcl[lane + 1], qb);
                        for (int32_t q = rb; q < re; ++q) sum += S.stage[q - qa];
                    }
                    wave_lds_sync();
                }
                if (lane < kGB) S.base[(b & 1) * kGB + lane] = sum;
                wave_lds_sync();
                if (lane == 0) lds_release(&S.cnt[2], b + 1);
            }
        }
    } else if (wv == 1) {
        // ------------------------------------------------------ scatter --
        // the batch's rows are packed (row i at [sx[i], sx[i+1])); the (col, val)
        // of the first kGSU * 64 positions are loaded before the chain is done
        // with the batch, so after the handoff only the atomics remain
        for (int32_t b = 0; b < NB; ++b) {
            const int32_t j = b * kGB + lane;
            int64_t beg = 0;
            int32_t z = 0;
            if (lane < kGB && j < H) {
                beg = a.plan_beg[g0 + j];
                z = a.plan_z[g0 + j];
            }
            const int32_t inc = wave_incl_scan(lane < kGB ? z : 0);
            int32_t* sx = S.cexcl;
            if (lane < kGB) {
                sx[lane + 1] = inc;
                S.cbeg[lane] = beg;
            }
            if (lane == 0) sx[0] = 0;
            const int32_t T = __shfl(inc, kGB - 1, 64);
            wave_lds_sync();
            int32_t cc[kGSU], ow[kGSU];
            double vv[kGSU];
            auto fetch = [&](int32_t q0) {
#pragma unroll
                for (int u = 0; u < kGSU; ++u) {
                    const int32_t q = q0 + 64 * u + lane;
                    cc[u] = -1;
                    vv[u] = 0.0;
                    ow[u] = 0;
                    if (q < T) {
                        const int o = gram_owner(sx, q);
                        const int64_t e = S.cbeg[o] + (q - sx[o]);
                        ow[u] = o;
                        cc[u] = a.col[e];
                        vv[u] = a.val[e];
                    }
                }
            };
            fetch(0);
            if (!wait_ge(&S.cnt[0], b + 1, &S.cnt[4], a.status)) break;       // the chain finished batch b
            if (MODE != MODE_MBCD && !wait_ge(&S.cnt[2], min(b + 2, NB), &S.cnt[4], a.status))
                break;                                                          // base(b+1) must not see batch b
            const double* cf = S.coef + (b & 1) * kGB;
            for (int32_t q0 = 0; q0 < T; q0 += 64 * kGSU) {
                if (q0 > 0) fetch(q0);
#pragma unroll
                for (int u = 0; u < kGSU; ++u) {
                    if (cc[u] >= 0) {
                        const double c = cf[ow[u]];
                        if (c != 0.0) unsafeAtomicAdd(dwk + cc[u], vv[u] * c);   // deltaW += update (CoCoA.scala:181-185)
                    }
                }
            }
            vm_drain();
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[1], b + 1);
        }
    } else {
        // -------------------------------------------------------- chain --
        bool ok = wait_ge(&S.cnt[3], min(2, NB), &S.cnt[4], a.status);
        double A = 0.0, Kx = 0.0, acc = 0.0, aa = 0.0;
        int32_t pd = -1;
        {
            const int b = lane >> 5;
            const int ri = b * kGB + (lane & 31);
            if (b < NB) {
                A = S.rA[ri];
                Kx = S.rKx[ri];
                pd = S.rPd[ri];
                const int32_t r = S.rR[ri];
                aa = r >= 0 ? alv[r] : 0.0;
            }
        }
        for (int32_t g = 0; ok && g < NB; ++g) {
            const int half = g & 1;
            if (MODE != MODE_MBCD && !wait_ge(&S.cnt[2], g + 1, &S.cnt[4], a.status)) break;
            // per-step constants of this batch: Cb = A * base + Kx
            if ((lane >> 5) == half) {
                const int ri = (g & 3) * kGB + (lane & 31);
                S.rCb[ri] = fma(A, S.base[lane], Kx);
            }
            wave_lds_sync();
            const int rb0 = (g & 3) * kGB;
            const double* grow = gt + (size_t)g * kGB * kGSlots;
            const int32_t m = min(kGB, H - g * kGB);
            // Gram rows straight from global memory, PF steps ahead
            constexpr int PF = 8;
            double gp[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u)
                gp[u] = (MODE != MODE_MBCD && u < m) ? __builtin_nontemporal_load(grow + u * kGSlots + lane) : 0.0;
            // step records (uniform LDS reads), one step ahead of their use
            double nA = S.rA[rb0], nCb = S.rCb[rb0], nRq = S.rRq[rb0], nY = S.rY[rb0];
            int32_t nR = S.rR[rb0], nF = S.rF[rb0];
            for (int32_t i0 = 0; i0 < m; i0 += PF) {
#pragma unroll
                for (int u = 0; u < PF; ++u) {
                    const int32_t i = i0 + u;
                    if (i < m) {
                        const int slot = half * kGB + i;
                        const double sA = nA, sCb = nCb, srq = nRq, sY = nY;
                        const int32_t sr = nR, sf = nF;
                        const int rn = rb0 + (i + 1 < m ? i + 1 : i);
                        nA = S.rA[rn];
                        nCb = S.rCb[rn];
                        nRq = S.rRq[rn];
                        nY = S.rY[rn];
                        nR = S.rR[rn];
                        nF = S.rF[rn];
                        const double sacc = readlane_d(acc, slot);
                        const double saa = readlane_d(aa, slot);
                        // CoCoA.scala:159-186 / MinibatchCD.scala:104-123
                        const double grad = fma(sA, sacc, sCb);
                        const double proj = saa <= 0.0 ? fmin(grad, 0.0) : (saa >= 1.0 ? fmax(grad, 0.0) : grad);
                        const bool go = proj != 0.0;
                        const double nt = fmin(fmax(fma(-grad, srq, saa), 0.0), 1.0);
                        const double na = go ? ((sf & 1) ? nt : 1.0) : saa;
                        const double cf = sY * (na - saa);
                        if (MODE != MODE_MBCD) {
                            acc = fma(cf, gp[u], acc);
                            gp[u] = i + PF < m ? __builtin_nontemporal_load(grow + (i + PF) * kGSlots + lane) : 0.0;
                        }
                        aa = pd == slot ? na : aa;
                        if (lane == 0) {
                            S.coef[slot] = cf;
                            if (go && sr >= 0) alv[sr] = na;
                        }
                    }
                }
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[0], g + 1);
            // refill this half with batch g + 2
            if (g + 2 < NB) {
                if (!wait_ge(&S.cnt[3], g + 3, &S.cnt[4], a.status)) break;
                if ((lane >> 5) == half) {
                    const int ri = ((g + 2) & 3) * kGB + (lane & 31);
                    A = S.rA[ri];
                    Kx = S.rKx[ri];
                    pd = S.rPd[ri];
                    const int32_t r = S.rR[ri];
                    acc = 0.0;
                    aa = r >= 0 ? alv[r] : 0.0;
                }
            }
        }
    }
    __syncthreads();
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
