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
//   base_s  = x_s . deltaW as of a batch boundary kGNB = 3 batches back, gathered
//             off the chain by a helper wave;
//   G(s, j) = x_s . x_j, the Gram entries of nearby steps, computed before the
//             round by gram_kernel (the sampled rows are known in advance:
//             java.util.Random does not depend on the data);
//   c_j     = y_j (alpha_new - alpha_old) / (lambda n), the scatter
//             coefficient of step j (CoCoA.scala:181).
//
// The chain wave keeps one accumulator per lane: lane l holds the pending
// correction of the step in window slot l (slot = step mod 48, three batches
// of 16).  Step j reads its own accumulator (v_readlane), applies the update
// rule, and adds c_j * G(., j) to every pending lane -- one FMA, no memory
// access and no reduction on the dependent path.
//
// Roles (one 384-thread workgroup per partition, one wave each):
//   chain      -- the H sequential steps (update rule, alpha in LDS);
//   memory x2  -- one per column class (device column parity): per batch b,
//                 deltaW += c_j x_j for the steps of batch b on the class's
//                 columns (fp64 atomics into the partition's private slice),
//                 then the gathers of x_s . deltaW for batch b+3 on them,
//                 software-pipelined one batch deep (issued now, summed next
//                 time) into the class's partial base;
//   loader     -- per-step records (constants of the update rule, the next
//                 occurrence of the same row in the window) and row layouts;
//   fetch x2   -- one per class: LDS DMA of the batch's class entries into the
//                 class's sub-ring.
// The waves hand off through counters in LDS (release / acquire, s_sleep
// while waiting), not workgroup barriers, so the chain never waits on a
// helper that is merely busy with a later batch.
//
// Ordering of the deltaW slice: base(b) must contain exactly the updates of
// batches <= b-3.  A column belongs to one class, so one memory wave issues,
// in this order, the atomics of batch b-3 to it and then the gathers of
// base(b), and the atomics of batch b-3 only after those gathers: one wave,
// one address stream, so the gathers see batch b-3 and nothing later.
// Batches b-3 .. b reach the steps of batch b through the Gram corrections
// (window of 48 steps = 3 batches of 16; lanes 48..63 of the chain idle.  A
// 64-step window measured the same solver time with 18% more Gram-row work,
// a 32-step one a 1.5% slower solver: r03 A/B).
//
// Numerics: fast mode (fused multiply-adds, reassociated dots, atomics); the
// results agree with the strict path / oracle within the north_star
// tolerance.  MbCD reads the stale w only (MinibatchCD.scala:104): no base,
// no Gram term, the chain is the update rule alone.
//
// Local SGD (MODE_LSGD, SGD.scala:87-139 with local = true) runs on the same
// machinery.  The reference shrinks its whole w copy every step (w *= 1 -
// step lambda, SGD.scala:119-120); here w = s (keep wInit + v), with the
// shrink in the scalar s and v = sum of u_j x_j, u_j = y_j step_j / s_j for the
// violators j (SGD.scala:124-129).  s depends only on the step index (t0 + i),
// so the loader forms it (and the step's constants) ahead of the chain, and
//   x_s . w_s = s_{s-1} (keep x_s.wInit + base_s + sum_j u_j G(s, j))
// with the same base / Gram split as above (the slice holds v).  A shrink of
// exactly 0 (step 1 of round 1) drops wInit: keep = 0, s = 1.  The epilogue
// writes deltaW = w - wInit = s keep wInit + s v - wInit (SGD.scala:133).
#pragma once
#include <type_traits>
#include "kernels.h"
#include "wave.h"

#ifdef COCOA_DIAG
#define COCOA_DIAG_ON 1  // diagnostic build: GramSolverArgs::diag may skip work (timing only)
#else
#define COCOA_DIAG_ON 0
#endif

namespace cocoa {

constexpr int kGB = 16;                  // steps per batch
constexpr int kGSlots = 64;              // lanes; Gram-row stride (doubles)
#ifndef COCOA_GWIN
#define COCOA_GWIN 48
#endif
constexpr int kGW = COCOA_GWIN;          // window slots (steps): slot of step s = s mod kGW
constexpr int kGNB = kGW / kGB;          // batches in the window
static_assert(kGW % kGB == 0 && kGW <= kGSlots && kGNB >= 2, "window");
constexpr int kGRing = 8;                // record / coefficient ring (batches)
constexpr int kXwPlan = 0, kXwProducer = 1;  // solver_gram_kernel's x.w source
constexpr uint64_t kXwPatience = 50000;  // cycles the loader polls x.w flags before forming x.w itself (~25 us)
#ifndef COCOA_GHOT
#define COCOA_GHOT 48  // (32: Gram rows 2.35 ms, 40: 2.28, 48: 2.26; r03 A/B)
#endif
constexpr int kGHot = COCOA_GHOT;        // dense hot columns of gram_kernel (device order: most frequent first)

// ----------------------------------------------------------- LDS handoff --
// The hand-offs order LDS data only (records, coefficients, layouts, staged
// entries, bases): LDS-only fences, so a release waits for the wave's LDS
// operations (lgkmcnt) and never for its outstanding global stores / atomics.
__device__ __forceinline__ int lds_acquire(const int* p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    return v;
}
__device__ __forceinline__ void lds_release(int* p, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
// n counters at once: one LDS round trip and one fence when all are >= v already
// (the common case), else wait_ge on each
__device__ __forceinline__ bool all_ge_now(const int* p, int n, int v) {
    bool ok = true;
    for (int i = 0; i < n; ++i) ok = ok && __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= v;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    return ok;
}
// L1-bypassing read of the deltaW slice (the scatter wave's atomics land in L2)
__device__ __forceinline__ double dw_load(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// gathers of hot columns (deltaW in LDS) load this instead: one line, factor 1
static __device__ double g_gram_one = 1.0;
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }    // vmcnt(0)
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xC07F); }  // lgkmcnt(0)

#ifdef COCOA_GS_CHECK  // debug variant: every global index checked (printf, access skipped)
#define GS_OK(cond, what, v)                                                                              \
    ((cond) ? true : (printf("gram_seq OOB %s %lld blk %d tid %d\n", what, (long long)(v), (int)blockIdx.x, \
                             (int)threadIdx.x), false))
#else
#define GS_OK(cond, what, v) ((void)(v), true)
#endif

// ================================================================ Gram ==
// Gt[k][j][slot] = x_s . x_j for the step s of window slot `slot` in j's
// window [16 floor(j/16), +kGW) with s > j; 0 otherwise.
// One workgroup per (partition, batch of 16 updaters); its kGW partners are the
// steps of the window (the updaters are partners 0..15).  The window's
// entries are packed partner by partner and loaded at once (256 per unit, up
// to kGramNU units in registers, owners found branch-free): one round trip to
// memory instead of one per row.  Then
//   hot columns (device index < kGHot, the most frequent): a dense image
//     XP[p][c] of the partners; G_hot = XP[0..15] XP^T with lanes =
//     partners and the updater values broadcast from LDS;
//   cold columns: an LDS hash (column -> list of (updater, value)) of the
//     updaters' cold entries, filled tile by tile; every partner cold entry
//     probes it.  A tile holds the updaters' COLD entries only, numbered in
//     position order (a block-wide ballot scan), so 1,024 cover a typical
//     batch (16 rows x ~76 entries, ~2/3 cold) and the LDS fits three
//     workgroups per CU (round 4; tiles of 2,048 packed positions, two per CU,
//     took 2.25 ms against 2.20).
// Windows longer than the register chunk reload it per tile (same results).
constexpr int kGramTable = 2048;     // hash slots (power of two, 2 x kGramTile)
constexpr int kGramTile = 1024;      // cold updater entries per hash tile
constexpr int kGramNU = 8;           // kGramThreads-entry units in registers
constexpr int kGramWGs = kGW <= 48 ? 3 : 2;  // workgroups per CU (LDS, and <= 80 VGPRs)
constexpr int kGramThreads = 512;    // 8 waves
constexpr int kGramCH = kGramNU * kGramThreads;
constexpr int kGHotS = kGHot + 1;    // XP row stride (doubles)

struct GramLds {
    double XP[kGW][kGHotS];          // hot image of the partners (updaters = rows 0..15)
    double acc[kGB][kGW];            // G of the updaters against the window
    int32_t tkey[kGramTable];
    int32_t thead[kGramTable];
    double eval[kGramTile];
    int16_t enext[kGramTile];
    int8_t eu[kGramTile];
    int64_t pbeg[kGSlots];
    int32_t pcum[kGSlots + 1];       // packed offsets of the partners
    int32_t cpre[kGramNU * (kGramThreads / 64)];  // cold-entry rank of each (unit, wave) in a chunk
    int32_t ctot;                                 // cold entries of the chunk
};
static_assert(sizeof(GramLds) * kGramWGs <= 160 * 1024, "gram_kernel LDS: kGramWGs workgroups per CU");
static_assert(kGramNU * (kGramThreads / 64) == 64, "one lane per (unit, wave) in the rank scan");
static_assert(kGramThreads == 512, "gram_kernel's hot part gives each of the 8 waves two updaters");
static_assert(kGramNU % 4 == 0, "gram_kernel probes four units at a time");

__device__ __forceinline__ uint32_t gram_hash(int32_t c) { return ((uint32_t)c * 2654435761u) >> 20; }  // 12 bits
static_assert(kGramTable <= 4096 && kGramTile <= 32767, "gram_hash bits / int16 list links");

// Gram rows of one updater batch g of partition k (every thread of the block)
__device__ __forceinline__ void gram_batch(const GramArgs& a, GramLds& L, int k, int g) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint64_t tph = a.prof ? __builtin_readcyclecounter() : 0;
    auto phase = [&](int i) {  // diagnostics: thread 0 adds the phase's cycles
        if (a.prof && tid == 0) {
            const uint64_t t = __builtin_readcyclecounter();
            atomicAdd((unsigned long long*)&a.prof[i], (unsigned long long)(t - tph));
            tph = t;
        }
    };
    const int32_t H = a.H;
    const int32_t j0 = g * kGB;
    const int32_t P = min(kGW, H - j0);         // partners [j0, j0 + P)
    const int32_t U = min(kGB, H - j0);          // updaters = partners [0, U)
    const int64_t p0 = a.part_ptr[k];
    const int32_t* smp = a.samples + (size_t)k * H;
    if (wv == 0) {
        int64_t b = 0;
        int32_t z = 0;
        if (lane < P) {
            const int64_t r = p0 + smp[j0 + lane];
            b = a.row_ptr[r];
            z = (int32_t)(a.row_ptr[r + 1] - b);
        }
        const int32_t inc = wave_incl_scan(z);
        L.pbeg[lane] = b;
        L.pcum[lane + 1] = inc;
        if (lane == 0) L.pcum[0] = 0;
    }
    for (int i = tid; i < kGW * kGHotS; i += kGramThreads) (&L.XP[0][0])[i] = 0.0;
    for (int i = tid; i < kGB * kGW; i += kGramThreads) (&L.acc[0][0])[i] = 0.0;
    __syncthreads();
    phase(0);
    const int32_t T = L.pcum[P], Q16 = L.pcum[U];
    // registers: a chunk of packed positions [qa, qa + kGramCH): column (-1 past
    // T), value, owner partner (4 per word)
    int32_t cc[kGramNU];
    double vv[kGramNU];
    uint32_t ow[kGramNU / 4];
    int32_t reg_qa = -1;
    auto load = [&](int32_t qa) {
        if (reg_qa == qa) return;
        reg_qa = qa;
        int o[kGramNU];
#pragma unroll
        for (int u = 0; u < kGramNU; ++u) {  // owners: independent binary searches, interleaved
            const int32_t q = min(qa + u * kGramThreads + tid, T - 1);
            int lo = 0;
#pragma unroll
            for (int st = kGSlots / 2; st >= 1; st >>= 1)
                if (L.pcum[lo + st] <= q) lo += st;
            o[u] = lo;
        }
#pragma unroll
        for (int u = 0; u < kGramNU; ++u) {
            const int32_t q = qa + u * kGramThreads + tid;
            const bool ok = q < T;
            const int64_t e = ok ? L.pbeg[o[u]] + (q - L.pcum[o[u]]) : 0;
            cc[u] = ok ? a.col[e] : -1;
            vv[u] = ok ? a.val[e] : 0.0;
        }
#pragma unroll
        for (int w = 0; w < kGramNU / 4; ++w)
            ow[w] = (uint32_t)o[4 * w] | ((uint32_t)o[4 * w + 1] << 8) | ((uint32_t)o[4 * w + 2] << 16) |
                    ((uint32_t)o[4 * w + 3] << 24);
    };
    auto owner_of = [&](int u) { return (int)((ow[u / 4] >> (8 * (u % 4))) & 0xFFu); };
    load(0);
    // hot image (duplicate columns of a row add up, as in the dot)
    for (int32_t qa = 0; qa < T; qa += kGramCH) {
        load(qa);
#pragma unroll
        for (int u = 0; u < kGramNU; ++u)
            if (cc[u] >= 0 && cc[u] < kGHot) atomicAdd(&L.XP[owner_of(u)][cc[u]], vv[u]);
    }
    phase(1);
    auto insert = [&](int32_t i, int u) {  // hash-list entry i of unit u's (cold updater) entry
        const int32_t c = cc[u];
        L.eval[i] = vv[u];
        L.eu[i] = (int8_t)owner_of(u);
        uint32_t h = gram_hash(c) & (kGramTable - 1);
        for (;;) {
            const int32_t old = atomicCAS(&L.tkey[h], -1, c);
            if (old == -1 || old == c) break;
            h = (h + 1) & (kGramTable - 1);
        }
        L.enext[i] = (int16_t)atomicExch(&L.thead[h], i);
    };
    // cold part, one hash tile of cold updater entries at a time: entry rank =
    // cold updater entries before it in position order (q = qa + 512 u + tid:
    // unit, wave, lane), the same in every tile's pass
    int32_t ncold = 0;
    for (int32_t ta = 0;; ta += kGramTile) {
        for (int i = tid; i < kGramTable; i += kGramThreads) {
            L.tkey[i] = -1;
            L.thead[i] = -1;
        }
        int32_t run = 0;  // cold entries of the chunks before qa
        for (int32_t qa = 0; qa < Q16; qa += kGramCH) {
            load(qa);
            uint64_t m[kGramNU];
#pragma unroll
            for (int u = 0; u < kGramNU; ++u) {
                const int32_t q = qa + u * kGramThreads + tid;
                m[u] = __ballot(q < Q16 && cc[u] >= kGHot);
                if (lane == 0) L.cpre[u * (kGramThreads / 64) + wv] = __popcll(m[u]);
            }
            __syncthreads();
            if (wv == 0) {
                const int32_t v = L.cpre[lane];
                const int32_t inc = wave_incl_scan(v);
                L.cpre[lane] = inc - v;
                if (lane == 63) L.ctot = inc;
            }
            __syncthreads();
            const uint64_t below = (1ull << lane) - 1;
#pragma unroll
            for (int u = 0; u < kGramNU; ++u) {
                if ((m[u] >> lane) & 1) {
                    const int32_t i = run + L.cpre[u * (kGramThreads / 64) + wv] + __popcll(m[u] & below) - ta;
                    if (i >= 0 && i < kGramTile) insert(i, u);
                }
            }
            run += L.ctot;
            __syncthreads();  // cpre / ctot of the next chunk
        }
        ncold = run;
        __syncthreads();
        phase(5);
        // entries of updater rows of column c from i on (list order), into partner pp
        auto walk = [&](int32_t i, int pp, double v) {
            for (; i >= 0; i = L.enext[i]) {
                const int uu = L.eu[i];
                if (pp > uu) atomicAdd(&L.acc[uu][pp], v * L.eval[i]);
            }
        };
        for (int32_t qa = 0; qa < T; qa += kGramCH) {
            load(qa);
            // four units at a time, in dependent rounds whose LDS reads go out
            // together: the home slot (key, head), the head entry (most cold columns
            // have one updater entry), then the rare rest one unit at a time
            // (longer lists, and probes that met another key)
#pragma unroll
            for (int u0 = 0; u0 < kGramNU; u0 += 4) {
                uint32_t h[4];
                int32_t key[4], hd[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    h[t] = gram_hash(cc[u0 + t]) & (kGramTable - 1);
                    key[t] = L.tkey[h[t]];
                    hd[t] = L.thead[h[t]];
                }
                bool act[4], hit[4];
                int32_t nx[4];
                int eu[4];
                double ev[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int u = u0 + t;
                    act[t] = cc[u] >= kGHot && owner_of(u) != 0;  // no updater before partner 0
                    hit[t] = act[t] && key[t] == cc[u];
                    const int32_t i0 = hit[t] ? hd[t] : 0;
                    ev[t] = L.eval[i0];
                    eu[t] = L.eu[i0];
                    nx[t] = L.enext[i0];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int u = u0 + t, pp = owner_of(u);
                    if (hit[t] && pp > eu[t]) atomicAdd(&L.acc[eu[t]][pp], vv[u] * ev[t]);
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int u = u0 + t, pp = owner_of(u);
                    const int32_t c = cc[u];
                    if (hit[t]) {
                        if (nx[t] >= 0) walk(nx[t], pp, vv[u]);
                    } else if (act[t] && key[t] != -1) {
                        uint32_t hh = (h[t] + 1) & (kGramTable - 1);
                        for (;;) {
                            const int32_t k2 = L.tkey[hh];
                            if (k2 == c) {
                                walk(L.thead[hh], pp, vv[u]);
                                break;
                            }
                            if (k2 == -1) break;
                            hh = (hh + 1) & (kGramTable - 1);
                        }
                    }
                }
            }
        }
        __syncthreads();
        phase(6);
        if (ta + kGramTile >= ncold) break;
    }
    phase(2);
    // hot part: wave wv -> updaters 2 wv, 2 wv + 1, lane = partner
    {
        double h0 = 0.0, h1 = 0.0;
        const int u0 = 2 * wv;
        const int pl = min(lane, kGW - 1);  // lanes past the window: discarded
#pragma unroll 8
        for (int c = 0; c < kGHot; ++c) {
            const double xp = L.XP[pl][c];
            h0 = fma(L.XP[u0][c], xp, h0);
            h1 = fma(L.XP[u0 + 1][c], xp, h1);
        }
        if (lane < kGW) {
            L.acc[u0][lane] += h0;  // sole writer of (u, lane) now
            L.acc[u0 + 1][lane] += h1;
        }
    }
    __syncthreads();
    phase(3);
    // Gt rows of the block's updaters: slot of partner p = (j0 + p) mod kGW (slots
    // past the window: zero)
    double* out = a.gt + ((size_t)k * a.nbatch * kGB + j0) * kGW;
    const int slot = ((g % kGNB) * kGB + lane) % kGW;
    for (int u = wv; u < kGB; u += kGramThreads / 64) {
        const double v = (u < U && lane > u && lane < P) ? L.acc[u][min(lane, kGW - 1)] : 0.0;
        if (lane < kGW) __builtin_nontemporal_store(v, out + (size_t)u * kGW + slot);
    }
    phase(4);
}

__global__ __launch_bounds__(kGramThreads, kGramWGs) void gram_kernel(GramArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramLds& L = *(GramLds*)lds_raw;
    // XCD-aware order: blocks land on the 8 XCDs round robin; one partition's
    // consecutive batches (3/4 of their partners shared) stay on one XCD, close
    // in time, so its L2 serves the re-reads
    int k, g;
    {
        const int64_t b = blockIdx.x;
        if (a.K % 8 == 0) {
            const int64_t kx = a.K / 8, i = b / 8;
            k = (int)((b % 8) + 8 * (i % kx));
            g = (int)(i / kx);
        } else {
            k = (int)(b % a.K);
            g = (int)(b / a.K);
        }
    }
    gram_batch(a, L, k, g);
}

// The same rows for a list of (partition, batch) pairs: the windows the
// sequential kernel below could not hold in its LDS pool (fb_n of them, at
// fb[2 i], fb[2 i + 1]); a block per pair, grid-stride.
__global__ __launch_bounds__(kGramThreads, kGramWGs) void gram_list_kernel(GramArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramLds& L = *(GramLds*)lds_raw;
    const int32_t n = *a.fb_n;
    for (int32_t i = blockIdx.x; i < n; i += gridDim.x) {
        if (!GS_OK(i < a.fb_cap && a.fb[2 * i] >= 0 && a.fb[2 * i] < a.K && a.fb[2 * i + 1] >= 0 &&
                       a.fb[2 * i + 1] < a.nbatch, "fb pair", i))
            continue;
        gram_batch(a, L, a.fb[2 * i], a.fb[2 * i + 1]);
        __syncthreads();  // (LDS reused by the next pair)
    }
}

// ===================================================== Gram rows, sequential ==
// gram_seq_kernel: one workgroup walks a contiguous chunk of one partition's
// batches in order and keeps the window's rows in LDS, so each batch is loaded,
// hashed and imaged once instead of once per window that holds it (three
// times), and each cold updater entry makes ONE lookup for the whole window
// instead of every partner entry probing the updaters' hash:
//
//   pool   -- the cold entries (device column >= kGHot) of the live batches
//             x-2 .. x, a ring of kGsPool records {column | step-in-batch << 27,
//             link, value}; batch x's entries at [pstart_x, pstart_x + n_x);
//   head   -- one list per hash bucket, newest first.  A link holds the
//             target's BATCH in its high bits (batch << 13 | slot), so a walk
//             for updater batch g stops at the first link into a batch < g
//             without reading it: entries of dead batches are never touched,
//             and their ring slots are reused without unlinking anything;
//   XP     -- the dense image of the hot columns, a ring of 4 batches x 16 rows;
//             the hot products of updater batch g against partner batches g,
//             g+1, g+2 are three 16 x 16 tiles over 48 columns on
//             v_mfma_f64_16x16x4f64 (12 per tile), stored to accH;
//   accC   -- the cold products, fp64 LDS atomics by the walks.
//
// Per batch x of the chunk (updater g = x - 2):
//   B1  hot entries of x into XP; cold counts per (register unit, wave);
//   B3  cold entries of x into the pool (ranks by a scan of the counts) and
//       their lists; the next batch's entries issued into registers;
//   C   MFMA tiles of g (waves 0-2); every wave walks g's cold entries;
//   D   Gt rows of g (accH + accC, as gram_kernel writes them); XP rows of
//       batch x+2 cleared; the batch metadata (row starts, packed offsets) of
//       x+2 written, x+3 / x+4 loaded, by wave 0.
// A batch whose cold entries do not fit the pool beside the two before it is
// not inserted; the windows that hold it (updaters x-2, x-1, x) go to the
// fallback list, recomputed afterwards by gram_list_kernel (the per-window
// kernel, any size).
// (r06i A/B, C2 beside the solver, 3 runs per partition: 512 threads and 48 hot
// columns 1.80 ms; 1,024 threads 1.24; 96 hot columns 1.57; both 1.16)
#ifndef COCOA_GS_THREADS
#define COCOA_GS_THREADS 1024
#endif
#ifndef COCOA_GS_HOT
#define COCOA_GS_HOT 96
#endif
constexpr int kGsThreads = COCOA_GS_THREADS;
constexpr int kGsWaves = kGsThreads / 64;
constexpr int kGsNU = 3072 / kGsThreads; // register units of kGsThreads entries: 3,072 entries of a batch at once
constexpr int kGsHot = COCOA_GS_HOT;     // dense (MFMA) columns: device order, most frequent first
constexpr int kGsHotS = kGsHot + 1;
#ifndef COCOA_GS_POOL
#define COCOA_GS_POOL 4608
#endif
// cold-entry ring: C2 windows hold 2,300 cold entries (column >= 96) on average,
// ~3,700 for 99.9% of them, so a handful per round go to the fallback list
constexpr int kGsPool = COCOA_GS_POOL;
constexpr int kGsSlotBits = 13;
static_assert(kGsPool <= (1 << kGsSlotBits), "link slot bits");
constexpr int kGsBuckets = 4096;         // gram_hash: 12 bits
constexpr int kGsMeta = 8;               // batch metadata ring
constexpr int kGsAhead = 3;              // batches whose entries are in flight (register sets)
static_assert(kGsAhead + 4 <= kGsMeta, "live metadata: batches x-2 .. x+kGsAhead+1");
constexpr int kGsColBits = 27;           // column bits of a pool record (step-in-batch above)
struct GsMetaRec {
    int64_t beg[kGB];                    // row starts of the batch's 16 steps
    int32_t pref[kGB + 1];               // packed offsets (entries of steps < i)
    int32_t pstart, pn;                  // the batch's cold entries in the pool
};
struct GramSeqLds {
    // pool records, split so a walk reads 8 bytes per visited record and the
    // value only on a column match: pcn = {column | step-in-batch << 27, link}
    int2 pcn[kGsPool];
    double pval[kGsPool];
    int32_t head[kGsBuckets];
    double XP[4 * kGB][kGsHotS];         // hot image, row = 16 (batch % 4) + step-in-batch
    double accH[kGB][kGW];
    double accC[kGB][kGW];
    GsMetaRec meta[kGsMeta];
    int32_t cnt[kGsNU * kGsWaves];
};
static_assert(sizeof(GramSeqLds) <= 160 * 1024, "gram_seq_kernel LDS");
static_assert(kGsNU * kGsWaves <= 64, "one lane per (unit, wave) count");
static_assert(kGsHot % 4 == 0, "MFMA k-steps of 4 hot columns");
// three partner batches (MFMA tiles): other windows (COCOA_GWIN) take gram_kernel
constexpr bool kGsWindowOK = kGW == 3 * kGB;

typedef double gs_d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kGsThreads, 1) void gram_seq_kernel(GramArgs a) {
  if constexpr (kGsWindowOK) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramSeqLds& L = *(GramSeqLds*)lds_raw;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // block b: partition b % K (the solver's XCD when K % 8 == 0), chunk b / K
    const int k = (int)(blockIdx.x % (unsigned)a.K), ch = (int)(blockIdx.x / (unsigned)a.K);
    const int32_t H = a.H, NB = a.nbatch;
    const int32_t gA = (int32_t)(((int64_t)NB * ch) / a.chunks), gB = (int32_t)(((int64_t)NB * (ch + 1)) / a.chunks);
    if (gA >= gB) return;
    const int64_t p0 = a.part_ptr[k];
    const int32_t* smp = a.samples + (size_t)k * H;
    double* gtk = a.gt + (size_t)k * NB * kGB * kGW;

    for (int i = tid; i < kGsBuckets; i += kGsThreads) L.head[i] = -1;
    for (int i = tid; i < 4 * kGB * kGsHotS; i += kGsThreads) (&L.XP[0][0])[i] = 0.0;
    for (int i = tid; i < kGB * kGW; i += kGsThreads) (&L.accC[0][0])[i] = 0.0;

    // ---- batch metadata (wave 0, lanes 0..15 = steps): samples -> row extents ----
    // in flight: row extents of batch mx (rb, re), samples of batch mx + 1 (ms)
    struct Ext {
        int64_t b, e;
    };
    Ext rx{0, 0};
    int32_t ms = -1;
    auto smp_of = [&](int32_t x) -> int32_t {  // sample of step lane of batch x (-1: none)
        const int32_t j = x * kGB + lane;
        return (lane < kGB && x < NB && j < H && GS_OK(j >= 0, "smp", j)) ? smp[j] : -1;
    };
    auto extents = [&](int32_t r) -> Ext {
        const bool ok = r >= 0 && GS_OK(p0 + r + 1 <= a.n_rows, "row_ptr", p0 + r);
        const int64_t i = ok ? p0 + r : 0;
        const int64_t b = a.row_ptr[i], e = a.row_ptr[i + 1];
        return ok ? Ext{b, e} : Ext{0, 0};
    };
    auto meta_write = [&](int32_t x, const Ext& q) {  // batch x's metadata from its row extents
        GsMetaRec& M = L.meta[x & (kGsMeta - 1)];
        const int32_t z = lane < kGB ? (int32_t)(q.e - q.b) : 0;
        const int32_t inc = wave_incl_scan(z);
        if (lane < kGB) {
            M.beg[lane] = q.b;
            M.pref[lane + 1] = inc;
        }
        if (lane == 0) M.pref[0] = 0;
    };
    // metadata kGsAhead + 1 batches ahead, entries kGsAhead batches ahead (registers)
    if (wv == 0) {
#pragma unroll
        for (int32_t i = 0; i <= kGsAhead; ++i) meta_write(gA + i, extents(smp_of(gA + i)));
        rx = extents(smp_of(gA + kGsAhead + 1));  // written in the first D phase
        ms = smp_of(gA + kGsAhead + 2);
        if (lane == 0) {
            L.meta[(gA - 1) & (kGsMeta - 1)].pstart = 0;  // the pool starts empty
            L.meta[(gA - 1) & (kGsMeta - 1)].pn = 0;
            L.meta[(gA - 2) & (kGsMeta - 1)].pn = 0;
        }
    }
    __syncthreads();

    // ---- a batch's entries in registers: q = u * kGsThreads + tid ----
    struct Ents {
        int32_t col[kGsNU];
        double val[kGsNU];
        int8_t own[kGsNU];
    };
    auto issue = [&](Ents& E, int32_t x) {  // entries [0, kGsNU * kGsThreads) of batch x
        const GsMetaRec& M = L.meta[x & (kGsMeta - 1)];
        const int32_t T = x < NB ? M.pref[kGB] : 0;
#pragma unroll
        for (int u = 0; u < kGsNU; ++u) {
            const int32_t q = u * kGsThreads + tid;
            int lo = 0;
            if (q < T) {
#pragma unroll
                for (int st = kGB / 2; st >= 1; st >>= 1)
                    if (M.pref[lo + st] <= q) lo += st;
            }
            E.own[u] = (int8_t)(q < T ? lo : -1);
        }
#pragma unroll
        for (int u = 0; u < kGsNU; ++u) {
            const int o = E.own[u];
            const int32_t q = u * kGsThreads + tid;
            const int64_t e = o >= 0 ? M.beg[o] + (q - M.pref[o]) : 0;
            const bool ok = o >= 0 && GS_OK(e >= 0 && e < a.nnz, "entry", e);
            E.col[u] = ok ? a.col[e] : -1;
            E.val[u] = ok ? a.val[e] : 0.0;
        }
    };
    static_assert(kGsAhead == 3, "the main loop rotates three register sets");
    Ents E0, E1, E2;
    issue(E0, gA);
    issue(E1, gA + 1);
    issue(E2, gA + 2);

    const uint64_t below = (1ull << lane) - 1;
    int32_t fb_next = gA;  // (thread 0) windows before it are on the fallback list already
    // diagnostics (a.prof): thread 0's cycles per phase, summed in registers and
    // added to the launch's totals once at the end (one atomic per phase and block)
    uint64_t tph = a.prof ? __builtin_readcyclecounter() : 0;
    uint64_t pc[7] = {0, 0, 0, 0, 0, 0, 0};
    auto phase = [&](int i) {
        if (a.prof && tid == 0) {
            const uint64_t t = __builtin_readcyclecounter();
            pc[i] += t - tph;
            tph = t;
        }
    };
    // one batch x (insert x, Gram rows of updater batch g = x - 2); E holds batch
    // x's entries and is refilled with batch x + kGsAhead's
    auto step = [&](const int32_t x, Ents& E) {
        const int32_t g = x - 2;
        const bool ins = x < NB;
        const int32_t T = ins ? L.meta[x & (kGsMeta - 1)].pref[kGB] : 0;
        const int xs = x & 3;
        // batch x's cold entries go in after the live ones of x-2, x-1
        const GsMetaRec& Mp = L.meta[(x - 1) & (kGsMeta - 1)];
        const int32_t base = (Mp.pstart + Mp.pn) % kGsPool;
        const int32_t live = Mp.pn + L.meta[(x - 2) & (kGsMeta - 1)].pn;
        // a batch longer than one register chunk is never inserted (fallback windows)
        bool ovf = T > kGsNU * kGsThreads;
        int32_t tot = 0;
        const bool body = T > 0 && !ovf;
        // B1: hot entries into the image; cold counts per (unit, wave)
        uint64_t m[kGsNU];
#pragma unroll
        for (int u = 0; u < kGsNU; ++u) {
            const int32_t c = body ? E.col[u] : -1;
            if (c >= 0 && c < kGsHot) atomicAdd(&L.XP[xs * kGB + E.own[u]][c], E.val[u]);
            m[u] = __ballot(c >= kGsHot);
            if (lane == 0) L.cnt[u * kGsWaves + wv] = __popcll(m[u]);
        }
        phase(0);
        // (every iteration: it also orders wave 0's metadata written in the last D
        // phase before the reads of issue() below)
        __syncthreads();
        phase(1);
        if (body) {
            // B3: ranks (every wave scans the counts itself) and the pool records
            const int32_t cv = lane < kGsNU * kGsWaves ? L.cnt[lane] : 0;
            const int32_t inc = wave_incl_scan(cv);
            tot = __builtin_amdgcn_readlane(inc, 63);
            ovf = live + tot > kGsPool;
            if (!ovf) {
#pragma unroll
                for (int u = 0; u < kGsNU; ++u) {
                    const int32_t ex = __builtin_amdgcn_readlane(inc - cv, uni(u * kGsWaves + wv));
                    if ((m[u] >> lane) & 1) {
                        const int32_t slot = (base + ex + __popcll(m[u] & below)) % kGsPool;
                        const int32_t c = E.col[u];
                        const int32_t link = (x << kGsSlotBits) | slot;
                        const int32_t old = atomicExch(&L.head[gram_hash(c) & (kGsBuckets - 1)], link);
                        L.pcn[slot] = make_int2(c | ((int32_t)E.own[u] << kGsColBits), old);
                        L.pval[slot] = E.val[u];
                    }
                }
            }
        }
        if (wv == 0 && lane == 0 && ins) {
            GsMetaRec& M = L.meta[x & (kGsMeta - 1)];
            M.pstart = base;
            M.pn = ovf ? 0 : tot;
            if (ovf) {  // windows holding batch x: recomputed by gram_list_kernel (each once)
                for (int32_t y = max(max(x - 2, gA), fb_next); y <= min(x, gB - 1); ++y) {
                    fb_next = y + 1;
                    const int32_t i = atomicAdd(a.fb_n, 1);
                    if (GS_OK(i < a.fb_cap, "fb", i)) {
                        a.fb[2 * i] = k;
                        a.fb[2 * i + 1] = y;
                    }
                }
            }
        }
        // batch x + kGsAhead's entries, in flight through the next kGsAhead batches
        issue(E, x + kGsAhead);
        phase(2);
        __syncthreads();  // (pool, lists, meta of x)
        phase(3);
        if (g >= gA) {
            // C: hot tiles on MFMA (waves 0..2: partner batch g + wv), then the cold walk
            const int gs = g & 3;
            if (wv < 3) {
                const int ps = (g + wv) & 3;
                gs_d4 acc = {0.0, 0.0, 0.0, 0.0};
                const int r = lane & 15, kq = lane >> 4;
#pragma unroll
                for (int kk = 0; kk < kGsHot / 4; ++kk) {
                    const double av = L.XP[gs * kGB + r][4 * kk + kq];
                    const double bv = L.XP[ps * kGB + r][4 * kk + kq];
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) L.accH[kq + 4 * i][wv * kGB + r] = acc[i];
            }
            const GsMetaRec& Mg = L.meta[g & (kGsMeta - 1)];
            const int32_t n = Mg.pn, ps0 = Mg.pstart;
            // waves 3.. take the first entries: the MFMA waves walk only what is
            // left past kGsThreads - 192 (C2: a batch holds ~770 cold entries)
            const int32_t wt = wv < 3 ? tid + (kGsThreads - 192) : tid - 192;
            for (int32_t i = wt; i < n; i += kGsThreads) {
                const int32_t se = (ps0 + i) % kGsPool;
                const int32_t ecu = L.pcn[se].x;
                const double ev = L.pval[se];
                const int32_t c = ecu & ((1 << kGsColBits) - 1), u = ecu >> kGsColBits;
                int32_t l = L.head[gram_hash(c) & (kGsBuckets - 1)];
                while (l >= 0 && (l >> kGsSlotBits) >= g) {
                    const int32_t sf = l & ((1 << kGsSlotBits) - 1);
                    const int2 f = L.pcn[sf];
                    if ((f.x & ((1 << kGsColBits) - 1)) == c) {
                        const int32_t p = ((l >> kGsSlotBits) - g) * kGB + (f.x >> kGsColBits);
                        if (p > u) atomicAdd(&L.accC[u][p], ev * L.pval[sf]);
                    }
                    l = f.y;
                }
            }
        }
        phase(4);
        __syncthreads();  // (accH, accC)
        phase(5);
        // D: Gt rows of g; XP rows of batch x+2 cleared (they held x-2 = g); metadata
        if (g >= gA) {
            const int32_t j0 = g * kGB, U = min(kGB, H - j0), P = min(kGW, H - j0);
            double* out = gtk + (size_t)j0 * kGW;
            for (int i = tid; i < kGB * kGW; i += kGsThreads) {
                const int u = i / kGW, p = i - u * kGW;
                const double v = (u < U && p > u && p < P) ? L.accH[u][p] + L.accC[u][p] : 0.0;
                const int64_t oi = (int64_t)(out - a.gt) + (int64_t)u * kGW + (j0 + p) % kGW;
                if (GS_OK(oi >= 0 && oi < a.gt_len, "gt", oi))
                    __builtin_nontemporal_store(v, out + (size_t)u * kGW + (j0 + p) % kGW);
                L.accC[u][p] = 0.0;
            }
        }
        {
            const int cs = (x + 2) & 3;
            for (int i = tid; i < kGB * kGsHotS; i += kGsThreads) (&L.XP[cs * kGB][0])[i] = 0.0;
        }
        if (wv == 0) {
            meta_write(x + kGsAhead + 1, rx);  // row extents loaded one batch ago
            rx = extents(ms);                  // batch x + kGsAhead + 2
            ms = smp_of(x + kGsAhead + 3);
        }
        phase(6);
        // (no barrier: the next B1 writes XP rows of x+1, cleared one batch ago, and
        // reads nothing D writes; its first barrier orders the rest)
    };
    for (int32_t x = gA; x < gB + 2; x += 3) {
        step(x, E0);
        if (x + 1 < gB + 2) step(x + 1, E1);
        if (x + 2 < gB + 2) step(x + 2, E2);
    }
    if (a.prof && tid == 0)
        for (int i = 0; i < 7; ++i) atomicAdd((unsigned long long*)&a.prof[i], (unsigned long long)pc[i]);
  }
}

// ============================================================== solver ==
// Per-step constants.  With sdot = x.deltaW (base + Gram corrections) the
// update rule of CoCoA.scala:159-186 is
//     grad = A sdot + Kx            A = y sigma' lambda n (CoCoA: y lambda n)
//     nt   = clamp(aa - grad / qii, 0, 1)
//          = clamp(AE - B sdot)     B = A / qii, E = Kx / qii, AE = aa - E
//     c    = y (nt - aa) / (lambda n) = Y nt - YA,   YA = Y aa
// and, while aa lies in [0, 1], nt is the new alpha whether or not the
// projected gradient vanishes: with aa = 0 and grad >= 0, or aa = 1 and
// grad <= 0, the clamp returns aa.  An alpha outside [0, 1] (scaling > 1 --
// CoCoA+ gamma > 1, CoCoA beta > K -- or an alpha set from outside) needs the
// explicit test of CoCoA.scala:166-172: with u = AE - B sdot = aa - grad/qii,
// the step is skipped (nt = aa) when aa <= 0 and u <= aa or aa >= 1 and
// u >= aa; that is the PROJ variant of the kernel.  An empty row (qii = 0) has
// grad = -lambda n < 0 and gets alpha = 1 unless skipped: B = 0 and E = -1e300,
// so u is huge for any aa.  MbCD (MinibatchCD.scala:104): A = 0, so B = 0.
//
// Column classes.  deltaW's columns are split into kGNC classes (device
// column c in class c % kGNC: the device order is by frequency, so the classes
// carry about the same entries); in fast mode every row stores its entries
// class by class (cocoa_set_train), so a row's entries of one class are one
// contiguous run.  Each class has its own fetch wave, LDS sub-ring and memory
// wave: the memory wave of class c scatters and gathers only columns of class
// c, so the per-column order "scatter of batch b, then gathers of batch b+3"
// still holds inside one wave's address stream, and the memory waves -- the
// issue-bound part of the round -- run side by side.  The chain adds the
// partial bases.
constexpr int kGWin = kGW + kGB;         // loader's look-back for alpha forwarding: the window + 1 batch
constexpr int kGUnitB = 64 * 13;         // bytes of one 64-entry ring unit
constexpr int kGOCol = 0, kGOLo = 256, kGOHi = 512, kGORow = 768;  // its fields
constexpr int kGGt = 4;                  // Gram-row ring (batches)
#ifndef COCOA_EARLY_RELEASE
#define COCOA_EARLY_RELEASE 0  // 1: memory waves free a staged batch's slots before its atomics (r06n: solver 2.34 -> 2.39 ms, not kept)
#endif
#ifndef COCOA_GPART
#define COCOA_GPART 16  // (32: 1.4% slower, 544 fewer LDS-resident deltaW columns; r03 A/B)
#endif
constexpr int kGPart = COCOA_GPART;      // product slots per row (lanes l, l + kGPart, ... share one)
// Shape of a workgroup with NC column classes (one memory wave and one fetch
// wave each): the one-workgroup solver has 2, the mirrored solver's halves
// kGramRuns / 2.  Staged entries: an LDS ring of kE positions, a sub-ring of
// kSub 64-entry units per class holding 4 live batches of up to kMaxU units
// (larger batches go direct).  With four classes the ring is halved (4,096
// positions, 4 units = 256 entries of a class per batch: 98.6% of C2's
// (batch, run) pairs with eight runs) so that the hot image keeps its LDS.
// Wave roles.  Wave w of the workgroup runs on SIMD w % 4, and which waves
// share a SIMD matters (r03 A/B on C2, two classes): chain + loader on one
// SIMD and the two fetch waves on another, 2.97 ms; chain + fetch 0 and
// loader + fetch 1, 2.85 ms; the memory waves keep a SIMD each (with four
// classes, two memory waves share each of SIMDs 2 and 3).  Waves: chain,
// loader, then groups of (memory, memory, fetch, fetch); the mirrored form adds
// the relay as the last wave.
#ifndef COCOA_GLAY4
#define COCOA_GLAY4 0  // (eight runs: the four memory waves on four SIMDs, A/B knob)
#endif
template <int NC>
struct GCfg {
    static constexpr int kE = NC == 2 ? 8192 : 4096;
    static constexpr int kSub = kE / 64 / NC;
    static constexpr int kMaxU = kSub / 4;
    static constexpr int kRChain = 0, kRLoader = 1, kRMem = 2, kRFetch = 2 + NC, kRIdle = 2 + 2 * NC,
                         kRRelay = 3 + 2 * NC;
    static constexpr int kWaves = 2 + 2 * NC;
    static constexpr int kThreads = 64 * kWaves;
    // counters (LDS, release / acquire); kCScat .. kCFetch: one per class; kCBase
    // + r: the partial base of column run r (kGramRuns of them: the one-workgroup
    // solver uses r < NC, one per class; the mirrored one every run)
    static constexpr int kCScat = 3, kCBase = kCScat + NC, kCFreed = kCBase + kGramRuns, kCFetch = kCFreed + NC;
    static_assert(kCFetch + NC <= 32, "counters");
    static_assert(NC == 2 || NC == 4, "classes");
    __device__ static int role(int w) {
        if (w == 0) return kRChain;
        if (w == 1) return kRLoader;
        if (w >= kWaves) return kRIdle;
        const int i = w - 2;
        if (COCOA_GLAY4 && NC == 4)  // the memory waves first: one on each SIMD
            return i < NC ? kRMem + i : kRFetch + (i - NC);
        const int g = i >> 2, j = i & 3;
        return j < 2 ? kRMem + 2 * g + j : kRFetch + 2 * g + (j - 2);
    }
};
constexpr int kCChain = 0, kCLoad = 1, kCAbort = 2;

struct GRec {                          // one step (64 B)
    double B, Y, AE, YA;               // AE, YA: set by the chain (its alpha prefetch or a forward)
    double E;
    double AA;                         // alpha before the step (PROJ: the projected-gradient skip test)
    int32_t r;                         // sampled row (partition-local); padding steps: the alpha sink
    int32_t fw;                        // ring position (mod 128) of the next step with the same row, -1
    int32_t fwd;                       // AE / YA already forwarded (the prefetched alpha is stale)
    int32_t pad;
};
static_assert(sizeof(GRec) == 64, "GRec layout");

struct GLay {                          // one batch's rows of one class, for the fetch and memory waves
    int64_t sb[kGB];                   // starts of the rows' class runs in the CSR
    int32_t sx[kGB + 1];               // packed offsets: row i at [sx[i], sx[i+1])
    int32_t pos;                       // sub-ring position of the staged entries (multiple of 64); -1: direct
    int32_t nu;                        // 64-entry units
    int32_t T;                         // entries
};

template <int NC>
struct GramSolverLdsT {
    int cnt[32];
    double lsgd_s;                     // MODE_LSGD: s after the last step (loader -> epilogue)
    int32_t lsgd_keep, lsgd_pad;       //   and whether wInit survived (no zero shrink)
    GRec rec[kGRing * kGB];            // ring: (b % kGRing) * kGB + i
    double coef[kGRing * 2 * kGB];     // c_j, same ring (chain -> memory waves); [kGB, 2 kGB) of a slot stay 0
    GLay lay[kGRing][NC];              // same ring (loader -> fetch / memory waves)
    double base[kGramRuns][kGSlots];   // partial base_s per class (mirrored: per run) and slot (memory waves -> chain)
    double part[NC][kGB + 1][kGPart];  // memory wave: row partial sums of a batch's products (+ a sink row)
    alignas(16) double gring[kGGt][kGB][kGW];      // Gram rows of batch x at [x % kGGt] (loader DMA -> chain)
    // staged entries (fetch waves -> memory waves), 64 per ring unit: columns, value
    // low words, value high words (the LDS DMA moves 4 bytes a lane), row bytes
    // (0xFF: past the batch's entries).  One address per lane and unit reaches all
    // four (immediate offsets; the two value words in one ds_read2).  Class c owns
    // units [c kSub, (c + 1) kSub).
    alignas(16) uint8_t ring[GCfg<NC>::kE / 64][kGUnitB];
};
static_assert(sizeof(GramSolverLdsT<2>) <= 160 * 1024 && sizeof(GramSolverLdsT<kGramRuns / 2>) <= 160 * 1024,
              "solver_gram_kernel LDS");

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
        E = -1e300;  // u = aa - E: the clamp gives 1 for every aa (and PROJ skips aa >= 1)
    }
    Y = y * a.inv_lam_n;
}

// the column run of class c of the mirrored solver's half h: half h owns the
// columns of parity h
__device__ __forceinline__ int gram_mirror_run(int c, int h) { return 2 * c + h; }

// packed position q of a batch's rows -> row: largest i with excl[i] <= q
__device__ __forceinline__ int gram_owner(const int32_t* excl, int32_t q) {
    int lo = 0;
#pragma unroll
    for (int st = kGB / 2; st >= 1; st >>= 1)
        if (excl[lo + st] <= q) lo += st;
    return lo;
}

// 4 or 16 bytes per lane from global memory straight into LDS (lds + size *
// lane).  (nt on these once-read streams measured no different: r03 A/B, 3.03
// vs 3.04 ms.)  The 12-byte form is no use for packed records: it writes lane l
// at lds + 16 l, leaving every fourth word (tools/ubench/dma_layout.hip).
__device__ __forceinline__ void lds_dma4(const void* g, void* lds) {
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}
__device__ __forceinline__ void lds_dma16(const void* g, void* lds) {
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// 0 for a unit of the batch (u < nu), 0xFF (row: no entry) past it.  The row byte is
// read unconditionally and or-ed with this: a branch around the read would make
// every unit wait for its LDS read before the next one goes out.
__device__ __forceinline__ uint32_t gram_pad(int32_t u, int32_t nu) {
    return (uint32_t)((nu - 1 - u) >> 31) & 0xFFu;
}
// ring unit of class c's sub-ring position pos (a multiple of 64) + 64 u
template <int NC>
__device__ __forceinline__ int32_t ring_unit(int c, int32_t pos, int32_t u) {
    constexpr int kSub = GCfg<NC>::kSub;
    return c * kSub + (((pos >> 6) + u) & (kSub - 1));
}
// lane's entry of a ring unit: (column, value, row byte)
template <class L>
__device__ __forceinline__ void ring_get(const L& S, int32_t us, int lane, int32_t& col, double& val,
                                         uint32_t& row) {
    const uint8_t* b = S.ring[us];
    col = *(const int32_t*)(b + kGOCol + 4 * lane);
    val = __hiloint2double(*(const int*)(b + kGOHi + 4 * lane), *(const int*)(b + kGOLo + 4 * lane));
    row = b[kGORow + lane];
}

// CoCoA.scala:166-178 on u = aa - grad / qii: the clamp, and with PROJ the
// projected-gradient skip for an alpha outside [0, 1]
template <bool PROJ>
__device__ __forceinline__ double gram_rule(double u, double aa) {
    const double nt = fmin(fmax(u, 0.0), 1.0);
    if (!PROJ) return nt;
    const bool skip = (aa <= 0.0 && u <= aa) || (aa >= 1.0 && u >= aa);
    return skip ? aa : nt;
}

// Roles (kGThreads threads, one workgroup per partition):
//   chain        -- the H dependent steps;
//   memory c     -- per batch b: deltaW += c_j x_j on class-c columns (batch b),
//                   then the gathers x_s . deltaW of batch b+3 on class-c columns,
//                   their products summed one batch later into base[c];
//   loader       -- records (update-rule constants, alpha forwarding marks) and
//                   the per-class row layouts, up to kGRing batches ahead;
//   fetch c      -- copy each batch's class-c (column, value) entries into the
//                   class's LDS sub-ring (LDS DMA), ahead of the gathers.
// MIRROR: two workgroups per partition (grid 2 K), each running the chain and
// the loader on identical inputs (so both form the same coefficients bit for
// bit) and the memory / fetch waves of the deltaW columns of its parity h; a
// seventh wave (relay) copies the other half's partial bases of every batch
// from xbase into LDS.  Each half thus scatters and gathers half the entries.
template <int MODE, bool HOTLDS, bool PROJ, int XWM, bool MIRROR = false>
__global__ __launch_bounds__(GCfg<MIRROR ? kGramRuns / 2 : kGramClasses>::kThreads + (MIRROR ? 64 : 0), 1)
void solver_gram_kernel(GramSolverArgs a) {
    constexpr bool XW = XWM == kXwProducer;  // x.w: plan_xw (kXwPlan) or the producer's flags
    // column classes: 2, or (mirrored) one per run of the half's parity
    constexpr int NC = MIRROR ? kGramRuns / 2 : kGramClasses;
    using C = GCfg<NC>;
    constexpr int kGSub = C::kSub, kGMaxU = C::kMaxU, kGNC = NC;
    constexpr int kRLoader = C::kRLoader, kRMem = C::kRMem, kRFetch = C::kRFetch, kRIdle = C::kRIdle,
                  kRRelay = C::kRRelay, kRChain = C::kRChain;
    constexpr int kCScat = C::kCScat, kCBase = C::kCBase, kCFreed = C::kCFreed, kCFetch = C::kCFetch;
    constexpr int kGWaves = C::kWaves, kGThreads = C::kThreads;
    using Lds = GramSolverLdsT<NC>;
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    Lds& S = *(Lds*)lds_raw;
    // LDS after the hand-off state: deltaW of the hot columns, a.hot doubles
    double* hotl = (double*)(lds_raw + ((sizeof(Lds) + 15) & ~(size_t)15));
    const int32_t hot = HOTLDS ? a.hot : 0;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int KP = MIRROR ? (int)(gridDim.x / 2) : (int)gridDim.x;
    // mirrored: block b -> (partition k, half h) with the two halves of a partition
    // dispatched next to one another and on one XCD (round-robin b % 8): groups of
    // 8 partitions, b = 16 (k / 8) + 8 h + k % 8; the last, partial group of
    // r = KP % 8 partitions, b = 16 (KP / 8) + r h + k % 8.  Both halves of a pair
    // must be resident at once (they wait on each other's bases): a pair is never
    // split across the dispatch of many other workgroups
    int k = (int)blockIdx.x, h = 0;
    if (MIRROR) {
        const int b = (int)blockIdx.x, full = KP >> 3, G = b >> 4;
        if (G < full) {
            h = (b >> 3) & 1;
            k = 8 * G + (b & 7);
        } else {
            const int r = KP & 7, rem = b - 16 * full;
            h = rem / r;
            k = 8 * full + rem % r;
        }
    }
    // hot columns [0, hotc), column c at hotl[hix(c)].  A mirrored half only
    // touches the columns of its parity (its runs 2 c + h), so its image holds those
    // alone: twice the hot columns in the same LDS (C2: 1,472 -> 2,944, 68% -> 75%
    // of the entries, round 5).
    constexpr bool PAR = MIRROR;
    const int32_t hotc = PAR ? 2 * hot : hot;
    auto hix = [&](int32_t c) -> int32_t { return PAR ? (c >> 1) : c; };
    constexpr int NRUN = MIRROR ? kGramRuns : kGNC;  // partial bases the chain sums
    constexpr int NTH = MIRROR ? kGThreads + 64 : kGThreads;
    const int32_t H = a.H, NB = (H + kGB - 1) / kGB;
    int role = C::role(wv);
    if (MIRROR && wv == kGWaves) role = kRRelay;
    role = __builtin_amdgcn_readfirstlane(role);
    const int64_t p0 = a.part_ptr[k];
    const int32_t nl = (int32_t)(a.part_ptr[k + 1] - p0);
    const size_t g0 = (size_t)k * H;
    double* dwk = a.dw + (size_t)k * a.d;
    // working alpha of the partition (global), plus a sink at [nl] for the padding steps
    double* alv = a.alpha_work + p0 + k + (MIRROR ? h * a.alpha_work_stride : 0);
    const double* gt = a.gt + (size_t)k * a.nbatch * kGB * kGW;
    int* abortf = &S.cnt[kCAbort];

    if (MODE != MODE_LSGD) {
        for (int32_t i = tid; i < nl; i += NTH) alv[i] = a.alpha[p0 + i];
        if (tid == 0) alv[nl] = 0.0;
    }
    for (int i = tid; i < kGramRuns * kGSlots; i += NTH) (&S.base[0][0])[i] = 0.0;  // batches 0 .. kGNB-1
    for (int32_t i = tid; i < hot; i += NTH) hotl[i] = 0.0;
    for (int i = tid; i < kGRing * 2 * kGB; i += NTH) S.coef[i] = 0.0;  // zero slots: rows past a batch
    if (tid < 32) S.cnt[tid] = 0;
    __syncthreads();
    if (tid < kGramRuns) S.cnt[kCBase + tid] = kGNB;
    __syncthreads();
    // MbCD mirrored: no bases tie the halves together, so half 1 flags that it has
    // copied alphaOld (above; every thread's load has landed, its value stored) and
    // half 0 waits for the flag before it writes the new alpha (epilogue)
    uint64_t* const mflag = (MIRROR && MODE == MODE_MBCD) ? a.xbase + (size_t)k * kGramRuns * kXbR * (2 * kGB) : nullptr;
    const uint64_t mtag = ((uint64_t)(a.xtag_epoch & 0xFFF) << 20) | 0xFFFFFu;
    if (MIRROR && MODE == MODE_MBCD && h == 1 && tid == 0) __hip_atomic_store(mflag, mtag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t wait_cycles = 0, wait_base_local = 0, wait_base_remote = 0;  // (diagnostics: the chain's base waits)
    uint64_t wait_load = 0, wait_scat = 0;  // (diagnostics: the chain's waits on the loader / the memory waves' ring)
    uint64_t* pw = a.prof ? &wait_cycles : nullptr;
    const uint64_t t_start = a.prof ? __builtin_readcyclecounter() : 0;

    if (role == kRLoader) {
        // ------------------------------------------------------- loader --
        int32_t cursor[kGNC];  // sub-ring position of the next staged batch, per class
#pragma unroll
        for (int c = 0; c < kGNC; ++c) cursor[c] = 0;
        // the step's inputs one batch ahead (registers)
        const int i = lane & (kGB - 1);
        int32_t xr = nl, xz = 0;
        int32_t xzc[kGramRuns - 1];  // ends of the column runs 0 .. R-2 in the row
        int32_t xpv = -1;            // the step's look-back: latest earlier step of its row in its window (plan)
        double xy = 0.0, xq = 0.0, xxw = 0.0;
        int64_t xbeg = 0;
        double ls = 1.0;   // MODE_LSGD: s before the batch (SGD.scala:119-120), wave-uniform
        int32_t lkeep = 1; //   wInit not yet dropped by a zero shrink
        // XW: x.w from xw_produce_kernel (beside this launch).  At the start of
        // every 16 batches, 16 lanes poll those batches' flags (sc1 loads) for
        // at most kXwPatience cycles; the batches found published load their x.w
        // with sc1 loads behind one agent acquire (the producer stored them sc1,
        // drained, then flagged).  A batch
        // not published by then (the launch's first batches before the producer
        // starts, or a device shared with other spinning grids) forms its x.w
        // here with the producer's summation when its record is consumed, so
        // the solver never waits on another grid's progress.
        uint32_t xw_ready = 0;  // bit i: batch (16 floor(b/16) + i) published
        bool xw_miss = false;   // the loaded batch forms its x.w in xw_inline
        auto xw_poll = [&](int32_t b) {
            const int32_t bb = b + (lane & 15);
            const bool need = lane < 16 && bb < NB;
            const int32_t* fp = a.xw_flag + (size_t)k * NB + (need ? bb : b);
            const uint64_t t0 = __builtin_readcyclecounter();
            uint64_t miss;
            for (;;) {
                const int32_t v = __hip_atomic_load(fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                miss = __ballot(need && v != a.xw_epoch);
                if (!miss || __builtin_readcyclecounter() - t0 > kXwPatience) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (pw) *pw += __builtin_readcyclecounter() - t0;
            xw_ready = (uint32_t)(__ballot(need) & ~miss);
            // The producer runs several workgroups per CU, outside the one-per-CU
            // geometry of MI355X_MICROARCH.md's sc1-load hand-off table, so the
            // sc1 loads alone are not the documented form: one agent acquire per
            // 16 batches (wave-uniform; this wave's own loads need no barrier).
            if (xw_ready) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        };
        // x.w of batch b's 16 steps from (xbeg, xz): four steps per pass, one
        // per 16 lanes, summed as xw_produce_kernel / plan_kernel sum them
        auto xw_inline = [&]() {
            double r4[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int s = 4 * p + (lane >> 4);
                const int64_t qb = __shfl(xbeg, s, 64);
                const int32_t qz = __shfl(xz, s, 64);
                double acc = 0.0;
                for (int32_t q = lane & 15; q < qz; q += 16) acc += a.val[qb + q] * a.w[a.xw_col[qb + q]];
                r4[p] = row16_sum(acc);
            }
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const double v = __shfl(r4[p], 16 * (lane & 3), 64);
                if ((lane >> 2) == p) xxw = v;
            }
        };
        auto load = [&](int32_t b) {
            if (XW && (b & 15) == 0) xw_poll(b);
            if (XW) xw_miss = !((xw_ready >> (b & 15)) & 1);
            const int32_t j = b * kGB + i;
            xr = nl;
            xz = 0;
#pragma unroll
            for (int c = 0; c < kGramRuns - 1; ++c) xzc[c] = 0;
            xpv = -1;
            xy = xq = xxw = 0.0;
            xbeg = 0;
            if (j < H) {  // (every lane: lane group g holds step lane & 15 too; same addresses, coalesced)
                xr = a.samples[g0 + j];
                xy = a.plan_y[g0 + j];
                xq = a.plan_q[g0 + j];
                if (!XW)
                    xxw = a.plan_xw[g0 + j];
                else if (!xw_miss)
                    xxw = __hip_atomic_load(const_cast<double*>(a.plan_xw) + (size_t)k * a.xw_stride + j,
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                xbeg = a.plan_beg[g0 + j];
                xz = a.plan_z[g0 + j];
                typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
                const int32_t* zp = a.plan_zc + (size_t)kGramRuns * (g0 + j);
                const i32x4 z4 = *(const i32x4*)(zp + kGramRuns - 4);  // (16-byte loads)
                if (kGramRuns == 8) {
                    const i32x4 zl = *(const i32x4*)zp;
#pragma unroll
                    for (int c = 0; c < 4; ++c) xzc[c] = zl[c];
                }
#pragma unroll
                for (int c = 0; c < 3; ++c) xzc[kGramRuns - 4 + c] = z4[c];
                xpv = z4[3];
            }
        };
        load(0);
        // (diagnostics: the loader's cycles per phase of an iteration)
        uint64_t lph[7] = {0, 0, 0, 0, 0, 0, 0};
        uint64_t ltp = pw ? __builtin_readcyclecounter() : 0;
        auto lstamp = [&](int i) {
            if (pw) {
                const uint64_t t = __builtin_readcyclecounter();
                lph[i] += t - ltp;
                ltp = t;
            }
        };
        // batch b's records and layouts; the Gram rows of batch b-4 (LDS DMA, their
        // completion published one iteration later: kCLoad = b+1 means records
        // <= b and Gram rows <= b-5 are in LDS)
        const int32_t NL = MODE != MODE_MBCD ? NB + kGGt + 1 : NB;
        for (int32_t b = 0; b < NL; ++b) {
            // ring slots (records b % kGRing, Gram rows (b-4) % kGGt) last held batch
            // b - kGRing: chain and both memory waves done with it
            if (!wait_ge(&S.cnt[kCChain], b - kGRing + 1, abortf, a.status, pw)) break;
            bool ok = true;
            if (!all_ge_now(&S.cnt[kCScat], kGNC, min(b, NB) - kGRing + 1)) {
#pragma unroll
                for (int c = 0; c < kGNC; ++c)
                    ok = ok && wait_ge(&S.cnt[kCScat + c], min(b, NB) - kGRing + 1, abortf, a.status, pw);
            }
            if (!ok) break;
            {
                const uint64_t td = pw ? __builtin_readcyclecounter() : 0;
                vm_drain();  // last iteration's loads and DMA
                if (pw) wait_base_local += __builtin_readcyclecounter() - td;  // (diagnostics: the loader's drain)
            }
            lstamp(0);
            if (b < NB) {
                const int32_t j = b * kGB + i;
                const bool valid = lane < kGB && j < H;
                const int32_t r = xr, z = xz, pv = xpv;
                // class c: entries [beg + zb[c], beg + ze[c+1]) -- runs [c R/2, (c + 1) R/2),
                // or (mirrored) run 2c + h
                int32_t zr[kGramRuns + 1];
                zr[0] = 0;
#pragma unroll
                for (int c = 0; c < kGramRuns - 1; ++c) zr[c + 1] = xzc[c];
                zr[kGramRuns] = z;
                int32_t ze[kGNC + 1], zb[kGNC];
#pragma unroll
                for (int c = 0; c < kGNC; ++c) {
                    const int r = gram_mirror_run(c, h);
                    zb[c] = MIRROR ? zr[r] : zr[c * (kGramRuns / 2)];
                    ze[c + 1] = MIRROR ? zr[r + 1] : zr[(c + 1) * (kGramRuns / 2)];
                }
                ze[0] = 0;
                if (XW && xw_miss) xw_inline();  // (wave-uniform)
                const double y = xy, q = xq, xw = xxw;
                const int64_t beg = xbeg;
                if (b + 1 < NB) load(b + 1);
                lstamp(1);
                // the rows' runs of each class, one class per 16-lane row of the wave
                // (lane group cl = lane >> 4 holds class cl of step lane & 15): one
                // DPP row scan for all classes
                const int cl = lane >> 4;
                int32_t zbl = zb[0], zel = ze[1];
#pragma unroll
                for (int c = 1; c < kGNC; ++c)
                    if (cl == c) {
                        zbl = zb[c];
                        zel = ze[c + 1];
                    }
                const int32_t incl = row16_incl_scan((cl < kGNC && j < H) ? zel - zbl : 0);
                int32_t T[kGNC], nu[kGNC];
#pragma unroll
                for (int c = 0; c < kGNC; ++c) {
                    T[c] = __builtin_amdgcn_readlane(incl, 16 * c + kGB - 1);
                    nu[c] = (T[c] + 63) >> 6;
                }
                wave_lds_sync();
                lstamp(2);
                // (each step's previous occurrence in its window: the plan's look-back, pv)
                lstamp(3);
                // MODE_LSGD: the step's shrink and s, in step order (SGD.scala:106, 119-120)
                // on the uniform running s, so every partition forms the same sequence
                double lB = 0.0, lAE = 0.0, lY = 0.0;
                if (MODE == MODE_LSGD) {
                    const double step = valid ? 1.0 / (a.lambda * (a.t0 + (double)(j + 1))) : 0.0;
                    const double scale = valid ? 1.0 - step * a.lambda : 1.0;
                    double sprev = 1.0, snew = 1.0;
                    int32_t kprev = 1;
                    for (int t = 0; t < kGB; ++t) {
                        const double sc = readlane_d(scale, t);
                        if (lane == t) {
                            sprev = ls;
                            kprev = lkeep;
                        }
                        if (sc == 0.0) {  // w *= 0: wInit and v dropped, s restarts
                            ls = 1.0;
                            lkeep = 0;
                        } else {
                            ls *= sc;
                        }
                        if (lane == t) snew = ls;
                    }
                    // eval = 1 - y x.w = AE - B (base + corrections); violators scatter
                    // u = y step / s (SGD.scala:115, 124-129)
                    lB = valid ? y * sprev : 0.0;
                    lAE = valid ? 1.0 - lB * (kprev ? xw : 0.0) : 0.0;
                    lY = valid ? (y * step) / snew : 0.0;
                }
                if (lane < kGB) {
                    GRec& R = S.rec[(b % kGRing) * kGB + lane];
                    double B = 0.0, E = 0.0, Y = 0.0;
                    if (MODE == MODE_LSGD) {
                        B = lB;
                        Y = lY;
                        R.AE = lAE;
                        R.YA = 0.0;
                    } else if (valid) {
                        gram_row_consts<MODE>(a, y, q, xw, B, E, Y);
                    }
                    R.B = B;
                    R.E = E;
                    R.Y = Y;
                    R.r = r;
                    R.fw = -1;
                    R.fwd = 0;
                }
                lstamp(4);
                {
                    // each lane group its class's layout: one store per field for all classes
                    int32_t tl = T[0], nl_ = nu[0], pl = nu[0] <= kGMaxU ? cursor[0] : -1;
#pragma unroll
                    for (int c = 1; c < kGNC; ++c)
                        if (cl == c) {
                            tl = T[c];
                            nl_ = nu[c];
                            pl = nu[c] <= kGMaxU ? cursor[c] : -1;
                        }
                    if (cl < kGNC) {
                        GLay& L = S.lay[b % kGRing][cl];
                        L.sx[i + 1] = incl;
                        L.sb[i] = beg + zbl;
                        if (i == 0) {
                            L.sx[0] = 0;
                            L.T = tl;
                            L.nu = nl_;
                            L.pos = pl;
                        }
                    }
#pragma unroll
                    for (int c = 0; c < kGNC; ++c)
                        if (nu[c] <= kGMaxU) cursor[c] += nu[c] * 64;
                }
                wave_lds_sync();
                // mark the earlier occurrence: step pv forwards its new alpha here
                if (MODE != MODE_LSGD && valid && pv >= 0) {
                    const int32_t js = pv;
                    S.rec[((js / kGB) % kGRing) * kGB + (js % kGB)].fw = j & (2 * kGSlots - 1);
                }
            }
            lstamp(5);
            const int32_t xg = b - kGGt;  // Gram rows of batch xg: 16 rows x 64 slots
            if (MODE != MODE_MBCD && xg >= 0 && xg < NB) {
                const uint32_t* src = (const uint32_t*)(gt + (size_t)xg * kGB * kGW);
                uint32_t* dst = (uint32_t*)&S.gring[xg % kGGt][0][0];
                static_assert((2 * kGB * kGW) % 256 == 0, "Gram-row DMA");
#pragma unroll
                for (int t = 0; t < 2 * kGB * kGW / 256; ++t) lds_dma16(src + t * 256 + 4 * lane, dst + t * 256);
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[kCLoad], b + 1);
            lstamp(6);
        }
        if (pw && lane == 0 && h == 0)
            for (int i = 0; i < 7; ++i) a.prof[(size_t)k * kProfStride + 56 + i] = lph[i];
        if (MODE == MODE_LSGD && lane == 0) {  // read after the final barrier
            S.lsgd_s = ls;
            S.lsgd_keep = lkeep;
        }
    } else if (role >= kRFetch && role < kRIdle) {
        // -------------------------------------------------------- fetch --
        const int c = role - kRFetch;
        for (int32_t x = 0; x < NB; ++x) {
            if (!wait_ge(&S.cnt[kCLoad], x + 1, abortf, a.status, pw)) break;
            const GLay& L = S.lay[x % kGRing][c];
            const int32_t pos = L.pos, nu = L.nu, T = L.T;
            if (pos >= 0 && nu > 0) {
                // sub-ring space: positions up to pos + 64 nu - 64 kGSub released by the memory wave
                if (!wait_ge(&S.cnt[kCFreed + c], pos + nu * 64 - kGSub * 64, abortf, a.status, pw)) break;
                for (int32_t u = 0; u < nu; ++u) {
                    const int32_t q = u * 64 + lane;
                    uint8_t* ub = S.ring[ring_unit<NC>(c, pos, u)];
                    const int o = gram_owner(L.sx, q);
                    if (q < T) {
                        const int64_t e = L.sb[o] + (q - L.sx[o]);
                        lds_dma4(a.col + e, ub + kGOCol);
                        lds_dma4((const uint32_t*)(a.val + e), ub + kGOLo);
                        lds_dma4((const uint32_t*)(a.val + e) + 1, ub + kGOHi);
                    }
                    ub[kGORow + lane] = q < T ? (uint8_t)o : (uint8_t)0xFF;
                }
                vm_drain();  // the DMA writes are in LDS
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[kCFetch + c], x + 1);
        }
    } else if (role >= kRMem && role < kRFetch) {
        // ------------------------------------------------------- memory --
        const int c = role - kRMem;  // this wave's column class
        const int bslot = MIRROR ? gram_mirror_run(c, h) : c;  // its partial base: class c, or (mirrored) its run
        // (mirrored) hand batch x's partial base to the other half: 16 doubles as 32
        // tagged 8-byte granules, sc1 stores (no drain, no flag: the tag is the flag)
        auto publish = [&](int32_t x) {
            if (!MIRROR || lane >= 2 * kGB) return;
            const double v = S.base[bslot][(x % kGNB) * kGB + (lane >> 1)];
            const uint64_t bits = (uint64_t)__double_as_longlong(v);
            const uint32_t tag = ((uint32_t)(a.xtag_epoch & 0xFFF) << 20) | (uint32_t)(x + 1);
            const uint64_t gr = ((uint64_t)tag << 32) | ((lane & 1) ? (bits >> 32) : (bits & 0xFFFFFFFFull));
            uint64_t* gp = a.xbase + (((size_t)k * kGramRuns + bslot) * kXbR + (x % kXbR)) * (2 * kGB) + lane;
            __hip_atomic_store(gp, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        const bool bases = MODE != MODE_MBCD;
        double hv[kGMaxU], dw[kGMaxU];  // in-flight gathers: staged value (x hot deltaW), loaded deltaW (or 1)
        uint32_t hrow[(kGMaxU + 5) / 6];  //   and their rows (5 bits per unit, 31 = no entry)
        int32_t xin = -1;               // batch whose gathers are in flight
        int32_t xnu = 0;                //   and its 64-entry units
        double(*part)[kGPart] = S.part[c];
        auto fetched = [&](int32_t x) { return wait_ge(&S.cnt[kCFetch + c], x + 1, abortf, a.status, pw); };
        uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint64_t tph = 0;
        auto stamp = [&](int i) {
            if (a.prof) {
                const uint64_t t = __builtin_readcyclecounter();
                ph[i] += t - tph;
                tph = t;
            }
        };
        // (diagnostic build: the atomics / products phase split in four)
        auto dstamp = [&](int i) {
            if (COCOA_DIAG_ON) stamp(i);
        };
        // KIND 0: a class mixing LDS-resident and slice columns (1 / 2, the round-5
        // hot-only / cold-only runs of COCOA_HOTRUNS, are gone); the mirrored
        // half's hot-only (LDS) / cold-only (slice) class of the COCOA_HOTRUNS layout
        auto mem_loop = [&](auto kind_c) {
            constexpr int KIND = decltype(kind_c)::value;
            auto dw_addk = [&](int32_t col, double v) {
                if (KIND == 1 || (KIND == 0 && HOTLDS && col < hotc))
                    __hip_atomic_fetch_add(hotl + hix(col), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    unsafeAtomicAdd(dwk + col, v);
            };
            auto dw_getk = [&](int32_t col) {
                return (KIND == 1 || (KIND == 0 && HOTLDS && col < hotc)) ? hotl[hix(col)] : dw_load(dwk + col);
            };
            for (int32_t b = 0; b < NB; ++b) {
                if (!wait_ge(&S.cnt[kCChain], b + 1, abortf, a.status, pw)) break;  // the chain finished batch b
                if (a.prof) tph = __builtin_readcyclecounter();
                // Scatter of batch b first, its LDS reads before the drain: the ring entries
                // and coefficients of b are read into registers while the gathers of batch
                // b+3 are still in flight; the drain then only orders those gathers before
                // b's atomics (the per-column order of the slice), and the products of b+3
                // are formed behind the atomics.
                {
                    const GLay& L = S.lay[b % kGRing][c];
                    const double* cf = S.coef + (b % kGRing) * (2 * kGB);
                    const int32_t pos = L.pos, nu_all = L.nu;
                    // (diag bit 4, timing only: half the units, as if the run were split in two)
                    const int32_t nu = (COCOA_DIAG_ON && (a.diag & 4)) ? (nu_all + 1) / 2 : nu_all;
                    int32_t scl[kGMaxU];
                    double sp[kGMaxU];
                    if (pos >= 0) {
                        if (!fetched(b)) break;
    #pragma unroll
                        for (int u0 = 0; u0 < kGMaxU; u0 += 4) {
                            if (u0 < nu) {
                                int rw[4];
                                double vl[4];
    #pragma unroll
                                for (int t = 0; t < 4; ++t) {
                                    uint32_t r8;
                                    ring_get(S, ring_unit<NC>(c, pos, u0 + t), lane, scl[u0 + t], vl[t], r8);
                                    rw[t] = r8 | gram_pad(u0 + t, nu);
                                }
    #pragma unroll
                                for (int t = 0; t < 4; ++t) {
                                    // a lane past the batch (row 0xFF) reads a zero slot; its ring
                                    // entry was never written, so it is dropped by the coefficient
                                    const double cc = cf[rw[t] & (2 * kGB - 1)];
                                    sp[u0 + t] = vl[t] * cc;
                                    if (cc == 0.0) scl[u0 + t] = -1;
                                }
                            }
                        }
                    }
                    stamp(3);
                    // staged: the ring entries and coefficients are in registers now, so the
                    // slots go back before the atomics (their release would otherwise also
                    // wait for this wave's LDS atomics into the hot columns)
                    wave_lds_sync();
                    if (COCOA_EARLY_RELEASE && pos >= 0 && lane == 0) {
                        lds_release(&S.cnt[kCScat + c], b + 1);  // coefficient / record / layout slot consumed
                        lds_release(&S.cnt[kCFreed + c], pos + nu_all * 64);
                    }
                    if (bases) vm_drain();  // the gathers of batch b+kGNB-1 have read the slice (MbCD: no gathers)
                    stamp(0);
                    if (pos >= 0) {
    #pragma unroll
                        for (int u = 0; u < kGMaxU; ++u)
                            if (u < nu && scl[u] >= 0 && !(COCOA_DIAG_ON && (a.diag & 1))) dw_addk(scl[u], sp[u]);
                        dstamp(4);
                    } else {
                        for (int i = 0; i < kGB; ++i) {
                            const double cv = cf[i];
                            if (cv == 0.0) continue;
                            const int32_t z = L.sx[i + 1] - L.sx[i];
                            const int64_t rb = L.sb[i];
                            for (int32_t e = lane; e < z; e += 64) dw_addk(a.col[rb + e], a.val[rb + e] * cv);
                        }
                    }
                    if (!COCOA_EARLY_RELEASE || pos < 0) {  // (the direct path read the layout and coefficients until here)
                        wave_lds_sync();
                        if (lane == 0) {
                            lds_release(&S.cnt[kCScat + c], b + 1);
                            if (!COCOA_EARLY_RELEASE && pos >= 0) lds_release(&S.cnt[kCFreed + c], pos + nu_all * 64);
                        }
                    }
                }
                // 1. products of the gathers in flight -> this class's part of the base of
                //    batch xin.  Each unit's product goes to (its row, lane mod 32) with a
                //    fire-and-forget LDS add (lanes l and l + 32 share a slot: different
                //    LDS lane groups, no conflict); 4 lanes per row add the slots up.
                if (xin >= 0) {
                    if (lane < kGPart) {
    #pragma unroll
                        for (int i = 0; i < kGB; ++i) part[i][lane] = 0.0;
                    }
                    wave_lds_sync();
                    dstamp(5);
    #pragma unroll
                    for (int u = 0; u < kGMaxU; ++u) {
                        if (u < xnu) {
                            const int row = min((int)((hrow[u / 6] >> (5 * (u % 6))) & 31u), kGB);  // 31: no entry
                            __hip_atomic_fetch_add(&part[row][lane & (kGPart - 1)], hv[u] * dw[u], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    }
                    wave_lds_sync();
                    dstamp(6);
                    const int rr = lane >> 2, qq = (lane & 3) * (kGPart / 4);
                    double s4 = 0.0;
    #pragma unroll
                    for (int t = 0; t < kGPart / 4; ++t) s4 += part[rr][qq + t];
                    s4 += dpp_row_d<0xB1>(s4);  // quad_perm [1,0,3,2]
                    s4 += dpp_row_d<0x4E>(s4);  // quad_perm [2,3,0,1]
                    if ((lane & 3) == 0) S.base[bslot][(xin % kGNB) * kGB + rr] = s4;
                    wave_lds_sync();
                    if (lane == 0) lds_release(&S.cnt[kCBase + bslot], xin + 1);
                    publish(xin);
                    xin = -1;
                }
                stamp(1);
                // 3. gathers of batch x = b + kGNB on this class's columns: they see batch
                //    b's updates (issued above, same wave, same addresses) and nothing later
                //    (the next atomics go out after step 1 has consumed these loads)
                const int32_t x = b + kGNB;
                if (bases && x < NB) {
                    const GLay& L = S.lay[x % kGRing][c];
                    const int32_t pos = L.pos, nu = (COCOA_DIAG_ON && (a.diag & 4)) ? (L.nu + 1) / 2 : L.nu;
                    if (pos >= 0) {
                        if (!fetched(x)) break;
                        dstamp(7);
    #pragma unroll
                        for (int w = 0; w < (kGMaxU + 5) / 6; ++w) hrow[w] = 0xFFFFFFFFu;  // units past nu: never read
                        // groups of 4 units (a group past the batch is skipped whole)
    #pragma unroll
                        for (int u0 = 0; u0 < kGMaxU; u0 += 4) {
                            if (u0 < nu) {
                                int rw[4];
                                int32_t cl[4];
                                double vl[4];
    #pragma unroll
                                for (int t = 0; t < 4; ++t) {
                                    uint32_t r8;
                                    ring_get(S, ring_unit<NC>(c, pos, u0 + t), lane, cl[t], vl[t], r8);
                                    rw[t] = r8 | gram_pad(u0 + t, nu);
                                }
                                double hx[4];
    #pragma unroll
                                for (int t = 0; t < 4; ++t) {
                                    const int u = u0 + t;
                                    const int32_t cc = rw[t] < kGB ? cl[t] : -1;
                                    // a hot (LDS) or empty lane loads the constant 1 -- one register
                                    // never mixes a global load with an LDS read (that would serialise)
                                    if (KIND == 1) {  // hot-only wave: LDS
                                        dw[u] = 1.0;
                                        hx[t] = hotl[cc >= 0 ? cc : 0];
                                    } else if (KIND == 2) {  // cold-only wave: the slice
                                        if (!(COCOA_DIAG_ON && (a.diag & 2))) dw[u] = dw_load(dwk + (cc >= 0 ? cc : 0));
                                    } else if (HOTLDS) {
                                        if (!(COCOA_DIAG_ON && (a.diag & 2))) dw[u] = dw_load(cc >= hotc ? dwk + cc : &g_gram_one);
                                        hx[t] = hotl[(cc >= 0 && cc < hotc) ? hix(cc) : 0];
                                    } else if (!(COCOA_DIAG_ON && (a.diag & 2))) {
                                        // a lane past the batch loads column 0: its product goes to the sink row
                                        dw[u] = dw_load(dwk + (cc >= 0 ? cc : 0));
                                    }
                                }
                                __builtin_amdgcn_sched_barrier(0);  // all reads of the group out before the products
    #pragma unroll
                                for (int t = 0; t < 4; ++t) {
                                    const int u = u0 + t;
                                    const bool ok = rw[t] < kGB;
                                    if (KIND == 1)
                                        hv[u] = ok ? vl[t] * hx[t] : 0.0;
                                    else if (KIND == 2)
                                        hv[u] = vl[t];
                                    else if (HOTLDS)
                                        hv[u] = ok ? ((cl[t] < hotc) ? vl[t] * hx[t] : vl[t]) : 0.0;
                                    else
                                        hv[u] = vl[t];  // past the batch: any value, summed into the sink row
                                    hrow[u / 6] = (hrow[u / 6] & ~(31u << (5 * (u % 6)))) | ((uint32_t)(ok ? rw[t] : 31) << (5 * (u % 6)));
                                }
                            }
                        }
                        xin = x;
                        xnu = nu;
                    } else {
                        // too long to stage: gathered and summed here
                        double* bs = S.base[bslot] + (x % kGNB) * kGB;
                        for (int i = 0; i < kGB; ++i) {
                            const int32_t z = L.sx[i + 1] - L.sx[i];
                            const int64_t rb = L.sb[i];
                            double acc = 0.0;
                            for (int32_t e = lane; e < z; e += 64) acc = fma(a.val[rb + e], dw_getk(a.col[rb + e]), acc);
                            const double t = wave_sum(acc);
                            if (lane == 0) bs[i] = t;
                        }
                        wave_lds_sync();
                        if (lane == 0) lds_release(&S.cnt[kCBase + bslot], x + 1);
                        publish(x);
                    }
                }
                stamp(2);
            }
        };
        mem_loop(std::integral_constant<int, 0>{});
        vm_drain();  // the last atomics land before the kernel ends
        if (a.prof && lane == 0) {
            for (int i = 0; i < 4; ++i) a.prof[(size_t)k * kProfStride + 64 + 4 * c + i] = ph[i];
            if (COCOA_DIAG_ON && c < 2)
                for (int i = 4; i < 8; ++i) a.prof[(size_t)k * kProfStride + 96 + 4 * c + i - 4] = ph[i];
        }
    } else if (MIRROR && role == kRRelay) {
        // -------------------------------------------------------- relay --
        // the other half's partial bases (its runs 2 c + hp, c < NC) of every batch
        // x >= kGNB, from its tagged granules into this half's LDS, two runs per poll
        if (MODE != MODE_MBCD) {
            const int hp = 1 - h;
            const int row = (lane >> 1) & (kGB - 1), half = lane & 1;
            const uint32_t thi = (uint32_t)(a.xtag_epoch & 0xFFF) << 20;
            bool ok = true;
            for (int32_t x = kGNB; ok && x < NB; ++x) {
                // base slot x % kGNB held batch x - kGNB: the chain is done with it
                if (!wait_ge(&S.cnt[kCChain], x - kGNB + 1, abortf, a.status, pw)) break;
                const uint32_t tag = thi | (uint32_t)(x + 1);
#pragma unroll
                for (int p = 0; p < NC / 2; ++p) {
                    const int run0 = gram_mirror_run(2 * p, hp), run1 = gram_mirror_run(2 * p + 1, hp);
                    const int run = (lane >> 5) ? run1 : run0;  // lanes 0-31: the pair's first run, 32-63: its second
                    uint64_t* gp = a.xbase + (((size_t)k * kGramRuns + run) * kXbR + (x % kXbR)) * (2 * kGB) + (lane & 31);
                    uint64_t gv = 0;
                    const uint64_t t0 = pw ? __builtin_readcyclecounter() : 0;
                    for (uint32_t it = 0;; ++it) {  // sc1 polls of the 64 granules until every tag matches
                        gv = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (__all((uint32_t)(gv >> 32) == tag)) break;
                        if (__hip_atomic_load(abortf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                            ok = false;
                            break;
                        }
                        if (it > (1u << 24)) {
                            __hip_atomic_store(abortf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (lane == 0) __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            ok = false;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    if (pw) *pw += __builtin_readcyclecounter() - t0;
                    if (!ok) break;
                    const uint32_t mine = (uint32_t)gv, other = (uint32_t)__shfl_xor((int)mine, 1, 64);
                    if (half == 0) S.base[run][(x % kGNB) * kGB + row] = __hiloint2double((int)other, (int)mine);
                    wave_lds_sync();
                    if (lane == 0) {
                        lds_release(&S.cnt[kCBase + run0], x + 1);
                        lds_release(&S.cnt[kCBase + run1], x + 1);
                    }
                }
            }
        }
    } else if (role == kRChain) {
        // -------------------------------------------------------- chain --
        // lane = window slot (step mod kGW): sdot = base + Gram corrections
        const int32_t ahead = MODE != MODE_MBCD ? kGGt + 2 : 0;  // kCLoad needed for batch g: g + 1 + kGNB (records), g + 6 (Gram rows)
        bool ok = wait_ge(&S.cnt[kCLoad], MODE != MODE_MBCD ? ahead : min(kGNB + 1, NB), abortf, a.status, pw);
        double acc = 0.0;
        if (MODE != MODE_LSGD && ok && lane < kGW && lane / kGB < NB) {  // (local SGD: the loader sets AE)
            GRec& R = S.rec[(lane / kGB) * kGB + (lane & (kGB - 1))];
            const double aa = alv[R.r];
            R.AE = aa - R.E;
            R.YA = R.Y * aa;
            if (PROJ) R.AA = aa;
        }
        wave_lds_sync();
        // (diagnostic build: the chain's cycles per part of a batch -- waits, head
        // loads, the 16 steps, the tail)
        uint64_t cph[4] = {0, 0, 0, 0};
        uint64_t ctp = (COCOA_DIAG_ON && pw) ? __builtin_readcyclecounter() : 0;
        auto cstamp = [&](int i) {
            if (COCOA_DIAG_ON && pw) {
                const uint64_t t = __builtin_readcyclecounter();
                cph[i] += t - ctp;
                ctp = t;
            }
        };
        // One batch.  Alpha of batch g+3 is loaded at the start of batch g (rows met
        // again in batches g .. g+3 are forwarded instead) and written into its
        // records at the end of batch g+1, a batch after the load: `aissue` / `afill`
        // alternate between two registers (no copy of a register still being loaded).
        auto batch = [&](int32_t g, double& aissue, const double& afill) -> bool {
            const int q4 = g % kGNB;          // this batch's quarter of the lanes
            const bool mine = lane / kGB == q4;
            if (MODE != MODE_MBCD) {
                if (!all_ge_now(&S.cnt[kCBase], NRUN, g + 1)) {
#pragma unroll
                    for (int c = 0; c < NRUN; ++c)  // (diagnostics: a mirrored half's own runs have parity h)
                        if (!wait_ge(&S.cnt[kCBase + c], g + 1, abortf, a.status,
                                     !pw ? nullptr : (MIRROR && (c & 1) != h) ? &wait_base_remote : &wait_base_local))
                            return false;
                }
                if (!wait_ge(&S.cnt[kCLoad], g + ahead, abortf, a.status, pw ? &wait_load : nullptr)) return false;
            } else if (!wait_ge(&S.cnt[kCLoad], min(g + kGNB + 1, NB), abortf, a.status, pw)) {
                return false;
            }
            // coefficient ring slot g % kGRing held batch g - kGRing: consumed by every memory wave?
            if (!all_ge_now(&S.cnt[kCScat], kGNC, g - kGRing + 1)) {
#pragma unroll
                for (int c = 0; c < kGNC; ++c)
                    if (!wait_ge(&S.cnt[kCScat + c], g - kGRing + 1, abortf, a.status, pw ? &wait_scat : nullptr))
                        return false;
            }
            cstamp(0);
            if (MODE != MODE_LSGD) {
                const int32_t g4 = g + kGNB;
                const GRec& R4 = S.rec[(g4 % kGRing) * kGB + (lane & (kGB - 1))];
                aissue = alv[(mine && g4 < NB) ? R4.r : nl];  // one load for every lane (the sink otherwise)
            }
            if (mine) {
                // (mirrored: runs in order 0..3 on both halves, so both chains add alike)
                double bsum = S.base[0][lane];
#pragma unroll
                for (int c = 1; c < NRUN; ++c) bsum += S.base[c][lane];
                acc += bsum;
            }
            double gcur[kGB];
            const int gl = min(lane, kGW - 1);  // lanes past the window: any value (never read back)
#pragma unroll
            for (int i = 0; i < kGB; ++i) gcur[i] = MODE != MODE_MBCD ? S.gring[g % kGGt][i][gl] : 0.0;
            double* cfo = S.coef + (g % kGRing) * (2 * kGB);
            const int slot0 = q4 * kGB;
            // this batch's records in the lanes of its quarter (lane slot0 + i holds step
            // i, next to its accumulator): every step evaluates the update rule on all
            // lanes at once and broadcasts one coefficient
            double rB = 0.0, rY = 0.0, rAE = 0.0, rYA = 0.0, rE = 0.0, rAA = 0.5;
            int32_t rR = nl, rF = -1;
            if (mine) {
                const GRec& R = S.rec[(g % kGRing) * kGB + (lane & (kGB - 1))];
                rB = R.B;
                rY = R.Y;
                rAE = R.AE;
                rYA = R.YA;
                rE = R.E;
                if (PROJ) rAA = R.AA;
                rR = R.r;
                rF = R.fw;
            }
            lgkm_drain();  // records and Gram rows in: no LDS wait inside the steps
            const uint32_t fwm = (uint32_t)(__ballot(mine && rF >= 0) >> slot0) & 0xFFFFu;  // steps that forward
            cstamp(1);
            // 16 steps, padding steps included (their record is inert: B = Y = YA = 0,
            // row = the sink).  Step i: nt = clamp(AE - B sdot) with sdot = acc on its
            // lane; c = Y nt - YA; acc += c G(., j).  Lanes of steps <= i have G = 0, so
            // a step's lane keeps its final sdot and the batch's nt / c are recomputed
            // once at the end for the alpha and coefficient stores.
#pragma unroll
            for (int i = 0; i < kGB; ++i) {
                if (MODE == MODE_LSGD) {
                    // SGD.scala:115, 124-129: eval = 1 - y x.w > 0 scatters u = y step / s
                    const double ev = fma(-rB, acc, rAE);
                    const double cf = readlane_d(ev > 0.0 ? rY : 0.0, slot0 + i);
                    acc = fma(cf, gcur[i], acc);
                    continue;
                }
                // CoCoA.scala:159-186 / MinibatchCD.scala:104-123 (see above)
                const double nt = gram_rule<PROJ>(fma(-rB, acc, rAE), rAA);
                if (MODE != MODE_MBCD) {
                    const double cf = readlane_d(fma(rY, nt, -rYA), slot0 + i);
                    acc = fma(cf, gcur[i], acc);
                }
                if (fwm & (1u << i)) {
                    // a later step (< kGWin steps on) samples the same row: its aa is nt
                    const double nts = readlane_d(nt, slot0 + i);
                    const int32_t sf = __builtin_amdgcn_readlane(rF, slot0 + i);
                    const int32_t sp = g * kGB + ((sf - g * kGB) & (2 * kGSlots - 1));
                    if (sp < (g + 1) * kGB) {
                        if (lane == slot0 + (sp - g * kGB)) {  // this batch: its lane's registers
                            rAE = nts - rE;
                            rYA = rY * nts;
                            if (PROJ) rAA = nts;
                        }
                        if (lane == slot0 + i) rR = nl;  // the later step stores the row's alpha
                    } else {
                        GRec& T = S.rec[((sp / kGB) % kGRing) * kGB + (sp % kGB)];
                        const double tE = T.E, tY = T.Y;
                        T.AE = nts - tE;
                        T.YA = tY * nts;
                        if (PROJ) T.AA = nts;
                        T.fwd = 1;
                    }
                }
            }
            cstamp(2);
            if (MODE == MODE_LSGD) {
                const double ev = fma(-rB, acc, rAE);
                if (mine) cfo[lane & (kGB - 1)] = ev > 0.0 ? rY : 0.0;
            } else {
                const double nt = gram_rule<PROJ>(fma(-rB, acc, rAE), rAA);
                const double cf = fma(rY, nt, -rYA);
                if (mine) {
                    alv[rR] = nt;
                    cfo[lane & (kGB - 1)] = cf;
                }
            }
            wave_lds_sync();
            if (lane == 0) lds_release(&S.cnt[kCChain], g + 1);
            // this batch's lanes now accumulate for batch g+kGNB
            if (mine) acc = 0.0;
            // alpha of batch g+kGNB-1 (loaded at the start of batch g-1 by the lanes
            // of batch g-1), unless a forward already set it
            const int32_t g3 = g + kGNB - 1;
            if (MODE != MODE_LSGD && g >= 1 && g3 < NB && lane / kGB == (g + kGNB - 1) % kGNB) {
                GRec& R3 = S.rec[(g3 % kGRing) * kGB + (lane & (kGB - 1))];
                if (!R3.fwd) {
                    R3.AE = afill - R3.E;
                    R3.YA = R3.Y * afill;
                    if (PROJ) R3.AA = afill;
                }
            }
            wave_lds_sync();
            cstamp(3);
            return true;
        };
        double aA = 0.0, aB = 0.0;
        for (int32_t g = 0; ok && g < NB; g += 2) {
            if (!batch(g, aA, aB)) break;
            if (g + 1 < NB && !batch(g + 1, aB, aA)) break;
        }
        if (COCOA_DIAG_ON && pw && lane == 0 && h == 0)
            for (int i = 0; i < 4; ++i) a.prof[(size_t)k * kProfStride + 50 + i] = cph[i];
    }
    if (a.prof && lane == 0 && h == 0 && wv < kGWaves) {
        // [k][128]: waves at 4 wv, chain waits at 48, loader phases at 56, memory phases at 64 + 4 c
        uint64_t* pr = a.prof + (size_t)k * kProfStride + wv * 4;
        pr[0] = wait_cycles + (role == kRChain ? wait_base_local + wait_base_remote + wait_load + wait_scat : 0);
        if (role == kRChain) {
            a.prof[(size_t)k * kProfStride + 48] = wait_load;
            a.prof[(size_t)k * kProfStride + 49] = wait_scat;
        }
        if (role == kRChain || role == kRLoader) {  // (loader: [2] its vm_drain cycles)
            pr[2] = wait_base_local;
            pr[3] = wait_base_remote;
        }
        pr[1] = __builtin_readcyclecounter() - t_start;
    }
    __syncthreads();
    if (MODE == MODE_LSGD) {
        // deltaW = w - wInit = s (keep wInit + v) - wInit (SGD.scala:133), the slice
        // holding v (L2: read past L1, like the gathers)
        const double sH = S.lsgd_s, f = S.lsgd_keep ? sH - 1.0 : -1.0;
        if (!MIRROR) {
            for (int64_t j = tid; j < a.d; j += NTH) {
                const double v = (HOTLDS && j < hot) ? hotl[j] : dw_load(dwk + j);
                dwk[j] = fma(sH, v, f * a.w[j]);
            }
        } else {
            // mirrored: this half's columns (parity h) only, their hot part in its
            // image; write-through, the other half writes the interleaved words
            for (int64_t j = 2 * (int64_t)tid + h; j < a.d; j += 2 * NTH) {
                const double v = (HOTLDS && j < hotc) ? hotl[hix((int32_t)j)] : dw_load(dwk + j);
                __hip_atomic_store(dwk + j, fma(sH, v, f * a.w[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    if (!MIRROR) {
        for (int32_t i = tid; i < hot; i += NTH) dwk[i] = hotl[i];  // the slice is zero there: plain stores
    } else {
        // this half's columns (parity h) only, write-through: the other half's
        // workgroup writes the interleaved words of the same lines, maybe from
        // another XCD's L2
        if (PAR) {
            for (int32_t j = tid; j < hot && 2 * (int64_t)j + h < a.d; j += NTH)
                __hip_atomic_store(dwk + 2 * j + h, hotl[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            for (int32_t i = 2 * tid + h; i < hot; i += 2 * NTH)
                __hip_atomic_store(dwk + i, hotl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (MIRROR && h != 0) return;  // alpha: the first half's (both hold the same)
    if (MIRROR && MODE == MODE_MBCD) {  // (half 1 has copied alphaOld: see above)
        if (tid == 0) {
            for (uint32_t it = 0; __hip_atomic_load(mflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != mtag; ++it) {
                if (it > (1u << 24)) {
                    __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
    }
    // alpha = alphaOld + (alpha - alphaOld) * scaling (CoCoA.scala:101, MinibatchCD.scala:127-128)
    if (a.raw_alpha) {
        for (int32_t i = tid; i < nl; i += NTH) a.alpha[p0 + i] = alv[i];
    } else {
        for (int32_t i = tid; i < nl; i += NTH) {
            const double old = a.alpha[p0 + i];
            a.alpha[p0 + i] = old + ((alv[i] - old) * a.scaling);
        }
    }
}

}  // namespace cocoa
