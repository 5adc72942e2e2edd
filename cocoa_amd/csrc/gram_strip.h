// Gram rows by partition strips (fast mode, solver_gram.h's window).
//
// gram_kernel (solver_gram.h) gives every (partition, batch) its own
// workgroup: the batch's 16 updater rows are hashed and the 48 rows of the
// window [16 g, 16 g + 48) probe the hash, so every row is loaded and probed
// by the three workgroups whose windows hold it.  Here one workgroup takes a
// strip of kGSB = 2 consecutive batches of one partition: the 32 updater rows
// of the strip are hashed once and the 64 rows of the strip's windows
// [16 g0, 16 g0 + 64) probe once, so a row is loaded and probed by two
// workgroups instead of three.  Same output, same layout:
//   Gt[k][j][slot] = x_s . x_j for the partner s of updater j's window
//   [16 floor(j/16), +48) with s > j (slot = s mod 48); 0 otherwise,
// the same entry products summed in another order (fast mode).
#pragma once
#include "solver_gram.h"

namespace cocoa {

constexpr int kGSB = 2;                      // batches per strip
constexpr int kGSU = kGSB * kGB;             // updaters per strip (32)
constexpr int kGSP = kGSU + kGW - kGB;       // partner rows of the strip's windows (64)
constexpr int kGSThreads = 1024;             // 16 waves, one workgroup per CU
constexpr int kGSNU = 6;                     // kGSThreads-entry units in registers (6,144 entries)
constexpr int kGSCH = kGSNU * kGSThreads;
constexpr int kGSTile = 4096;                // updater positions per hash tile (32 rows of ~76 entries: one tile)
constexpr int kGSTable = 8192;               // hash slots
static_assert(kGSP == 64, "the strip's partners are one wave's lanes");
static_assert(kGSNU % 2 == 0, "owners packed 4 per word");

struct GramStripLds {
    double XP[kGSP][kGHotS];                 // hot image of the partners (updaters = rows 0..31)
    double acc[kGSU][kGW];                   // G of the updaters against their windows
    int32_t tkey[kGSTable];
    int32_t thead[kGSTable];
    double eval[kGSTile];
    int16_t enext[kGSTile];
    int8_t eu[kGSTile];
    int64_t pbeg[kGSP];
    int32_t pcum[kGSP + 1];
};
static_assert(sizeof(GramStripLds) <= 160 * 1024, "gram_strip_kernel LDS");
static_assert(kGSTable == 8192 && kGSTile <= 32767, "gs_hash bits / int16 list links");
__device__ __forceinline__ uint32_t gs_hash(int32_t c) { return ((uint32_t)c * 2654435761u) >> 19; }  // 13 bits

__global__ __launch_bounds__(kGSThreads, 1) void gram_strip_kernel(GramArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    GramStripLds& L = *(GramStripLds*)lds_raw;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // XCD-aware order as in gram_kernel: one partition's consecutive strips on one XCD
    int k, st;
    {
        const int64_t b = blockIdx.x;
        if (a.K % 8 == 0) {
            const int64_t kx = a.K / 8, i = b / 8;
            k = (int)((b % 8) + 8 * (i % kx));
            st = (int)(i / kx);
        } else {
            k = (int)(b % a.K);
            st = (int)(b / a.K);
        }
    }
    const int32_t H = a.H;
    const int32_t j0 = st * kGSU;
    const int32_t P = min(kGSP, H - j0);  // partners [j0, j0 + P)
    const int32_t U = min(kGSU, H - j0);  // updaters = partners [0, U)
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
    for (int i = tid; i < kGSP * kGHotS; i += kGSThreads) (&L.XP[0][0])[i] = 0.0;
    for (int i = tid; i < kGSU * kGW; i += kGSThreads) (&L.acc[0][0])[i] = 0.0;
    __syncthreads();
    const int32_t T = L.pcum[P], QU = L.pcum[U];
    // registers: a chunk of packed positions [qa, qa + kGSCH): column (-1 past
    // T), value, owner partner (4 per word)
    int32_t cc[kGSNU];
    double vv[kGSNU];
    uint32_t ow[(kGSNU + 3) / 4];
    int32_t reg_qa = -1;
    auto load = [&](int32_t qa) {
        if (reg_qa == qa) return;
        reg_qa = qa;
        int o[kGSNU];
#pragma unroll
        for (int u = 0; u < kGSNU; ++u) {  // owners: independent binary searches, interleaved
            const int32_t q = min(qa + u * kGSThreads + tid, max(T - 1, 0));
            int lo = 0;
#pragma unroll
            for (int s2 = kGSP / 2; s2 >= 1; s2 >>= 1)
                if (L.pcum[lo + s2] <= q) lo += s2;
            o[u] = lo;
        }
#pragma unroll
        for (int u = 0; u < kGSNU; ++u) {
            const int32_t q = qa + u * kGSThreads + tid;
            const bool ok = q < T;
            const int64_t e = ok ? L.pbeg[o[u]] + (q - L.pcum[o[u]]) : 0;
            cc[u] = ok ? a.col[e] : -1;
            vv[u] = ok ? a.val[e] : 0.0;
        }
#pragma unroll
        for (int w = 0; w < (kGSNU + 3) / 4; ++w) ow[w] = 0;
#pragma unroll
        for (int u = 0; u < kGSNU; ++u) ow[u / 4] |= (uint32_t)o[u] << (8 * (u % 4));
    };
    auto owner_of = [&](int u) { return (int)((ow[u / 4] >> (8 * (u % 4))) & 0xFFu); };
    // hot image (duplicate columns of a row add up, as in the dot)
    for (int32_t qa = 0; qa < T; qa += kGSCH) {
        load(qa);
#pragma unroll
        for (int u = 0; u < kGSNU; ++u)
            if (cc[u] >= 0 && cc[u] < kGHot) atomicAdd(&L.XP[owner_of(u)][cc[u]], vv[u]);
    }
    // updater u (strip-relative) pairs with partner p when p is in u's window
    // [16 floor(u/16), +48) and p > u; its accumulator column is p - 16 floor(u/16)
    // cold part, one hash tile of updater positions at a time
    for (int32_t ta = 0; ta < QU; ta += kGSTile) {
        for (int i = tid; i < kGSTable; i += kGSThreads) {
            L.tkey[i] = -1;
            L.thead[i] = -1;
        }
        __syncthreads();
        const int32_t tb = min(QU, ta + kGSTile);
        for (int32_t qa = (ta / kGSCH) * kGSCH; qa < tb; qa += kGSCH) {
            load(qa);
#pragma unroll
            for (int u = 0; u < kGSNU; ++u) {
                const int32_t q = qa + u * kGSThreads + tid;
                const int32_t c = cc[u];
                if (q >= ta && q < tb && c >= kGHot) {
                    const int32_t i = q - ta;
                    L.eval[i] = vv[u];
                    L.eu[i] = (int8_t)owner_of(u);
                    uint32_t h = gs_hash(c) & (kGSTable - 1);
                    for (;;) {
                        const int32_t old = atomicCAS(&L.tkey[h], -1, c);
                        if (old == -1 || old == c) break;
                        h = (h + 1) & (kGSTable - 1);
                    }
                    L.enext[i] = (int16_t)atomicExch(&L.thead[h], i);
                }
            }
        }
        __syncthreads();
        // entries of updater rows of column c from i on (list order), into partner pp
        auto walk = [&](int32_t i, int pp, double v) {
            for (; i >= 0; i = L.enext[i]) {
                const int uu = L.eu[i];
                const int wb = (uu / kGB) * kGB;
                if (pp > uu && pp < wb + kGW) atomicAdd(&L.acc[uu][pp - wb], v * L.eval[i]);
            }
        };
        for (int32_t qa = 0; qa < T; qa += kGSCH) {
            load(qa);
            // two units at a time: the home slot (key, head), the head entry, then the
            // rare rest one unit at a time (longer lists, probes that met another key)
#pragma unroll
            for (int u0 = 0; u0 < kGSNU; u0 += 2) {
                uint32_t h[2];
                int32_t key[2], hd[2];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    h[t] = gs_hash(cc[u0 + t]) & (kGSTable - 1);
                    key[t] = L.tkey[h[t]];
                    hd[t] = L.thead[h[t]];
                }
                bool act[2], hit[2];
                int32_t nx[2];
                int eu[2];
                double ev[2];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int u = u0 + t;
                    act[t] = cc[u] >= kGHot && owner_of(u) != 0;  // no updater before partner 0
                    hit[t] = act[t] && key[t] == cc[u];
                    const int32_t i0 = hit[t] ? hd[t] : 0;
                    ev[t] = L.eval[i0];
                    eu[t] = L.eu[i0];
                    nx[t] = L.enext[i0];
                }
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int u = u0 + t, pp = owner_of(u);
                    const int wb = (eu[t] / kGB) * kGB;
                    if (hit[t] && pp > eu[t] && pp < wb + kGW) atomicAdd(&L.acc[eu[t]][pp - wb], vv[u] * ev[t]);
                }
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int u = u0 + t, pp = owner_of(u);
                    const int32_t c = cc[u];
                    if (hit[t]) {
                        if (nx[t] >= 0) walk(nx[t], pp, vv[u]);
                    } else if (act[t] && key[t] != -1) {
                        uint32_t hh = (h[t] + 1) & (kGSTable - 1);
                        for (;;) {
                            const int32_t k2 = L.tkey[hh];
                            if (k2 == c) {
                                walk(L.thead[hh], pp, vv[u]);
                                break;
                            }
                            if (k2 == -1) break;
                            hh = (hh + 1) & (kGSTable - 1);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
    // hot part: wave wv -> updaters 2 wv, 2 wv + 1, lane = window position
    {
        const int u0 = 2 * wv;                   // 16 waves x 2 = the 32 updaters
        const int wb = (u0 / kGB) * kGB;         // both updaters share a batch (u0 even)
        const int pl = min(wb + min(lane, kGW - 1), kGSP - 1);
        double h0 = 0.0, h1 = 0.0;
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
    // Gt rows of the strip's updaters: slot of window position l of batch g = (16 (g % 3) + l) % 48;
    // positions past the partners / not after the updater: zero
    for (int u = wv; u < kGSU; u += kGSThreads / 64) {
        const int g = st * kGSB + u / kGB;
        if (g >= a.nbatch) continue;
        const int wb = (u / kGB) * kGB;
        const int p = wb + lane;                 // partner (strip-relative) of window position lane
        const double v = (u < U && p > u && p < P && lane < kGW) ? L.acc[u][min(lane, kGW - 1)] : 0.0;
        const int slot = ((g % kGNB) * kGB + lane) % kGW;
        double* out = a.gt + ((size_t)k * a.nbatch * kGB + (size_t)g * kGB + (u % kGB)) * kGW;
        if (lane < kGW) __builtin_nontemporal_store(v, out + slot);
    }
}

}  // namespace cocoa
