// Fast sparse evaluation pass, one wave per tile (OptUtils.scala:57-98).
//
// The block-tiled pass (eval_stream_kernel, r01-r03) moved a 4,096-entry tile
// per 512-thread block through LDS between two workgroup barriers, so each
// tile paid its loads, then its w gathers, then the barrier chain, one after
// the other; 40% of HBM on C2.  Here every wave owns
// its tiles outright:
//   - a tile is a run of whole rows of at most 256 U - 4 entries and 63 rows
//     (make_tiles), read from the 4-entry-aligned base with 16-byte loads (U
//     units of 4 entries per lane: values 2 x 16 B, columns 8 B as uint16 or
//     16 B as int32) plus one row_ptr value per lane;
//   - the wave runs its tiles software-pipelined: the w gathers of tile i are
//     issued before the stream loads of tile i+1, so waiting for the gathers
//     (vmcnt counts in issue order) never waits for the next tile's stream,
//     and the tile bounds run two tiles ahead;
//   - products go to the wave's own LDS region and 16-lane groups sum the rows
//     (one DPP row each); a wave's LDS operations complete in order, so no
//     barrier is needed -- the only workgroup barriers are the final
//     reduction's.
// A row longer than a tile is its own "tile" and is summed by the wave in a
// plain loop.  Results: per-row x.w (train rows, for the next round's step
// plan), hinge sum, test error count, alpha sum and ||w||^2 as block partials
// reduced in a fixed order (run-to-run deterministic).
#pragma once
#include "kernels.h"
#include "wave.h"

namespace cocoa {

typedef int32_t ew_i32x4 __attribute__((ext_vector_type(4)));
typedef double ew_f64x2 __attribute__((ext_vector_type(2)));
typedef uint16_t ew_u16x4 __attribute__((ext_vector_type(4)));

constexpr int kEwRows = 63;  // rows per wave tile (row_ptr values fit one register per lane)
__host__ __device__ constexpr int ew_tile_entries(int U) { return 256 * U - 4; }

// 4 column indices at entry k, kept as loaded (uint16 x 4 in two dwords, or
// int32 x 4) and unpacked only when the gathers are issued: an unpack right
// after the load would make the wave wait for it -- and, as loads complete in
// issue order, for every gather issued before it.
template <bool C16>
struct EwCols {
    typedef uint32_t raw __attribute__((ext_vector_type(C16 ? 2 : 4)));
    static __device__ __forceinline__ raw load(const int32_t* c32, const uint16_t* c16, int64_t k) {
        if (C16) return __builtin_nontemporal_load((const raw*)(c16 + k));
        return __builtin_nontemporal_load((const raw*)(c32 + k));
    }
    static __device__ __forceinline__ int32_t at(const raw& v, int i) {
        if (C16) return (int32_t)((v[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
        return (int32_t)v[i];
    }
};

template <int U, bool C16>
struct EwTile {
    typename EwCols<C16>::raw c[U];
    ew_f64x2 v0[U], v1[U];
    int64_t rp;  // row_ptr[r0 + lane] (lane <= nr)
    double y;    // y[r0 + lane] (lane < nr)
};

// compiler-only fence: keeps the issue order of the loads on either side
__device__ __forceinline__ void ew_order() { __asm__ volatile("" ::: "memory"); }
// the value stays live (and in its registers) up to this point
__device__ __forceinline__ void ew_keep(int64_t& x) { __asm__ volatile("" : "+v"(x)); }

template <int U, int BLOCK, bool C16, bool NOGATHER = false>
__global__ __launch_bounds__(BLOCK) void eval_wave_kernel(EvalArgs a) {
    constexpr int W = BLOCK / 64;
    constexpr int SPAN = 256 * U;
    __shared__ double prod[W][SPAN];
    __shared__ double red[W];
    __shared__ double xwb[W][64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int sub = lane & 15, grp = lane >> 4;
    double* P = prod[wv];
    double* XW = xwb[wv];
    double hinge = 0.0, err = 0.0;
    const int64_t ntr = a.n_tiles, ntot = a.n_tiles + a.n_t_tiles;
    const int64_t gw = (int64_t)blockIdx.x * W + wv, nw = (int64_t)gridDim.x * W;

    // tile bounds: rows [r0, r1), entries [e0, e1)
    struct Bounds {
        int64_t r0, r1, e0, e1;
    };
    // (a prefetch past the last tile reads the last tile again: never used)
    auto bounds = [&](int64_t t) {
        t = min(t, ntot - 1);
        const bool test = t >= ntr;
        const int64_t tt = test ? t - ntr : t;
        const int64_t* tl = test ? a.t_tiles : a.tiles;
        const int64_t* te = tl + (test ? a.n_t_tiles : a.n_tiles) + 1;
        return Bounds{tl[tt], tl[tt + 1], te[tt], te[tt + 1]};
    };
    // Every call issues the same loads, whatever the tile (a long row: its
    // first units, unused), so the compiler's wait counts stay exact.
    auto load = [&](int64_t t, const Bounds& b, EwTile<U, C16>& d) {
        const bool test = min(t, ntot - 1) >= ntr;
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const int32_t* cl = test ? a.t_col : a.col;
        const uint16_t* cl16 = test ? a.t_col16 : a.col16;
        const double* vl = test ? a.t_val : a.val;
        const double* yy = test ? a.t_y : a.y;
        const int nr = (int)(b.r1 - b.r0);
        d.rp = rp[b.r0 + min(lane, nr)];
        d.y = yy[b.r0 + max(0, min(lane, nr - 1))];
        const int64_t base = b.e0 & ~(int64_t)3, span = b.e1 - base;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // lanes past the tile reload its first unit (in bounds, never summed)
            const int64_t k = 4 * ((int64_t)u * 64 + lane);
            const int64_t kk = k < span ? k : 0;
            d.c[u] = EwCols<C16>::load(cl, cl16, base + kk);
            d.v0[u] = __builtin_nontemporal_load((const ew_f64x2*)(vl + base + kk));
            d.v1[u] = __builtin_nontemporal_load((const ew_f64x2*)(vl + base + kk + 2));
        }
    };
    auto finish_row = [&](bool test, int64_t r, double dot, double yv) {
        if (!test) {
            hinge += jmax(1 - yv * dot, 0.0);  // OptUtils.scala:57-61
            if (a.row_xw) a.row_xw[r] = dot;
        } else {
            err += (dot * yv > 0) ? 0.0 : 1.0;  // OptUtils.scala:95-98
        }
    };

    int64_t t = gw;
    Bounds bc = bounds(t), bn = bounds(t + nw);
    EwTile<U, C16> cur, nxt;
    load(t, bc, cur);
    for (; t < ntot; t += nw) {
        const bool test = t >= ntr;
        const int64_t T = bc.e1 - bc.e0;
        if (T > ew_tile_entries(U)) {  // one row longer than a tile
            const int32_t* cl = test ? a.t_col : a.col;
            const double* vl = test ? a.t_val : a.val;
            double acc = 0.0;
            for (int64_t q = bc.e0 + lane; q < bc.e1; q += 64) acc = fma(vl[q], a.w[cl[q]], acc);
            const double dot = wave_sum(acc);
            if (lane == 0) finish_row(test, bc.r0, dot, (test ? a.t_y : a.y)[bc.r0]);
            const Bounds bnn = bounds(t + 2 * nw);
            load(t + nw, bn, cur);
            bc = bn;
            bn = bnn;
            continue;
        }
        // 1. w gathers of this tile
        double x[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NOGATHER) {
                x[u][0] = x[u][1] = x[u][2] = x[u][3] = 1.0;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) x[u][i] = a.w[EwCols<C16>::at(cur.c[u], i)];
            }
        }
        ew_order();
        // 2. the next tile's stream (and the bounds of the one after)
        Bounds bnn = bounds(t + 2 * nw);
        load(t + nw, bn, nxt);
        ew_order();
        // 3. products into the wave's LDS region (waits for the gathers only)
        const int64_t base = bc.e0 & ~(int64_t)3;
        const int sh = (int)(bc.e0 - base);
        const int span = (int)(bc.e1 - base);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = 4 * (u * 64 + lane);
            if (k < span) {
                *(ew_f64x2*)(P + k) = ew_f64x2{cur.v0[u].x * x[u][0], cur.v0[u].y * x[u][1]};
                *(ew_f64x2*)(P + k + 2) = ew_f64x2{cur.v1[u].x * x[u][2], cur.v1[u].y * x[u][3]};
            }
        }
        wave_lds_sync();
        // 4. row sums: 16-lane group grp takes rows grp, grp + 4, ...
        const int nr = (int)(bc.r1 - bc.r0);
        const int64_t rb = bc.e0 - sh;  // = base
        for (int r0 = 0; r0 < nr; r0 += 4) {
            const int r = r0 + grp;
            const int rr = min(r, nr - 1);
            // (both shuffles with every lane active: a lane of a row past nr may be the source)
            const int b = (int)(__shfl(cur.rp, rr) - rb), e1 = (int)(__shfl(cur.rp, rr + 1) - rb);
            const int e = r < nr ? e1 : b;
            // four independent LDS reads in flight per pass (a C2 row: two passes)
            // (reads past the row stay inside P and are dropped by a select)
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
            for (int q = b + sub; q < e; q += 64) {
                const double p0 = P[q], p1 = P[min(q + 16, SPAN - 1)], p2 = P[min(q + 32, SPAN - 1)],
                             p3 = P[min(q + 48, SPAN - 1)];
                a0 += p0;
                a1 += q + 16 < e ? p1 : 0.0;
                a2 += q + 32 < e ? p2 : 0.0;
                a3 += q + 48 < e ? p3 : 0.0;
            }
            const double dot = row16_sum((a0 + a1) + (a2 + a3));
            if (sub == 0 && r < nr) XW[r] = dot;
        }
        // the rows' objective terms lane by lane (lane r: row r, its y in cur.y);
        // no global store inside the loop above, or the compiler drains every
        // outstanding load (the next tile's) before entering it
        wave_lds_sync();
        if (lane < nr) finish_row(test, bc.r0 + lane, XW[lane], cur.y);
        wave_lds_sync();  // the next tile's products overwrite P
        // keep the prefetched bounds whole and untouched until here: a load whose
        // destination register is reused early (a dead upper half) makes the wave
        // wait for it, and so for every load issued before it
        ew_keep(bnn.r0);
        ew_keep(bnn.r1);
        ew_keep(bnn.e0);
        ew_keep(bnn.e1);
        cur = nxt;
        bc = bn;
        bn = bnn;
    }
    const int64_t gt = (int64_t)blockIdx.x * BLOCK + tid, gs = (int64_t)gridDim.x * BLOCK;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    double s[4] = {hinge, al, w2, err};
    for (int i = 0; i < 4; ++i) {
        const double v = wave_sum(s[i]);
        __syncthreads();
        if (lane == 0) red[wv] = v;
        __syncthreads();
        double acc = 0.0;
        for (int j = 0; j < W; ++j) acc += red[j];
        s[i] = acc;
    }
    if (tid == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s[0];
        p[1] = s[1];
        p[2] = s[2];
        p[3] = s[3];
    }
}

}  // namespace cocoa
