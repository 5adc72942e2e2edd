// Fast translation unit (-ffp-contract=fast): wave-tree dot products and
// fused multiply-adds.  Results agree with the strict path within the 1e-9
// relative tolerance of BASELINE.json's north_star.
#include <cstdlib>

#include "kernels.h"
#include "solver2_impl.h"
#include "solver_impl.h"
#include "wave.h"

namespace cocoa {

void launch_solver_fast(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                        hipStream_t s) {
    launch_solver_impl<false>(mode, vec_lds, alpha_lds, a, grid, lds, s);
}

void launch_solver2_fast(int mode, const Solver2Args& a, int grid, size_t lds, hipStream_t s) {
    launch_solver2_impl<false>(mode, a, grid, lds, s);
}

void launch_plan_fast(const PlanArgs& a, hipStream_t s) { launch_plan_impl<false>(a, s); }

// ----------------------------------------------------------- fused eval --
// One pass over train + test CSR (OptUtils.scala:57-98) as a CSR stream:
// each block takes a tile of whole rows holding <= kEvalTile entries, streams
// the tile's (col, val) entries with coalesced loads (8 entries per thread in
// flight), gathers w (L2-resident), parks the products in LDS, then 16-lane
// groups (one DPP row each) sum the rows.  A row longer than a tile is summed
// by the whole block.  The same launch sums alpha and ||w||^2.  Block partials
// -> fixed-order final reduction (deterministic run to run).
constexpr int kEvalBlock = 256;
constexpr int kEvalUnroll = 8;
constexpr int kEvalBlocksPerCU = 6;  // 24 KB LDS per block

__device__ __forceinline__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(kEvalBlock) void eval_fast_kernel(EvalArgs a) {
    __shared__ double prod[kEvalTile];
    __shared__ int32_t roff[kEvalTile + 1];
    __shared__ double red[4];
    const int tid = threadIdx.x;
    const int sub = tid & 15, grp = tid >> 4;
    double hinge = 0.0, err = 0.0;
    const int64_t ntiles = a.n_tiles + a.n_t_tiles;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const bool test = t >= a.n_tiles;
        const int64_t tt = test ? t - a.n_tiles : t;
        const int64_t* tl = test ? a.t_tiles : a.tiles;
        const int64_t* te = tl + (test ? a.n_t_tiles : a.n_tiles) + 1;  // entry offsets of the boundaries
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const int32_t* cl = test ? a.t_col : a.col;
        const double* vl = test ? a.t_val : a.val;
        const double* yy = test ? a.t_y : a.y;
        const int64_t r0 = tl[tt], r1 = tl[tt + 1];
        const int64_t e0 = te[tt], e1 = te[tt + 1];
        const int64_t T = e1 - e0;
        if (T > kEvalTile) {
            // one long row: the whole block reduces it
            double acc = 0.0;
            for (int64_t q = e0 + tid; q < e1; q += kEvalBlock) acc += vl[q] * a.w[cl[q]];
            const double dot = block_sum(acc, red);
            if (tid == 0) {
                if (!test) hinge += jmax(1 - yy[r0] * dot, 0.0);
                else err += (dot * yy[r0] > 0) ? 0.0 : 1.0;
            }
            continue;
        }
        const int nr = (int)(r1 - r0);
        for (int i = tid; i <= nr; i += kEvalBlock) roff[i] = (int32_t)(rp[r0 + i] - e0);
        int32_t c[kEvalUnroll];
        double v[kEvalUnroll];
#pragma unroll
        for (int u = 0; u < kEvalUnroll; ++u) {
            const int64_t i = tid + (int64_t)u * kEvalBlock;
            c[u] = 0;
            v[u] = 0.0;
            if (i < T) {
                c[u] = cl[e0 + i];
                v[u] = vl[e0 + i];
            }
        }
#pragma unroll
        for (int u = 0; u < kEvalUnroll; ++u) {
            const int64_t i = tid + (int64_t)u * kEvalBlock;
            if (i < T) prod[i] = v[u] * a.w[c[u]];
        }
        __syncthreads();
        for (int r = grp; r < nr; r += kEvalBlock / 16) {
            const int32_t b = roff[r], e = roff[r + 1];
            double acc = 0.0;
            for (int32_t q = b + sub; q < e; q += 16) acc += prod[q];
            const double dot = row16_sum(acc);
            if (sub == 0) {
                if (!test) hinge += jmax(1 - yy[r0 + r] * dot, 0.0);
                else err += (dot * yy[r0 + r] > 0) ? 0.0 : 1.0;
            }
        }
        __syncthreads();
    }
    const int64_t gt = (int64_t)blockIdx.x * kEvalBlock + tid;
    const int64_t gs = (int64_t)gridDim.x * kEvalBlock;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    const double s0 = block_sum(hinge, red);
    const double s1 = block_sum(al, red);
    const double s2 = block_sum(w2, red);
    const double s3 = block_sum(err, red);
    if (tid == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
        p[3] = s3;
    }
}

// Eval v2/v3: the (col, val, row_ptr) loads of a block's next tile are issued
// before the current tile's row sums, so one tile of HBM reads is always in
// flight behind the LDS work.  Same tiles, same per-row 16-lane DPP sums and
// the same fixed-order block partials as eval v1.
//   WLDS (v2): one 1024-thread block per CU that first copies the hot head of
//              w (device feature order = descending frequency) into LDS;
//   v3:        256-thread blocks, several per CU, w gathered from L1/L2.
constexpr int kEvalHotW = 16384;  // doubles of w staged in LDS by v2 (128 KiB)
constexpr int kEval3BlocksPerCU = 6;

template <int BLOCK>
struct EvalTileRegs {
    static constexpr int PER = kEvalTile / BLOCK;            // entries per thread
    static constexpr int RO = (kEvalTile + 1 + BLOCK - 1) / BLOCK;  // row offsets per thread
    int64_t r0 = 0, e0 = 0, T = -1;  // T < 0: no tile
    int32_t nr = 0;
    bool test = false, longrow = false;
    int32_t c[PER];
    double v[PER];
    int32_t ro[RO];
};

template <int BLOCK>
__device__ __forceinline__ void eval_fetch(const EvalArgs& a, int64_t t, int64_t ntiles, EvalTileRegs<BLOCK>& x) {
    using R = EvalTileRegs<BLOCK>;
    const int tid = threadIdx.x;
    x.T = -1;
    if (t >= ntiles) return;
    x.test = t >= a.n_tiles;
    const int64_t tt = x.test ? t - a.n_tiles : t;
    const int64_t* tl = x.test ? a.t_tiles : a.tiles;
    const int64_t* te = tl + (x.test ? a.n_t_tiles : a.n_tiles) + 1;
    const int64_t* rp = x.test ? a.t_row_ptr : a.row_ptr;
    const int32_t* cl = x.test ? a.t_col : a.col;
    const double* vl = x.test ? a.t_val : a.val;
    const int64_t r0 = tl[tt], r1 = tl[tt + 1];
    const int64_t e0 = te[tt], e1 = te[tt + 1];
    x.r0 = r0;
    x.e0 = e0;
    x.T = e1 - e0;
    x.nr = (int32_t)(r1 - r0);
    x.longrow = x.T > kEvalTile;
    if (x.longrow) return;
#pragma unroll
    for (int u = 0; u < R::PER; ++u) {
        const int64_t i = tid + (int64_t)u * BLOCK;
        x.c[u] = 0;
        x.v[u] = 0.0;
        if (i < x.T) {
            x.c[u] = __builtin_nontemporal_load(cl + e0 + i);
            x.v[u] = __builtin_nontemporal_load(vl + e0 + i);
        }
    }
#pragma unroll
    for (int u = 0; u < R::RO; ++u) {
        const int i = tid + u * BLOCK;
        x.ro[u] = i <= x.nr ? (int32_t)(rp[r0 + i] - e0) : 0;
    }
}

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

template <int BLOCK, bool WLDS>
__global__ __launch_bounds__(BLOCK) void eval_pf_kernel(EvalArgs a) {
    using R = EvalTileRegs<BLOCK>;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    double* wh = (double*)lds;                                  // [kEvalHotW] (WLDS)
    double* prod = wh + (WLDS ? kEvalHotW : 0);                 // [kEvalTile]
    int32_t* roff = (int32_t*)(prod + kEvalTile);               // [kEvalTile + 1] (+pad)
    double* red = (double*)(roff + kEvalTile + 4);              // [BLOCK / 64]
    const int tid = threadIdx.x;
    const int sub = tid & 15, grp = tid >> 4;
    const int hw = WLDS ? (int)(a.d < kEvalHotW ? a.d : kEvalHotW) : 0;
    if (WLDS)
        for (int j = tid; j < hw; j += BLOCK) wh[j] = a.w[j];
    auto wv = [&](int32_t c) { return (WLDS && c < hw) ? wh[c] : a.w[c]; };
    double hinge = 0.0, err = 0.0;
    const int64_t ntiles = a.n_tiles + a.n_t_tiles;
    R cur, nxt;
    eval_fetch<BLOCK>(a, blockIdx.x, ntiles, cur);
    if (WLDS) __syncthreads();
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (cur.longrow) {
            const int64_t* rp = cur.test ? a.t_row_ptr : a.row_ptr;
            const int32_t* cl = cur.test ? a.t_col : a.col;
            const double* vl = cur.test ? a.t_val : a.val;
            const double* yy = cur.test ? a.t_y : a.y;
            const int64_t e1 = rp[cur.r0 + 1];
            double acc = 0.0;
            for (int64_t q = cur.e0 + tid; q < e1; q += BLOCK) acc += vl[q] * wv(cl[q]);
            const double dot = block_sum_n<BLOCK>(acc, red);
            if (tid == 0) {
                if (!cur.test) hinge += jmax(1 - yy[cur.r0] * dot, 0.0);
                else err += (dot * yy[cur.r0] > 0) ? 0.0 : 1.0;
            }
            eval_fetch<BLOCK>(a, t + gridDim.x, ntiles, nxt);
            cur = nxt;
            continue;
        }
#pragma unroll
        for (int u = 0; u < R::RO; ++u) {
            const int i = tid + u * BLOCK;
            if (i <= cur.nr) roff[i] = cur.ro[u];
        }
#pragma unroll
        for (int u = 0; u < R::PER; ++u) {
            const int64_t i = tid + (int64_t)u * BLOCK;
            if (i < cur.T) prod[i] = cur.v[u] * wv(cur.c[u]);
        }
        __syncthreads();
        // next tile's HBM reads go out before the LDS row sums of this one
        eval_fetch<BLOCK>(a, t + gridDim.x, ntiles, nxt);
        const double* yy = cur.test ? a.t_y : a.y;
        for (int r = grp; r < cur.nr; r += BLOCK / 16) {
            const int32_t b = roff[r], e = roff[r + 1];
            double acc = 0.0;
            for (int32_t q = b + sub; q < e; q += 16) acc += prod[q];
            const double dot = row16_sum(acc);
            if (sub == 0) {
                if (!cur.test) hinge += jmax(1 - yy[cur.r0 + r] * dot, 0.0);
                else err += (dot * yy[cur.r0 + r] > 0) ? 0.0 : 1.0;
            }
        }
        __syncthreads();
        cur = nxt;
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
    if (tid == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
        p[3] = s3;
    }
}

__global__ __launch_bounds__(256) void eval_final_kernel(const double* partials, int blocks, double* out) {
    __shared__ double red[4][4];
    const int tid = threadIdx.x;
    double v[4] = {0, 0, 0, 0};
    for (int b = tid; b < blocks; b += 256)
        for (int i = 0; i < 4; ++i) v[i] += partials[(size_t)b * 4 + i];
    for (int i = 0; i < 4; ++i) {
        const double s = wave_sum(v[i]);
        if ((tid & 63) == 0) red[i][tid >> 6] = s;
    }
    __syncthreads();
    if (tid < 4) out[tid] = ((red[tid][0] + red[tid][1]) + red[tid][2]) + red[tid][3];
}

int eval_fast_blocks(int64_t n_tiles, int64_t n_t_tiles) {
    int64_t b = n_tiles + n_t_tiles;
    const int64_t cap = 256 * kEvalBlocksPerCU;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (int)b;
}

void launch_eval_fast(const EvalArgs& a, int blocks, hipStream_t s) {
    eval_fast_kernel<<<blocks, kEvalBlock, 0, s>>>(a);
    eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
}

int eval2_blocks(int version, int64_t n_tiles, int64_t n_t_tiles) {
    int64_t b = n_tiles + n_t_tiles;
    const int64_t cap = version == 2 ? 256 : 256 * kEval3BlocksPerCU;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (int)b;
}

template <int BLOCK, bool WLDS>
static void launch_pf(const EvalArgs& a, int blocks, hipStream_t s) {
    const size_t lds = sizeof(double) * ((WLDS ? kEvalHotW : 0) + kEvalTile) + sizeof(int32_t) * (kEvalTile + 4) +
                       sizeof(double) * (BLOCK / 64);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)eval_pf_kernel<BLOCK, WLDS>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    eval_pf_kernel<BLOCK, WLDS><<<blocks, BLOCK, lds, s>>>(a);
    eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
}

void launch_eval2(int version, const EvalArgs& a, int blocks, hipStream_t s) {
    if (version == 2)
        launch_pf<1024, true>(a, blocks, s);
    else
        launch_pf<256, false>(a, blocks, s);
}

}  // namespace cocoa

namespace cocoa {

// Eval v4: the v1 tile stream with 16-byte loads.  A tile [e0, e1) is read from
// the 4-entry-aligned base e0 & ~3, so each thread moves 4 consecutive entries
// per unit with one 16-B col load and two 16-B val loads (v1 moves 4 B + 8 B
// per lane).  Row offsets inside a tile are 16-bit (a tile holds <= TILE <=
// 65536 entries), which leaves room for more blocks per CU.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// GATHER: 1 = w gathered from global (the product); diagnostics (wrong values,
// timing only): 0 = no gather, 2 = 1 lane in 8 gathers, 3 = gathered from a
// 2048-double LDS copy of the head of w.
// SAUX >= 0: the tile stream goes through buffer loads with that cache-policy
// word (16 = sc1: bypasses the CU's L1, so the stream does not evict the
// gathered head of w; 2 = nt; 18 = sc1 + nt) instead of nontemporal globals.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int AUX>
__device__ __forceinline__ u32x4 stream_ld128(const void* base, int32_t voff) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)p);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(p >> 32));
    void* pu = (void*)(((uint64_t)hi << 32) | lo);
    const auto r = __builtin_amdgcn_make_buffer_rsrc(pu, (short)0, 0x7FFFFFF0, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, AUX);
}

template <int TILE, int BLOCK, int GATHER, int SAUX = -1>
__global__ __launch_bounds__(BLOCK) void eval_v4_kernel(EvalArgs a) {
    constexpr int UNITS = TILE / (4 * BLOCK);  // 4-entry units per thread (base alignment adds one)
    __shared__ double prod[TILE + 4];
    __shared__ double wl[GATHER == 3 ? 2048 : 1];
    if (GATHER == 3) {
        for (int j = threadIdx.x; j < 2048; j += BLOCK) wl[j] = j < a.d ? a.w[j] : 0.0;
        __syncthreads();
    }
    auto wg = [&](double v, int32_t c) -> double {
        if (GATHER == 1) return v * a.w[c];
        if (GATHER == 2) return (c & 7) == 0 ? v * a.w[c] : v;
        if (GATHER == 3) return v * wl[c & 2047];
        if (GATHER == 5) return v * a.w[c & 2047];
        if (GATHER == 6) return v * a.w[c >> 31];  // every lane reads w[0]: one line per instruction
        return v;
    };
    __shared__ uint16_t roff[TILE + 2];
    __shared__ double red[BLOCK / 64];
    const int tid = threadIdx.x;
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
        const double* vl = test ? a.t_val : a.val;
        const double* yy = test ? a.t_y : a.y;
        const int64_t r0 = tl[tt], r1 = tl[tt + 1];
        const int64_t e0 = te[tt], e1 = te[tt + 1];
        const int64_t T = e1 - e0;
        if (T > TILE) {
            double acc = 0.0;
            for (int64_t q = e0 + tid; q < e1; q += BLOCK) acc += wg(vl[q], cl[q]);
            const double dot = block_sum_n<BLOCK>(acc, red);
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
        for (int i = tid; i <= nr; i += BLOCK) roff[i] = (uint16_t)(rp[r0 + i] - e0);
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
                if (SAUX >= 0) {
                    c[u] = __builtin_bit_cast(i32x4, stream_ld128<SAUX < 0 ? 0 : SAUX>(cl + base, (int32_t)(4 * k)));
                    v0[u] = __builtin_bit_cast(f64x2, stream_ld128<SAUX < 0 ? 0 : SAUX>(vl + base, (int32_t)(8 * k)));
                    v1[u] = __builtin_bit_cast(f64x2, stream_ld128<SAUX < 0 ? 0 : SAUX>(vl + base, (int32_t)(8 * k + 16)));
                } else if (SAUX == -2) {  // plain global loads (default cache policy)
                    c[u] = *(const i32x4*)(cl + base + k);
                    v0[u] = *(const f64x2*)(vl + base + k);
                    v1[u] = *(const f64x2*)(vl + base + k + 2);
                } else {
                    c[u] = __builtin_nontemporal_load((const i32x4*)(cl + base + k));
                    v0[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k));
                    v1[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k + 2));
                }
            }
        }
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            if (k < span) {
                // entries past e1 inside the last unit are never summed (roff bounds rows)
                const double p0 = wg(v0[u].x, c[u].x);
                const double p1 = wg(v0[u].y, c[u].y);
                const double p2 = wg(v1[u].x, c[u].z);
                const double p3 = wg(v1[u].y, c[u].w);
                *(f64x2*)(prod + k) = f64x2{p0, p1};
                *(f64x2*)(prod + k + 2) = f64x2{p2, p3};
            }
        }
        __syncthreads();
        for (int r = grp; r < nr; r += BLOCK / 16) {
            const int b = roff[r] + sh, e = roff[r + 1] + sh;
            double acc = 0.0;
            for (int q = b + sub; q < e; q += 16) acc += prod[q];
            const double dot = row16_sum(acc);
            if (sub == 0) {
                if (!test) {
                    hinge += jmax(1 - yy[r0 + r] * dot, 0.0);
                    if (a.row_xw) a.row_xw[r0 + r] = dot;
                } else {
                    err += (dot * yy[r0 + r] > 0) ? 0.0 : 1.0;
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
    if (tid == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
        p[3] = s3;
    }
}

// Eval v7: v4 with the per-tile dependent round trips taken off the critical
// path.  v4 waits on row_ptr before it issues the tile's stream (its roff loop
// comes first), reads y only after each row's dot, and reads the tile bounds
// only when the tile starts: up to five serialized memory latencies per tile.
// Here the next tile's bounds are read one tile ahead, the row_ptr and y
// values go to registers in the same batch as the stream, and LDS is written
// only after the batch lands.  Same arithmetic as v4.
template <int TILE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void eval_v7_kernel(EvalArgs a) {
    constexpr int UNITS = TILE / (4 * BLOCK);
    __shared__ double prod[TILE + 4];
    __shared__ uint16_t roff[TILE + 2];
    __shared__ double ys[BLOCK];  // y of the tile's first BLOCK rows
    __shared__ double red[BLOCK / 64];
    const int tid = threadIdx.x;
    const int sub = tid & 15, grp = tid >> 4;
    double hinge = 0.0, err = 0.0;
    const int64_t ntiles = a.n_tiles + a.n_t_tiles;
    auto bounds = [&](int64_t t, int64_t& r0, int64_t& r1, int64_t& e0, int64_t& e1) {
        const bool test = t >= a.n_tiles;
        const int64_t tt = test ? t - a.n_tiles : t;
        const int64_t* tl = test ? a.t_tiles : a.tiles;
        const int64_t* te = tl + (test ? a.n_t_tiles : a.n_tiles) + 1;
        r0 = tl[tt];
        r1 = tl[tt + 1];
        e0 = te[tt];
        e1 = te[tt + 1];
    };
    int64_t nr0 = 0, nr1 = 0, ne0 = 0, ne1 = 0;
    if ((int64_t)blockIdx.x < ntiles) bounds(blockIdx.x, nr0, nr1, ne0, ne1);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t r0 = nr0, r1 = nr1, e0 = ne0, e1 = ne1;
        if (t + gridDim.x < ntiles) bounds(t + gridDim.x, nr0, nr1, ne0, ne1);
        const bool test = t >= a.n_tiles;
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const int32_t* cl = test ? a.t_col : a.col;
        const double* vl = test ? a.t_val : a.val;
        const double* yy = test ? a.t_y : a.y;
        const int64_t T = e1 - e0;
        if (T > TILE) {
            double acc = 0.0;
            for (int64_t q = e0 + tid; q < e1; q += BLOCK) acc += vl[q] * a.w[cl[q]];
            const double dot = block_sum_n<BLOCK>(acc, red);
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
                c[u] = __builtin_nontemporal_load((const i32x4*)(cl + base + k));
                v0[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k));
                v1[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k + 2));
            }
        }
        const int64_t rpv = tid <= nr ? rp[r0 + tid] : 0;  // same batch as the stream
        const double yv = tid < nr ? yy[r0 + tid] : 0.0;
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            if (k < span) {
                const double p0 = v0[u].x * a.w[c[u].x];
                const double p1 = v0[u].y * a.w[c[u].y];
                const double p2 = v1[u].x * a.w[c[u].z];
                const double p3 = v1[u].y * a.w[c[u].w];
                *(f64x2*)(prod + k) = f64x2{p0, p1};
                *(f64x2*)(prod + k + 2) = f64x2{p2, p3};
            }
        }
        if (tid <= nr) roff[tid] = (uint16_t)(rpv - e0);
        if (tid < nr) ys[tid] = yv;
        for (int i = tid + BLOCK; i <= nr; i += BLOCK) roff[i] = (uint16_t)(rp[r0 + i] - e0);  // tiles of tiny rows
        __syncthreads();
        for (int r = grp; r < nr; r += BLOCK / 16) {
            const int b = roff[r] + sh, e = roff[r + 1] + sh;
            double acc = 0.0;
            for (int q = b + sub; q < e; q += 16) acc += prod[q];
            const double dot = row16_sum(acc);
            if (sub == 0) {
                const double yr = r < BLOCK ? ys[r] : yy[r0 + r];
                if (!test) {
                    hinge += jmax(1 - yr * dot, 0.0);
                    if (a.row_xw) a.row_xw[r0 + r] = dot;
                } else {
                    err += (dot * yr > 0) ? 0.0 : 1.0;
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
    if (tid == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
        p[3] = s3;
    }
}

int eval4_tile(int variant) { return variant == 1 || variant == 3 || variant >= 4 ? 4096 : 2048; }

// variant: 0 = tile 2048 / 8 blocks per CU, 1 = tile 4096 / 4 per CU,
//          2 = tile 2048 without the w gather (diagnostic: stream-only time),
//          3 = tile 4096 / 4 per CU, 512 threads
int eval4_blocks(int variant, int64_t n_tiles, int64_t n_t_tiles) {
    const int per_cu = (variant >= 8 && variant <= 10) ? 2 : (variant == 1 || variant >= 3 ? 3 : 7);  // LDS: 41 KB / 20.5 KB per block
    int64_t b = n_tiles + n_t_tiles;
    if (b > 256 * per_cu) b = 256 * per_cu;
    return (int)(b < 1 ? 1 : b);
}

void launch_eval4(int variant, const EvalArgs& a, int blocks, hipStream_t s) {
    if (variant == 1)
        eval_v4_kernel<4096, 256, 1><<<blocks, 256, 0, s>>>(a);
    else if (variant == 2)
        eval_v4_kernel<2048, 256, 0><<<blocks, 256, 0, s>>>(a);
    else if (variant == 3)
        eval_v4_kernel<4096, 512, 1><<<blocks, 512, 0, s>>>(a);
    else if (variant == 4)
        eval_v4_kernel<4096, 512, 2><<<blocks, 512, 0, s>>>(a);
    else if (variant == 5)
        eval_v4_kernel<4096, 512, 3><<<blocks, 512, 0, s>>>(a);
    else if (variant == 6)
        eval_v4_kernel<4096, 512, 0><<<blocks, 512, 0, s>>>(a);
    else if (variant == 7)
        eval_v4_kernel<4096, 512, 5><<<blocks, 512, 0, s>>>(a);
    else if (variant == 8)
        eval_v4_kernel<4096, 1024, 1><<<blocks, 1024, 0, s>>>(a);
    else if (variant == 9)
        eval_v4_kernel<4096, 1024, 5><<<blocks, 1024, 0, s>>>(a);
    else if (variant == 10)
        eval_v4_kernel<4096, 1024, 0><<<blocks, 1024, 0, s>>>(a);
    else if (variant == 11)
        eval_v4_kernel<4096, 512, 6><<<blocks, 512, 0, s>>>(a);
    else if (variant == 12)
        eval_v7_kernel<4096, 512><<<blocks, 512, 0, s>>>(a);
    else if (variant == 14)
        eval_v4_kernel<4096, 512, 1, 16><<<blocks, 512, 0, s>>>(a);
    else if (variant == 15)
        eval_v4_kernel<4096, 512, 1, 18><<<blocks, 512, 0, s>>>(a);
    else if (variant == 16)
        eval_v4_kernel<4096, 512, 1, 2><<<blocks, 512, 0, s>>>(a);
    else if (variant == 17)
        eval_v4_kernel<4096, 512, 1, 0><<<blocks, 512, 0, s>>>(a);
    else if (variant == 18)
        eval_v4_kernel<4096, 512, 1, -2><<<blocks, 512, 0, s>>>(a);
    else if (variant == 13)
        eval_v7_kernel<4096, 256><<<blocks, 256, 0, s>>>(a);
    else
        eval_v4_kernel<2048, 256, 1><<<blocks, 256, 0, s>>>(a);
    eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
}

// Eval v6: wave tiles.  v4's block-wide tile (stream -> gather -> LDS ->
// barrier -> row sums -> barrier) keeps a whole 512-thread block in one phase
// at a time, so a CU's HBM stream stalls while its blocks wait on the w gather.
// Here every wave owns its own tile of whole rows (<= WT entries, tiles built
// with cap WT) and its own LDS slice, and the only synchronisation is the
// in-wave LDS ordering fence: the waves of a CU drift apart and one wave's
// gather hides behind the others' streams.  PF = 1 also issues the next tile's
// stream loads before this tile's gathers (register double buffer).
// Same sums as v4 (OptUtils.scala:65-98 hinge / error, row order inside a
// 16-lane DPP tree: fast mode).
template <int WT>
struct WaveTile {
    static constexpr int U = WT / 256 + 1;  // 4-entry units per lane (alignment adds one)
    i32x4 c[U];
    f64x2 v0[U], v1[U];
    int64_t r0, r1, e0, e1;
    bool test;
};

template <int WT>
__device__ __forceinline__ void wave_tile_load(const EvalArgs& a, int64_t t, int lane, WaveTile<WT>& x) {
    x.test = t >= a.n_tiles;
    const int64_t tt = x.test ? t - a.n_tiles : t;
    const int64_t* tl = x.test ? a.t_tiles : a.tiles;
    const int64_t* te = tl + (x.test ? a.n_t_tiles : a.n_tiles) + 1;
    x.r0 = tl[tt];
    x.r1 = tl[tt + 1];
    x.e0 = te[tt];
    x.e1 = te[tt + 1];
    const int32_t* cl = x.test ? a.t_col : a.col;
    const double* vl = x.test ? a.t_val : a.val;
    const int64_t base = x.e0 & ~(int64_t)3;
    const int64_t span = (x.e1 - x.e0 > WT) ? 0 : x.e1 - base;  // a long row is streamed separately
#pragma unroll
    for (int u = 0; u < WaveTile<WT>::U; ++u) {
        const int64_t k = 4 * ((int64_t)u * 64 + lane);
        x.c[u] = i32x4{0, 0, 0, 0};
        x.v0[u] = f64x2{0.0, 0.0};
        x.v1[u] = x.v0[u];
        if (k < span) {
            x.c[u] = __builtin_nontemporal_load((const i32x4*)(cl + base + k));
            x.v0[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k));
            x.v1[u] = __builtin_nontemporal_load((const f64x2*)(vl + base + k + 2));
        }
    }
}

template <int WT, int BLOCK, int PF>
__global__ __launch_bounds__(BLOCK) void eval_v6_kernel(EvalArgs a) {
    constexpr int NW = BLOCK / 64;
    __shared__ double prod_s[NW][WT + 4];
    __shared__ uint16_t roff_s[NW][WT + 2];
    __shared__ double red[NW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double* prod = prod_s[wv];
    uint16_t* roff = roff_s[wv];
    const int sub = lane & 15, grp = lane >> 4;
    double hinge = 0.0, err = 0.0;
    const int64_t ntiles = a.n_tiles + a.n_t_tiles;
    const int64_t nwaves = (int64_t)gridDim.x * NW;
    int64_t t = (int64_t)blockIdx.x * NW + wv;
    WaveTile<WT> cur, nxt;
    if (PF && t < ntiles) wave_tile_load<WT>(a, t, lane, cur);
    for (; t < ntiles; t += nwaves) {
        if (PF) {
            if (t + nwaves < ntiles) wave_tile_load<WT>(a, t + nwaves, lane, nxt);
        } else {
            wave_tile_load<WT>(a, t, lane, cur);
        }
        const bool test = cur.test;
        const int64_t* rp = test ? a.t_row_ptr : a.row_ptr;
        const double* yy = test ? a.t_y : a.y;
        const int64_t r0 = cur.r0, e0 = cur.e0, e1 = cur.e1;
        if (e1 - e0 > WT) {  // one long row: strided stream + wave tree
            const int32_t* cl = test ? a.t_col : a.col;
            const double* vl = test ? a.t_val : a.val;
            double acc = 0.0;
            for (int64_t q = e0 + lane; q < e1; q += 64) acc += vl[q] * a.w[cl[q]];
            const double dot = wave_sum(acc);
            if (lane == 0) {
                if (!test) {
                    hinge += jmax(1 - yy[r0] * dot, 0.0);
                    if (a.row_xw) a.row_xw[r0] = dot;
                } else {
                    err += (dot * yy[r0] > 0) ? 0.0 : 1.0;
                }
            }
        } else {
            const int nr = (int)(cur.r1 - r0);
            const int64_t base = e0 & ~(int64_t)3;
            const int sh = (int)(e0 - base);
            const int64_t span = e1 - base;
            for (int i = lane; i <= nr; i += 64) roff[i] = (uint16_t)(rp[r0 + i] - e0);
#pragma unroll
            for (int u = 0; u < WaveTile<WT>::U; ++u) {
                const int64_t k = 4 * ((int64_t)u * 64 + lane);
                if (k < span) {
                    const double p0 = cur.v0[u].x * a.w[cur.c[u].x];
                    const double p1 = cur.v0[u].y * a.w[cur.c[u].y];
                    const double p2 = cur.v1[u].x * a.w[cur.c[u].z];
                    const double p3 = cur.v1[u].y * a.w[cur.c[u].w];
                    *(f64x2*)(prod + k) = f64x2{p0, p1};
                    *(f64x2*)(prod + k + 2) = f64x2{p2, p3};
                }
            }
            wave_lds_sync();
            for (int r = grp; r < nr; r += 4) {
                const int b = roff[r] + sh, e = roff[r + 1] + sh;
                double acc = 0.0;
                for (int q = b + sub; q < e; q += 16) acc += prod[q];
                const double dot = row16_sum(acc);
                if (sub == 0) {
                    if (!test) {
                        hinge += jmax(1 - yy[r0 + r] * dot, 0.0);
                        if (a.row_xw) a.row_xw[r0 + r] = dot;
                    } else {
                        err += (dot * yy[r0 + r] > 0) ? 0.0 : 1.0;
                    }
                }
            }
            wave_lds_sync();  // this tile's LDS reads finish before the next tile's writes
        }
        if (PF) cur = nxt;
    }
    const int64_t gt = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * BLOCK;
    double al = 0.0, w2 = 0.0;
    for (int64_t i = gt; i < a.n; i += gs) al += a.alpha[i];
    for (int64_t j = gt; j < a.d; j += gs) w2 += a.w[j] * a.w[j];
    const double s0 = block_sum_n<BLOCK>(hinge, red);
    const double s1 = block_sum_n<BLOCK>(al, red);
    const double s2 = block_sum_n<BLOCK>(w2, red);
    const double s3 = block_sum_n<BLOCK>(err, red);
    if (threadIdx.x == 0) {
        double* p = a.partials + (size_t)blockIdx.x * 4;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
        p[3] = s3;
    }
}

// variant: 0 = WT 512 / 256 threads, 1 = WT 512 prefetched, 2 = WT 1024 / 128
// threads, 3 = WT 256 / 256 threads.  Blocks per CU from the LDS footprint
// (160 KB per CU) and the 32-wave cap.
int eval6_tile(int variant) { return variant == 2 ? 1024 : variant == 3 ? 256 : 512; }

int eval6_blocks(int variant, int64_t n_tiles, int64_t n_t_tiles) {
    const int wt = eval6_tile(variant);
    const int nw = variant == 2 ? 2 : 4;
    const int lds = nw * (wt * 10 + 40) + 64;
    int per_cu = (160 * 1024) / lds;
    if (per_cu * nw > 32) per_cu = 32 / nw;
    const char* e = std::getenv("COCOA_EVAL6_PERCU");
    if (e && std::atoi(e) > 0 && std::atoi(e) < per_cu) per_cu = std::atoi(e);
    int64_t b = (n_tiles + n_t_tiles + nw - 1) / nw;
    if (b > 256 * per_cu) b = 256 * per_cu;
    return (int)(b < 1 ? 1 : b);
}

void launch_eval6(int variant, const EvalArgs& a, int blocks, hipStream_t s) {
    if (variant == 1)
        eval_v6_kernel<512, 256, 1><<<blocks, 256, 0, s>>>(a);
    else if (variant == 2)
        eval_v6_kernel<1024, 128, 0><<<blocks, 128, 0, s>>>(a);
    else if (variant == 3)
        eval_v6_kernel<256, 256, 0><<<blocks, 256, 0, s>>>(a);
    else
        eval_v6_kernel<512, 256, 0><<<blocks, 256, 0, s>>>(a);
    eval_final_kernel<<<1, 256, 0, s>>>(a.partials, blocks, a.out);
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
