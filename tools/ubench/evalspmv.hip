// Eval-pass micro-benchmark on the C2 shape (rcv1-shaped, n = 677,399 train +
// 50,000 test rows, d = 47,236, ~75.6 nnz/row): the shipped fast eval
// (cocoa::launch_eval_fast from libcocoa_hip.so) against eval_wave_kernel
// variants, each timed with HIP events over 20 launches and checked against a
// host double-precision evaluation of the same rows (row x.w, hinge sum,
// test errors, alpha sum, ||w||^2).
//   ./evalspmv [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "cocoa_capi.h"
#include "eval_wave.h"

using namespace cocoa;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

namespace cocoa {
bool launch_eval_fast(const EvalArgs& a, int blocks, hipStream_t s);
int eval_fast_blocks(int64_t n, int64_t n_test);
}

__global__ void final_kernel(const double* p, int blocks, double* out) {
    if (threadIdx.x < 4) {
        double s = 0.0;
        for (int b = 0; b < blocks; ++b) s += p[(size_t)b * 4 + threadIdx.x];
        out[threadIdx.x] = s;
    }
}


// Column-sorted tiles (diagnostic): each tile's entries sorted by column so a
// gather instruction's lanes share cache lines; pos = the entry's offset from
// the tile's first entry, so each product lands in its row order slot in LDS.
typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));
typedef double f64x2_t __attribute__((ext_vector_type(2)));
typedef uint16_t u16x4_t __attribute__((ext_vector_type(4)));
struct SortedArgs {
    const uint16_t* scol;  // sorted columns (train | test, concatenated per side)
    const uint16_t* spos;
    const double* sval;
    const uint16_t* t_scol;
    const uint16_t* t_spos;
    const double* t_sval;
};
template <int TILE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void eval_sorted_kernel(EvalArgs a, SortedArgs z) {
    constexpr int UNITS = TILE / (4 * BLOCK);
    __shared__ double prod[TILE + 4];
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
        const uint16_t* sc = test ? z.t_scol : z.scol;
        const uint16_t* sp = test ? z.t_spos : z.spos;
        const double* sv = test ? z.t_sval : z.sval;
        const double* yy = test ? a.t_y : a.y;
        const int64_t r0 = tl[tt], r1 = tl[tt + 1];
        const int64_t e0 = te[tt], e1 = te[tt + 1];
        const int nr = (int)(r1 - r0);
        for (int i = tid; i <= nr; i += BLOCK) roff[i] = (uint16_t)(rp[r0 + i] - e0);
        const int64_t base = e0 & ~(int64_t)3;
        const int sh = (int)(e0 - base);
        const int64_t span = e1 - base;
        u16x4_t c[UNITS + 1], q[UNITS + 1];
        f64x2_t v0[UNITS + 1], v1[UNITS + 1];
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            c[u] = u16x4_t{0, 0, 0, 0};
            q[u] = c[u];
            v0[u] = f64x2_t{0.0, 0.0};
            v1[u] = v0[u];
            if (k < span) {
                c[u] = __builtin_nontemporal_load((const u16x4_t*)(sc + base + k));
                q[u] = __builtin_nontemporal_load((const u16x4_t*)(sp + base + k));
                v0[u] = __builtin_nontemporal_load((const f64x2_t*)(sv + base + k));
                v1[u] = __builtin_nontemporal_load((const f64x2_t*)(sv + base + k + 2));
            }
        }
#pragma unroll
        for (int u = 0; u <= UNITS; ++u) {
            const int64_t k = 4 * ((int64_t)u * BLOCK + tid);
            // entries of the unit inside [e0, e1): pos is their row-order offset from e0
            if (k < span) {
                const double p0 = v0[u].x * a.w[c[u].x], p1 = v0[u].y * a.w[c[u].y];
                const double p2 = v1[u].x * a.w[c[u].z], p3 = v1[u].y * a.w[c[u].w];
                if (k + 0 >= sh && k + 0 < span) prod[q[u].x] = p0;
                if (k + 1 >= sh && k + 1 < span) prod[q[u].y] = p1;
                if (k + 2 >= sh && k + 2 < span) prod[q[u].z] = p2;
                if (k + 3 >= sh && k + 3 < span) prod[q[u].w] = p3;
            }
        }
        __syncthreads();
        for (int r = grp; r < nr; r += BLOCK / 16) {
            const int b = roff[r], e = roff[r + 1];
            double acc = 0.0;
            for (int qq = b + sub; qq < e; qq += 16) acc += prod[qq];
            const double dot = cocoa::row16_sum(acc);
            if (sub == 0) {
                if (!test) {
                    hinge += cocoa::jmax(1 - yy[r0 + r] * dot, 0.0);
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
    double s4[4] = {hinge, al, w2, err};
    for (int i = 0; i < 4; ++i) {
        double v = cocoa::wave_sum(s4[i]);
        __syncthreads();
        if ((tid & 63) == 0) red[tid >> 6] = v;
        __syncthreads();
        double acc = 0.0;
        for (int j = 0; j < BLOCK / 64; ++j) acc += red[j];
        s4[i] = acc;
    }
    if (tid == 0)
        for (int i = 0; i < 4; ++i) a.partials[(size_t)blockIdx.x * 4 + i] = s4[i];
}


// Split CSR (diagnostic): each row's entries of the HOT most frequent columns
// in one CSR, the rest in another; w[0, HOT) in LDS, so the hot entries issue
// no texture-addresser gather.  One tile = whole rows, both segments loaded
// 4 entries per lane, products parked in LDS (hot segment, then cold), and
// 16-lane groups sum each row over its two segments.
struct SplitArgs {
    const int64_t* rph;  const uint16_t* ch; const double* vh;   // hot CSR (train)
    const int64_t* rpc;  const uint16_t* cc; const double* vc;   // cold CSR (train)
    const int64_t* trph; const uint16_t* tch; const double* tvh; // test
    const int64_t* trpc; const uint16_t* tcc; const double* tvc;
};
template <int TILE, int BLOCK, int HOT>
__global__ __launch_bounds__(BLOCK) void eval_split_kernel(EvalArgs a, SplitArgs z) {
    constexpr int UN = TILE / (4 * BLOCK) + 1;  // units per segment per thread (alignment adds one)
    __shared__ double whot[HOT];
    __shared__ double prod[TILE + 16];  // hot + cold entries of a tile <= TILE (+ alignment)
    __shared__ uint16_t roh[TILE + 2], roc[TILE + 2];
    __shared__ double red[BLOCK / 64];
    const int tid = threadIdx.x;
    const int sub = tid & 15, grp = tid >> 4;
    for (int j = tid; j < HOT; j += BLOCK) whot[j] = a.w[j];
    __syncthreads();
    double hinge = 0.0, err = 0.0;
    const int64_t ntiles = a.n_tiles + a.n_t_tiles;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const bool test = t >= a.n_tiles;
        const int64_t tt = test ? t - a.n_tiles : t;
        const int64_t* tl = test ? a.t_tiles : a.tiles;
        const int64_t* rph = test ? z.trph : z.rph;
        const int64_t* rpc = test ? z.trpc : z.rpc;
        const uint16_t* ch = test ? z.tch : z.ch;
        const uint16_t* cc = test ? z.tcc : z.cc;
        const double* vh = test ? z.tvh : z.vh;
        const double* vc = test ? z.tvc : z.vc;
        const double* yy = test ? a.t_y : a.y;
        const int64_t r0 = tl[tt], r1 = tl[tt + 1];
        const int nr = (int)(r1 - r0);
        const int64_t eh0 = rph[r0], eh1 = rph[r1], ec0 = rpc[r0], ec1 = rpc[r1];
        const int64_t bh = eh0 & ~(int64_t)3, bc = ec0 & ~(int64_t)3;
        const int shh = (int)(eh0 - bh), shc = (int)(ec0 - bc);
        const int sph = (int)(eh1 - bh), spc = (int)(ec1 - bc);
        const int offc = (sph + 3) & ~3;  // cold products after the hot ones, 16-B aligned
        for (int i = tid; i <= nr; i += BLOCK) {
            roh[i] = (uint16_t)(rph[r0 + i] - eh0 + shh);
            roc[i] = (uint16_t)(rpc[r0 + i] - ec0 + shc + offc);
        }
        u16x4_t hc[UN], ccol[UN];
        f64x2_t h0[UN], h1[UN], c0[UN], c1[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int k = 4 * (u * BLOCK + tid);
            hc[u] = ccol[u] = u16x4_t{0, 0, 0, 0};
            h0[u] = h1[u] = c0[u] = c1[u] = f64x2_t{0.0, 0.0};
            if (k < sph) {
                hc[u] = __builtin_nontemporal_load((const u16x4_t*)(ch + bh + k));
                h0[u] = __builtin_nontemporal_load((const f64x2_t*)(vh + bh + k));
                h1[u] = __builtin_nontemporal_load((const f64x2_t*)(vh + bh + k + 2));
            }
            if (k < spc) {
                ccol[u] = __builtin_nontemporal_load((const u16x4_t*)(cc + bc + k));
                c0[u] = __builtin_nontemporal_load((const f64x2_t*)(vc + bc + k));
                c1[u] = __builtin_nontemporal_load((const f64x2_t*)(vc + bc + k + 2));
            }
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int k = 4 * (u * BLOCK + tid);
            if (k < sph) {
                *(f64x2_t*)(prod + k) = f64x2_t{h0[u].x * whot[min((int)hc[u].x, HOT - 1)], h0[u].y * whot[min((int)hc[u].y, HOT - 1)]};
                *(f64x2_t*)(prod + k + 2) = f64x2_t{h1[u].x * whot[min((int)hc[u].z, HOT - 1)], h1[u].y * whot[min((int)hc[u].w, HOT - 1)]};
            }
            if (k < spc) {
                *(f64x2_t*)(prod + offc + k) = f64x2_t{c0[u].x * a.w[ccol[u].x], c0[u].y * a.w[ccol[u].y]};
                *(f64x2_t*)(prod + offc + k + 2) = f64x2_t{c1[u].x * a.w[ccol[u].z], c1[u].y * a.w[ccol[u].w]};
            }
        }
        __syncthreads();
        for (int r = grp; r < nr; r += BLOCK / 16) {
            double acc = 0.0;
            for (int q = roh[r] + sub; q < roh[r + 1]; q += 16) acc += prod[q];
            for (int q = roc[r] + sub; q < roc[r + 1]; q += 16) acc += prod[q];
            const double dot = cocoa::row16_sum(acc);
            if (sub == 0) {
                if (!test) {
                    hinge += cocoa::jmax(1 - yy[r0 + r] * dot, 0.0);
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
    double s4[4] = {hinge, al, w2, err};
    for (int i = 0; i < 4; ++i) {
        double v = cocoa::wave_sum(s4[i]);
        __syncthreads();
        if ((tid & 63) == 0) red[tid >> 6] = v;
        __syncthreads();
        double acc = 0.0;
        for (int j = 0; j < BLOCK / 64; ++j) acc += red[j];
        s4[i] = acc;
    }
    if (tid == 0)
        for (int i = 0; i < 4; ++i) a.partials[(size_t)blockIdx.x * 4 + i] = s4[i];
}

template <class T>
static T* dev(const std::vector<T>& h, size_t pad_bytes = 64) {
    T* p = nullptr;
    const size_t b = sizeof(T) * h.size();
    CK(hipMalloc(&p, b + pad_bytes));
    CK(hipMemset((char*)p + b, 0, pad_bytes));
    if (b) CK(hipMemcpy(p, h.data(), b, hipMemcpyHostToDevice));
    return p;
}

static std::vector<int64_t> tiles(const std::vector<int64_t>& rp, int64_t cap, int64_t row_cap) {
    const int64_t n = (int64_t)rp.size() - 1;
    std::vector<int64_t> t{0};
    int64_t r = 0;
    while (r < n) {
        const int64_t start = r, e0 = rp[r];
        if (rp[r + 1] - e0 > cap) {
            ++r;
        } else {
            while (r < n && rp[r + 1] - e0 <= cap && r - start < row_cap) ++r;
        }
        t.push_back(r);
    }
    const size_t nb = t.size();
    for (size_t i = 0; i < nb; ++i) t.push_back(rp[t[i]]);
    return t;
}

struct Side {
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
    std::vector<uint16_t> col16;
    std::vector<double> val, y;
};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    const bool all = argc > 2 ? std::strcmp(argv[2], "all") == 0 : true;  // "shipped": the library's kernel only
    const char* ev = std::getenv("COCOA_EVAL_VARIANT");
    const int64_t n = 677399, nt = 50000;
    const int32_t d = 47236;
    cocoa_dataset ds{};
    if (cocoa_gen_synthetic(0, n + nt, d, 75.6, 1, 12345, 0, 16, &ds)) {
        std::fprintf(stderr, "gen failed: %s\n", cocoa_last_error(nullptr));
        return 1;
    }
    // device feature order: by descending frequency (as cocoa_set_train)
    std::vector<int64_t> freq(d, 0);
    for (int64_t q = 0; q < ds.row_ptr[n]; ++q) freq[ds.col[q]]++;
    std::vector<int32_t> order(d), perm(d);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return freq[a] > freq[b]; });
    for (int32_t j = 0; j < d; ++j) perm[order[j]] = j;
    Side tr, te;
    auto fill = [&](Side& s, int64_t r0, int64_t r1) {
        const int64_t e0 = ds.row_ptr[r0];
        for (int64_t r = r0; r <= r1; ++r) s.rp.push_back(ds.row_ptr[r] - e0);
        for (int64_t q = e0; q < ds.row_ptr[r1]; ++q) {
            s.col.push_back(perm[ds.col[q]]);
            s.col16.push_back((uint16_t)perm[ds.col[q]]);
            s.val.push_back(ds.val[q]);
        }
        s.y.assign(ds.y + r0, ds.y + r1);
    };
    fill(tr, 0, n);
    fill(te, n, n + nt);
    std::vector<double> w(d), alpha(n);
    uint64_t st = 88172645463325252ull;
    auto rnd = [&]() {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        return (double)(st >> 11) * (1.0 / 9007199254740992.0);
    };
    for (auto& x : w) x = (rnd() - 0.5) * 0.2;
    for (auto& x : alpha) x = rnd();
    // host reference
    std::vector<double> xw(n);
    double hinge = 0.0, errs = 0.0, asum = 0.0, w2 = 0.0;
    for (int64_t r = 0; r < n; ++r) {
        double s = 0.0;
        for (int64_t q = tr.rp[r]; q < tr.rp[r + 1]; ++q) s += tr.val[q] * w[tr.col[q]];
        xw[r] = s;
        hinge += std::max(1 - tr.y[r] * s, 0.0);
    }
    for (int64_t r = 0; r < nt; ++r) {
        double s = 0.0;
        for (int64_t q = te.rp[r]; q < te.rp[r + 1]; ++q) s += te.val[q] * w[te.col[q]];
        errs += (s * te.y[r] > 0) ? 0.0 : 1.0;
    }
    for (double a : alpha) asum += a;
    for (double x : w) w2 += x * x;
    const double bytes = 12.0 * (double)(tr.val.size() + te.val.size()) + 8.0 * (n + 1) + 16.0 * n + 8.0 * d +
                         8.0 * (nt + 1) + 8.0 * nt;
    std::printf("C2 eval: train nnz %zu, test nnz %zu, algorithmic bytes %.1f MB\n", tr.val.size(), te.val.size(),
                bytes / 1e6);

    EvalArgs a{};
    a.row_ptr = dev(tr.rp);
    a.col = dev(tr.col);
    a.col16 = dev(tr.col16);
    a.val = dev(tr.val);
    a.y = dev(tr.y);
    a.alpha = dev(alpha);
    a.n = n;
    a.t_row_ptr = dev(te.rp);
    a.t_col = dev(te.col);
    a.t_col16 = dev(te.col16);
    a.t_val = dev(te.val);
    a.t_y = dev(te.y);
    a.n_test = nt;
    a.w = dev(w);
    a.d = d;
    std::vector<double> zeros(8 * 4096 + n, 0.0);
    double* partials = dev(zeros);
    double* out = dev(std::vector<double>(4, 0.0));
    double* rxw = dev(std::vector<double>(n, 0.0));
    a.partials = partials;
    a.out = out;
    a.row_xw = rxw;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto check = [&](const char* name, float ms) {
        double o[4];
        std::vector<double> gx(n);
        CK(hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost));
        CK(hipMemcpy(gx.data(), rxw, sizeof(double) * n, hipMemcpyDeviceToHost));
        double md = 0.0;
        for (int64_t r = 0; r < n; ++r) md = std::max(md, std::fabs(gx[r] - xw[r]) / std::max(1e-300, std::fabs(xw[r]) + 1e-12));
        const bool ok = std::fabs(o[0] - hinge) <= 1e-11 * std::fabs(hinge) && std::fabs(o[1] - asum) <= 1e-11 * asum &&
                        std::fabs(o[2] - w2) <= 1e-11 * w2 && o[3] == errs && md < 1e-9;
        std::printf("%-28s %8.4f ms  %6.3f TB/s  %5.1f%% of 8 TB/s   %s (hinge rel %.2e, xw max rel %.2e, err %g/%g)\n",
                    name, ms, bytes / (ms * 1e-3) / 1e12, 100.0 * bytes / (ms * 1e-3) / 8e12, ok ? "OK" : "MISMATCH",
                    std::fabs(o[0] - hinge) / hinge, md, o[3], errs);
        CK(hipMemset(rxw, 0, sizeof(double) * n));
    };
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };

    {  // shipped kernel
        // the library's tile size for this variant (COCOA_EVAL_VARIANT 6-9: 2,048)
        const int64_t cap = (ev && std::atoi(ev) >= 6 && std::atoi(ev) <= 9) ? 2048 : 4096;
        const auto t4 = tiles(tr.rp, cap, cap), tt4 = tiles(te.rp, cap, cap);
        EvalArgs b = a;
        b.tiles = dev(t4);
        b.n_tiles = (int64_t)t4.size() / 2 - 1;
        b.t_tiles = dev(tt4);
        b.n_t_tiles = (int64_t)tt4.size() / 2 - 1;
        const int nb = eval_fast_blocks(b.n_tiles, b.n_t_tiles);
        const float ms = timeit([&] { launch_eval_fast(b, nb, s); });
        char nm[64];
        std::snprintf(nm, sizeof nm, "shipped (variant %s)", ev ? ev : "0");
        check(nm, ms);
    }
    if (!all) return 0;
    auto run_wave = [&](const char* name, auto kern, int U, int block, int blocks_per_cu) {
        const auto t1 = tiles(tr.rp, ew_tile_entries(U), kEwRows), tt1 = tiles(te.rp, ew_tile_entries(U), kEwRows);
        EvalArgs b = a;
        b.tiles = dev(t1);
        b.n_tiles = (int64_t)t1.size() / 2 - 1;
        b.t_tiles = dev(tt1);
        b.n_t_tiles = (int64_t)tt1.size() / 2 - 1;
        const int nb = 256 * blocks_per_cu;
        const float ms = timeit([&] {
            kern<<<nb, block, 0, s>>>(b);
            final_kernel<<<1, 64, 0, s>>>(b.partials, nb, b.out);
        });
        char nm[96];
        std::snprintf(nm, sizeof nm, "%s U%d b%d x%d", name, U, block, blocks_per_cu);
        check(nm, ms);
    };
    {  // column-sorted 4,096-entry tiles
        const auto t4 = tiles(tr.rp, 4096, 4096), tt4 = tiles(te.rp, 4096, 4096);
        auto sorted = [&](const Side& sd, const std::vector<int64_t>& tl, std::vector<uint16_t>& sc,
                          std::vector<uint16_t>& sp, std::vector<double>& sv) {
            const size_t nnz = sd.val.size();
            sc.assign(nnz, 0);
            sp.assign(nnz, 0);
            sv.assign(nnz, 0.0);
            const size_t nt = tl.size() / 2 - 1;
            std::vector<int> idx;
            for (size_t i = 0; i < nt; ++i) {
                const int64_t e0 = tl[nt + 1 + i], e1 = tl[nt + 1 + i + 1];
                idx.resize((size_t)(e1 - e0));
                std::iota(idx.begin(), idx.end(), 0);
                std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return sd.col16[e0 + x] < sd.col16[e0 + y]; });
                for (int64_t q = 0; q < e1 - e0; ++q) {
                    sc[e0 + q] = sd.col16[e0 + idx[q]];
                    sp[e0 + q] = (uint16_t)idx[q];
                    sv[e0 + q] = sd.val[e0 + idx[q]];
                }
            }
        };
        std::vector<uint16_t> sc, sp, tsc, tsp;
        std::vector<double> sv, tsv;
        sorted(tr, t4, sc, sp, sv);
        sorted(te, tt4, tsc, tsp, tsv);
        SortedArgs z{dev(sc), dev(sp), dev(sv), dev(tsc), dev(tsp), dev(tsv)};
        EvalArgs b = a;
        b.tiles = dev(t4);
        b.n_tiles = (int64_t)t4.size() / 2 - 1;
        b.t_tiles = dev(tt4);
        b.n_t_tiles = (int64_t)tt4.size() / 2 - 1;
        const int nb = 768;
        const float ms = timeit([&] {
            eval_sorted_kernel<4096, 512><<<nb, 512, 0, s>>>(b, z);
            final_kernel<<<1, 64, 0, s>>>(b.partials, nb, b.out);
        });
        check("column-sorted tiles 4096", ms);
    }
    {  // split CSR: hot columns' entries (w in LDS) and the rest
        auto split = [&](const Side& sd, int hot, std::vector<int64_t>& rh, std::vector<uint16_t>& ch,
                         std::vector<double>& vh, std::vector<int64_t>& rc, std::vector<uint16_t>& cc,
                         std::vector<double>& vc) {
            rh.assign(1, 0);
            rc.assign(1, 0);
            ch.clear(); vh.clear(); cc.clear(); vc.clear();
            for (size_t r = 0; r + 1 < sd.rp.size(); ++r) {
                for (int64_t q = sd.rp[r]; q < sd.rp[r + 1]; ++q) {
                    if (sd.col16[q] < hot) { ch.push_back(sd.col16[q]); vh.push_back(sd.val[q]); }
                    else { cc.push_back(sd.col16[q]); vc.push_back(sd.val[q]); }
                }
                rh.push_back((int64_t)ch.size());
                rc.push_back((int64_t)cc.size());
            }
        };
        auto run_split = [&](const char* name, auto kern, int hot, int tile, int block, int nb) {
            std::vector<int64_t> rh, rc, trh, trc;
            std::vector<uint16_t> ch, cc, tch, tcc;
            std::vector<double> vh, vc, tvh, tvc;
            split(tr, hot, rh, ch, vh, rc, cc, vc);
            split(te, hot, trh, tch, tvh, trc, tcc, tvc);
            SplitArgs z{dev(rh), dev(ch), dev(vh), dev(rc), dev(cc), dev(vc),
                        dev(trh), dev(tch), dev(tvh), dev(trc), dev(tcc), dev(tvc)};
            const auto t4 = tiles(tr.rp, tile, tile), tt4 = tiles(te.rp, tile, tile);
            EvalArgs b = a;
            b.tiles = dev(t4);
            b.n_tiles = (int64_t)t4.size() / 2 - 1;
            b.t_tiles = dev(tt4);
            b.n_t_tiles = (int64_t)tt4.size() / 2 - 1;
            const float ms = timeit([&] {
                kern<<<nb, block, 0, s>>>(b, z);
                final_kernel<<<1, 64, 0, s>>>(b.partials, nb, b.out);
            });
            check(name, ms);
        };
        run_split("split hot2048 t4096 b512x2", eval_split_kernel<4096, 512, 2048>, 2048, 4096, 512, 512);
        run_split("split hot4096 t4096 b512x2", eval_split_kernel<4096, 512, 4096>, 4096, 4096, 512, 512);
        run_split("split hot2048 t2048 b256x4", eval_split_kernel<2048, 256, 2048>, 2048, 2048, 256, 1024);
        run_split("split hot4096 t2048 b256x3", eval_split_kernel<2048, 256, 4096>, 4096, 2048, 256, 768);
        run_split("split hot1024 t2048 b256x5", eval_split_kernel<2048, 256, 1024>, 1024, 2048, 256, 1280);
        run_split("split hot2048 t2048 b512x3", eval_split_kernel<2048, 512, 2048>, 2048, 2048, 512, 768);
    }
    run_wave("wave", eval_wave_kernel<4, 512, true>, 4, 512, 2);
    run_wave("wave", eval_wave_kernel<4, 256, true>, 4, 256, 4);
    run_wave("wave", eval_wave_kernel<2, 512, true>, 2, 512, 3);
    run_wave("wave", eval_wave_kernel<2, 256, true>, 2, 256, 6);
    run_wave("wave", eval_wave_kernel<3, 256, true>, 3, 256, 5);
    run_wave("wave-nogather", eval_wave_kernel<4, 512, true, true>, 4, 512, 2);
    std::printf("done\n");
    return 0;
}
