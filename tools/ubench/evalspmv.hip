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
void launch_eval_fast(const EvalArgs& a, int blocks, hipStream_t s);
int eval_fast_blocks(int64_t n, int64_t n_test);
}

__global__ void final_kernel(const double* p, int blocks, double* out) {
    if (threadIdx.x < 4) {
        double s = 0.0;
        for (int b = 0; b < blocks; ++b) s += p[(size_t)b * 4 + threadIdx.x];
        out[threadIdx.x] = s;
    }
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
        const auto t4 = tiles(tr.rp, 4096, 4096), tt4 = tiles(te.rp, 4096, 4096);
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
    run_wave("wave", eval_wave_kernel<4, 512, true>, 4, 512, 2);
    run_wave("wave", eval_wave_kernel<4, 256, true>, 4, 256, 4);
    run_wave("wave", eval_wave_kernel<2, 512, true>, 2, 512, 3);
    run_wave("wave", eval_wave_kernel<2, 256, true>, 2, 256, 6);
    run_wave("wave", eval_wave_kernel<3, 256, true>, 3, 256, 5);
    run_wave("wave-nogather", eval_wave_kernel<4, 512, true, true>, 4, 512, 2);
    std::printf("done\n");
    return 0;
}
