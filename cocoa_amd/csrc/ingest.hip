// GPU-side LIBSVM ingest: OptUtils.loadLIBSVMData (OptUtils.scala:11-53) with
// the tokenising and number parsing on the device.
//
//   1. the file goes to HBM once;
//   2. line starts: per 64 KB block a 256-thread workgroup counts newlines,
//      the host scans the block counts, a second pass writes every line start
//      in file order (block-local LDS scan);
//   3. count pass, one wave per line: trims the line (Java String.trim), splits
//      it on single spaces (String.split(' ')), applies the label rule
//      (OptUtils.scala:36-37) and parses every "index:value" token
//      (OptUtils.scala:41-42) -- lanes find the token starts with ballots, the
//      lane at a token start parses it;
//   4. the host builds row_ptr and the Hadoop-split partitions from the counts;
//   5. write pass: the same tokenising, entries stored at row_ptr.
//
// A line is parsed on the device when it is "simple": only [0-9 + - . e E :]
// between single spaces after trimming, indices of at most 9 digits inside
// [1, numFeatures], and values on the exact fast path of decimal conversion
// (at most 19 significant digits, m <= 2^53 and |exponent| <= 22: m * 10^e or
// m / 10^-e is one correctly rounded IEEE operation, the same double as the
// JDK's Double.parseDouble / strtod).  Any other line (tabs inside, "NaN",
// hex floats, type suffixes, long mantissas, malformed or out-of-range tokens)
// is flagged and parsed by the host with the CPU loader's rules, so results
// and exceptions are those of cocoa_load_libsvm, byte for byte.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cocoa_capi.h"
#include "common.h"
#include "libsvm.h"

namespace cocoa {
namespace {

constexpr int kNlBlock = 65536;  // bytes per newline-scan workgroup

__global__ __launch_bounds__(256) void nl_count_kernel(const char* buf, int64_t S, int64_t* counts) {
    const int64_t b0 = (int64_t)blockIdx.x * kNlBlock;
    int c = 0;
    for (int64_t i = b0 + threadIdx.x; i < min(S, b0 + kNlBlock); i += 256) c += buf[i] == '\n';
    __shared__ int red[256];
    red[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[blockIdx.x] = red[0];
}

// line starts p (p == 0, or buf[p-1] == '\n', p < S) in file order: thread t of
// a block owns bytes [b0 + 256 t, b0 + 256 (t + 1)); off = newlines before the block
__global__ __launch_bounds__(256) void nl_write_kernel(const char* buf, int64_t S, const int64_t* off,
                                                       int64_t* line_beg) {
    const int64_t b0 = (int64_t)blockIdx.x * kNlBlock;
    const int64_t t0 = b0 + (int64_t)threadIdx.x * (kNlBlock / 256), t1 = min(S, t0 + kNlBlock / 256);
    int c = 0;
    for (int64_t i = t0; i < t1; ++i) c += buf[i] == '\n';
    __shared__ int sc[257];
    sc[threadIdx.x + 1] = c;
    if (threadIdx.x == 0) sc[0] = 0;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int i = 1; i <= 256; ++i) sc[i] += sc[i - 1];
    __syncthreads();
    // line 0 starts at byte 0; the line after newline number j (0-based) is line j + 1
    int64_t o = off[blockIdx.x] + sc[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 0 && S > 0) line_beg[0] = 0;
    for (int64_t i = t0; i < t1; ++i)
        if (buf[i] == '\n') {
            ++o;
            if (i + 1 < S) line_beg[o] = i + 1;
        }
}

__device__ __forceinline__ bool ws(unsigned char c) { return c <= ' '; }
__device__ __forceinline__ bool simple_char(unsigned char c) {
    return (c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E' || c == ':' || c == ' ';
}

// exact powers of ten (1e0 .. 1e22 are representable)
__device__ __forceinline__ double pow10_exact(int e) {
    constexpr double t[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                              1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    return t[e];
}

// "index:value" at [p, e): true and (col, val) when it is on the device's fast path
__device__ bool parse_entry(const char* p, const char* e, int32_t d, int32_t* col, double* val) {
    bool neg = false;
    if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
    int64_t idx = 0;
    int nd = 0;
    while (p < e && *p >= '0' && *p <= '9') {
        idx = idx * 10 + (*p++ - '0');
        if (++nd > 9) return false;
    }
    if (nd == 0 || neg || p >= e || *p != ':') return false;
    ++p;
    if (idx < 1 || idx > d) return false;  // ArrayIndexOutOfBounds: the host reports it
    bool vneg = false;
    if (p < e && (*p == '+' || *p == '-')) vneg = *p++ == '-';
    uint64_t m = 0;
    int sig = 0, frac = 0, digits = 0;
    bool dot = false;
    for (; p < e; ++p) {
        const char c = *p;
        if (c >= '0' && c <= '9') {
            ++digits;
            if (dot) ++frac;
            if (m == 0 && c == '0') continue;  // leading zeros
            if (++sig > 19) return false;
            m = m * 10 + (uint64_t)(c - '0');
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            break;
        }
    }
    if (digits == 0) return false;
    int ex = 0;
    if (p < e && (*p == 'e' || *p == 'E')) {
        ++p;
        bool eneg = false;
        if (p < e && (*p == '+' || *p == '-')) eneg = *p++ == '-';
        int en = 0;
        while (p < e && *p >= '0' && *p <= '9') {
            ex = ex * 10 + (*p++ - '0');
            if (++en > 4) return false;
        }
        if (en == 0) return false;
        if (eneg) ex = -ex;
    }
    if (p != e) return false;
    const int e10 = ex - frac;
    double v;
    if (m == 0) {
        v = 0.0;
    } else {
        if (m > (1ull << 53) || e10 < -22 || e10 > 22) return false;
        v = e10 >= 0 ? (double)m * pow10_exact(e10) : (double)m / pow10_exact(-e10);
    }
    *col = (int32_t)(idx - 1);
    *val = vneg ? -v : v;
    return true;
}

// label token [p, e): +1 iff it contains '+' or parses (Integer.parseInt) to 1
__device__ bool parse_label(const char* p, const char* e, double* y) {
    for (const char* q = p; q < e; ++q)
        if (*q == '+') {
            *y = 1.0;
            return true;
        }
    bool neg = false;
    if (p < e && *p == '-') neg = true, ++p;
    int64_t v = 0;
    int nd = 0;
    for (; p < e; ++p) {
        if (*p < '0' || *p > '9') return false;
        v = v * 10 + (*p - '0');
        if (++nd > 9) return false;
    }
    if (nd == 0) return false;
    *y = (!neg && v == 1) ? 1.0 : -1.0;
    return true;
}

// One wave per line.  WRITE = false: count entries, label, flag; WRITE = true:
// store the entries of unflagged lines at row_ptr[r].
template <bool WRITE>
__global__ __launch_bounds__(256) void line_kernel(const char* buf, int64_t S, const int64_t* line_beg, int64_t n,
                                                   int32_t d, int32_t* cnt, double* y, uint8_t* flag,
                                                   const int64_t* row_ptr, int32_t* col, double* val) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const uint64_t lt = (1ull << lane) - 1;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += nw) {
        if (WRITE && flag[r]) continue;
        const int64_t lb = line_beg[r];
        const int64_t le = r + 1 < n ? line_beg[r + 1] - 1 : S;  // excludes the newline
        // String.trim: first / last byte > ' '
        int64_t tb = le, te = lb;
        for (int64_t base = lb; base < le; base += 64) {
            const int64_t q = base + lane;
            const uint64_t m = __ballot(q < le && !ws((unsigned char)buf[q]));
            if (m) {
                tb = base + __builtin_ctzll(m);
                break;
            }
        }
        for (int64_t base = le; base > tb; base -= 64) {
            const int64_t q = base - 1 - lane;
            const uint64_t m = __ballot(q >= tb && !ws((unsigned char)buf[q]));
            if (m) {
                te = base - __builtin_ctzll(m);  // one past the last non-blank byte
                break;
            }
        }
        bool bad = te <= tb;  // blank line: the host raises the reference's exception
        int32_t k = 0;
        double lab = 0.0;
        int64_t lab_end = te;
        if (!bad) {
            // end of the label token: first ' '
            for (int64_t base = tb; base < te; base += 64) {
                const int64_t q = base + lane;
                const uint64_t m = __ballot(q < te && buf[q] == ' ');
                if (m) {
                    lab_end = base + __builtin_ctzll(m);
                    break;
                }
            }
            bad = !parse_label(buf + tb, buf + lab_end, &lab);
        }
        const int64_t r0 = WRITE ? row_ptr[r] : 0;
        for (int64_t base = lab_end; !bad && base < te; base += 64) {
            const int64_t q = base + lane;
            const bool in = q < te;
            const unsigned char c = in ? (unsigned char)buf[q] : ' ';
            const bool start = in && q > lab_end && buf[q - 1] == ' ';
            // anything but [0-9+-.eE:] and single spaces goes to the host
            const bool odd = in && (!simple_char(c) || (c == ' ' && q > lab_end && buf[q - 1] == ' ') ||
                                    (start && c == ' '));
            if (__ballot(odd)) {
                bad = true;
                break;
            }
            const uint64_t sm = __ballot(start);
            bool ok = true;
            if (start) {
                int64_t e = q;
                while (e < te && buf[e] != ' ') ++e;
                int32_t cj;
                double vj;
                ok = parse_entry(buf + q, buf + e, d, &cj, &vj);
                if (WRITE && ok) {
                    const int64_t o = r0 + k + __popcll(sm & lt);
                    col[o] = cj;
                    val[o] = vj;
                }
            }
            if (__ballot(!ok)) bad = true;
            k += __popcll(sm);
        }
        if (!WRITE && lane == 0) {
            flag[r] = bad ? 1 : 0;
            cnt[r] = bad ? 0 : k;
            y[r] = lab;
        }
    }
}

struct DBuf {
    void* p = nullptr;
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T* as() {
        return (T*)p;
    }
};

}  // namespace
}  // namespace cocoa

using namespace cocoa;

#define ICHK(x)                                                                        \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) throw Error(COCOA_E_HIP, std::string("HIP: ") + hipGetErrorString(e_)); \
    } while (0)

extern "C" int cocoa_load_libsvm_gpu(int device, const char* path, int32_t num_splits, int32_t num_features,
                                     cocoa_dataset* out) {
    if (!path || !out || num_splits < 1 || num_features < 1)
        return host_error(COCOA_E_ARG, "cocoa_load_libsvm_gpu: bad argument");
    std::memset(out, 0, sizeof(*out));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev)
        return host_error(COCOA_E_NODEV, "cocoa_load_libsvm_gpu: no such HIP device");
    char* hbuf = nullptr;
    hipStream_t s = nullptr;
    try {
        ICHK(hipSetDevice(device));
        FILE* f = std::fopen(path, "rb");
        if (!f) return host_error(COCOA_E_IO, std::string("cannot open ") + path);
        std::fseek(f, 0, SEEK_END);
        const int64_t S = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        // pageable buffer: pinning the whole file costs more than HIP's staged copy
        hbuf = (char*)std::malloc((size_t)S + 1);
        if (!hbuf) {
            std::fclose(f);
            return host_error(COCOA_E_ARG, "cocoa_load_libsvm_gpu: out of host memory");
        }
        if (S > 0 && std::fread(hbuf, 1, (size_t)S, f) != (size_t)S) {
            std::fclose(f);
            std::free(hbuf);
            return host_error(COCOA_E_IO, std::string("read error on ") + path);
        }
        std::fclose(f);
        ICHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const std::vector<int64_t> starts = hadoop_split_starts(S, num_splits);
        const int K = std::min((int)starts.size(), (int)num_splits);  // coalesce(numSplits)

        DBuf dtext, dcnt_blk, doff, dbeg, dcnt, dy, dflag, drp, dcol, dval;
        ICHK(hipMalloc(&dtext.p, (size_t)S + 1));
        if (S > 0) ICHK(hipMemcpyAsync(dtext.p, hbuf, (size_t)S, hipMemcpyHostToDevice, s));
        // 2. line starts
        const int64_t nb = std::max<int64_t>(1, (S + kNlBlock - 1) / kNlBlock);
        ICHK(hipMalloc(&dcnt_blk.p, sizeof(int64_t) * (size_t)nb));
        ICHK(hipMalloc(&doff.p, sizeof(int64_t) * (size_t)nb));
        if (S > 0) nl_count_kernel<<<(unsigned)nb, 256, 0, s>>>(dtext.as<char>(), S, dcnt_blk.as<int64_t>());
        std::vector<int64_t> blk((size_t)nb, 0), off((size_t)nb, 0);
        if (S > 0) ICHK(hipMemcpyAsync(blk.data(), dcnt_blk.p, sizeof(int64_t) * (size_t)nb, hipMemcpyDeviceToHost, s));
        ICHK(hipStreamSynchronize(s));
        int64_t nl = 0;
        for (int64_t i = 0; i < nb; ++i) off[(size_t)i] = nl, nl += blk[(size_t)i];
        const int64_t n = S == 0 ? 0 : nl + (hbuf[S - 1] == '\n' ? 0 : 1);  // lines that start before S
        ICHK(hipMalloc(&dbeg.p, sizeof(int64_t) * (size_t)std::max<int64_t>(n, 1) + 8));
        if (S > 0) {
            ICHK(hipMemcpyAsync(doff.p, off.data(), sizeof(int64_t) * (size_t)nb, hipMemcpyHostToDevice, s));
            nl_write_kernel<<<(unsigned)nb, 256, 0, s>>>(dtext.as<char>(), S, doff.as<int64_t>(), dbeg.as<int64_t>());
        }
        // 3. count pass
        const size_t nn = (size_t)std::max<int64_t>(n, 1);
        ICHK(hipMalloc(&dcnt.p, sizeof(int32_t) * nn));
        ICHK(hipMalloc(&dy.p, sizeof(double) * nn));
        ICHK(hipMalloc(&dflag.p, nn));
        const unsigned lgrid = (unsigned)std::min<int64_t>(std::max<int64_t>((n + 3) / 4, 1), 256 * 8);
        if (n > 0)
            line_kernel<false><<<lgrid, 256, 0, s>>>(dtext.as<char>(), S, dbeg.as<int64_t>(), n, num_features,
                                                     dcnt.as<int32_t>(), dy.as<double>(), dflag.as<uint8_t>(),
                                                     nullptr, nullptr, nullptr);
        std::vector<int64_t> line_beg(nn);
        std::vector<int32_t> cnt(nn);
        std::vector<uint8_t> flag(nn);
        std::vector<double> yv(nn);
        if (n > 0) {
            ICHK(hipMemcpyAsync(line_beg.data(), dbeg.p, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost, s));
            ICHK(hipMemcpyAsync(cnt.data(), dcnt.p, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
            ICHK(hipMemcpyAsync(flag.data(), dflag.p, (size_t)n, hipMemcpyDeviceToHost, s));
            ICHK(hipMemcpyAsync(yv.data(), dy.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, s));
        }
        ICHK(hipStreamSynchronize(s));
        // 4. flagged lines on the host (in file order: the first malformed line raises)
        struct Host {
            int64_t r;
            std::vector<int32_t> c;
            std::vector<double> v;
        };
        std::vector<Host> hosted;
        for (int64_t r = 0; r < n; ++r) {
            if (!flag[(size_t)r]) continue;
            const int64_t p = line_beg[(size_t)r];
            const int64_t e = r + 1 < n ? line_beg[(size_t)r + 1] - 1 : S;
            const int64_t cap = std::count(hbuf + p, hbuf + e, ':');
            Host h{r, std::vector<int32_t>((size_t)std::max<int64_t>(cap, 1)),
                   std::vector<double>((size_t)std::max<int64_t>(cap, 1))};
            int64_t z = 0;
            std::string msg;
            const int rc = libsvm_parse_line(hbuf + p, hbuf + e, r, num_features, &yv[(size_t)r], h.c.data(),
                                             h.v.data(), &z, &msg);
            if (rc != COCOA_OK) {
                (void)hipStreamDestroy(s);
                std::free(hbuf);
                return host_error(rc, msg);
            }
            h.c.resize((size_t)z);
            h.v.resize((size_t)z);
            cnt[(size_t)r] = (int32_t)z;
            hosted.push_back(std::move(h));
        }
        // row_ptr and partitions (Hadoop split of each line's first byte)
        int64_t nnz = 0;
        for (int64_t r = 0; r < n; ++r) nnz += cnt[(size_t)r];
        if (!dataset_alloc(out, n, nnz, K)) throw Error(COCOA_E_ARG, "out of host memory");
        out->n_rows = n;
        out->num_features = num_features;
        out->num_parts = K;
        out->nnz = nnz;
        out->row_ptr[0] = 0;
        LinePartitioner lp(starts, K);
        for (int64_t r = 0; r < n; ++r) {
            out->row_ptr[r + 1] = out->row_ptr[r] + cnt[(size_t)r];
            out->part_ptr[lp.part(line_beg[(size_t)r]) + 1]++;
            out->y[r] = yv[(size_t)r];
        }
        for (int k = 1; k <= K; ++k) out->part_ptr[k] += out->part_ptr[k - 1];
        // 5. write pass
        ICHK(hipMalloc(&drp.p, sizeof(int64_t) * (size_t)(n + 1)));
        ICHK(hipMalloc(&dcol.p, sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1)));
        ICHK(hipMalloc(&dval.p, sizeof(double) * (size_t)std::max<int64_t>(nnz, 1)));
        ICHK(hipMemcpyAsync(drp.p, out->row_ptr, sizeof(int64_t) * (size_t)(n + 1), hipMemcpyHostToDevice, s));
        if (n > 0)
            line_kernel<true><<<lgrid, 256, 0, s>>>(dtext.as<char>(), S, dbeg.as<int64_t>(), n, num_features,
                                                    dcnt.as<int32_t>(), dy.as<double>(), dflag.as<uint8_t>(),
                                                    drp.as<int64_t>(), dcol.as<int32_t>(), dval.as<double>());
        if (nnz > 0) {
            ICHK(hipMemcpyAsync(out->col, dcol.p, sizeof(int32_t) * (size_t)nnz, hipMemcpyDeviceToHost, s));
            ICHK(hipMemcpyAsync(out->val, dval.p, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToHost, s));
        }
        ICHK(hipStreamSynchronize(s));
        ICHK(hipGetLastError());
        for (const Host& h : hosted) {
            const int64_t o = out->row_ptr[h.r];
            std::copy(h.c.begin(), h.c.end(), out->col + o);
            std::copy(h.v.begin(), h.v.end(), out->val + o);
        }
        (void)hipStreamDestroy(s);
        std::free(hbuf);
        return COCOA_OK;
    } catch (const Error& e) {
        if (s) (void)hipStreamDestroy(s);
        if (hbuf) std::free(hbuf);
        cocoa_dataset_free(out);
        return host_error(e.code, e.what());
    }
}
