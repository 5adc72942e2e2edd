// Host-side data layer of libcocoa_hip.so (no device code).
//
//  * cocoa_load_libsvm   -- OptUtils.loadLIBSVMData (OptUtils.scala:11-53),
//    including the Hadoop-1.0.4 FileInputFormat byte-split rule that decides
//    which rows land in which partition, and Scala/Java token semantics.
//  * cocoa_gen_synthetic -- seeded synthetic problems of the BASELINE.json
//    shapes (rcv1-like, epsilon-like, url-like).
//  * cocoa_jrandom_ints  -- java.util.Random on the host.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cocoa_capi.h"
#include "common.h"
#include "jdouble.h"
#include "jrandom.h"
#include "libsvm.h"

namespace cocoa {

// ---------------------------------------------------------------- LIBSVM --
namespace {

inline bool java_ws(char c) { return (unsigned char)c <= ' '; }

// Integer.parseInt (Scala String.toInt)
bool parse_int(const char* b, const char* e, int32_t* out) {
    if (b >= e) return false;
    bool neg = false;
    if (*b == '+' || *b == '-') {
        neg = *b == '-';
        ++b;
    }
    if (b >= e) return false;
    long long v = 0;
    for (; b < e; ++b) {
        if (*b < '0' || *b > '9') return false;
        v = v * 10 + (*b - '0');
        if (v > 2147483648LL) return false;
    }
    if (neg) v = -v;
    if (v > 2147483647LL) return false;
    *out = (int32_t)v;
    return true;
}

// Double.parseDouble for decimal / NaN / Infinity spellings (strtod is correctly
// rounded like the JDK; a trailing f/F/d/D type suffix is accepted like Java).
bool parse_double(const char* b, const char* e, double* out) {
    while (b < e && java_ws(*b)) ++b;
    while (e > b && java_ws(e[-1])) --e;
    if (b >= e || e - b > 120) return false;
    std::string s(b, e);
    if (s.size() > 1 && std::strchr("fFdD", s.back())) s.pop_back();
    if (s == "NaN" || s == "+NaN" || s == "-NaN") {
        *out = std::nan("");
        return true;
    }
    if (s == "Infinity" || s == "+Infinity") {
        *out = INFINITY;
        return true;
    }
    if (s == "-Infinity") {
        *out = -INFINITY;
        return true;
    }
    for (char c : s)
        if (!((c >= '0' && c <= '9') || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-')) return false;
    char* end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    if (end != s.c_str() + s.size()) return false;
    *out = v;
    return true;
}

// Hadoop 1.0.4 FileInputFormat.getSplits on a local file of `size` bytes.
std::vector<int64_t> split_starts(int64_t size, int num_splits) {
    const int64_t goal = size / std::max(num_splits, 1);
    const int64_t block = 32LL << 20;  // LocalFileSystem default block size
    const int64_t split = std::max<int64_t>(1, std::min(goal, block));
    std::vector<int64_t> starts;
    int64_t rem = size;
    while ((double)rem / (double)split > 1.1) {  // SPLIT_SLOP
        starts.push_back(size - rem);
        rem -= split;
    }
    if (rem != 0) starts.push_back(size - rem);
    if (starts.empty()) starts.push_back(0);
    return starts;
}

}  // namespace

std::vector<int64_t> hadoop_split_starts(int64_t size, int num_splits) { return split_starts(size, num_splits); }

}  // namespace cocoa

using namespace cocoa;

static thread_local std::string g_host_err;
const char* cocoa_host_last_error() { return g_host_err.c_str(); }

static int host_fail(int code, const std::string& msg) {
    g_host_err = msg;
    cocoa_set_global_error(msg);
    return code;
}
namespace cocoa {
int host_error(int code, const std::string& msg) { return host_fail(code, msg); }
}

extern "C" void cocoa_dataset_free(cocoa_dataset* ds) {
    if (!ds) return;
    std::free(ds->row_ptr);
    std::free(ds->col);
    std::free(ds->val);
    std::free(ds->y);
    std::free(ds->part_ptr);
    std::memset(ds, 0, sizeof(*ds));
}

namespace cocoa {
bool dataset_alloc(cocoa_dataset* ds, int64_t n, int64_t nnz, int32_t K);
}
static bool ds_alloc(cocoa_dataset* ds, int64_t n, int64_t nnz, int32_t K) { return cocoa::dataset_alloc(ds, n, nnz, K); }
bool cocoa::dataset_alloc(cocoa_dataset* ds, int64_t n, int64_t nnz, int32_t K) {
    ds->row_ptr = (int64_t*)std::malloc(sizeof(int64_t) * (size_t)(n + 1));
    ds->col = (int32_t*)std::malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1));
    ds->val = (double*)std::malloc(sizeof(double) * (size_t)std::max<int64_t>(nnz, 1));
    ds->y = (double*)std::malloc(sizeof(double) * (size_t)std::max<int64_t>(n, 1));
    ds->part_ptr = (int64_t*)std::calloc((size_t)K + 1, sizeof(int64_t));
    return ds->row_ptr && ds->col && ds->val && ds->y && ds->part_ptr;
}

// One LIBSVM line (OptUtils.scala:31-50): label rule ("+" anywhere, or the
// integer 1 -> +1, else -1), then "index:value" tokens split on single spaces,
// index - 1 checked against numFeatures.  Writes y, the entries and their
// count; on a malformed line returns the reference's exception kind.
int cocoa::libsvm_parse_line(const char* b, const char* le, int64_t r, int32_t num_features, double* y, int32_t* col,
                             double* val, int64_t* z, std::string* msg) {
    int64_t k = 0;
    while (b < le && java_ws(*b)) ++b;  // line.trim()
    while (le > b && java_ws(le[-1])) --le;
    // line.split(' '): tokens separated by single spaces; trailing empties dropped
    const char* tok = b;
    bool first = true;
    for (;;) {
        const char* te = tok;
        while (te < le && *te != ' ') ++te;
        if (first) {
            const bool plus = std::memchr(tok, '+', (size_t)(te - tok)) != nullptr;
            double lab = -1.0;
            if (plus) {
                lab = 1.0;
            } else {
                int32_t v;
                if (!parse_int(tok, te, &v)) {
                    *msg = "NumberFormatException: label on line " + std::to_string(r + 1);
                    return COCOA_E_PARSE;
                }
                if (v == 1) lab = 1.0;
            }
            *y = lab;
            first = false;
        } else {
            bool rest_blank = true;
            for (const char* q = tok; q < le; ++q)
                if (*q != ' ') {
                    rest_blank = false;
                    break;
                }
            if (rest_blank) break;
            const char* c = (const char*)std::memchr(tok, ':', (size_t)(te - tok));
            if (!c || c + 1 >= te || std::memchr(c + 1, ':', (size_t)(te - c - 1))) {
                *msg = "MatchError: feature token on line " + std::to_string(r + 1);
                return COCOA_E_PARSE;
            }
            int32_t idx;
            double v;
            if (!parse_int(tok, c, &idx) || !parse_double(c + 1, te, &v)) {
                *msg = "NumberFormatException: feature on line " + std::to_string(r + 1);
                return COCOA_E_PARSE;
            }
            const int64_t j = (int64_t)idx - 1;
            if (j < 0 || j >= num_features) {
                *msg = "ArrayIndexOutOfBoundsException: feature index " + std::to_string(idx) + " on line " +
                       std::to_string(r + 1) + " (numFeatures=" + std::to_string(num_features) + ")";
                return COCOA_E_RANGE;
            }
            col[k] = (int32_t)j;
            val[k] = v;
            ++k;
        }
        if (te >= le) break;
        tok = te + 1;
    }
    *z = k;
    return COCOA_OK;
}

extern "C" int cocoa_load_libsvm(const char* path, int32_t num_splits, int32_t num_features, cocoa_dataset* out) {
    if (!path || !out || num_splits < 1) return host_fail(COCOA_E_ARG, "cocoa_load_libsvm: bad argument");
    std::memset(out, 0, sizeof(*out));
    FILE* f = std::fopen(path, "rb");
    if (!f) return host_fail(COCOA_E_IO, std::string("cannot open ") + path);
    std::fseek(f, 0, SEEK_END);
    const int64_t S = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<char> buf((size_t)S + 1, 0);
    if (S > 0 && std::fread(buf.data(), 1, (size_t)S, f) != (size_t)S) {
        std::fclose(f);
        return host_fail(COCOA_E_IO, std::string("read error on ") + path);
    }
    std::fclose(f);
    const std::vector<int64_t> starts = split_starts(S, num_splits);
    const int ns = (int)starts.size();
    const int K = std::min(ns, (int)num_splits);  // coalesce(numSplits)

    // Multithreaded ingest (one pass per stage, threads over byte / line
    // ranges); results and error reporting are those of the sequential parse:
    // the first malformed line in file order raises.
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                                 S / (1 << 20) + 1}));
    auto run = [&](auto&& fn) {
        std::vector<std::thread> th;
        for (int i = 1; i < nt; ++i) th.emplace_back(fn, i);
        fn(0);
        for (auto& x : th) x.join();
    };
    // pass 1: line starts and per-line ':' counts (an upper bound of the line's nnz)
    std::vector<std::vector<int64_t>> lb(nt), lc(nt);
    run([&](int i) {
        const int64_t c0 = S * i / nt, c1 = S * (i + 1) / nt;
        int64_t p = c0;
        if (p > 0) {  // first line starting inside [c0, c1)
            const char* nl = (const char*)std::memchr(buf.data() + p - 1, '\n', (size_t)(S - p + 1));
            p = nl ? (nl - buf.data()) + 1 : S;
        }
        while (p < c1) {
            const char* nl = (const char*)std::memchr(buf.data() + p, '\n', (size_t)(S - p));
            const int64_t e = nl ? nl - buf.data() : S;
            int64_t cc = 0;
            for (int64_t q = p; q < e; ++q) cc += buf[(size_t)q] == ':';
            lb[(size_t)i].push_back(p);
            lc[(size_t)i].push_back(cc);
            p = e + 1;
        }
    });
    std::vector<int64_t> line_beg, cap{0};
    for (int i = 0; i < nt; ++i) {
        line_beg.insert(line_beg.end(), lb[(size_t)i].begin(), lb[(size_t)i].end());
        for (int64_t c : lc[(size_t)i]) cap.push_back(cap.back() + c);
        std::vector<int64_t>().swap(lb[(size_t)i]);
        std::vector<int64_t>().swap(lc[(size_t)i]);
    }
    const int64_t n = (int64_t)line_beg.size();
    if (!ds_alloc(out, n, cap.back(), K)) return host_fail(COCOA_E_ARG, "out of host memory");
    out->n_rows = n;
    out->num_features = num_features;
    out->num_parts = K;

    // pass 2: parse lines in parallel, each into its slot at cap[r]
    std::vector<int64_t> zr((size_t)n, 0);
    std::vector<int64_t> bad_line((size_t)nt, n);
    std::vector<int> bad_code((size_t)nt, COCOA_OK);
    std::vector<std::string> bad_msg((size_t)nt);
    run([&](int i) {
        const int64_t r0 = n * i / nt, r1 = n * (i + 1) / nt;
        for (int64_t r = r0; r < r1; ++r) {
            const int64_t p = line_beg[(size_t)r];
            const int64_t e = r + 1 < n ? line_beg[(size_t)r + 1] - 1 : S;
            std::string msg;
            const int rc = libsvm_parse_line(buf.data() + p, buf.data() + e, r, num_features, out->y + r,
                                      out->col + cap[(size_t)r], out->val + cap[(size_t)r], &zr[(size_t)r], &msg);
            if (rc != COCOA_OK) {
                bad_line[(size_t)i] = r;
                bad_code[(size_t)i] = rc;
                bad_msg[(size_t)i] = msg;
                return;
            }
        }
    });
    for (int i = 0; i < nt; ++i)
        if (bad_code[(size_t)i] != COCOA_OK) {  // threads own increasing line ranges: the first is the earliest
            cocoa_dataset_free(out);
            return host_fail(bad_code[(size_t)i], bad_msg[(size_t)i]);
        }

    // pass 3: partitions (Hadoop split of the line's first byte), row_ptr, and
    // compaction of the slots (in place, moving left, only where a line had
    // fewer entries than ':' characters)
    int64_t nnz = 0;
    LinePartitioner lp(starts, K);
    out->row_ptr[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        out->part_ptr[lp.part(line_beg[(size_t)r]) + 1]++;
        const int64_t z = zr[(size_t)r], src = cap[(size_t)r];
        if (src != nnz && z > 0) {
            std::memmove(out->col + nnz, out->col + src, sizeof(int32_t) * (size_t)z);
            std::memmove(out->val + nnz, out->val + src, sizeof(double) * (size_t)z);
        }
        nnz += z;
        out->row_ptr[r + 1] = nnz;
    }
    for (int k = 1; k <= K; ++k) out->part_ptr[k] += out->part_ptr[k - 1];
    out->nnz = nnz;
    return COCOA_OK;
}

// ------------------------------------------------------------- synthetic --
namespace {

// Walker alias table for O(1) sampling of a discrete distribution.
struct Alias {
    std::vector<double> prob;
    std::vector<int32_t> alias;
    explicit Alias(const std::vector<double>& w) {
        const size_t n = w.size();
        prob.resize(n);
        alias.resize(n);
        double tot = 0;
        for (double x : w) tot += x;
        std::vector<double> p(n);
        std::vector<int32_t> small, large;
        for (size_t i = 0; i < n; ++i) {
            p[i] = w[i] * (double)n / tot;
            (p[i] < 1.0 ? small : large).push_back((int32_t)i);
        }
        while (!small.empty() && !large.empty()) {
            const int32_t s = small.back(), l = large.back();
            small.pop_back();
            prob[(size_t)s] = p[(size_t)s];
            alias[(size_t)s] = l;
            p[(size_t)l] = (p[(size_t)l] + p[(size_t)s]) - 1.0;
            if (p[(size_t)l] < 1.0) {
                large.pop_back();
                small.push_back(l);
            }
        }
        for (int32_t i : large) prob[(size_t)i] = 1.0, alias[(size_t)i] = i;
        for (int32_t i : small) prob[(size_t)i] = 1.0, alias[(size_t)i] = i;
    }
    int32_t draw(std::mt19937_64& g) const {
        const uint64_t u = g();
        const size_t i = (size_t)((u >> 11) % prob.size());
        const double f = (double)(g() >> 11) * (1.0 / 9007199254740992.0);
        return f < prob[i] ? (int32_t)i : alias[i];
    }
};

uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

template <class F>
void parallel_blocks(int64_t nblocks, int threads, F&& fn) {
    std::atomic<int64_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&] {
            for (int64_t b; (b = next.fetch_add(1)) < nblocks;) fn(b);
        });
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" int cocoa_gen_synthetic(int32_t kind, int64_t n, int32_t d, double mean_nnz, int32_t K, uint64_t seed,
                                   int64_t first_row, int32_t threads, cocoa_dataset* out) {
    if (!out || n < 1 || d < 1 || K < 1 || K > n || kind < 0 || kind > 2 || first_row < 0 || first_row % 4096)
        return host_fail(COCOA_E_ARG, "cocoa_gen_synthetic: bad argument");
    std::memset(out, 0, sizeof(*out));
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    threads = std::min(threads, 64);
    const int64_t BR = 4096;  // rows per RNG block (result independent of thread count)
    const int64_t nb = (n + BR - 1) / BR;
    const uint64_t b0 = (uint64_t)(first_row / BR);  // global block index of row 0 (rank shards)

    // planted separator and the column permutation / popularity
    std::mt19937_64 g0(splitmix(seed));
    std::normal_distribution<double> N01(0.0, 1.0);
    std::vector<double> wstar((size_t)d);
    for (auto& x : wstar) x = N01(g0);
    std::vector<int32_t> perm((size_t)d);
    for (int32_t j = 0; j < d; ++j) perm[(size_t)j] = j;
    std::shuffle(perm.begin(), perm.end(), g0);
    const double zipf_s = kind == 2 ? 1.2 : 1.1;
    std::vector<double> pw((size_t)d), idf((size_t)d);
    for (int32_t r = 0; r < d; ++r) {
        pw[(size_t)r] = std::pow((double)(r + 1), -zipf_s);
        idf[(size_t)r] = 1.0 + std::log((double)(r + 1));
    }
    Alias zipf(pw);

    // pass 1: row lengths
    std::vector<int64_t> len((size_t)n);
    const double sig = 0.8, mu = std::log(std::max(mean_nnz, 1.0)) - 0.5 * sig * sig;
    const int64_t zmax = kind == 1 ? d : std::min<int64_t>(d, kind == 0 ? 2000 : 4000);
    parallel_blocks(nb, threads, [&](int64_t b) {
        std::mt19937_64 g(splitmix(seed ^ (0x1000000ULL + b0 + (uint64_t)b)));
        std::normal_distribution<double> nd(0.0, 1.0);
        for (int64_t r = b * BR; r < std::min(n, (b + 1) * BR); ++r) {
            int64_t z;
            if (kind == 1) {
                z = d;
            } else {
                z = (int64_t)std::llround(std::exp(mu + sig * nd(g)));
                z = std::max<int64_t>(1, std::min(z, zmax));
            }
            len[(size_t)r] = z;
        }
    });
    int64_t nnz = 0;
    for (int64_t r = 0; r < n; ++r) nnz += len[(size_t)r];
    if (!ds_alloc(out, n, nnz, K)) {
        cocoa_dataset_free(out);
        return host_fail(COCOA_E_ARG, "out of host memory");
    }
    out->row_ptr[0] = 0;
    for (int64_t r = 0; r < n; ++r) out->row_ptr[r + 1] = out->row_ptr[r] + len[(size_t)r];
    out->n_rows = n;
    out->num_features = d;
    out->num_parts = K;
    out->nnz = nnz;
    for (int32_t k = 0; k <= K; ++k) out->part_ptr[k] = (int64_t)(((__int128)n * k) / K);

    // pass 2: columns, values, labels
    parallel_blocks(nb, threads, [&](int64_t b) {
        std::mt19937_64 g(splitmix(seed ^ (0x2000000ULL + b0 + (uint64_t)b)));
        std::normal_distribution<double> nd(0.0, 1.0);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        std::vector<int32_t> ranks;
        std::vector<uint8_t> seen;
        if (kind != 1) seen.assign((size_t)d, 0);
        for (int64_t r = b * BR; r < std::min(n, (b + 1) * BR); ++r) {
            const int64_t z = len[(size_t)r], o = out->row_ptr[r];
            int32_t* c = out->col + o;
            double* v = out->val + o;
            if (kind == 1) {
                for (int64_t j = 0; j < z; ++j) c[j] = (int32_t)j, v[j] = nd(g);
            } else {
                ranks.clear();
                while ((int64_t)ranks.size() < z) {
                    const int32_t rk = zipf.draw(g);
                    if (!seen[(size_t)rk]) seen[(size_t)rk] = 1, ranks.push_back(rk);
                }
                for (int32_t rk : ranks) seen[(size_t)rk] = 0;
                std::vector<std::pair<int32_t, double>> e((size_t)z);
                for (int64_t j = 0; j < z; ++j) {
                    const int32_t rk = ranks[(size_t)j];
                    double val;
                    if (kind == 0) {
                        const double tf = 1.0 + std::floor(-std::log(1.0 - U(g)) * 1.5);
                        val = (1.0 + std::log(tf)) * idf[(size_t)rk];
                    } else {
                        val = U(g) < 0.9 ? 1.0 : 1.0 + std::floor(U(g) * 4.0);
                    }
                    e[(size_t)j] = {perm[(size_t)rk], val};
                }
                std::sort(e.begin(), e.end());
                for (int64_t j = 0; j < z; ++j) c[j] = e[(size_t)j].first, v[j] = e[(size_t)j].second;
            }
            double s2 = 0.0;
            for (int64_t j = 0; j < z; ++j) s2 += v[j] * v[j];
            const double inv = s2 > 0 ? 1.0 / std::sqrt(s2) : 0.0;
            double m = 0.0;
            for (int64_t j = 0; j < z; ++j) {
                v[j] *= inv;
                m += v[j] * wstar[(size_t)c[j]];
            }
            out->y[r] = (m + 0.1 * nd(g)) > 0.0 ? 1.0 : -1.0;
        }
    });
    return COCOA_OK;
}

extern "C" int cocoa_jrandom_ints(int64_t seed, int32_t bound, int32_t count, int32_t* out) {
    if (!out || count < 0) return host_fail(COCOA_E_ARG, "cocoa_jrandom_ints: bad argument");
    JRandom r(seed);
    for (int32_t i = 0; i < count; ++i) out[i] = bound > 0 ? r.next_int(bound) : r.next(32);
    return COCOA_OK;
}

// java.lang.Double.toString of the reference's JVM (JDK 7/8 FloatingDecimal)
extern "C" int cocoa_java_double_string(double x, char* buf, int32_t cap) {
    if (!buf || cap <= 0) return COCOA_E_ARG;
    const std::string t = cocoa::jdouble::to_string(x);
    if ((int32_t)t.size() + 1 > cap) return COCOA_E_ARG;
    std::memcpy(buf, t.c_str(), t.size() + 1);
    return COCOA_OK;
}
