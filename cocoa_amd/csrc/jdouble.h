// java.lang.Double.toString as JDK 7/8 printed it (the reference's runtime:
// Spark 1.3.1 / Scala 2.10).  sun.misc.FloatingDecimal's BinaryToASCIIBuffer
// does not always give the shortest round-tripping digits (JDK-4511638,
// changed in JDK 19: 2.0E23 prints as "1.9999999999999998E23").  Restated
// here: the long fast path (developLongDigits with its insignificant-digit
// rounding), estimateDecExp, the int / long / big-integer digit loops with
// their stopping tests and last-digit rounding, and the compatible-format
// layout.  Same algorithm as cocoa_amd/jdouble.py (tests/test_jdouble.py
// compares the two).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace cocoa {
namespace jdouble {

// minimal unsigned big integer (base 2^32, little endian) for the hard case
struct Big {
    std::vector<uint32_t> w;
    explicit Big(uint64_t v = 0) {
        while (v) {
            w.push_back((uint32_t)v);
            v >>= 32;
        }
    }
    void trim() {
        while (!w.empty() && w.back() == 0) w.pop_back();
    }
    void mul_small(uint32_t m) {
        uint64_t c = 0;
        for (auto& x : w) {
            const uint64_t t = (uint64_t)x * m + c;
            x = (uint32_t)t;
            c = t >> 32;
        }
        if (c) w.push_back((uint32_t)c);
    }
    void shl(int n) {
        if (w.empty() || n == 0) return;
        const int ws = n / 32, bs = n % 32;
        std::vector<uint32_t> r((size_t)ws, 0);
        uint32_t c = 0;
        for (auto x : w) {
            r.push_back(bs ? (x << bs) | c : x);
            c = bs ? x >> (32 - bs) : 0;
        }
        if (c) r.push_back(c);
        w.swap(r);
    }
    void mul_pow5(int n) {
        for (; n >= 13; n -= 13) mul_small(1220703125u);  // 5^13
        uint32_t p = 1;
        for (int i = 0; i < n; ++i) p *= 5;
        if (p > 1) mul_small(p);
    }
    static int cmp(const Big& a, const Big& b) {
        if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
        for (size_t i = a.w.size(); i-- > 0;)
            if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
        return 0;
    }
    void sub(const Big& b) {  // *this >= b
        int64_t c = 0;
        for (size_t i = 0; i < w.size(); ++i) {
            const int64_t t = (int64_t)w[i] - (i < b.w.size() ? b.w[i] : 0) + c;
            w[i] = (uint32_t)t;
            c = t < 0 ? -1 : 0;
        }
        trim();
    }
    static Big add(const Big& a, const Big& b) {
        Big r;
        const size_t n = std::max(a.w.size(), b.w.size());
        uint64_t c = 0;
        for (size_t i = 0; i < n; ++i) {
            const uint64_t t = (uint64_t)(i < a.w.size() ? a.w[i] : 0) + (i < b.w.size() ? b.w[i] : 0) + c;
            r.w.push_back((uint32_t)t);
            c = t >> 32;
        }
        if (c) r.w.push_back((uint32_t)c);
        return r;
    }
    static Big pow52(int p5, int p2) {
        Big r(1);
        r.mul_pow5(p5);
        r.shl(p2);
        return r;
    }
};

static const int kN5Bits[] = {0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31,
                              33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61};
static const int kInsignificant[] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6,
                                     6, 6, 7, 7, 7, 8, 8, 8, 9, 9, 9, 9, 10, 10, 10, 11, 11, 11, 12, 12,
                                     12, 12, 13, 13, 13, 14, 14, 14, 15, 15, 15, 15, 16, 16, 16, 17, 17, 17,
                                     18, 18, 18, 19};

inline uint64_t pow5_u64(int n) {
    uint64_t p = 1;
    for (int i = 0; i < n; ++i) p *= 5;
    return p;
}

struct Digits {
    std::vector<int> d;
    int dec_exponent = 0;
    void roundup() {
        int i = (int)d.size() - 1;
        int q = d[(size_t)i];
        if (q == 9) {
            while (q == 9 && i > 0) {
                d[(size_t)i] = 0;
                q = d[(size_t)--i];
            }
            if (q == 9) {
                dec_exponent += 1;
                d[0] = 1;
                return;
            }
        }
        d[(size_t)i] = q + 1;
    }
};

inline Digits develop_long_digits(int dec_exponent, int64_t lvalue, int insignificant) {
    if (insignificant != 0) {
        const int64_t pow10 = (int64_t)(pow5_u64(insignificant) << insignificant);
        const int64_t residue = lvalue % pow10;
        lvalue /= pow10;
        dec_exponent += insignificant;
        if (residue >= (pow10 >> 1)) lvalue++;
    }
    std::vector<int> out;
    int64_t c = lvalue % 10;
    lvalue /= 10;
    while (c == 0) {
        dec_exponent++;
        c = lvalue % 10;
        lvalue /= 10;
    }
    while (lvalue != 0) {
        out.push_back((int)c);
        dec_exponent++;
        c = lvalue % 10;
        lvalue /= 10;
    }
    out.push_back((int)c);
    Digits r;
    r.d.assign(out.rbegin(), out.rend());
    r.dec_exponent = dec_exponent + 1;
    return r;
}

inline int estimate_dec_exp(uint64_t fract_bits, int bin_exp) {
    uint64_t b = (0x3FFull << 52) | (fract_bits & ((1ull << 52) - 1));
    double d2;
    std::memcpy(&d2, &b, 8);
    const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + (double)bin_exp * 0.301029995663981;
    return (int)std::floor(d);
}

// the int / long loops: Java's wraparound arithmetic on W-bit signed integers
template <class T, class U>
inline void small_loop(uint64_t fract_bits, int B5, int B2, int S5, int S2, int M5, int M2, int& dec_exp,
                       std::vector<int>& digits, bool& low, bool& high, int64_t& low_diff) {
    auto w = [](U x) { return (T)x; };
    T b = w((U)w((U)fract_bits * (U)pow5_u64(B5)) << B2);
    const T s = w((U)pow5_u64(S5) << S2);
    T m = w((U)pow5_u64(M5) << M2);
    const T tens = w((U)s * 10u);
    int q = (int)(b / s);
    b = w((U)10 * (U)(b % s));
    m = w((U)m * 10u);
    low = b < m;
    high = w((U)b + (U)m) > tens;
    if (q == 0 && !high)
        dec_exp--;
    else
        digits.push_back(q);
    if (dec_exp < -3 || dec_exp >= 8) high = low = false;
    while (!low && !high) {
        q = (int)(b / s);
        b = w((U)10 * (U)(b % s));
        m = w((U)m * 10u);
        if (m > 0) {
            low = b < m;
            high = w((U)b + (U)m) > tens;
        } else {
            low = high = true;
        }
        digits.push_back(q);
    }
    low_diff = (int64_t)w((U)w((U)b << 1) - (U)tens);
}

inline Digits dtoa(int bin_exp, uint64_t fract_bits, int n_sig_bits) {
    const int tail_zeros = __builtin_ctzll(fract_bits);
    const int n_fract_bits = 52 + 1 - tail_zeros;
    const int n_tiny_bits = std::max(0, n_fract_bits - bin_exp - 1);
    if (bin_exp <= 62 && bin_exp >= -21) {
        if (n_tiny_bits < 27 && n_fract_bits + kN5Bits[n_tiny_bits] < 64 && n_tiny_bits == 0) {
            int insignificant = 0;
            if (bin_exp > n_sig_bits) {
                const int p2 = bin_exp - n_sig_bits - 1;
                insignificant = (p2 > 1 && p2 < (int)(sizeof(kInsignificant) / sizeof(int))) ? kInsignificant[p2] : 0;
            }
            const uint64_t fb = bin_exp >= 52 ? fract_bits << (bin_exp - 52) : fract_bits >> (52 - bin_exp);
            return develop_long_digits(0, (int64_t)fb, insignificant);
        }
    }
    int dec_exp = estimate_dec_exp(fract_bits, bin_exp);
    int B5 = std::max(0, -dec_exp);
    int B2 = B5 + n_tiny_bits + bin_exp;
    int S5 = std::max(0, dec_exp);
    int S2 = S5 + n_tiny_bits;
    int M5 = B5;
    int M2 = B2 - n_sig_bits;
    fract_bits >>= tail_zeros;
    B2 -= n_fract_bits - 1;
    const int common2 = std::min(B2, S2);
    B2 -= common2;
    S2 -= common2;
    M2 -= common2;
    if (n_fract_bits == 1) M2 -= 1;
    if (M2 < 0) {
        B2 -= M2;
        S2 -= M2;
        M2 = 0;
    }
    const int b_bits = n_fract_bits + B2 + (B5 < 27 ? kN5Bits[B5] : B5 * 3);
    const int ten_s_bits = S2 + 1 + (S5 + 1 < 27 ? kN5Bits[S5 + 1] : (S5 + 1) * 3);
    std::vector<int> digits;
    bool low = false, high = false;
    int64_t low_diff = 0;
    if (b_bits < 64 && ten_s_bits < 64) {
        if (b_bits < 32 && ten_s_bits < 32)
            small_loop<int32_t, uint32_t>(fract_bits, B5, B2, S5, S2, M5, M2, dec_exp, digits, low, high, low_diff);
        else
            small_loop<int64_t, uint64_t>(fract_bits, B5, B2, S5, S2, M5, M2, dec_exp, digits, low, high, low_diff);
    } else {
        Big Bv(fract_bits);
        Bv.mul_pow5(B5);
        Bv.shl(B2);
        const Big Sv = Big::pow52(S5, S2);
        Big Mv = Big::pow52(M5 + 1, M2 + 1);
        const Big tenS = Big::pow52(S5 + 1, S2 + 1);
        auto quorem = [&]() {
            int q = 0;
            while (Big::cmp(Bv, Sv) >= 0) {
                Bv.sub(Sv);
                ++q;
            }
            Bv.mul_small(10);
            return q;
        };
        int q = quorem();
        low = Big::cmp(Bv, Mv) < 0;
        high = Big::cmp(Big::add(Bv, Mv), tenS) >= 0;
        if (q == 0 && !high)
            dec_exp--;
        else
            digits.push_back(q);
        if (dec_exp < -3 || dec_exp >= 8) high = low = false;
        while (!low && !high) {
            q = quorem();
            Mv.mul_small(10);
            low = Big::cmp(Bv, Mv) < 0;
            high = Big::cmp(Big::add(Bv, Mv), tenS) >= 0;
            digits.push_back(q);
        }
        if (high && low) {
            Big b2 = Bv;
            b2.shl(1);
            low_diff = Big::cmp(b2, tenS);
        }
    }
    Digits r;
    r.d = digits;
    r.dec_exponent = dec_exp + 1;
    if (high) {
        if (low) {
            if (low_diff == 0) {
                if (r.d.back() & 1) r.roundup();
            } else if (low_diff > 0) {
                r.roundup();
            }
        } else {
            r.roundup();
        }
    }
    return r;
}

inline std::string to_string(double x) {
    if (x != x) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
    uint64_t bits;
    std::memcpy(&bits, &x, 8);
    const bool neg = (bits >> 63) != 0;
    uint64_t fract_bits = bits & ((1ull << 52) - 1);
    int bin_exp = (int)((bits >> 52) & 0x7FF);
    int n_sig;
    if (bin_exp == 0) {
        if (fract_bits == 0) return neg ? "-0.0" : "0.0";
        const int lz = __builtin_clzll(fract_bits);
        const int shift = lz - (63 - 52);
        fract_bits <<= shift;
        bin_exp = 1 - shift;
        n_sig = 64 - lz;
    } else {
        fract_bits |= 1ull << 52;
        n_sig = 53;
    }
    bin_exp -= 1023;
    const Digits r = dtoa(bin_exp, fract_bits, n_sig);
    std::string ds;
    for (int c : r.d) ds.push_back((char)('0' + c));
    const int n = (int)ds.size(), e = r.dec_exponent;
    std::string out = neg ? "-" : "";
    if (e > 0 && e < 8) {
        const int k = std::min(n, e);
        out += ds.substr(0, (size_t)k);
        if (k < e)
            out += std::string((size_t)(e - k), '0') + ".0";
        else
            out += "." + (k < n ? ds.substr((size_t)k) : std::string("0"));
    } else if (e <= 0 && e > -3) {
        out += "0." + std::string((size_t)(-e), '0') + ds;
    } else {
        out += ds.substr(0, 1) + "." + (n > 1 ? ds.substr(1) : std::string("0")) + "E";
        out += e <= 0 ? "-" + std::to_string(-e + 1) : std::to_string(e - 1);
    }
    return out;
}

}  // namespace jdouble
}  // namespace cocoa
