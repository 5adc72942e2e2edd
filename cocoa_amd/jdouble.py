"""java.lang.Double.toString as the reference's JVM printed it.

The reference (Spark 1.3.1 / Scala 2.10) ran on JDK 7/8, whose
sun.misc.FloatingDecimal does not always emit the shortest round-tripping
digits (JDK-4511638, fixed in JDK 19): e.g. 2.0E23 prints as
"1.9999999999999998E23".  This module restates that algorithm (the
BinaryToASCIIBuffer.dtoa digit generation with its long fast path, the
int / long / big-integer Steele-White loops and their stopping and rounding
rules, and the compatible-format layout) so the driver's stdout lines
(CoCoA.scala:53-57, OptUtils.scala printSummaryStats*) read as the reference's.
Exact integers stand in for FDBigInteger; the int and long loops keep Java's
32- / 64-bit wraparound.  The C++ driver carries the same restatement
(csrc/jdouble.h); tests/test_jdouble.py checks both against each other and
against known JDK 8 outputs.
"""
import math
import struct

EXP_SHIFT = 52
FRACT_HOB = 1 << 52
SIGNIF_MASK = (1 << 52) - 1
EXP_BIAS = 1023
MAX_SMALL_BIN_EXP = 62
MIN_SMALL_BIN_EXP = -(63 // 3)
N_5_BITS = [0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61]
LONG_5_POW = [5 ** i for i in range(27)]
SMALL_5_POW = [5 ** i for i in range(14)]
INSIGNIFICANT_DIGITS = [0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7,
                        8, 8, 8, 9, 9, 9, 9, 10, 10, 10, 11, 11, 11, 12, 12, 12, 12, 13, 13, 13, 14, 14, 14,
                        15, 15, 15, 15, 16, 16, 16, 17, 17, 17, 18, 18, 18, 19]


def _wrap(x, bits):
    m = 1 << bits
    x &= m - 1
    return x - m if x >= (m >> 1) else x


def _ntz(x):
    return (x & -x).bit_length() - 1


def _bits(d):
    return struct.unpack("<q", struct.pack("<d", d))[0]


def _from_bits(b):
    return struct.unpack("<d", struct.pack("<q", b))[0]


def _estimate_dec_exp(fract_bits, bin_exp):
    d2 = _from_bits((0x3FF << 52) | (fract_bits & SIGNIF_MASK))
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    return math.floor(d)


class _Digits:
    def __init__(self):
        self.digits = []
        self.dec_exponent = 0

    def roundup(self):
        ds = self.digits
        i = len(ds) - 1
        q = ds[i]
        if q == 9:
            while q == 9 and i > 0:
                ds[i] = 0
                i -= 1
                q = ds[i]
            if q == 9:
                self.dec_exponent += 1
                ds[0] = 1
                return
        ds[i] = q + 1


def _develop_long_digits(dec_exponent, lvalue, insignificant):
    if insignificant != 0:
        pow10 = LONG_5_POW[insignificant] << insignificant
        residue = lvalue % pow10
        lvalue //= pow10
        dec_exponent += insignificant
        if residue >= (pow10 >> 1):
            lvalue += 1
    c = lvalue % 10
    lvalue //= 10
    while c == 0:
        dec_exponent += 1
        c = lvalue % 10
        lvalue //= 10
    out = []
    while lvalue != 0:
        out.append(c)
        dec_exponent += 1
        c = lvalue % 10
        lvalue //= 10
    out.append(c)
    r = _Digits()
    r.digits = out[::-1]
    r.dec_exponent = dec_exponent + 1
    return r


def _dtoa(bin_exp, fract_bits, n_sig_bits):
    tail_zeros = _ntz(fract_bits)
    n_fract_bits = EXP_SHIFT + 1 - tail_zeros
    n_tiny_bits = max(0, n_fract_bits - bin_exp - 1)
    if MIN_SMALL_BIN_EXP <= bin_exp <= MAX_SMALL_BIN_EXP:
        if n_tiny_bits < len(LONG_5_POW) and n_fract_bits + N_5_BITS[n_tiny_bits] < 64:
            if n_tiny_bits == 0:
                insignificant = 0
                if bin_exp > n_sig_bits:
                    p2 = bin_exp - n_sig_bits - 1
                    insignificant = INSIGNIFICANT_DIGITS[p2] if 1 < p2 < len(INSIGNIFICANT_DIGITS) else 0
                if bin_exp >= EXP_SHIFT:
                    fb = fract_bits << (bin_exp - EXP_SHIFT)
                else:
                    fb = fract_bits >> (EXP_SHIFT - bin_exp)
                return _develop_long_digits(0, fb, insignificant)
    dec_exp = _estimate_dec_exp(fract_bits, bin_exp)
    B5 = max(0, -dec_exp)
    B2 = B5 + n_tiny_bits + bin_exp
    S5 = max(0, dec_exp)
    S2 = S5 + n_tiny_bits
    M5 = B5
    M2 = B2 - n_sig_bits
    fract_bits >>= tail_zeros
    B2 -= n_fract_bits - 1
    common2 = min(B2, S2)
    B2 -= common2
    S2 -= common2
    M2 -= common2
    if n_fract_bits == 1:
        M2 -= 1
    if M2 < 0:
        B2 -= M2
        S2 -= M2
        M2 = 0
    b_bits = n_fract_bits + B2 + (N_5_BITS[B5] if B5 < len(N_5_BITS) else B5 * 3)
    ten_s_bits = S2 + 1 + (N_5_BITS[S5 + 1] if S5 + 1 < len(N_5_BITS) else (S5 + 1) * 3)
    digits = []
    if b_bits < 64 and ten_s_bits < 64:
        W = 32 if (b_bits < 32 and ten_s_bits < 32) else 64
        p5 = SMALL_5_POW if W == 32 else LONG_5_POW
        b = _wrap(_wrap(fract_bits * p5[B5], W) << B2, W)
        s = _wrap(p5[S5] << S2, W)
        m = _wrap(p5[M5] << M2, W)
        tens = _wrap(s * 10, W)
        q = b // s
        b = _wrap(10 * (b % s), W)
        m = _wrap(m * 10, W)
        low = b < m
        high = _wrap(b + m, W) > tens
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q = b // s
            b = _wrap(10 * (b % s), W)
            m = _wrap(m * 10, W)
            if m > 0:
                low = b < m
                high = _wrap(b + m, W) > tens
            else:
                low = high = True
            digits.append(q)
        low_diff = _wrap(_wrap(b << 1, W) - tens, W)
    else:
        Bv = fract_bits * 5 ** B5 * 2 ** B2
        Sv = 5 ** S5 * 2 ** S2
        Mv = 5 ** (M5 + 1) * 2 ** (M2 + 1)
        tenS = 5 ** (S5 + 1) * 2 ** (S2 + 1)
        q, Bv = Bv // Sv, (Bv % Sv) * 10
        low = Bv < Mv
        high = Bv + Mv >= tenS
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q, Bv = Bv // Sv, (Bv % Sv) * 10
            Mv *= 10
            low = Bv < Mv
            high = Bv + Mv >= tenS
            digits.append(q)
        low_diff = ((Bv << 1) > tenS) - ((Bv << 1) < tenS) if (high and low) else 0
    r = _Digits()
    r.digits = digits
    r.dec_exponent = dec_exp + 1
    if high:
        if low:
            if low_diff == 0:
                if digits[-1] & 1:
                    r.roundup()
            elif low_diff > 0:
                r.roundup()
        else:
            r.roundup()
    return r


def _layout(neg, r):
    ds = "".join(chr(48 + c) for c in r.digits)
    n = len(ds)
    e = r.dec_exponent
    out = "-" if neg else ""
    if 0 < e < 8:
        k = min(n, e)
        out += ds[:k]
        if k < e:
            out += "0" * (e - k) + ".0"
        else:
            out += "." + (ds[k:] if k < n else "0")
    elif -3 < e <= 0:
        out += "0." + "0" * (-e) + ds
    else:
        out += ds[0] + "." + (ds[1:] if n > 1 else "0") + "E"
        out += ("-" + str(-e + 1)) if e <= 0 else str(e - 1)
    return out


def java_double_tostring(x):
    """Double.toString(x) of JDK 7/8 (FloatingDecimal.toJavaFormatString)."""
    x = float(x)
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    bits = _bits(x)
    neg = bits < 0
    fract_bits = bits & SIGNIF_MASK
    bin_exp = (bits >> 52) & 0x7FF
    if bin_exp == 0:
        if fract_bits == 0:
            return "-0.0" if neg else "0.0"
        lz = 64 - fract_bits.bit_length()
        shift = lz - (63 - EXP_SHIFT)
        fract_bits <<= shift
        bin_exp = 1 - shift
        n_sig = 64 - lz
    else:
        fract_bits |= FRACT_HOB
        n_sig = EXP_SHIFT + 1
    bin_exp -= EXP_BIAS
    return _layout(neg, _dtoa(bin_exp, fract_bits, n_sig))
