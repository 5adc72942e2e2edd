"""java.lang.Double.toString of the reference's JVM (JDK 7/8 FloatingDecimal),
restated in cocoa_amd/jdouble.py and csrc/jdouble.h (the driver's stdout and
cocoa_java_double_string): known JDK 8 outputs, including the non-shortest
ones JDK-4511638 documents, the layout rules (plain form for 1e-3 <= |x| <
1e7, E-form otherwise), round trip of every output, and the two
restatements against each other on random doubles.  Host-only."""
import ctypes
import math
import struct

import numpy as np
import pytest

from cocoa_amd import _capi
from cocoa_amd.jdouble import java_double_tostring as jstr

KNOWN = [
    (0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (-1.0, "-1.0"), (0.1, "0.1"), (0.5, "0.5"), (100.0, "100.0"),
    (1e7, "1.0E7"), (9999999.0, "9999999.0"), (12345678.9, "1.23456789E7"), (0.001, "0.001"), (1e-4, "1.0E-4"),
    (1e-5, "1.0E-5"), (0.0013, "0.0013"), (123456.789, "123456.789"), (0.30000000000000004, "0.30000000000000004"),
    (5e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"),
    (2.2250738585072014e-308, "2.2250738585072014E-308"), (float("nan"), "NaN"), (float("inf"), "Infinity"),
    (float("-inf"), "-Infinity"),
    # JDK <= 18 (FloatingDecimal) digits that are not the shortest: JDK-4511638
    (2e23, "1.9999999999999998E23"), (8.41e21, "8.409999999999999E21"),
]


@pytest.mark.parametrize("x,s", KNOWN)
def test_known_jdk8_strings(x, s):
    assert jstr(x) == s


def _c(x):
    buf = ctypes.create_string_buffer(64)
    assert _capi.lib().cocoa_java_double_string(x, buf, 64) == 0
    return buf.value.decode()


def _rand_doubles(n, seed):
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2 ** 63 - 1, size=n, dtype=np.int64)
    xs = [struct.unpack("<d", struct.pack("<q", int(b)))[0] for b in bits]
    xs = [x for x in xs if math.isfinite(x)]
    # and the magnitudes the objectives take (1e-12 .. 1e3), both signs
    xs += list(rng.standard_normal(n) * 10.0 ** rng.uniform(-12, 3, n))
    xs += [float(v) for v in rng.integers(1, 10 ** 9, size=n // 4)]
    return xs


def test_round_trip():
    for x in _rand_doubles(4000, 1):
        s = jstr(x)
        assert float(s) == x, (x, s)


def test_layout_forms():
    for x in _rand_doubles(2000, 2):
        s = jstr(x)
        ax = abs(x)
        if ax == 0:
            continue
        if 1e-3 <= ax < 1e7:
            assert "E" not in s and "." in s, (x, s)
        else:
            assert "E" in s and "." in s.split("E")[0], (x, s)


def test_c_restatement_matches_python():
    for x in _rand_doubles(3000, 3) + [v for v, _ in KNOWN]:
        assert _c(x) == jstr(x), x


def test_c_abi_argument_errors():
    assert _capi.lib().cocoa_java_double_string(1.0, None, 64) != 0
    buf = ctypes.create_string_buffer(4)
    assert _capi.lib().cocoa_java_double_string(2e23, buf, 4) != 0
