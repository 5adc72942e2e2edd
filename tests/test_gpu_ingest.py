"""GPU-side LIBSVM ingest (cocoa_load_libsvm_gpu, csrc/ingest.hip) against the
multithreaded host loader (cocoa_load_libsvm, itself pinned to the oracle's
parse in test_host.py): identical datasets -- row_ptr, columns, values bit for
bit, labels, Hadoop-split partitions -- and identical exceptions, on the demo
files, on generated files of every token form the reference accepts, and on
malformed files.  Reference: OptUtils.scala:11-53 (loadLIBSVMData).
"""
import os

import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import gen_synthetic, load_libsvm

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def same(a, b):
    assert np.array_equal(a.row_ptr, b.row_ptr)
    assert np.array_equal(a.col, b.col)
    assert a.val.tobytes() == b.val.tobytes()  # bitwise, incl. signed zeros
    assert np.array_equal(a.y, b.y)
    assert np.array_equal(a.part_ptr, b.part_ptr)
    assert a.num_features == b.num_features


@pytest.mark.parametrize("name,K", [("small_train.dat", 4), ("small_test.dat", 4), ("small_train.dat", 1),
                                    ("small_train.dat", 7), ("small_test.dat", 13)])
def test_demo_files(name, K):
    p = os.path.join(GOLD, name)
    same(load_libsvm(p, K, 9947, device=0), load_libsvm(p, K, 9947))


def write_rows(path, ds, fmt, rng, extras=()):
    lines = []
    for r in range(ds.n):
        b, e = ds.row_ptr[r], ds.row_ptr[r + 1]
        lab = rng.choice(["+1", "-1", "1", "0", "2", "01", "-0"]) if ds.y[r] > 0 else "-1"
        toks = [lab] + ["%d:%s" % (c + 1, fmt(v, rng)) for c, v in zip(ds.col[b:e], ds.val[b:e])]
        lines.append(" ".join(toks))
    lines.extend(extras)
    with open(path, "w", newline="") as f:
        f.write("\n".join(lines) + "\n")


def fmt_mixed(v, rng):
    k = rng.integers(0, 9)
    if k == 0:
        return repr(float(v))                 # shortest round trip (often 17 digits: host path)
    if k == 1:
        return "%.6e" % v                     # exponent form
    if k == 2:
        return "%.3E" % v
    if k == 3:
        return ("%.5f" % v).rstrip("0")     # "0.123" / "5." forms
    if k == 4:
        return ("%.4f" % v).lstrip("0")     # ".1234"
    if k == 5:
        return "%.15g" % v
    if k == 6:
        return "%.18g" % v                   # 18 significant digits: device path when m <= 2^53
    return "%.7g" % v


@pytest.mark.parametrize("K", [1, 4, 9])
def test_generated_rcv1_like_file(tmp_path, K):
    rng = np.random.default_rng(K)
    ds = gen_synthetic("rcv1", 3000, 5000, 30.0, 1, 7)
    extras = [
        "  +1 3:0.5 7:1e-3  ",              # trimmed
        "-1 2:1.5\r",                        # CRLF line end (String.trim drops \r)
        "1",                                 # label only
        "-1 4:-0 5:-.0 6:0e5 7:5.",         # signed zeros, bare dot forms
        "+1 1:0.1 2:1e22 3:1e-22 4:123456789012345678 5:9007199254740993",  # fast-path edges
        "-1 1:NaN 2:Infinity",               # host path
        "1 1:0x1p3",                         # rejected by the host rules -> error? (kept out below)
    ][:-1]
    p = tmp_path / "rows.txt"
    write_rows(str(p), ds, fmt_mixed, rng, extras)
    a = load_libsvm(str(p), K, 5000, device=0)
    b = load_libsvm(str(p), K, 5000)
    same(a, b)
    assert a.n == 3000 + 6


def test_tabs_and_odd_tokens_take_the_host_path(tmp_path):
    p = tmp_path / "odd.txt"
    p.write_text("1 1:0.5\t2:0.25\n-1 3:1.0d 4:2f\n+1 5:+3 +6:4\n-1 7:1.2345678901234567890123\n")
    with pytest.raises(cocoa_amd.CocoaError) as e1:
        load_libsvm(str(p), 2, 10)
    with pytest.raises(type(e1.value)) as e2:
        load_libsvm(str(p), 2, 10, device=0)
    assert str(e1.value) == str(e2.value)
    q = tmp_path / "ok.txt"
    q.write_text("-1 3:1.0d 4:2f\n+1 5:+3 +6:4\n-1 7:1.2345678901234567890123 8:1e400 9:1e-400\n")
    same(load_libsvm(str(q), 2, 10, device=0), load_libsvm(str(q), 2, 10))


@pytest.mark.parametrize("text", [
    "1 1:2  3:4\n",          # empty token (double space): MatchError
    "1 0:2\n",               # index 0 -> -1: out of range
    "1 11:2\n",              # index past numFeatures
    "x 1:2\n",               # label: NumberFormatException
    "1 1:2\n\n-1 2:3\n",     # blank line: NumberFormatException on its label
    "1 1:2:3\n",             # MatchError
    "1 1:abc\n",             # NumberFormatException
    "1 :2\n",
])
def test_errors_match_the_host_loader(tmp_path, text):
    p = tmp_path / "bad.txt"
    p.write_text(text)
    with pytest.raises(cocoa_amd.CocoaError) as e1:
        load_libsvm(str(p), 1, 10)
    with pytest.raises(type(e1.value)) as e2:
        load_libsvm(str(p), 1, 10, device=0)
    assert str(e1.value) == str(e2.value)


def test_empty_and_unterminated_files(tmp_path):
    p = tmp_path / "empty.txt"
    p.write_text("")
    a, b = load_libsvm(str(p), 3, 10, device=0), load_libsvm(str(p), 3, 10)
    same(a, b)
    assert a.n == 0
    q = tmp_path / "last.txt"
    q.write_text("1 1:2\n-1 2:3")           # no newline after the last line
    same(load_libsvm(str(q), 2, 10, device=0), load_libsvm(str(q), 2, 10))
