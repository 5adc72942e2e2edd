"""CPU tests of the product's host side: the C-ABI library loads and exports
every symbol include/cocoa_capi.h declares, the LIBSVM loader / Hadoop split
matches the oracle and the reference's token rules, host java.util.Random,
the synthetic generators, and Java double formatting.  No GPU compute."""
import os
import re

import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import _capi as C
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
TRAIN = os.path.join(G, "data", "small_train.dat")
TEST = os.path.join(G, "data", "small_test.dat")


def header_functions():
    src = open(os.path.join(ROOT, "include", "cocoa_capi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(cocoa_[a-z0-9_]+)\s*\(", src))
    return sorted(n for n in names if not n.endswith("_cb"))


def test_library_exports_every_declared_symbol():
    lib = C.lib()
    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
        assert n in C.SIGNATURES, n
    assert lib.cocoa_version() == 3


def test_no_cpu_fallback_without_device():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(cocoa_amd.NoDeviceError):
        cocoa_amd.Engine()


@pytest.mark.parametrize("fn,K", [(TRAIN, 4), (TEST, 4), (TRAIN, 7), (TRAIN, 1), (TEST, 13)])
def test_loader_matches_oracle(fn, K):
    a = cocoa_amd.load_libsvm(fn, K, 9947)
    b = oracle.Data.load_libsvm(fn, K, 9947)
    for f in ("row_ptr", "col", "val", "y", "part_ptr"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_loader_demo_partitions():
    a = cocoa_amd.load_libsvm(TRAIN, 4, 9947)
    assert a.partition_sizes().tolist() == [522, 510, 577, 391]
    assert a.nnz == 94790 and a.n == 2000
    t = cocoa_amd.load_libsvm(TEST, 4, 9947)
    assert t.partition_sizes().tolist() == [168, 148, 180, 104]
    assert (np.diff(t.row_ptr) == 0).sum() == 2


def _write(tmp_path, text):
    p = tmp_path / "f.dat"
    p.write_bytes(text.encode())
    return str(p)


def test_loader_label_rules(tmp_path):
    # label +1 iff the token contains '+' or parses to 1 (OptUtils.scala:35-37)
    p = _write(tmp_path, "+1 1:1\n1 1:1\n-1 1:1\n0 1:1\n2 1:1\n+0 1:1\n+7 2:0.5\n")
    d = cocoa_amd.load_libsvm(p, 1, 3)
    assert d.y.tolist() == [1, 1, -1, -1, -1, 1, 1]
    assert d.col.tolist() == [0] * 6 + [1]


@pytest.mark.parametrize("text,exc", [
    ("1.0 3:4\n", cocoa_amd.NumberFormatError),          # "1.0".toInt
    ("1 3\n", cocoa_amd.NumberFormatError),              # MatchError on Array(i)
    ("1 3:4:5\n", cocoa_amd.NumberFormatError),          # MatchError on 3 parts
    ("1 x:4\n", cocoa_amd.NumberFormatError),
    ("1 3:abc\n", cocoa_amd.NumberFormatError),
    ("1  3:4\n", cocoa_amd.NumberFormatError),           # split(' ') -> empty token
    ("1 0:4\n", cocoa_amd.IndexOutOfBoundsError),        # index 0 -> -1
    ("1 9:4\n", cocoa_amd.IndexOutOfBoundsError),        # >= numFeatures
    ("\n", cocoa_amd.NumberFormatError),                 # "".toInt
])
def test_loader_errors(tmp_path, text, exc):
    with pytest.raises(exc):
        cocoa_amd.load_libsvm(_write(tmp_path, text), 1, 8)


def test_loader_whitespace_and_suffixes(tmp_path):
    p = _write(tmp_path, "  1 1:1.5 2:2e-1   \n-1 3:4d \n")
    d = cocoa_amd.load_libsvm(p, 1, 4)
    assert d.val.tolist() == [1.5, 0.2, 4.0]
    assert d.y.tolist() == [1, -1]


def test_host_jrandom_known_answers():
    assert cocoa_amd.jrandom_ints(0, 0, 1)[0] == -1155484576
    assert cocoa_amd.jrandom_ints(42, 0, 1)[0] == -1170105035
    assert cocoa_amd.jrandom_ints(42, 10, 10).tolist() == [0, 3, 8, 4, 0, 5, 5, 8, 9, 3]
    for seed, bound in ((1, 522), (1, 512), (7, 3), (-5, 2**30 + 1), (123, 1500000001)):
        assert np.array_equal(cocoa_amd.jrandom_ints(seed, bound, 300), oracle.jrandom_ints(seed, bound, 300))


@pytest.mark.parametrize("kind,n,d,z", [("rcv1", 3000, 2000, 40.0), ("url", 2000, 50000, 30.0), ("epsilon", 300, 64, 0)])
def test_synthetic_generator(kind, n, d, z):
    a = cocoa_amd.gen_synthetic(kind, n, d, z, 8, 12345, threads=3)
    b = cocoa_amd.gen_synthetic(kind, n, d, z, 8, 12345, threads=1)
    for f in ("row_ptr", "col", "val", "y", "part_ptr"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert a.n == n and a.num_parts == 8 and set(np.unique(a.y)) <= {-1.0, 1.0}
    rows = np.diff(a.row_ptr)
    assert rows.min() >= 1
    for r in range(0, n, 97):
        c = a.col[a.row_ptr[r]:a.row_ptr[r + 1]]
        v = a.val[a.row_ptr[r]:a.row_ptr[r + 1]]
        assert np.all(np.diff(c) > 0) and c.min() >= 0 and c.max() < d
        assert abs(np.sum(v * v) - 1.0) < 1e-12
    assert 0.2 < (a.y > 0).mean() < 0.8


def test_java_double_strings():
    j = cocoa_amd.jstr
    assert j(0.1) == "0.1" and j(1e-4) == "1.0E-4" and j(0.001) == "0.001" and j(1e7) == "1.0E7"
    assert j(9999999.0) == "9999999.0" and j(-0.025) == "-0.025" and j(2.5e-10) == "2.5E-10"
    assert j(0.0) == "0.0" and j(float("nan")) == "NaN" and j(12345678.9) == "1.23456789E7"


def _big_file(tmp_path, copies=6):
    """The demo train file repeated: > 1 MB, so the loader runs its
    multithreaded line split / parse / compaction passes."""
    raw = open(TRAIN, "rb").read()
    p = tmp_path / "big.dat"
    p.write_bytes(raw * copies)
    return str(p), raw


@pytest.mark.parametrize("K", [1, 4, 9])
def test_loader_multithreaded_matches_oracle(tmp_path, K):
    fn, raw = _big_file(tmp_path)
    assert len(raw) * 6 > (1 << 21)
    a = cocoa_amd.load_libsvm(fn, K, 9947)
    b = oracle.Data.load_libsvm(fn, K, 9947)
    for f in ("row_ptr", "col", "val", "y", "part_ptr"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_loader_multithreaded_reports_first_bad_line(tmp_path):
    fn, raw = _big_file(tmp_path)
    lines = open(fn, "rb").read().split(b"\n")
    n = len(lines)
    lines[int(n * 0.7)] = b"1 7:1 0:2"        # index 0 -> ArrayIndexOutOfBounds, later in the file
    lines[int(n * 0.3)] = b"1 3:1 x:4"        # NumberFormatException, earlier: this one is reported
    bad = tmp_path / "bad.dat"
    bad.write_bytes(b"\n".join(lines))
    with pytest.raises(cocoa_amd.NumberFormatError, match="line %d" % (int(n * 0.3) + 1)):
        cocoa_amd.load_libsvm(str(bad), 4, 9947)


def test_loader_multithreaded_trailing_blanks(tmp_path):
    """Lines ending in a blank token (line.trim() then split(' ')) through the
    multithreaded passes, against the oracle's sequential parse."""
    fn, raw = _big_file(tmp_path, 5)
    text = open(fn, "rb").read().replace(b"\n", b" \n", 50)
    p = tmp_path / "ws.dat"
    p.write_bytes(text)
    a = cocoa_amd.load_libsvm(str(p), 3, 9947)
    b = oracle.Data.load_libsvm(str(p), 3, 9947)
    for f in ("row_ptr", "col", "val", "y", "part_ptr"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
