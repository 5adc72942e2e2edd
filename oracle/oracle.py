"""ctypes binding for the CPU oracle (oracle/cocoa_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline.  The product
(cocoa_amd/) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

METHODS = {"cocoa+": 0, "cocoa": 1, "mbcd": 2, "mbsgd": 3, "localsgd": 4}

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_f64p = ctypes.POINTER(ctypes.c_double)


class OracleData(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("d", ctypes.c_int32), ("K", ctypes.c_int32),
                ("row_ptr", _i64p), ("col", _i32p), ("val", _f64p), ("y", _f64p),
                ("part_ptr", _i64p), ("owns", ctypes.c_int)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_jrandom_ints.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _i32p]
        L.oracle_load_libsvm.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.POINTER(OracleData), ctypes.c_char_p, ctypes.c_int]
        L.oracle_free_data.argtypes = [ctypes.POINTER(OracleData)]
        L.oracle_local_sdca.argtypes = [_i64p, _i32p, _f64p, _f64p, ctypes.c_int32, ctypes.c_int32, _f64p,
                                        ctypes.c_int32, ctypes.c_double, ctypes.c_int32, _f64p, _f64p,
                                        ctypes.c_int32, ctypes.c_int, ctypes.c_double, _f64p, _f64p]
        L.oracle_run_create.restype = ctypes.c_void_p
        L.oracle_run_create.argtypes = [ctypes.POINTER(OracleData), ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int32,
                                        ctypes.c_int]
        L.oracle_run_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_run_round.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.oracle_run_local.argtypes = [ctypes.c_void_p, ctypes.c_int32, _f64p]
        L.oracle_run_apply.argtypes = [ctypes.c_void_p, _f64p]
        L.oracle_run_set_global_parts.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.oracle_run_eval.argtypes = [ctypes.c_void_p, ctypes.POINTER(OracleData), _f64p]
        for f in ("oracle_run_get_w", "oracle_run_get_alpha", "oracle_run_set_w", "oracle_run_set_alpha"):
            getattr(L, f).argtypes = [ctypes.c_void_p, _f64p]
        L.oracle_samples.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _i32p]
        L.oracle_row_sqnorm.argtypes = [ctypes.POINTER(OracleData), _f64p]
        L.oracle_primal.restype = ctypes.c_double
        L.oracle_primal.argtypes = [ctypes.POINTER(OracleData), _f64p, ctypes.c_double]
        L.oracle_dual.restype = ctypes.c_double
        L.oracle_dual.argtypes = [ctypes.POINTER(OracleData), _f64p, _f64p, ctypes.c_double]
        L.oracle_error_count.restype = ctypes.c_int64
        L.oracle_error_count.argtypes = [ctypes.POINTER(OracleData), _f64p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def jrandom_ints(seed, bound, count):
    out = np.zeros(count, np.int32)
    lib().oracle_jrandom_ints(seed, bound, count, _p(out, _i32p))
    return out


def samples(seed_plus_t, n_local, H):
    out = np.zeros(H, np.int32)
    lib().oracle_samples(seed_plus_t, n_local, H, _p(out, _i32p))
    return out


class Data:
    """Partitioned CSR held as numpy arrays (kept alive for the C side)."""

    def __init__(self, row_ptr, col, val, y, part_ptr, d):
        self.row_ptr = np.ascontiguousarray(row_ptr, np.int64)
        self.col = np.ascontiguousarray(col, np.int32)
        self.val = np.ascontiguousarray(val, np.float64)
        self.y = np.ascontiguousarray(y, np.float64)
        self.part_ptr = np.ascontiguousarray(part_ptr, np.int64)
        self.d = int(d)
        self.n = len(self.y)
        self.K = len(self.part_ptr) - 1
        self.c = OracleData(self.n, self.d, self.K, _p(self.row_ptr, _i64p), _p(self.col, _i32p),
                            _p(self.val, _f64p), _p(self.y, _f64p), _p(self.part_ptr, _i64p), 0)

    @classmethod
    def load_libsvm(cls, path, num_splits, num_feats):
        D = OracleData()
        err = ctypes.create_string_buffer(512)
        rc = lib().oracle_load_libsvm(path.encode(), num_splits, num_feats, ctypes.byref(D), err, 512)
        if rc != 0:
            raise ValueError(err.value.decode())
        n, K = D.n, D.K
        nnz = D.row_ptr[n]
        obj = cls(np.ctypeslib.as_array(D.row_ptr, (n + 1,)).copy(), np.ctypeslib.as_array(D.col, (max(nnz, 1),))[:nnz].copy(),
                  np.ctypeslib.as_array(D.val, (max(nnz, 1),))[:nnz].copy(), np.ctypeslib.as_array(D.y, (n,)).copy(),
                  np.ctypeslib.as_array(D.part_ptr, (K + 1,)).copy(), D.d)
        lib().oracle_free_data(ctypes.byref(D))
        return obj

    def row_sqnorm(self):
        out = np.zeros(self.n, np.float64)
        lib().oracle_row_sqnorm(ctypes.byref(self.c), _p(out, _f64p))
        return out

    def primal(self, w, lam):
        return lib().oracle_primal(ctypes.byref(self.c), _p(np.ascontiguousarray(w, np.float64), _f64p), lam)

    def dual(self, w, alpha, lam):
        return lib().oracle_dual(ctypes.byref(self.c), _p(np.ascontiguousarray(w, np.float64), _f64p),
                                 _p(np.ascontiguousarray(alpha, np.float64), _f64p), lam)

    def error_count(self, w):
        return lib().oracle_error_count(ctypes.byref(self.c), _p(np.ascontiguousarray(w, np.float64), _f64p))


def local_sdca(data, part, w, H, lam, n, alpha, seed, plus, sigma):
    """CoCoA.localSDCA on partition `part` (w, alpha mutated in place like the reference)."""
    r0, r1 = int(data.part_ptr[part]), int(data.part_ptr[part + 1])
    rp = np.ascontiguousarray(data.row_ptr[r0:r1 + 1])
    dw = np.zeros(data.d, np.float64)
    da = np.zeros(r1 - r0, np.float64)
    alpha_old = alpha.copy()
    lib().oracle_local_sdca(_p(rp, _i64p), _p(data.col, _i32p), _p(data.val, _f64p), _p(data.y[r0:r1].copy(), _f64p),
                            r1 - r0, data.d, _p(w, _f64p), H, lam, n, _p(alpha, _f64p), _p(alpha_old, _f64p), seed,
                            1 if plus else 0, sigma, _p(dw, _f64p), _p(da, _f64p))
    return da, dw


class Run:
    """runCoCoA / runMbCD / runSGD round-by-round (oracle)."""

    def __init__(self, data, method, n, H, lam, beta=1.0, gamma=1.0, seed=0, nthreads=1):
        self.data = data
        self.h = lib().oracle_run_create(ctypes.byref(data.c), METHODS[method], n, H, lam, beta, gamma, seed, nthreads)

    def round(self, t):
        lib().oracle_run_round(self.h, t)

    def set_global_parts(self, Kg):
        lib().oracle_run_set_global_parts(self.h, Kg)

    def round_local(self, t, out):
        lib().oracle_run_local(self.h, t, _p(out, _f64p))

    def round_apply(self, dw_sum):
        lib().oracle_run_apply(self.h, _p(np.ascontiguousarray(dw_sum, np.float64), _f64p))

    def eval(self, test=None):
        out = np.zeros(6, np.float64)
        lib().oracle_run_eval(self.h, ctypes.byref(test.c) if test is not None else None, _p(out, _f64p))
        return {"primal": out[0], "dual": out[1], "gap": out[2], "test_err": int(out[3]),
                "hinge_sum": out[4], "alpha_sum": out[5]}

    def w(self):
        out = np.zeros(self.data.d, np.float64)
        lib().oracle_run_get_w(self.h, _p(out, _f64p))
        return out

    def alpha(self):
        out = np.zeros(self.data.n, np.float64)
        lib().oracle_run_get_alpha(self.h, _p(out, _f64p))
        return out

    def set_state(self, w, alpha):
        lib().oracle_run_set_w(self.h, _p(np.ascontiguousarray(w, np.float64), _f64p))
        lib().oracle_run_set_alpha(self.h, _p(np.ascontiguousarray(alpha, np.float64), _f64p))

    def close(self):
        if self.h:
            lib().oracle_run_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
