"""ctypes binding of libcocoa_hip.so (include/cocoa_capi.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``) and
loaded from this package directory.  There is no CPU fallback: if the library
or a HIP device is missing, the calls raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# COCOA_LIB may point at a diagnostic build (e.g. build/diag/libcocoa_hip.so)
LIB_PATH = os.environ.get("COCOA_LIB") or os.path.join(HERE, "libcocoa_hip.so")

COCOA_OK = 0
E_ARG, E_PARSE, E_RANGE, E_IO, E_HIP, E_STATE, E_NODEV = -1, -2, -3, -4, -5, -6, -7

METHOD_COCOA_PLUS, METHOD_COCOA, METHOD_MBCD, METHOD_MBSGD, METHOD_LOCALSGD = 0, 1, 2, 3, 4
METHODS = {"cocoa+": 0, "cocoa": 1, "mbcd": 2, "mbsgd": 3, "localsgd": 4}
K_SAMPLE, K_SOLVER, K_FOLD, K_APPLY, K_EVAL, K_PLAN, K_GRAM, K_XW = 0, 1, 2, 3, 4, 5, 6, 7
KERNEL_NAMES = ["sample", "solver", "fold", "apply", "eval", "plan", "gram", "xw"]
SOLVERS = {"auto": 0, "chain": 1, "gram": 2, "dense": 3}


class CocoaError(RuntimeError):
    """Base error; subclasses mirror the reference's JVM exception kinds."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class IllegalArgumentError(CocoaError, ValueError):
    pass


class NumberFormatError(CocoaError, ValueError):
    pass


class IndexOutOfBoundsError(CocoaError, IndexError):
    pass


class NoDeviceError(CocoaError):
    pass


_EXC = {E_ARG: IllegalArgumentError, E_PARSE: NumberFormatError, E_RANGE: IndexOutOfBoundsError,
        E_IO: CocoaError, E_HIP: CocoaError, E_STATE: CocoaError, E_NODEV: NoDeviceError}


class Params(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("num_rounds", ctypes.c_int32), ("local_iters", ctypes.c_int32),
                ("_pad", ctypes.c_int32), ("lambda_", ctypes.c_double), ("beta", ctypes.c_double),
                ("gamma", ctypes.c_double)]


class Debug(ctypes.Structure):
    _fields_ = [("debug_iter", ctypes.c_int32), ("seed", ctypes.c_int32), ("chkpt_iter", ctypes.c_int32),
                ("_pad", ctypes.c_int32)]


class EvalResult(ctypes.Structure):
    _fields_ = [("primal", ctypes.c_double), ("dual", ctypes.c_double), ("gap", ctypes.c_double),
                ("test_error", ctypes.c_double), ("hinge_sum", ctypes.c_double), ("alpha_sum", ctypes.c_double),
                ("w_sqnorm", ctypes.c_double), ("test_err_count", ctypes.c_int64), ("test_rows", ctypes.c_int64)]

    def as_dict(self):
        return {f[0]: getattr(self, f[0]) for f in self._fields_}


class Dataset(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("num_features", ctypes.c_int32), ("num_parts", ctypes.c_int32),
                ("nnz", ctypes.c_int64), ("row_ptr", ctypes.POINTER(ctypes.c_int64)),
                ("col", ctypes.POINTER(ctypes.c_int32)), ("val", ctypes.POINTER(ctypes.c_double)),
                ("y", ctypes.POINTER(ctypes.c_double)), ("part_ptr", ctypes.POINTER(ctypes.c_int64))]


ROUND_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(EvalResult))

# exported symbols and their signatures; tests check every one is exported
_i32, _i64, _f64, _vp, _int = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.c_int
_pi32, _pi64, _pf64 = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
SIGNATURES = {
    "cocoa_version": (_int, []),
    "cocoa_create": (_int, [_int, _int, _vp, ctypes.POINTER(_vp)]),
    "cocoa_create_multi": (_int, [_i32, _pi32, _int, ctypes.POINTER(_vp)]),
    "cocoa_num_devices": (_int, [_vp, _pi32, _pi32, _i32]),
    "cocoa_destroy": (_int, [_vp]),
    "cocoa_last_error": (ctypes.c_char_p, [_vp]),
    "cocoa_set_train": (_int, [_vp, _i32, _pi64, _pi64, _pi32, _pf64, _pf64, _i64, _i32, _i32, _i32]),
    "cocoa_set_test": (_int, [_vp, _pi64, _pi32, _pf64, _pf64, _i64]),
    "cocoa_set_train_dense": (_int, [_vp, _i32, _pi64, _pf64, _pf64, _i64, _i32, _i32, _i32]),
    "cocoa_set_test_dense": (_int, [_vp, _pf64, _pf64, _i64]),
    "cocoa_init": (_int, [_vp, ctypes.POINTER(Params), ctypes.POINTER(Debug), _int, _pf64]),
    "cocoa_round_local": (_int, [_vp, _i32]),
    "cocoa_dw_sum_device_ptr": (_int, [_vp, ctypes.POINTER(_vp)]),
    "cocoa_set_dw_sum_buffer": (_int, [_vp, _vp]),
    "cocoa_round_apply": (_int, [_vp]),
    "cocoa_round": (_int, [_vp, _i32]),
    "cocoa_eval": (_int, [_vp, ctypes.POINTER(EvalResult)]),
    "cocoa_eval_async": (_int, [_vp]),
    "cocoa_eval_wait": (_int, [_vp, ctypes.POINTER(EvalResult)]),
    "cocoa_eval_begin": (_int, [_vp]),
    "cocoa_eval_end": (_int, [_vp, ctypes.POINTER(EvalResult)]),
    "cocoa_eval_finish": (_int, [_vp, _f64, _f64, _f64, _i64, _i64, ctypes.POINTER(EvalResult)]),
    "cocoa_run": (_int, [_vp, ctypes.POINTER(Params), ctypes.POINTER(Debug), _int, _pf64, ROUND_CB, _vp]),
    "cocoa_get_w": (_int, [_vp, _pf64]),
    "cocoa_get_alpha": (_int, [_vp, _pf64]),
    "cocoa_set_w": (_int, [_vp, _pf64]),
    "cocoa_set_alpha": (_int, [_vp, _pf64]),
    "cocoa_checkpoint_save": (_int, [_vp, ctypes.c_char_p, _i32]),
    "cocoa_checkpoint_load": (_int, [_vp, ctypes.c_char_p, ctypes.POINTER(_i32)]),
    "cocoa_set_checkpoint_dir": (_int, [_vp, ctypes.c_char_p]),
    "cocoa_checkpoint_file": (_int, [_vp, _int, ctypes.c_char_p, _i64]),
    "cocoa_resume": (_int, [_vp, ctypes.POINTER(Params), ctypes.POINTER(Debug), _int, ctypes.c_char_p, ROUND_CB,
                            _vp]),
    "cocoa_local_sdca": (_int, [_vp, _i32, _pf64, _i32, _f64, _i32, _pf64, _i32, _int, _f64, _pf64, _pf64]),
    "cocoa_samples": (_int, [_vp, _i32, _i32, _i32, _pi32]),
    "cocoa_stats_enable": (_int, [_vp, _int]),
    "cocoa_stats_kernels": (_int, [_vp, ctypes.c_uint32]),
    "cocoa_kernel_stats": (_int, [_vp, _int, _pf64, _pi64]),
    "cocoa_stats_reset": (_int, [_vp]),
    "cocoa_plan_info": (_int, [_vp, ctypes.c_char_p, _int]),
    "cocoa_gram_fallback_count": (_int, [_vp, ctypes.POINTER(_i32)]),
    "cocoa_debug_gram_rows": (_int, [_vp, _i32, _pf64, _i64]),
    "cocoa_solver_profile": (_int, [_vp, _int]),
    "cocoa_solver_profile_read": (_int, [_vp, ctypes.POINTER(ctypes.c_uint64), _i64]),
    "cocoa_sync": (_int, [_vp]),
    "cocoa_load_libsvm": (_int, [ctypes.c_char_p, _i32, _i32, ctypes.POINTER(Dataset)]),
    "cocoa_load_libsvm_gpu": (_int, [_i32, ctypes.c_char_p, _i32, _i32, ctypes.POINTER(Dataset)]),
    "cocoa_gen_synthetic": (_int, [_i32, _i64, _i32, _f64, _i32, ctypes.c_uint64, _i64, _i32,
                                    ctypes.POINTER(Dataset)]),
    "cocoa_dataset_free": (None, [ctypes.POINTER(Dataset)]),
    "cocoa_java_double_string": (_int, [ctypes.c_double, ctypes.c_char_p, _i32]),
    "cocoa_jrandom_ints": (_int, [_i64, _i32, _i32, _pi32]),
    "cocoa_set_solver": (_int, [_vp, _int]),
    "cocoa_comm_unique_id": (_int, [_int, ctypes.c_char_p]),
    "cocoa_comm_init": (_int, [_vp, _int, _i32, _i32, ctypes.c_char_p]),
    "cocoa_comm_info": (_int, [_vp, _pi32, _pi32, _pi32]),
    "cocoa_comm_create": (_int, [_int, _i32, _i32, ctypes.c_char_p, _int, ctypes.POINTER(_vp)]),
    "cocoa_comm_destroy": (_int, [_vp]),
    "cocoa_comm_allreduce": (_int, [_vp, _pf64, _i64]),
    "cocoa_comm_ordered_sum": (_int, [_vp, _pf64, _i64]),
}

TRANSPORTS = {"rccl": 0, "host": 1, "local": 2}
UID_BYTES = 128

_lib = None


def lib():
    """Load libcocoa_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CocoaError(E_NODEV, "libcocoa_hip.so not built: run `make` or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name, None)
            if f is None:  # an older library (A/B runs); tests/test_capi_symbols.py checks the shipped one
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != COCOA_OK:
        msg = lib().cocoa_last_error(ctx)
        msg = msg.decode() if msg else "error %d" % rc
        raise _EXC.get(rc, CocoaError)(rc, msg)


def ptr(a, t):
    return a.ctypes.data_as(t)


def f64p(a):
    return a.ctypes.data_as(_pf64)


def i64p(a):
    return a.ctypes.data_as(_pi64)


def i32p(a):
    return a.ctypes.data_as(_pi32)
