"""Engine: one libcocoa_hip context (one GPU, one stream) holding one rank's
partitions.  Thin, typed wrapper over include/cocoa_capi.h."""
import ctypes
import os
import json

import numpy as np

from . import _capi as C


def comm_unique_id(transport="rccl"):
    """cocoa_comm_unique_id: made once on rank 0, then handed to every rank
    (HOST opens rank 0's listening socket in this process)."""
    buf = ctypes.create_string_buffer(C.UID_BYTES)
    C.check(C.lib().cocoa_comm_unique_id(C.TRANSPORTS[transport], buf))
    return buf.raw


class Comm:
    """Stand-alone communicator on host buffers (cocoa_comm_create): the two
    reductions the engine uses between ranks, without a context or a GPU for
    the HOST transport."""

    def __init__(self, transport, rank, world, uid, device=-1):
        h = ctypes.c_void_p()
        C.check(C.lib().cocoa_comm_create(C.TRANSPORTS[transport], rank, world, uid, device, ctypes.byref(h)))
        self.h = h

    def allreduce(self, x):
        x = np.ascontiguousarray(x, np.float64).copy()
        C.check(C.lib().cocoa_comm_allreduce(self.h, C.f64p(x), len(x)))
        return x

    def ordered_sum(self, x):
        x = np.ascontiguousarray(x, np.float64).copy()
        C.check(C.lib().cocoa_comm_ordered_sum(self.h, C.f64p(x), len(x)))
        return x

    def close(self):
        if getattr(self, "h", None):
            C.lib().cocoa_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _dense_rows(data, chunk=1 << 14):
    """Rows that store every feature 0..d-1 in index order (epsilon-shaped, C3):
    the value array is then the row-major matrix itself."""
    n, d = data.n, data.num_features
    if n < 1 or len(data.col) != n * d:
        return False
    if not np.array_equal(data.row_ptr, np.arange(n + 1, dtype=np.int64) * d):
        return False
    cols = data.col.reshape(n, d)
    ar = np.arange(d, dtype=np.int32)
    return all(np.array_equal(cols[r:r + chunk], np.broadcast_to(ar, (min(chunk, n - r), d)))
               for r in range(0, n, chunk))


class Engine:
    def __init__(self, device=0, strict=False, stream=None, devices=None):
        """stream: a hipStream_t handle as int (e.g. torch.cuda.current_stream().cuda_stream).
        devices: a list of device ordinals -> ONE context over all of them
        (cocoa_create_multi): the partitions are split over the devices and
        every round / eval exchanges between them internally.

        A process that also uses torch on the GPU must initialise torch's HIP
        runtime (torch ships its own libamdhip64) before the first Engine opens
        the device, e.g. `import torch; torch.cuda.init()` first."""
        h = ctypes.c_void_p()
        if devices is not None:
            devs = np.ascontiguousarray(devices, np.int32)
            C.check(C.lib().cocoa_create_multi(len(devs), C.i32p(devs), 1 if strict else 0, ctypes.byref(h)))
        else:
            C.check(C.lib().cocoa_create(int(device), 1 if strict else 0, ctypes.c_void_p(stream or 0),
                                         ctypes.byref(h)))
        self.h = h
        self.strict = strict
        self.d = 0
        self.n_rows = 0
        self._keep = []

    # -- data ----------------------------------------------------------------
    def set_train(self, data, part_begin=0, num_parts_global=None):
        data = data.contiguous()
        K = data.num_parts
        Kg = K if num_parts_global is None else num_parts_global
        if _dense_rows(data):  # no column array crosses the ABI (cocoa_set_train_dense)
            self.set_train_dense(data.val.reshape(data.n, data.num_features), data.y, data.part_ptr, part_begin, Kg)
            return
        C.check(C.lib().cocoa_set_train(self.h, K, C.i64p(data.part_ptr), C.i64p(data.row_ptr), C.i32p(data.col),
                                        C.f64p(data.val), C.f64p(data.y), data.n, data.num_features, part_begin, Kg),
                self.h)
        self.d = data.num_features
        self.n_rows = data.n
        self.K_loc, self.K_glob, self.part_begin = K, Kg, part_begin

    def set_test(self, data):
        data = data.contiguous()
        if self.d and data.num_features == self.d and _dense_rows(data):
            self.set_test_dense(data.val.reshape(data.n, data.num_features), data.y)
            return
        C.check(C.lib().cocoa_set_test(self.h, C.i64p(data.row_ptr), C.i32p(data.col), C.f64p(data.val),
                                       C.f64p(data.y), data.n), self.h)

    def set_train_dense(self, X, y, part_ptr, part_begin=0, num_parts_global=None):
        """Dense rows (cocoa_set_train_dense): X float64 [n, d] row-major."""
        X = np.ascontiguousarray(X, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        pp = np.ascontiguousarray(part_ptr, np.int64)
        K = len(pp) - 1
        Kg = K if num_parts_global is None else num_parts_global
        C.check(C.lib().cocoa_set_train_dense(self.h, K, C.i64p(pp), C.f64p(X), C.f64p(y), X.shape[0], X.shape[1],
                                              part_begin, Kg), self.h)
        self.d = X.shape[1]
        self.n_rows = X.shape[0]
        self.K_loc, self.K_glob, self.part_begin = K, Kg, part_begin

    def set_test_dense(self, X, y):
        X = np.ascontiguousarray(X, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        C.check(C.lib().cocoa_set_test_dense(self.h, C.f64p(X), C.f64p(y), X.shape[0]), self.h)

    # -- ranks ---------------------------------------------------------------
    def comm_init(self, transport, rank, world, uid):
        """Attach a communicator (cocoa_comm_init): round / eval / run then
        exchange deltaW and the objective sums between the ranks internally."""
        C.check(C.lib().cocoa_comm_init(self.h, C.TRANSPORTS[transport], rank, world, uid), self.h)

    def devices(self):
        """Device ordinals of this context (one for cocoa_create)."""
        n = ctypes.c_int32()
        buf = np.zeros(64, np.int32)
        C.check(C.lib().cocoa_num_devices(self.h, ctypes.byref(n), C.i32p(buf), len(buf)), self.h)
        return [int(x) for x in buf[:n.value]]

    def comm_info(self):
        t, r, w = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        C.check(C.lib().cocoa_comm_info(self.h, ctypes.byref(t), ctypes.byref(r), ctypes.byref(w)), self.h)
        names = {v: k for k, v in C.TRANSPORTS.items()}
        return {"transport": names.get(t.value), "rank": r.value, "world": w.value}

    # -- solver --------------------------------------------------------------
    def set_solver(self, kind):
        """Fast-mode SDCA solver: "auto" (default), "chain", "gram" or "dense" (cocoa_set_solver)."""
        C.check(C.lib().cocoa_set_solver(self.h, C.SOLVERS[kind]), self.h)

    def init(self, method, n, num_rounds, local_iters, lam, beta=1.0, gamma=1.0, debug_iter=10, seed=0,
             chkpt_iter=100, w_init=None):
        self.params = C.Params(n, num_rounds, local_iters, 0, lam, beta, gamma)
        self.debug = C.Debug(debug_iter, seed, chkpt_iter, 0)
        wi = None if w_init is None else np.ascontiguousarray(w_init, np.float64)
        C.check(C.lib().cocoa_init(self.h, ctypes.byref(self.params), ctypes.byref(self.debug),
                                   C.METHODS[method] if isinstance(method, str) else int(method),
                                   C.f64p(wi) if wi is not None else None), self.h)

    def round(self, t):
        C.check(C.lib().cocoa_round(self.h, t), self.h)

    def round_local(self, t):
        C.check(C.lib().cocoa_round_local(self.h, t), self.h)

    def round_apply(self):
        C.check(C.lib().cocoa_round_apply(self.h), self.h)

    def dw_sum_ptr(self):
        p = ctypes.c_void_p()
        C.check(C.lib().cocoa_dw_sum_device_ptr(self.h, ctypes.byref(p)), self.h)
        return p.value

    def set_dw_sum_buffer(self, device_ptr):
        C.check(C.lib().cocoa_set_dw_sum_buffer(self.h, ctypes.c_void_p(device_ptr or 0)), self.h)

    def eval(self):
        r = C.EvalResult()
        C.check(C.lib().cocoa_eval(self.h, ctypes.byref(r)), self.h)
        return r.as_dict()

    def eval_async(self):
        """cocoa_eval_async: enqueue the objectives of the current state beside
        the next round (one device, fast mode); collect them with eval_wait."""
        C.check(C.lib().cocoa_eval_async(self.h), self.h)

    def eval_wait(self):
        r = C.EvalResult()
        C.check(C.lib().cocoa_eval_wait(self.h, ctypes.byref(r)), self.h)
        return r.as_dict()

    def eval_begin(self):
        """cocoa_eval_begin: the in-line evaluation of the current state, its
        read-back deferred to eval_end (enqueue the next round in between)."""
        C.check(C.lib().cocoa_eval_begin(self.h), self.h)

    def eval_end(self):
        r = C.EvalResult()
        C.check(C.lib().cocoa_eval_end(self.h, ctypes.byref(r)), self.h)
        return r.as_dict()

    def eval_finish(self, hinge_sum, alpha_sum, w_sq, err, test_rows):
        r = C.EvalResult()
        C.check(C.lib().cocoa_eval_finish(self.h, hinge_sum, alpha_sum, w_sq, int(err), int(test_rows),
                                          ctypes.byref(r)), self.h)
        return r.as_dict()

    def run(self, method, n, num_rounds, local_iters, lam, beta=1.0, gamma=1.0, debug_iter=10, seed=0,
            w_init=None, callback=None, chkpt_iter=100, resume_from=None):
        """cocoa_run (or cocoa_resume from a checkpoint file): T rounds with
        evaluation every debug_iter rounds and, when a checkpoint directory is
        set, a checkpoint every chkpt_iter rounds (CoCoA.scala:51-62)."""
        self.params = C.Params(n, num_rounds, local_iters, 0, lam, beta, gamma)
        self.debug = C.Debug(debug_iter, seed, chkpt_iter, 0)

        def _cb(user, t, ev):
            if callback is not None:
                callback(t, ev.contents.as_dict())

        cb = C.ROUND_CB(_cb)
        m = C.METHODS[method] if isinstance(method, str) else int(method)
        if resume_from is not None:
            assert w_init is None, "a resumed run takes w from the checkpoint"
            C.check(C.lib().cocoa_resume(self.h, ctypes.byref(self.params), ctypes.byref(self.debug), m,
                                         os.fsencode(resume_from), cb, None), self.h)
            return
        wi = None if w_init is None else np.ascontiguousarray(w_init, np.float64)
        C.check(C.lib().cocoa_run(self.h, ctypes.byref(self.params), ctypes.byref(self.debug), m,
                                  C.f64p(wi) if wi is not None else None, cb, None), self.h)

    def set_checkpoint_dir(self, path):
        """Periodic checkpoints inside run() (None turns them off)."""
        C.check(C.lib().cocoa_set_checkpoint_dir(self.h, None if path is None else os.fsencode(path)), self.h)

    def checkpoint_file(self, method):
        """Path of run()'s periodic checkpoint for `method` on this rank."""
        buf = ctypes.create_string_buffer(4096)
        m = C.METHODS[method] if isinstance(method, str) else int(method)
        C.check(C.lib().cocoa_checkpoint_file(self.h, m, buf, len(buf)), self.h)
        return os.fsdecode(buf.value)

    def w(self):
        out = np.zeros(self.d, np.float64)
        C.check(C.lib().cocoa_get_w(self.h, C.f64p(out)), self.h)
        return out

    def alpha(self):
        out = np.zeros(self.n_rows, np.float64)
        C.check(C.lib().cocoa_get_alpha(self.h, C.f64p(out)), self.h)
        return out

    def set_w(self, w):
        w = np.ascontiguousarray(w, np.float64)
        C.check(C.lib().cocoa_set_w(self.h, C.f64p(w)), self.h)

    def set_alpha(self, a):
        a = np.ascontiguousarray(a, np.float64)
        C.check(C.lib().cocoa_set_alpha(self.h, C.f64p(a)), self.h)

    def save_checkpoint(self, path, t):
        """(t, w, alpha) of this rank to `path` (cocoa_checkpoint_save)."""
        C.check(C.lib().cocoa_checkpoint_save(self.h, os.fsencode(path), int(t)), self.h)

    def load_checkpoint(self, path):
        """Restore w and alpha from `path`; returns the round t to resume after."""
        t = ctypes.c_int32(0)
        C.check(C.lib().cocoa_checkpoint_load(self.h, os.fsencode(path), ctypes.byref(t)), self.h)
        return t.value

    def local_sdca(self, part, w, local_iters, lam, n, alpha, seed, plus, sigma):
        """CoCoA.localSDCA on partition `part` (CoCoA.scala:130).  w and alpha are
        updated in place like the reference; returns (deltaAlpha, deltaW)."""
        assert w.dtype == np.float64 and alpha.dtype == np.float64
        dw = np.zeros(self.d, np.float64)
        da = np.zeros(len(alpha), np.float64)
        C.check(C.lib().cocoa_local_sdca(self.h, part, C.f64p(w), local_iters, lam, n, C.f64p(alpha), seed,
                                         1 if plus else 0, sigma, C.f64p(dw), C.f64p(da)), self.h)
        return da, dw

    def samples(self, part, seed_plus_t, count):
        out = np.zeros(count, np.int32)
        C.check(C.lib().cocoa_samples(self.h, part, seed_plus_t, count, C.i32p(out)), self.h)
        return out

    # -- profiling -----------------------------------------------------------
    def stats_enable(self, on=True):
        C.check(C.lib().cocoa_stats_enable(self.h, 1 if on else 0), self.h)

    def stats_kernels(self, names=None):
        """Bracket only these kernels (names from KERNEL_NAMES; None: all) while stats are on."""
        mask = 0xFFFFFFFF if names is None else sum(1 << C.KERNEL_NAMES.index(n) for n in names)
        C.check(C.lib().cocoa_stats_kernels(self.h, mask), self.h)

    def stats_reset(self):
        C.check(C.lib().cocoa_stats_reset(self.h), self.h)

    def kernel_stats(self):
        out = {}
        for i, name in enumerate(C.KERNEL_NAMES):
            ms = ctypes.c_double()
            cnt = ctypes.c_int64()
            rc = C.lib().cocoa_kernel_stats(self.h, i, ctypes.byref(ms), ctypes.byref(cnt))
            if rc == C.E_ARG and i >= C.K_XW:  # a library built before this kernel id existed (A/B runs)
                continue
            C.check(rc, self.h)
            out[name] = {"total_ms": ms.value, "launches": cnt.value}
        return out

    def solver_profile(self, on=True):
        C.check(C.lib().cocoa_solver_profile(self.h, 1 if on else 0), self.h)

    def solver_profile_read(self, count=None):
        """Raw counters: [K_loc][32] of the solver, then (count > 32 K_loc) the
        gram_kernel phase sums.  Default: the solver part as [K_loc][2][16]."""
        n = self.K_loc * 32 if count is None else count
        out = np.zeros(n, np.uint64)
        C.check(C.lib().cocoa_solver_profile_read(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                  len(out)), self.h)
        return out.reshape(self.K_loc, 2, 16) if count is None else out

    def gram_rows(self, t):
        """cocoa_debug_gram_rows: round t's Gram rows, shape [K_loc, nbatch * 16, 48]."""
        p = self.plan()
        K, H = p["K_loc"], self.params.local_iters
        nb = (H + 15) // 16
        out = np.zeros(K * nb * 16 * 48, np.float64)
        C.check(C.lib().cocoa_debug_gram_rows(self.h, int(t), C.f64p(out), out.size), self.h)
        return out.reshape(K, nb * 16, 48)

    def plan(self):
        buf = ctypes.create_string_buffer(2048)
        C.check(C.lib().cocoa_plan_info(self.h, buf, 2048), self.h)
        return json.loads(buf.value.decode())

    def gram_fallback_count(self):
        """Windows the last Gram-row launch sent to the per-window kernel (-1: none in use)."""
        v = ctypes.c_int32(0)
        C.check(C.lib().cocoa_gram_fallback_count(self.h, ctypes.byref(v)), self.h)
        return v.value

    def sync(self):
        C.check(C.lib().cocoa_sync(self.h), self.h)

    def close(self):
        if getattr(self, "h", None):
            C.lib().cocoa_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
