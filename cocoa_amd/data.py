"""Partitioned CSR datasets (the engine's view of ``RDD[LabeledPoint]``).

``LabeledPoint(label, features)`` (OptClasses.scala:8) rows are stored as one
CSR with rows kept in file order and partition k owning rows
``[part_ptr[k], part_ptr[k+1])`` -- exactly the partitions
``OptUtils.loadLIBSVMData`` (OptUtils.scala:11-53) produces.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _capi as C


@dataclass
class LabeledData:
    row_ptr: np.ndarray   # int64 [n+1]
    col: np.ndarray       # int32 [nnz], 0-based
    val: np.ndarray       # float64 [nnz]
    y: np.ndarray         # float64 [n], +1/-1
    part_ptr: np.ndarray  # int64 [K+1]
    num_features: int

    @property
    def n(self):
        return len(self.y)

    @property
    def num_parts(self):
        return len(self.part_ptr) - 1

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def count(self):
        """RDD.count()"""
        return self.n

    def partition_sizes(self):
        return np.diff(self.part_ptr)

    def shard(self, k0, k1):
        """Partitions [k0, k1) as a stand-alone dataset (one rank's share)."""
        r0, r1 = int(self.part_ptr[k0]), int(self.part_ptr[k1])
        e0, e1 = int(self.row_ptr[r0]), int(self.row_ptr[r1])
        return LabeledData(self.row_ptr[r0:r1 + 1] - e0, self.col[e0:e1], self.val[e0:e1], self.y[r0:r1],
                           self.part_ptr[k0:k1 + 1] - r0, self.num_features)

    def row_range(self, r0, r1):
        e0, e1 = int(self.row_ptr[r0]), int(self.row_ptr[r1])
        return LabeledData(self.row_ptr[r0:r1 + 1] - e0, self.col[e0:e1], self.val[e0:e1], self.y[r0:r1],
                           np.array([0, r1 - r0], np.int64), self.num_features)

    def contiguous(self):
        return LabeledData(*(np.ascontiguousarray(a) for a in (self.row_ptr, self.col, self.val, self.y,
                                                                self.part_ptr)), self.num_features)


def _from_c(ds):
    n, K, nnz = ds.n_rows, ds.num_parts, ds.nnz
    out = LabeledData(np.ctypeslib.as_array(ds.row_ptr, (n + 1,)).copy(),
                      np.ctypeslib.as_array(ds.col, (max(nnz, 1),))[:nnz].copy(),
                      np.ctypeslib.as_array(ds.val, (max(nnz, 1),))[:nnz].copy(),
                      np.ctypeslib.as_array(ds.y, (max(n, 1),))[:n].copy(),
                      np.ctypeslib.as_array(ds.part_ptr, (K + 1,)).copy(), ds.num_features)
    C.lib().cocoa_dataset_free(ctypes.byref(ds))
    return out


def load_libsvm(path, num_splits, num_features, device=None):
    """OptUtils.loadLIBSVMData(sc, filename, numSplits, numFeats) (OptUtils.scala:11).
    device: a HIP device ordinal to tokenise and parse on (cocoa_load_libsvm_gpu);
    None: the multithreaded host parse (cocoa_load_libsvm)."""
    ds = C.Dataset()
    if device is None:
        C.check(C.lib().cocoa_load_libsvm(path.encode(), num_splits, num_features, ctypes.byref(ds)))
    else:
        C.check(C.lib().cocoa_load_libsvm_gpu(int(device), path.encode(), num_splits, num_features, ctypes.byref(ds)))
    return _from_c(ds)


SYNTH_KINDS = {"rcv1": 0, "epsilon": 1, "url": 2}


def gen_synthetic(kind, n, d, mean_nnz, num_parts, seed, threads=0, first_row=0):
    """Seeded synthetic problem of a BASELINE.json shape.
    Rows [first_row, first_row+n) of the seeded stream (first_row % 4096 == 0)."""
    ds = C.Dataset()
    C.check(C.lib().cocoa_gen_synthetic(SYNTH_KINDS[kind], n, d, float(mean_nnz), num_parts, seed, first_row,
                                        threads, ctypes.byref(ds)))
    return _from_c(ds)


def jrandom_ints(seed, bound, count):
    """java.util.Random(seed).nextInt(bound) x count (host)."""
    out = np.zeros(count, np.int32)
    C.check(C.lib().cocoa_jrandom_ints(seed, bound, count, C.i32p(out)))
    return out
