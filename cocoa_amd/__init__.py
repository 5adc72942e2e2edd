"""cocoa_amd -- MI355X-native engine for the per-round CoCoA / CoCoA+ hot path
of calvinmccarter/cocoa (local SDCA, deltaW aggregation, primal/dual/gap and
test-error evaluation), built on hand-written gfx950 HIP kernels behind the C
ABI in include/cocoa_capi.h.  See DESIGN.md."""
from ._capi import CocoaError, IllegalArgumentError, IndexOutOfBoundsError, NoDeviceError, NumberFormatError  # noqa
from .data import LabeledData, gen_synthetic, jrandom_ints, load_libsvm  # noqa
from .engine import Engine  # noqa
from .solvers import CoCoA, DebugParams, MinibatchCD, OptUtils, Params, SGD, jstr  # noqa

__all__ = ["Engine", "LabeledData", "load_libsvm", "gen_synthetic", "jrandom_ints", "CoCoA", "MinibatchCD", "SGD",
           "OptUtils", "Params", "DebugParams", "jstr", "CocoaError"]
