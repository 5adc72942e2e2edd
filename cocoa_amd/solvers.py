"""Host-side mirror of the reference's solver / utility API, backed by the HIP
engine (one GPU).  Names, argument meaning, printed lines and error kinds
follow the Scala reference so a caller can switch over unchanged:

  CoCoA.runCoCoA(data, params, debug, plus)      CoCoA.scala:22-66
  CoCoA.localSDCA(localData, wInit, ...)          CoCoA.scala:130-192
  MinibatchCD.runMbCD(data, params, debug)        MinibatchCD.scala:19-61
  SGD.runSGD(data, params, debug, local)          SGD.scala:21-70
  OptUtils.loadLIBSVMData / computePrimalObjective / computeDualObjective /
           computeDualityGap / computeClassificationError /
           printSummaryStatsPrimalDual / printSummaryStats   OptUtils.scala
  Params, DebugParams                             OptClasses.scala:21-42
"""
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from .data import LabeledData, load_libsvm
from .engine import Engine
from .jdouble import java_double_tostring


def jstr(x):
    """java.lang.Double.toString as the reference's JVM (JDK 7/8) printed it
    (cocoa_amd/jdouble.py: sun.misc.FloatingDecimal restated)."""
    return java_double_tostring(x)


@dataclass
class Params:
    """OptClasses.scala:21-29 (`loss` is accepted and unused, as in CoCoA)."""
    loss: Optional[Callable] = None
    n: int = 0
    wInit: Optional[np.ndarray] = None
    numRounds: int = 200
    localIters: int = 1
    lambda_: float = 0.01
    beta: float = 1.0
    gamma: float = 1.0


@dataclass
class DebugParams:
    """OptClasses.scala:38-42."""
    testData: Optional[LabeledData] = None
    debugIter: int = 10
    seed: int = 0
    chkptIter: int = 100


class _Printer:
    out = print


def _engine_for(data, debug, strict, device):
    eng = Engine(device=device, strict=strict)
    eng.set_train(data)
    if debug is not None and debug.testData is not None:
        eng.set_test(debug.testData)
    return eng


def _run(method, name, data, params, debug, strict, device, primal_dual, printer):
    p = printer or _Printer.out
    K = data.num_parts
    p(f"\nRunning {name} on {params.n} data examples, distributed over {K} workers")
    eng = _engine_for(data, debug, strict, device)
    eng.init(method, params.n, params.numRounds, params.localIters, params.lambda_, params.beta, params.gamma,
             debug.debugIter, debug.seed, debug.chkptIter, params.wInit)
    for t in range(1, params.numRounds + 1):
        eng.round(t)
        if debug.debugIter > 0 and t % debug.debugIter == 0:
            ev = eng.eval()
            p("Iteration: " + str(t))
            p("primal objective: " + jstr(ev["primal"]))
            if primal_dual:
                p("primal-dual gap: " + jstr(ev["gap"]))
            if debug.testData is not None:
                p("test error: " + jstr(ev["test_error"]))
    w = eng.w()
    alpha = eng.alpha()
    alphas = [alpha[data.part_ptr[k]:data.part_ptr[k + 1]] for k in range(K)]
    eng.close()
    return w, alphas


class CoCoA:
    @staticmethod
    def runCoCoA(data, params, debug, plus, strict=False, device=0, printer=None):
        """Returns (w, alpha per partition)."""
        return _run("cocoa+" if plus else "cocoa", "CoCoA+" if plus else "CoCoA", data, params, debug, strict,
                    device, True, printer)

    @staticmethod
    def localSDCA(localData, wInit, localIters, lambda_, n, alpha, alphaOld, seed, plus, sigma, strict=False,
                  device=0):
        """One partition's local SDCA.  Mutates `alpha` (and `wInit` when not
        plus) in place like the reference; returns (deltaAlpha, deltaW)."""
        data = localData if localData.num_parts == 1 else localData.row_range(0, localData.n)
        eng = Engine(device=device, strict=strict)
        eng.set_train(data)
        _, dw = eng.local_sdca(0, wInit, localIters, lambda_, n, alpha, seed, plus, sigma)
        eng.close()
        return alpha - alphaOld, dw


class MinibatchCD:
    @staticmethod
    def runMbCD(data, params, debug, strict=False, device=0, printer=None):
        return _run("mbcd", "Mini-batch CD", data, params, debug, strict, device, True, printer)


class SGD:
    @staticmethod
    def runSGD(data, params, debug, local, strict=False, device=0, printer=None):
        p = printer or _Printer.out
        # SGD.scala:29 prints its own banner
        name = f"SGD (with local updates = {'true' if local else 'false'})"
        w, _ = _run("localsgd" if local else "mbsgd", name, data, params, debug, strict, device, False,
                    lambda s: p(s))
        return w


class OptUtils:
    @staticmethod
    def loadLIBSVMData(sc, filename, numSplits, numFeats):
        """`sc` is ignored (no SparkContext)."""
        return load_libsvm(filename, numSplits, numFeats)

    @staticmethod
    def _eval(data, w, alpha=None, lam=0.0, test=None, strict=True, device=0):
        eng = Engine(device=device, strict=strict)
        eng.set_train(data)
        if test is not None:
            eng.set_test(test)
        eng.init("cocoa+", data.n, 0, 0, lam)
        eng.set_w(w)
        if alpha is not None:
            eng.set_alpha(np.concatenate([np.asarray(a, np.float64) for a in alpha]) if isinstance(alpha, list)
                          else alpha)
        ev = eng.eval()
        eng.close()
        return ev

    @staticmethod
    def computePrimalObjective(data, w, lambda_, strict=True, device=0):
        return OptUtils._eval(data, w, None, lambda_, strict=strict, device=device)["primal"]

    @staticmethod
    def computeDualObjective(data, w, alpha, lambda_, strict=True, device=0):
        return OptUtils._eval(data, w, alpha, lambda_, strict=strict, device=device)["dual"]

    @staticmethod
    def computeDualityGap(data, w, alpha, lambda_, strict=True, device=0):
        return OptUtils._eval(data, w, alpha, lambda_, strict=strict, device=device)["gap"]

    @staticmethod
    def computeClassificationError(data, w, strict=True, device=0):
        return OptUtils._eval(data, w, None, 0.0, test=data, strict=strict, device=device)["test_error"]

    @staticmethod
    def printSummaryStatsPrimalDual(algName, data, w, alpha, lambda_, testData, printer=None, strict=True, device=0):
        p = printer or _Printer.out
        ev = OptUtils._eval(data, w, alpha, lambda_, test=testData, strict=strict, device=device)
        s = algName + " has finished running. Summary Stats: "
        s += "\n Total Objective Value: " + jstr(ev["primal"])
        s += "\n Duality Gap: " + jstr(ev["gap"])
        if testData is not None:
            s += "\n Test Error: " + jstr(ev["test_error"])
        p(s + "\n")

    @staticmethod
    def printSummaryStats(algName, data, w, lambda_, testData, printer=None, strict=True, device=0):
        p = printer or _Printer.out
        ev = OptUtils._eval(data, w, None, lambda_, test=testData, strict=strict, device=device)
        s = algName + " has finished running. Summary Stats: "
        s += "\n Total Objective Value: " + jstr(ev["primal"])
        if testData is not None:
            s += "\n Test Error: " + jstr(ev["test_error"])
        p(s + "\n")
