#!/usr/bin/env python3
"""Independent pure-Python restatement of calvinmccarter/cocoa's hot path.

Test infrastructure only.  It regenerates the committed golden fixtures
``tests/golden/c1_*.json`` for config C1 (the reference's demo:
``run-demo-local.sh:1-9`` -> K=4, lambda=1e-3, localIterFrac=0.1 (H=50),
numRounds=100, debugIter=10, seed=0, numFeatures=9947).

It is written separately from ``oracle/cocoa_oracle.c`` so the two
restatements cross-check each other bit for bit (Python floats are IEEE
doubles with no fused multiply-add; sums are explicit left-to-right loops).
Parity with the JVM reference itself is unpinned (no JVM here, no reference
tests); see the oracle header for the assumptions about breeze/Spark.

Usage: python tests/golden/make_golden.py [--data /root/reference/data]
(the demo data files are copied as fixtures into tests/golden/data/).
"""
import argparse
import hashlib
import json
import math
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


# --- java.util.Random (JDK) -------------------------------------------------
class JRandom:
    MULT = 0x5DEECE66D
    MASK = (1 << 48) - 1

    def __init__(self, seed):
        self.s = (seed ^ self.MULT) & self.MASK

    def next(self, bits):
        self.s = (self.s * self.MULT + 0xB) & self.MASK
        v = self.s >> (48 - bits)
        if v >= 1 << 31:
            v -= 1 << 32
        return v

    def next_int(self, bound=None):
        if bound is None:
            return self.next(32)
        r = self.next(31)
        m = bound - 1
        if bound & m == 0:
            return (bound * r) >> 31
        u = r
        while True:
            r = u % bound
            t = (u - r + m) & 0xFFFFFFFF
            if t < (1 << 31):
                return r
            u = self.next(31)


# --- LIBSVM + Hadoop 1.0.4 split (OptUtils.scala:11-53) ---------------------
def hadoop_split_starts(size, num_splits):
    goal = size // max(num_splits, 1)
    split = max(1, min(goal, 32 * 1024 * 1024))
    starts, rem = [], size
    while rem / split > 1.1:
        starts.append(size - rem)
        rem -= split
    if rem:
        starts.append(size - rem)
    return starts or [0]


def load_libsvm(path, num_splits, num_feats):
    raw = open(path, "rb").read()
    starts = hadoop_split_starts(len(raw), num_splits)
    assert len(starts) == num_splits, "demo files never need coalescing"
    rows, offs, pos = [], [], 0
    for line in raw.split(b"\n"):
        if pos < len(raw):
            rows.append(line.decode())
            offs.append(pos)
        pos += len(line) + 1
    part_of = []
    for o in offs:
        k = 0
        while k + 1 < len(starts) and o >= starts[k + 1]:
            k += 1
        part_of.append(k)
    data = []
    for line in rows:
        parts = line.strip().split(" ")
        lab = 1.0 if ("+" in parts[0] or int(parts[0]) == 1) else -1.0
        idx, val = [], []
        for tok in parts[1:]:
            i, j = tok.split(":")
            idx.append(int(i) - 1)
            val.append(float(j))
        data.append((lab, idx, val))
    K = num_splits
    parts = [[data[r] for r in range(len(data)) if part_of[r] == k] for k in range(K)]
    return parts


# --- breeze arithmetic (sequential, from 0.0) -------------------------------
def dot(idx, val, dense):
    s = 0.0
    for i, v in zip(idx, val):
        s += v * dense[i]
    return s


def norm2(vals):
    s = 0.0
    for v in vals:
        s += v * v
    return math.sqrt(s)


def jmax(a, b):
    if a != a:
        return a
    if a == 0.0 and b == 0.0:
        return b if math.copysign(1.0, a) < 0 else a
    return a if a >= b else b


def jmin(a, b):
    if a != a:
        return a
    if a == 0.0 and b == 0.0:
        return a if math.copysign(1.0, a) < 0 else b
    return a if a <= b else b


# --- CoCoA.localSDCA (CoCoA.scala:130-192) ----------------------------------
def local_sdca(local, w, H, lam, n, alpha, seed, plus, sigma):
    r = JRandom(seed)
    d = len(w)
    dW = [0.0] * d
    lam_n = lam * n
    for _ in range(H):
        i = r.next_int(len(local))
        y, idx, val = local[i]
        if plus:
            g = (y * (dot(idx, val, w) + (sigma * dot(idx, val, dW))) - 1.0) * lam_n
        else:
            g = (y * (dot(idx, val, w)) - 1.0) * lam_n
        pg = g
        if alpha[i] <= 0.0:
            pg = jmin(g, 0.0)
        elif alpha[i] >= 1.0:
            pg = jmax(g, 0.0)
        if abs(pg) != 0.0:
            nr = norm2(val)
            xn = nr * nr
            q = xn * sigma if plus else xn
            na = 1.0
            if q != 0.0:
                na = jmin(jmax(alpha[i] - (g / q), 0.0), 1.0)
            c = (y * (na - alpha[i])) / lam_n
            for j, v in zip(idx, val):
                u = v * c
                if not plus:
                    w[j] += u
                dW[j] += u
            alpha[i] = na
    return dW


def mbcd_local(local, w, H, lam, n, alpha, seed):
    r = JRandom(seed)
    dW = [0.0] * len(w)
    lam_n = lam * n
    for _ in range(H):
        i = r.next_int(len(local))
        y, idx, val = local[i]
        g = (y * (dot(idx, val, w)) - 1.0) * lam_n
        pg = g
        if alpha[i] <= 0.0:
            pg = jmin(g, 0.0)
        elif alpha[i] >= 1.0:
            pg = jmax(g, 0.0)
        if abs(pg) != 0.0:
            nr = norm2(val)
            q = nr * nr
            na = 1.0
            if q != 0.0:
                na = jmin(jmax(alpha[i] - (g / q), 0.0), 1.0)
            c = (y * (na - alpha[i])) / lam_n
            for j, v in zip(idx, val):
                dW[j] += v * c
            alpha[i] = na
    return dW


def sgd_local(local, w_init, lam, t0, H, is_local, seed):
    r = JRandom(seed)
    w = np.array(w_init, dtype=np.float64)
    dW = np.zeros_like(w)
    for i in range(1, H + 1):
        step = 1.0 / (lam * (t0 + i))
        k = r.next_int(len(local))
        y, idx, val = local[k]
        ev = 1.0 - (y * dot(idx, val, w))
        if is_local:
            w *= 1.0 - (step * lam)
        if ev > 0:
            for j, v in zip(idx, val):
                u = v * y
                dW[j] += u
                if is_local:
                    w[j] += u * step
        if is_local:
            dW = w - np.asarray(w_init)
    return list(dW)


# --- OptUtils (OptUtils.scala:57-98) ----------------------------------------
def hinge_sum(parts, w):
    tot = None
    for p in parts:
        acc = None
        for (y, idx, val) in p:
            h = jmax(1 - y * (dot(idx, val, w)), 0.0)
            acc = h if acc is None else acc + h
        if acc is not None:
            tot = acc if tot is None else tot + acc
    return tot


def n_rows(parts):
    return sum(len(p) for p in parts)


def primal(parts, w, lam):
    nr = norm2(w)
    return hinge_sum(parts, w) / n_rows(parts) + (0.5 * lam * (nr * nr))


def dual(parts, w, alphas, lam):
    tot = None
    for a in alphas:
        s = 0.0
        for v in a:
            s += v
        tot = s if tot is None else tot + s
    nr = norm2(w)
    return (-lam / 2 * (nr * nr)) + (tot / n_rows(parts))


def err_count(parts, w):
    c = 0
    for p in parts:
        for (y, idx, val) in p:
            if not ((dot(idx, val, w)) * y > 0):
                c += 1
    return c


def sha(vec):
    return hashlib.sha256(struct.pack("<%dd" % len(vec), *vec)).hexdigest()


def wrap32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


# --- drivers: runCoCoA / runMbCD / runSGD -----------------------------------
def run(method, parts, test, d, T, H, lam, beta, gamma, seed, debug_iter):
    K = len(parts)
    n = n_rows(parts)
    w = [0.0] * d
    alphas = [[0.0] * len(p) for p in parts]
    if method == "cocoa+":
        scaling = gamma
    elif method == "cocoa":
        scaling = beta / K
    elif method in ("mbcd", "mbsgd"):
        scaling = beta / wrap32(K * H)
    else:
        scaling = beta / K
    trace = []
    for t in range(1, T + 1):
        s = wrap32(seed + t)
        dws = []
        if method in ("cocoa+", "cocoa", "mbcd"):
            new_alphas = []
            for k in range(K):
                a = list(alphas[k])
                old = list(alphas[k])
                if method == "mbcd":
                    dw = mbcd_local(parts[k], w, H, lam, n, a, s)
                else:
                    wk = list(w)  # the task deserialises its own copy of w
                    dw = local_sdca(parts[k], wk, H, lam, n, a, s, method == "cocoa+", K * gamma)
                new_alphas.append([o + ((x - o) * scaling) for x, o in zip(a, old)])
                dws.append(dw)
            alphas = new_alphas
            mult = scaling
        else:
            step = 1 / (lam * t)
            if method == "mbsgd":
                sc = 1.0 - (step * lam)
                w = [x * sc for x in w]
            t0 = float(wrap32((t - 1) * H * K))
            for k in range(K):
                dws.append(sgd_local(parts[k], w, lam, t0, H, method == "localsgd", s))
            mult = scaling if method == "localsgd" else step * scaling
        tot = list(dws[0])
        for dw in dws[1:]:
            tot = [a + b for a, b in zip(tot, dw)]
        w = [a + (b * mult) for a, b in zip(w, tot)]
        if debug_iter > 0 and t % debug_iter == 0:
            P = primal(parts, w, lam)
            rec = {"t": t, "primal": P.hex()}
            if method in ("cocoa+", "cocoa", "mbcd"):
                D = dual(parts, w, alphas, lam)
                rec["dual"] = D.hex()
                rec["gap"] = (P - D).hex()
            rec["test_err"] = err_count(test, w)
            trace.append(rec)
    flat_alpha = [v for a in alphas for v in a]
    return {
        "trace": trace,
        "w_sha256": sha(w),
        "alpha_sha256": sha(flat_alpha),
        "w_head": [v.hex() for v in w[:64]],
        "w_norm2": norm2(w).hex(),
        "alpha_sum": math.fsum(flat_alpha).hex(),
        "train_err": err_count(parts, w),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default="/root/reference/data")
    ap.add_argument("--rounds", type=int, default=100)
    args = ap.parse_args()
    os.makedirs(os.path.join(HERE, "data"), exist_ok=True)
    for fn in ("small_train.dat", "small_test.dat"):
        dst = os.path.join(HERE, "data", fn)
        src = os.path.join(args.data, fn)
        if os.path.exists(src) and not os.path.exists(dst):
            open(dst, "wb").write(open(src, "rb").read())
    train = load_libsvm(os.path.join(HERE, "data", "small_train.dat"), 4, 9947)
    test = load_libsvm(os.path.join(HERE, "data", "small_test.dat"), 4, 9947)
    cfg = dict(K=4, d=9947, lam=1e-3, beta=1.0, gamma=1.0, seed=0, debug_iter=10, T=args.rounds)
    n = n_rows(train)
    H = max(int(0.1 * n / 4), 1)
    cfg["H"] = H
    meta = {
        "config": cfg,
        "train_part_sizes": [len(p) for p in train],
        "test_part_sizes": [len(p) for p in test],
        "train_part_nnz": [sum(len(r[1]) for r in p) for p in train],
        "jrandom": {
            "seed0_nextInt": [JRandom(0).next_int() for _ in range(1)],
            "seed42_nextInt": JRandom(42).next_int(),
            "seed42_nextInt10": (lambda r: [r.next_int(10) for _ in range(10)])(JRandom(42)),
            "seed1_nextInt522": (lambda r: [r.next_int(522) for _ in range(8)])(JRandom(1)),
            "seed1_nextInt512": (lambda r: [r.next_int(512) for _ in range(5)])(JRandom(1)),
        },
        "row_sqnorm_head": [(lambda nr: (nr * nr).hex())(norm2(r[2])) for r in train[0][:16]],
    }
    json.dump(meta, open(os.path.join(HERE, "c1_meta.json"), "w"), indent=1)
    # one localSDCA call in isolation (CoCoA.localSDCA is public, CoCoA.scala:130)
    for plus in (True, False):
        w = [0.0] * 9947
        for j in range(0, 9947, 7):
            w[j] = ((j % 13) - 6) * 1e-3
        a = [0.0] * len(train[1])
        for j in range(0, len(a), 3):
            a[j] = 0.5
        w_in = list(w)
        dw = local_sdca(train[1], w, 200, 1e-3, n, a, 7, plus, 4.0)
        json.dump({"plus": plus, "H": 200, "lam": 1e-3, "n": n, "seed": 7, "sigma": 4.0, "part": 1,
                   "w_in_sha256": sha(w_in), "w_out_sha256": sha(w), "dw_sha256": sha(dw),
                   "alpha_sha256": sha(a), "dw_sum": math.fsum(dw).hex()},
                  open(os.path.join(HERE, "c1_localsdca_%s.json" % ("plus" if plus else "cocoa")), "w"), indent=1)
    for method in ("cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"):
        res = run(method, train, test, 9947, args.rounds, H, 1e-3, 1.0, 1.0, 0, 10)
        res["method"] = method
        json.dump(res, open(os.path.join(HERE, "c1_%s.json" % method.replace("+", "plus")), "w"), indent=1)
        print(method, res["trace"][-1])


if __name__ == "__main__":
    main()
