"""CPU oracle (oracle/cocoa_oracle.c) pinned against the golden fixtures made
by the independent Python restatement (tests/golden/make_golden.py), JDK
java.util.Random known answers, the Hadoop split sizes of the demo data and
the liblinear optimum of the demo problem."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle

G = os.path.join(os.path.dirname(__file__), "golden")
TRAIN = os.path.join(G, "data", "small_train.dat")
TEST = os.path.join(G, "data", "small_test.dat")


def _j(name):
    return json.load(open(os.path.join(G, name)))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, "<f8").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def c1():
    return oracle.Data.load_libsvm(TRAIN, 4, 9947), oracle.Data.load_libsvm(TEST, 4, 9947)


def test_jdk_random_known_answers():
    # java.util.Random known answers (JDK spec algorithm)
    assert oracle.jrandom_ints(0, 0, 1)[0] == -1155484576
    assert oracle.jrandom_ints(42, 0, 1)[0] == -1170105035
    assert oracle.jrandom_ints(1, 0, 3).tolist() == [-1155869325, 431529176, 1761283695]
    assert oracle.jrandom_ints(42, 10, 10).tolist() == [0, 3, 8, 4, 0, 5, 5, 8, 9, 3]
    meta = _j("c1_meta.json")["jrandom"]
    assert oracle.jrandom_ints(1, 522, 8).tolist() == meta["seed1_nextInt522"]
    assert oracle.jrandom_ints(1, 512, 5).tolist() == meta["seed1_nextInt512"] == [374, 51, 209, 208, 106]


def test_jdk_random_rejection_branch():
    # bound close to 2^31 forces the rejection loop often; compare with a direct Python LCG
    from tests.golden.make_golden import JRandom
    for bound in (2**30 + 1, 1500000001, 3, 7, 2**20):
        r = JRandom(12345)
        exp = [r.next_int(bound) for _ in range(200)]
        assert oracle.jrandom_ints(12345, bound, 200).tolist() == exp


def test_demo_partition_sizes(c1):
    tr, te = c1
    meta = _j("c1_meta.json")
    assert np.diff(tr.part_ptr).tolist() == meta["train_part_sizes"] == [522, 510, 577, 391]
    assert np.diff(te.part_ptr).tolist() == meta["test_part_sizes"] == [168, 148, 180, 104]
    nnz = [int(tr.row_ptr[tr.part_ptr[k + 1]] - tr.row_ptr[tr.part_ptr[k]]) for k in range(4)]
    assert nnz == meta["train_part_nnz"]
    assert tr.n == 2000 and te.n == 600 and tr.row_ptr[-1] == 94790 and te.row_ptr[-1] == 23730
    # two label-only rows in the test file (lines 55 and 343)
    assert (np.diff(te.row_ptr) == 0).sum() == 2


def test_row_sqnorm(c1):
    tr, _ = c1
    head = [float.fromhex(h) for h in _j("c1_meta.json")["row_sqnorm_head"]]
    assert tr.row_sqnorm()[:16].tolist() == head


@pytest.mark.parametrize("plus", [True, False])
def test_local_sdca_unit(c1, plus):
    tr, _ = c1
    fx = _j("c1_localsdca_%s.json" % ("plus" if plus else "cocoa"))
    w = np.zeros(9947)
    w[::7] = ((np.arange(0, 9947, 7) % 13) - 6) * 1e-3
    assert sha(w) == fx["w_in_sha256"]
    part = fx["part"]
    nl = int(tr.part_ptr[part + 1] - tr.part_ptr[part])
    a = np.zeros(nl)
    a[::3] = 0.5
    da, dw = oracle.local_sdca(tr, part, w, fx["H"], fx["lam"], fx["n"], a, fx["seed"], plus, fx["sigma"])
    assert sha(dw) == fx["dw_sha256"]
    assert sha(a) == fx["alpha_sha256"]
    assert sha(w) == fx["w_out_sha256"]  # w mutated only when !plus (CoCoA.scala:182-184)


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
def test_run_matches_golden_bitwise(c1, method):
    tr, te = c1
    fx = _j("c1_%s.json" % method.replace("+", "plus"))
    cfg = _j("c1_meta.json")["config"]
    run = oracle.Run(tr, method, tr.n, cfg["H"], cfg["lam"], cfg["beta"], cfg["gamma"], cfg["seed"], nthreads=2)
    recs = {r["t"]: r for r in fx["trace"]}
    for t in range(1, cfg["T"] + 1):
        run.round(t)
        if t in recs:
            ev = run.eval(te)
            assert ev["primal"].hex() == recs[t]["primal"], t
            if "dual" in recs[t]:
                assert ev["dual"].hex() == recs[t]["dual"], t
                assert ev["gap"].hex() == recs[t]["gap"], t
            assert ev["test_err"] == recs[t]["test_err"], t
    assert sha(run.w()) == fx["w_sha256"]
    assert [v.hex() for v in run.w()[:64]] == fx["w_head"]
    if method in ("cocoa+", "cocoa", "mbcd"):
        assert sha(run.alpha()) == fx["alpha_sha256"]
    assert tr.error_count(run.w()) == fx["train_err"]


def test_threads_do_not_change_results(c1):
    tr, _ = c1
    ws = []
    for nt in (1, 4):
        run = oracle.Run(tr, "cocoa+", tr.n, 50, 1e-3, nthreads=nt)
        for t in range(1, 6):
            run.round(t)
        ws.append((run.w(), run.alpha()))
    assert np.array_equal(ws[0][0], ws[1][0]) and np.array_equal(ws[0][1], ws[1][1])


def test_cocoa_plus_approaches_liblinear_optimum(c1):
    tr, _ = c1
    pstar = _j("c1_liblinear.json")["primal_opt"]
    run = oracle.Run(tr, "cocoa+", tr.n, 50, 1e-3, nthreads=4)
    last = None
    for t in range(1, 1201):
        run.round(t)
        if t % 100 == 0:
            ev = run.eval()
            assert ev["gap"] >= 0.0                 # weak duality
            assert ev["dual"] <= pstar + 1e-9       # D(alpha) <= P* <= P(w)
            last = ev
    assert last["primal"] - pstar < 2e-4
    assert last["gap"] < 1e-3
