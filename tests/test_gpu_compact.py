"""Compact deltaW slices (config C4 layout): partition k's slice holds only the
distinct columns of its rows, the fold gathers each column's entries in
partition order (CoCoA.scala:47, the dense fold with its zero terms dropped).

The layout changes where deltaW lives, not the arithmetic: every dot still
sums the row's entries in stored order.  Which columns the Gram solver keeps in
LDS follows the slice order, so the order of the fast-mode deltaW adds can
differ between the layouts: a run with compact slices agrees with the same run
with dense slices to 1e-12, and both agree with the oracle within 1e-9.  COCOA_DW_COMPACT (read by cocoa_set_train) forces the
layout on small problems.
"""
import numpy as np
import pytest

from cocoa_amd import Engine, configs
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9


def run(sh, method, compact, monkeypatch, rounds=4, strict=False, solver="gram"):
    monkeypatch.setenv("COCOA_DW_COMPACT", "1" if compact else "0")
    e = Engine(strict=strict)
    e.set_train(sh.train, part_begin=sh.part_begin, num_parts_global=sh.k_glob)
    e.set_test(sh.test)
    e.set_solver(solver)
    e.init(method, sh.n_glob, rounds, sh.H, sh.lam)
    assert e.plan()["dw_compact"] == (1 if compact else 0)
    evs = []
    for t in range(1, rounds + 1):
        e.round(t)
        evs.append(e.eval())
    return e, evs


def test_cocoa_keeps_dense_slices(monkeypatch):
    """CoCoA's task-local copy of w is indexed by the global column."""
    sh = configs.share("c4", n=8000, d=100000, parts=8, n_test=100)
    monkeypatch.setenv("COCOA_DW_COMPACT", "1")
    e = Engine(strict=False)
    e.set_train(sh.train)
    e.init("cocoa", sh.n_glob, 1, sh.H, sh.lam)
    assert e.plan()["dw_compact"] == 0
    e.init("cocoa+", sh.n_glob, 1, sh.H, sh.lam)
    assert e.plan()["dw_compact"] == 1


@pytest.mark.parametrize("method", ["cocoa+", "mbcd"])
def test_compact_slices_match_dense_slices(method, monkeypatch):
    sh = configs.share("c4", n=40000, d=400000, parts=32, n_test=2000)
    a, ea = run(sh, method, True, monkeypatch)
    b, eb = run(sh, method, False, monkeypatch)
    p = a.plan()
    assert p["max_u"] * 4 < sh.train.num_features and p["sum_u"] > 0
    wb = b.w()
    assert np.max(np.abs(a.w() - wb)) <= 1e-12 * np.max(np.abs(wb))
    assert np.max(np.abs(a.alpha() - b.alpha())) <= 1e-12
    for x, y in zip(ea, eb):
        assert abs(x["gap"] - y["gap"]) <= 1e-12 * abs(y["primal"]) and x["test_err_count"] == y["test_err_count"]


def test_compact_slices_vs_oracle(monkeypatch):
    sh = configs.share("c4", n=40000, d=400000, parts=32, n_test=2000)
    e, evs = run(sh, "cocoa+", True, monkeypatch)
    od = oracle.Data(sh.train.row_ptr, sh.train.col, sh.train.val, sh.train.y, sh.train.part_ptr,
                     sh.train.num_features)
    ot = oracle.Data(sh.test.row_ptr, sh.test.col, sh.test.val, sh.test.y, sh.test.part_ptr, sh.test.num_features)
    r = oracle.Run(od, "cocoa+", sh.n_glob, sh.H, sh.lam, nthreads=16)
    for t in range(1, 5):
        r.round(t)
    rv = r.eval(ot)
    ev = evs[-1]
    assert abs(ev["primal"] - rv["primal"]) <= REL * abs(rv["primal"])
    assert abs(ev["gap"] - rv["gap"]) <= REL * abs(rv["primal"])
    assert ev["test_err_count"] == rv["test_err"]
    wr = r.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))


def test_c4_share_uses_compact_slices():
    """One GPU's 8-way share of C4 (K_loc = 128, d = 3,231,961) picks the compact
    layout by default: 128 x 3.23 M dense doubles would be 3.3 GB."""
    sh = configs.share("c4", rank=0, world=8, scaling="strong", n_test=1000)
    e = Engine(strict=False)
    e.set_train(sh.train, part_begin=sh.part_begin, num_parts_global=sh.k_glob)
    e.init("cocoa+", sh.n_glob, 1, sh.H, sh.lam)
    p = e.plan()
    assert p["dw_compact"] == 1 and p["dw_dbuf"] == 1 and p["solver"] == "gram" and p["fold"] == "blocks"
    assert p["max_u"] * 8 < sh.train.num_features


@pytest.mark.parametrize("method", ["cocoa+", "mbcd"])
def test_compact_slices_strict_chain_bitwise_vs_oracle(method, monkeypatch):
    """The chain solver (strict mode) on compact slices: bitwise equal to the
    oracle, whose deltaW is dense (the fold's dropped terms are exact zeros)."""
    sh = configs.share("c4", n=20000, d=300000, parts=16, n_test=1000)
    e, evs = run(sh, method, True, monkeypatch, rounds=3, strict=True, solver="auto")
    assert e.plan()["solver"] == "chain"
    od = oracle.Data(sh.train.row_ptr, sh.train.col, sh.train.val, sh.train.y, sh.train.part_ptr,
                     sh.train.num_features)
    ot = oracle.Data(sh.test.row_ptr, sh.test.col, sh.test.val, sh.test.y, sh.test.part_ptr, sh.test.num_features)
    r = oracle.Run(od, method, sh.n_glob, sh.H, sh.lam, nthreads=16)
    for t in range(1, 4):
        r.round(t)
    assert np.array_equal(e.w(), r.w())
    assert np.array_equal(e.alpha(), r.alpha())
    rv = r.eval(ot)
    assert evs[-1]["gap"].hex() == rv["gap"].hex() and evs[-1]["test_err_count"] == rv["test_err"]


def test_compact_slices_fast_chain_vs_oracle(monkeypatch):
    sh = configs.share("c4", n=20000, d=300000, parts=16, n_test=1000)
    e, evs = run(sh, "cocoa+", True, monkeypatch, rounds=3, solver="chain")
    od = oracle.Data(sh.train.row_ptr, sh.train.col, sh.train.val, sh.train.y, sh.train.part_ptr,
                     sh.train.num_features)
    r = oracle.Run(od, "cocoa+", sh.n_glob, sh.H, sh.lam, nthreads=16)
    for t in range(1, 4):
        r.round(t)
    wr = r.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - r.alpha())) <= REL


@pytest.mark.parametrize("solver", ["gram", "chain"])
def test_block_fold_matches_gather_fold(solver, monkeypatch):
    """Fast mode folds compact slices by column blocks (double-buffered sets,
    fold_blocks_kernel); a single slice set keeps the per-column gather fold
    that zeroes as it reads.  Same rounds, same results within 1e-12 (the
    block fold reassociates the partition sums)."""
    sh = configs.share("c4", n=40000, d=400000, parts=32, n_test=2000)
    monkeypatch.setenv("COCOA_DW_PRIVATE", "0")  # (the same slot layout in both runs: test_gpu_private.py)
    monkeypatch.setenv("COCOA_DW_DBUF", "0")
    b, eb = run(sh, "cocoa+", True, monkeypatch, rounds=4, solver=solver)
    assert b.plan()["fold"] == "gather" and b.plan()["dw_dbuf"] == 0
    monkeypatch.delenv("COCOA_DW_DBUF")
    a, ea = run(sh, "cocoa+", True, monkeypatch, rounds=4, solver=solver)
    assert a.plan()["fold"] == "blocks" and a.plan()["dw_dbuf"] == 1
    wb = b.w()
    assert np.max(np.abs(a.w() - wb)) <= 1e-12 * np.max(np.abs(wb))
    assert np.max(np.abs(a.alpha() - b.alpha())) <= 1e-12
    for x, y in zip(ea, eb):
        assert abs(x["gap"] - y["gap"]) <= 1e-12 * abs(y["primal"]) and x["test_err_count"] == y["test_err_count"]


def test_chain_hot_slice_positions_in_lds_are_bitwise_neutral(monkeypatch):
    """Fast CoCoA+ on compact slices keeps each slice's first positions (the
    partition's most frequent columns) in LDS for the launch (SolverArgs::hot).
    Where a value lives does not change the solver's arithmetic; the same rounds
    with COCOA_CHAIN_HOT=0 agree to 1e-12 (the block fold's fp64 atomic adds,
    where work items share a column block, reassociate between runs)."""
    sh = configs.share("c4", n=20000, d=300000, parts=16, n_test=1000)
    # (the slot per distinct column: with private columns these 16 slices fit LDS whole)
    monkeypatch.setenv("COCOA_DW_PRIVATE", "0")
    a, ea = run(sh, "cocoa+", True, monkeypatch, rounds=3, solver="chain")
    assert a.plan()["chain_hot"] >= 1024 and a.plan()["vec_lds"] == 0, a.plan()
    monkeypatch.setenv("COCOA_CHAIN_HOT", "0")
    b, eb = run(sh, "cocoa+", True, monkeypatch, rounds=3, solver="chain")
    assert b.plan()["chain_hot"] == 0
    wb = b.w()
    assert np.max(np.abs(a.w() - wb)) <= 1e-12 * np.max(np.abs(wb))
    assert np.max(np.abs(a.alpha() - b.alpha())) <= 1e-12
    for x, y in zip(ea, eb):
        assert abs(x["gap"] - y["gap"]) <= 1e-12 * abs(y["primal"]) and x["test_err_count"] == y["test_err_count"]
