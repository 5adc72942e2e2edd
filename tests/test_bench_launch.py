"""bench.py's own N-rank launcher: `bench.py --gpus N`
spawns N ranks before any GPU call and relays rank 0's JSON line, and a rank
whose WORLD_SIZE differs from --gpus fails.  The CPU tests use --launch-probe
(each rank returns before touching a device); the GPU test runs two ranks of a
small weak-scaled C2 shard over the HOST transport on the box's one GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _clean_env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.strip().startswith("{")]


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-probe"], cwd=ROOT, env=_clean_env(),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    assert lines[0]["world"] == n and lines[0]["rank"] == 0
    assert lines[0]["master"].startswith("127.0.0.1:")


def test_bench_world_mismatch_fails():
    env = dict(_clean_env(), RANK="0", WORLD_SIZE="2", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-probe"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_host_transport():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--transport", "host", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--no-gap", "--n", "40000", "--parts", "16", "--n-test", "4000"],
                       cwd=ROOT, env=_clean_env(), capture_output=True, text=True, timeout=380)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["comm"] == {"transport": "host", "world": 2}
    assert d["config"]["K_total"] == 32 and d["value"] > 0


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_comm_rule_eight_ranks_must_run_rccl():
    """an 8-rank line exits non-zero unless the library's
    communicator runs the requested transport (RCCL) over all 8 ranks."""
    b = _bench_module()
    ok = {"transport": "rccl", "rank": 3, "world": 8}
    assert b.comm_mismatch("rccl", 3, 8, ok) is None
    assert "runs host" in b.comm_mismatch("rccl", 3, 8, dict(ok, transport="host"))
    assert b.comm_mismatch("rccl", 3, 8, dict(ok, world=4))
    assert b.comm_mismatch("rccl", 3, 8, dict(ok, rank=0))
    assert b.comm_mismatch("rccl", 3, 8, None)
    assert b.comm_mismatch("rccl", 0, 1, None) is None  # one rank: no exchange
    assert b.comm_mismatch("host", 1, 2, {"transport": "host", "rank": 1, "world": 2}) is None


def test_launch_probe_reports_transport():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], cwd=ROOT, env=_clean_env(),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_lines(p.stdout)[0]
    assert d["transport"] == "rccl" and d["world"] == 2
