"""bench.py's one-line JSON contract on a short run of the headline workload:
BASELINE.json's metric and unit, a positive whole-job value, the roofline
block of the dominant kernel (frac <= 1), vs_baseline null (BASELINE.md
publishes no number), and the configuration it names."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_bench_json_line_contract():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--no-gap"], cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["metric"] == base["metric"]
    assert d["unit"] == "coord updates/s" and d["value"] > 0 and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["vs_baseline"] is None and d["dtype"] == "f64"
    assert d["config"]["workload"].startswith("C2") and d["config"]["eval_flow"].startswith("deferred")
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] <= 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    assert d["ms_per_step"] > 0 and abs(d["value"] - d["config"]["K_total"] * d["config"]["H"] /
                                        (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]
