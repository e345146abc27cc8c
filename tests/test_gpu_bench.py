"""bench.py on the GPU: the one JSON line the driver parses (contract keys, roofline, config 2 shape)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["higher_is_better"] is True
    assert d["config"]["width"] == 1920 and d["config"]["height_per_gpu"] == 1080
    assert d["config"]["spp"] == 16 and d["config"]["bounces"] == 8 and d["config"]["seed"] == 12345
    assert d["intersections_per_step"] == 56746603  # the oracle's count for config 2
    assert d["value"] > 1e9
    rf = d["roofline"]
    assert 0 < rf["frac"] < 1 and rf["peak"] == 157.3 and rf["achieved"] == pytest.approx(rf["frac"] * rf["peak"])
