"""bench.py on the GPU: the one JSON line the driver parses (contract keys, roofline, config shapes)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=110):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def test_bench_json_line():
    d = run_bench("--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "setup_ms", "value_per_gpu"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["higher_is_better"] is True and d["scaling"] == "weak"
    c = d["config"]
    assert c["width"] == 1920 and c["height_per_gpu"] == 1080 and c["config"] == 2
    assert c["spp"] == 16 and c["bounces"] == 8 and c["seed"] == 12345
    assert d["intersections_per_step"] == 56746603  # the oracle's count for config 2
    assert d["value"] > 1e9 and d["value_per_gpu"] == d["value"]
    rf = d["roofline"]
    assert 0 < rf["frac"] < 1 and rf["peak"] == 157.3 and rf["achieved"] == pytest.approx(rf["frac"] * rf["peak"])
    assert rf["ops_per_unit_reference_lut"] < rf["ops_per_unit"] and rf["frac_reference_lut"] < rf["frac"]
    assert rf["frac_reference"] == rf["frac"]
    if rf.get("frac_counters") and rf["frac_executed"] is not None:  # a profile of this shape with the FLOP pass
        assert 0 < rf["frac_executed"] < rf["frac_counters"] < 1
    assert d["setup_ms"]["set_scene_repeat_ms"] < d["setup_ms"]["set_scene_ms"] + 1.0
    # the 4D view's frame loop at properties.txt's sizes: overlapped launches against serial ones (bench.py
    # refuses to print a line when their images or counts differ); the speed-up is reported, not asserted
    # (a wall-clock ratio on a shared box)
    sl = d["sections_loop_leg"]
    assert sl["overlapped"]["intersections_per_frame"] == sl["serial"]["intersections_per_frame"] > 0
    assert sl["speedup"] > 0
    # the sustained-clock leg: the same frames after as many frames of load (never the value)
    st = d["steady_clock_leg"]
    assert st["intersections_per_step"] == d["intersections_per_step"] and st["frames"] >= 2 and st["value"] > 1e9
    if rf.get("frac_counters"):
        assert st["frac_counters"] > rf["frac_counters"] * 0.9  # the same work over a time at least as short


def test_bench_strong_config4_one_gpu():
    """Config 4 in strong mode on one GPU: the whole 3840x2160 frame per step, efficiency 1 by definition."""
    d = run_bench("--config", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", timeout=115)
    assert d["scaling"] == "strong" and d["n_gpus"] == 1
    c = d["config"]
    assert (c["scene"], c["width"], c["height"], c["spp"], c["bounces"]) == ("tiger_two_mirrors", 3840, 2160, 64, 12)
    assert d["efficiency"] == pytest.approx(1.0)
    assert d["intersections_per_step"] <= d["nominal_bound_per_step"]


@pytest.mark.parametrize("args", [["--steps", "3", "--warmup", "1"],  # weak, config 2, one gather after the frames
                                  ["--config", "4", "--steps", "1", "--warmup", "0"]])  # strong, T1 leg, gather per frame
def test_bench_two_ranks_rehearsal(args):
    """bench.py --gpus 2 starts two ranks itself (torch.distributed.run) and runs the whole multi-rank
    path: band plan, per-rank regions, padded gather + un-permute on rank 0, max-over-ranks timing, the
    strong-scaling T1 leg. On this one-GPU box both ranks render on GPU 0 and the gather runs over gloo
    (RT4_BENCH_REHEARSE=1); the 8-GPU RCCL run is the driver's."""
    env = dict(os.environ, RT4_BENCH_REHEARSE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu-baseline", "--no-ops",
                        *args], capture_output=True, text=True, timeout=115, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value_per_gpu"] == pytest.approx(d["value"] / 2)
    assert "gloo rehearsal" in d["config"]["parallelism"] and d["gather_ms"] > 0
    if "--config" in args:
        assert d["scaling"] == "strong" and d["t1_ms"] > 0 and 0 < d["efficiency"]
        assert d["config"]["height"] == 2160 and d["config"]["height_per_gpu"] == 1080
    else:
        assert d["scaling"] == "weak" and d["config"]["height"] == 2160
        assert d["intersections_per_step"] > 2 * 5e7  # both ranks' 1920x1080 shares


def test_bench_two_ranks_gather_failure_exits_cleanly():
    """rank 1's part of the gather fails (RT4_GATHER_FAIL_RANK=1, the two-rank rehearsal on
    this box). Rank 1 posts the error to the store and exits; rank 0, waiting in the gather for rank 1's shard,
    exits too (shard.exit_failed). bench.py ends with a non-zero status naming rank 1, no JSON line, no hang."""
    env = dict(os.environ, RT4_BENCH_REHEARSE="1", RT4_GATHER_FAIL_RANK="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-ops", "--no-reuse-leg", "--no-fbf-leg", "--no-sections-leg"],
                       capture_output=True, text=True, timeout=115, cwd=ROOT, env=env)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "rank 1: GatherError: gather failure injected" in r.stderr, r.stderr[-3000:]
    assert '"metric"' not in r.stdout
