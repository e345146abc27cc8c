"""bench.py's host-side logic on the CPU: the BASELINE config presets, the host-CPU report, the row
samples of the CPU-baseline and op-count legs, the executed-op count of the oracle, and the lookup of
the PMC traffic figure (only a profile of the same workload and kernel version counts)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("cfg,scene,w,h,spp,b,fmt,mode,prog,gather", [
    (2, "sphere", 1920, 1080, 16, 8, "f32", "weak", False, "final"),
    (3, "hypercube", 1920, 1080, 16, 8, "f32", "weak", False, "final"),
    (4, "tiger_two_mirrors", 3840, 2160, 64, 12, "f32", "strong", False, "every"),
    (5, "all_primitives", 3840, 2160, 16, 8, "f16", "strong", True, "final"),
])
def test_config_presets(cfg, scene, w, h, spp, b, fmt, mode, prog, gather):
    """BASELINE.json configs[1..4]."""
    a = bench.parse_args(["--config", str(cfg)])
    assert (a.scene, a.width, a.height, a.spp, a.bounces, a.format, a.mode, a.progressive, a.gather) == \
        (scene, w, h, spp, b, fmt, mode, prog, gather)


def test_default_is_config2_and_overrides_win():
    a = bench.parse_args([])
    assert a.config == 2 and a.gpus == 1 and a.mode == "weak" and not a.primary_reuse
    a = bench.parse_args(["--config", "4", "--strong", "--width", "640", "--format", "f16", "--gather", "final"])
    assert (a.width, a.height, a.format, a.gather, a.mode) == (640, 2160, "f16", "final", "strong")
    a = bench.parse_args(["--weak", "--config", "5"])
    assert a.mode == "weak" and a.gather == "final"


def test_host_cpus_respects_the_share(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    c = bench.host_cpus()
    assert c["threads"] == min(3, c["usable"]) and c["nproc"] >= c["usable"] >= 1 and c["model"]
    monkeypatch.delenv("OMP_NUM_THREADS")
    monkeypatch.delenv("RT4_CPU_THREADS", raising=False)
    assert bench.host_cpus()["threads"] == bench.host_cpus()["usable"]


def test_row_region_samples_the_frame(rt4):
    reg, step = bench.row_region(rt4, 1920, 1080, 16, y0_hint=7)
    assert step == 1080 // 16 and reg.band_rows == 1 and reg.band_step == step and reg.w == 1920
    rows = [reg.y0 + i * step for i in range(reg.h)]
    assert rows[0] == 7 % step and rows[-1] < 1080 and len(rows) >= 16
    reg, step = bench.row_region(rt4, 64, 10, 100)  # more rows wanted than the frame has: every row
    assert step == 1 and reg.h == 10


def test_executed_ops_drop_the_newton_loop(rt4):
    """ops_per_unit: the executed count drops the Newton loop's ops (~3.25 iterations of two
    volume_by_w per diffuse bounce) and nothing else, so the gap is a fixed share per diffuse bounce."""
    scene = rt4.Scene.named("sphere")
    u = rt4.make_uniforms(96, 60, samples=2, reflections=3, seed=5)
    opu, opu_exec, n = bench.ops_per_unit(rt4, scene, u, 96, 60, 4)
    assert n > 0 and 0 < opu_exec < opu
    sky = rt4.make_uniforms(96, 60, samples=2, reflections=3, seed=5, fi=0.0, te=80.0)  # looking up: sky only
    opu, opu_exec, _ = bench.ops_per_unit(rt4, scene, sky, 96, 60, 4)
    assert opu_exec == opu  # no hit, no diffuse bounce, no Newton loop


def test_pmc_profile_needs_the_same_workload_kernel_and_shape(tmp_path, monkeypatch):
    prof = tmp_path / "profiles" / "rx"
    prof.mkdir(parents=True)
    cfg = {"scene": "sphere", "width": 1920, "height_per_gpu": 1080, "spp": 16, "bounces": 8, "seed": 12345,
           "sampler_lut": True, "frame_format": "f32", "kernel_version": "r02-test", "progressive": False}
    (prof / "pmc_config2.json").write_text(json.dumps({"config": cfg, "frames_per_dispatch": 20,
                                                       "derived": {"hbm_bytes_per_launch": 123.0}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_profile(dict(cfg), 20)[0]["derived"]["hbm_bytes_per_launch"] == 123.0
    assert bench.pmc_profile(dict(cfg), 5) == (None, None)  # another launch shape
    for k, v in (("kernel_version", "r02-other"), ("spp", 8), ("frame_format", "f16")):
        assert bench.pmc_profile(dict(cfg, **{k: v}), 20) == (None, None)


def test_committed_profiles_cover_every_config_of_the_current_kernel(rt4):
    """The traffic and frac_counters figures of every config's bench line come from a committed profile of
    the kernel version librt4.so reports, taken at the bench's launch shape (profiles/r03_*/pmc_config*.json:
    20 frames per pipelined dispatch, 32 for config 5, or one per dispatch where the scene runs frame by
    frame)."""
    version = rt4.lib.rt4_build_info().decode().split()[2]
    for cfg in (2, 3, 4, 5):
        a = bench.parse_args(["--config", str(cfg)])
        config = {"scene": a.scene, "width": a.width, "height_per_gpu": a.height, "spp": a.spp, "bounces": a.bounces,
                  "seed": a.seed, "sampler_lut": True, "frame_format": a.format, "kernel_version": version,
                  "progressive": bool(a.progressive)}
        found = [bench.pmc_profile(config, f)[0] for f in (1, 20, 32)]
        prof = next((p for p in found if p), None)
        assert prof and prof["derived"].get("hbm_bytes_per_launch", 0) > 0, (cfg, version)
        assert prof["counters"].get("SQ_THREAD_CYCLES_VALU", 0) > 0, (cfg, version)
        # the FLOP pass behind roofline.frac_executed (round 6): executed fp32 FLOPs below the lane-ops
        c = prof["counters"]
        assert c.get("SQ_INSTS_VALU_FLOPS_FP32", 0) > 0, (cfg, version)
        assert 0 < c["SQ_INSTS_VALU_FLOPS_FP32"] < 2 * c["SQ_INSTS_VALU"], (cfg, version)


def test_gather_ceiling_is_the_committed_probe():
    """roofline.gather_rate_frac divides by the measured 32 MiB random-gather ceiling (profiles/r03_mall)."""
    assert abs(bench.gather_ceiling() - 65.69e9) < 1e6


def test_bench_gives_its_process_eight_hardware_queues():
    """bench.py sets GPU_MAX_HW_QUEUES for its own process before the HIP runtime starts (the overlapped small
    frames' 8 side streams); --hw-queues 0 keeps the environment's value."""
    assert bench.parse_args([]).hw_queues == 8
    assert bench.parse_args(["--hw-queues", "0"]).hw_queues == 0
    src = open(bench.__file__).read()
    main = src[src.index("def main():"):]
    assert main.index('os.environ["GPU_MAX_HW_QUEUES"]') < main.index("import torch")
