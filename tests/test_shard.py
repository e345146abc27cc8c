"""Pixel-band sharding (4d_ray_tracing_amd/shard.py) on the CPU: gloo process groups of world size 2,
3 and 8 on frame heights that do not divide evenly (2160 = the 4K frame of BASELINE configs 4/5,
1081 = a short last band), the CPU oracle as each rank's renderer, one padded gather to rank 0 ->
the assembled frame must equal a single full render bit for bit (the RNG depends only on the pixel,
shader.frag:104-108). The same plan drives librt4.so on the GPU
(tests/test_gpu_shard.py, bench.py)."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, scene_name, width, height, out_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    import oracle_lib

    plan = shard.make_plan(width, height=height, world=world, band=8)
    scene = rt4.Scene.named(scene_name)
    u = rt4.make_uniforms(plan.width, plan.height, samples=1, reflections=2, seed=31337)
    reg = rt4.region(**plan.region_args(rank))
    local = np.zeros((plan.rows_max, plan.width, 4), np.float32)  # padded shard: rows past reg.h stay 0
    n = 0
    if reg.h:
        _, n, _, _ = oracle_lib.render(scene.desc, u, reg, frame=local, threads=1)
    image = shard.gather_frame(torch.from_numpy(local), plan, rank)
    total = torch.tensor([n], dtype=torch.int64)
    dist.all_reduce(total)
    if rank == 0:
        np.save(os.path.join(out_dir, "image.npy"), image.numpy())
        np.save(os.path.join(out_dir, "n.npy"), total.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height", [(2, 2160), (3, 1081), (8, 2160), (8, 1081)])
def test_banded_gather_equals_full_frame(tmp_path, world, height):
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    import oracle_lib

    width = 12
    tmp.spawn(_worker, args=(world, _free_port(), "cylinder4d", width, height, str(tmp_path)), nprocs=world, join=True)
    image = np.load(tmp_path / "image.npy")
    n = int(np.load(tmp_path / "n.npy")[0])
    u = rt4.make_uniforms(width, height, samples=1, reflections=2, seed=31337)
    full, n_full, _, _ = oracle_lib.render(rt4.Scene.named("cylinder4d").desc, u, rt4.region(width, height), threads=4)
    assert image.shape == full.shape
    assert n == n_full
    assert np.array_equal(image.view(np.uint32), full.view(np.uint32))


@pytest.mark.parametrize("height", [1, 7, 8, 9, 63, 1080, 1081, 2160, 2161, 4320])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("band", [1, 8, 16])
def test_plan_rows_partition_the_frame(height, world, band):
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    plan = shard.make_plan(1920, height=height, world=world, band=band)
    rows = [plan.rows(r) for r in range(world)]
    assert sum(rows) == height
    assert plan.rows_max == max(1, max(rows))
    # round-robin bands: shares differ by at most one band
    assert max(rows) - min(rows) <= band
    owned = sorted(plan.image_row(r, i) for r in range(world) for i in range(rows[r]))
    assert owned == list(range(height))
    for r in range(world):
        for i in range(rows[r]):
            assert plan.owner(plan.image_row(r, i)) == (r, i)
    # the row index of the padded gather agrees with image_row(), numpy and torch alike
    tag = np.full((world, plan.rows_max, 1, 4), -1, np.int64)
    for r in range(world):
        for i in range(rows[r]):
            tag[r, i] = plan.image_row(r, i)
    img = shard.unpermute(tag, plan)
    assert (img[:, 0, 0] == np.arange(height)).all()
    timg = shard.unpermute(torch.from_numpy(tag), plan)
    assert (timg[:, 0, 0].numpy() == np.arange(height)).all()


def test_4k_over_8_ranks_is_balanced():
    """BASELINE configs 4/5: 3840x2160 over 8 GPUs in 8-row bands -> 270 bands, 6 ranks x 34 + 2 x 33;
    the largest share is 0.7 % above the mean (the bound on strong-scaling efficiency from the split)."""
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    plan = shard.make_plan(3840, height=2160, world=8)
    assert [plan.bands(r) for r in range(8)] == [34] * 6 + [33] * 2
    assert plan.rows_max == 272
    assert plan.rows_max / (2160 / 8) < 1.01


def test_bad_plans_raise():
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    for w, h, n in [(0, 10, 1), (10, 0, 1), (10, 10, 0)]:
        with pytest.raises(ValueError):
            shard.make_plan(w, height=h, world=n)
    with pytest.raises(ValueError):
        shard.make_plan(10, height=10, world=2, band=0)
    # height is keyword-only: round 1's positional (width, rows_per_rank, world) call fails loudly
    with pytest.raises(TypeError):
        shard.make_plan(1920, 1080, 8)


@pytest.mark.parametrize("height", [1, 7, 8, 9, 17, 1080, 1081, 2160, 2161])
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("band", [1, 8, 16])
def test_c_abi_band_plan_equals_shard_py(rt4, height, world, band):
    """rt4_band_plan (the C++ multi-GPU host's plan, librt4.so) is shard.py's arithmetic: the same region
    and rows_max for every rank (host code only, no GPU)."""
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    plan = shard.make_plan(640, height=height, world=world, band=band)
    for rank in range(world):
        reg, rows_max = rt4.band_plan(640, height, world, rank, band=band)
        want = plan.region_args(rank)
        got = dict(w=reg.w, h=reg.h, x0=reg.x0, y0=reg.y0, band_rows=reg.band_rows, band_step=reg.band_step)
        assert got == want, (rank, got, want)
        assert rows_max == plan.rows_max


def test_c_abi_band_plan_rejects_bad_arguments(rt4):
    for args in [(0, 10, 1, 0), (10, 0, 1, 0), (10, 10, 0, 0), (10, 10, 2, 2), (10, 10, 2, -1)]:
        with pytest.raises(rt4.RT4Error):
            rt4.band_plan(*args)
    with pytest.raises(rt4.RT4Error):
        rt4.band_plan(10, 10, 2, 0, band=0)


def _rt4_render(rt4):
    exe = os.path.join(os.path.dirname(rt4.LIB_PATH), "rt4_render")
    if not os.path.exists(exe):
        pytest.skip("lib/rt4_render not built")
    return exe


def test_cpp_host_bands_error_path_exits_cleanly(rt4, tmp_path):
    """rt4_render --gpus N (csrc/rt4_render.cpp render_bands) when a rank's set-up fails: every rank agrees
    on the failure before anything collective runs, skips the gather and the un-permute, and the program
    exits with status 1 naming the failed rank, without hanging and without writing an image.
    Here (no GPU) every rank fails at hipSetDevice; RT4_RENDER_FAIL_RANK makes the outcome the same on a
    machine with a GPU (test_gpu_shard.py runs the injected failure on the MI355X)."""
    import subprocess

    exe = _rt4_render(rt4)
    props = os.path.join(ROOT, "properties.txt")
    pre = str(tmp_path / "bands")
    env = dict(os.environ, RT4_RENDER_FAIL_RANK="1")
    r = subprocess.run([exe, "-p", props, "-s", "sphere", "-n", "2", "-W", "64", "-H", "40", "--gpus", "3",
                        "--rehearse", "-o", pre], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 1, r.stdout + r.stderr
    assert "rank 1" in r.stderr, r.stderr
    assert not os.path.exists(pre + "_yxz.ppm")


def _gather_fail_worker(rank, world, port, out_dir):
    os.environ["RT4_GATHER_FAIL_RANK"] = "1"
    sys.path.insert(0, ROOT)
    # the store lives in the test process, as torchrun's agent hosts it for bench.py's ranks
    store = dist.TCPStore("127.0.0.1", port, world, is_master=False)
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    plan = shard.make_plan(16, height=40, world=world, band=8)
    local = torch.zeros((plan.rows_max, plan.width, 4))

    def log(text):
        with open(os.path.join(out_dir, f"rank{rank}.log"), "w") as f:
            f.write(text)

    try:  # bench.py's gather_once: any failure of the collective ends the rank via shard.exit_failed
        shard.gather_frame(local, plan, rank)
    except Exception as e:  # noqa: BLE001
        shard.exit_failed(rank, f"{type(e).__name__}: {e}", log=log)
    try:  # a non-root rank's gather may complete (its send is done); its next collective then fails
        dist.barrier()
    except Exception as e:  # noqa: BLE001
        shard.exit_failed(rank, f"{type(e).__name__}: {e}", log=log)
    log("gather returned")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_failure_on_one_rank_ends_every_rank(tmp_path, world):
    """VERDICT r04 item 5 (bench.py's gather, shard.gather_frame): rank 1's part of the gather fails
    (RT4_GATHER_FAIL_RANK). It posts the error to the process group's store and exits; the other ranks fail in
    their gather (the root, waiting for rank 1's shard) or in their next collective (a rank whose send completed)
    when its connection closes (gloo), and exit too. Every rank ends with status 1 and names rank 1; none hangs."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _free_port()
    store = dist.TCPStore("127.0.0.1", port, world, is_master=True, wait_for_workers=False)  # noqa: F841
    procs = [ctx.Process(target=_gather_fail_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank hung after the gather failure"
    assert [p.exitcode for p in procs] == [1] * world
    for r in range(world):
        text = (tmp_path / f"rank{r}.log").read_text()
        assert "rank 1: GatherError: gather failure injected" in text, (r, text)


def test_unreachable_store_ends_the_wait(monkeypatch):
    """when the rank that hosts the store has exited after a failure, a peer's gather never completes and
    its store reads raise. wait_or_failure must then report a failure ('store unreachable') instead of polling
    forever; a plain failure() call (report paths) still returns None."""
    shard = importlib.import_module("4d_ray_tracing_amd.shard")

    class GoneStore:
        def check(self, keys):
            raise RuntimeError("Connection reset by peer")

    monkeypatch.setattr(shard, "_store", lambda: GoneStore())
    assert shard.failure() is None
    msg = shard.failure(unreachable_is_failure=True)
    assert msg is not None and msg.startswith("store unreachable") and "Connection reset" in msg

    class Pending:  # a device event that never completes (the gather the dead rank never joins)
        def record(self, stream=None):
            pass

        def query(self):
            return False

    monkeypatch.setattr(torch.cuda, "Event", Pending)
    assert shard.wait_or_failure(check_s=0.001).startswith("store unreachable")
