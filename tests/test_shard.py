"""Pixel-band sharding (4d_ray_tracing_amd/shard.py) on the CPU: gloo process groups of world size 2 and
3, the CPU oracle as each rank's renderer, one gather to rank 0 -> the assembled frame must equal a
single full render bit for bit (the RNG depends only on the pixel)."""
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


def _worker(rank, world, port, scene_name, out_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    import oracle_lib

    plan = shard.make_plan(width=40, rows_per_rank=16, world=world, band=8)
    scene = rt4.Scene.named(scene_name)
    u = rt4.make_uniforms(plan.width, plan.height, samples=2, reflections=3, seed=31337)
    reg = rt4.region(**plan.region_args(rank))
    frame, n, _, _ = oracle_lib.render(scene.desc, u, reg, threads=2)
    image = shard.gather_frame(torch.from_numpy(frame), plan, rank)
    total = torch.tensor([n], dtype=torch.int64)
    dist.all_reduce(total)
    if rank == 0:
        np.save(os.path.join(out_dir, "image.npy"), image.numpy())
        np.save(os.path.join(out_dir, "n.npy"), total.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_banded_gather_equals_full_frame(tmp_path, world):
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    import oracle_lib

    tmp.spawn(_worker, args=(world, _free_port(), "cylinder4d", str(tmp_path)), nprocs=world, join=True)
    image = np.load(tmp_path / "image.npy")
    n = int(np.load(tmp_path / "n.npy")[0])
    plan = shard.make_plan(width=40, rows_per_rank=16, world=world, band=8)
    u = rt4.make_uniforms(plan.width, plan.height, samples=2, reflections=3, seed=31337)
    full, n_full, _, _ = oracle_lib.render(rt4.Scene.named("cylinder4d").desc, u, rt4.region(plan.width, plan.height))
    assert n == n_full
    assert np.array_equal(image.view(np.uint32), full.view(np.uint32))


def test_plan_rows_partition_the_frame():
    shard = importlib.import_module("4d_ray_tracing_amd.shard")
    for world in (1, 2, 4, 8):
        plan = shard.make_plan(1920, 1080, world)
        rows = sorted(plan.image_row(r, i) for r in range(world) for i in range(plan.rows_per_rank))
        assert rows == list(range(plan.height))
        # the numpy un-permute agrees with image_row()
        tag = np.zeros((world, plan.rows_per_rank, 1, 4), np.int64)
        for r in range(world):
            for i in range(plan.rows_per_rank):
                tag[r, i] = plan.image_row(r, i)
        plan1 = shard.BandPlan(1, plan.rows_per_rank, world, plan.band)
        img = shard.unpermute(tag, plan1)
        assert (img[:, 0, 0] == np.arange(plan.height)).all()
    with pytest.raises(ValueError):
        shard.make_plan(1920, 1081, 2)
