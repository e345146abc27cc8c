"""Pixel-band sharding of one frame over the GPUs of a node.

Every pixel is independent (the RNG depends only on the pixel's scr_coord bits, the seed and its own
call index: shader.frag:104-108), so a frame splits into disjoint pixel sets with no exchange during
rendering. Rows are dealt out in bands of `band` rows, round-robin over ranks, so each rank gets the
same mix of cheap sky rows and expensive object rows. Each rank renders its bands into a contiguous
buffer (rt4_region band layout, include/rt4.h); one gather to the root and a device-side
un-permute assemble the image. The assembled image is bit-identical to a 1-GPU render.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class BandPlan:
    width: int
    rows_per_rank: int
    world: int
    band: int

    @property
    def height(self) -> int:
        return self.rows_per_rank * self.world

    def region_args(self, rank: int) -> dict:
        """Keyword arguments of rt4.region() for `rank` (local row i -> image row, include/rt4.h)."""
        if self.world == 1:
            return dict(w=self.width, h=self.rows_per_rank, x0=0, y0=0, band_rows=0, band_step=0)
        return dict(w=self.width, h=self.rows_per_rank, x0=0, y0=rank * self.band, band_rows=self.band,
                    band_step=self.band * self.world)

    def image_row(self, rank: int, i: int) -> int:
        if self.world == 1:
            return i
        return (i // self.band) * self.band * self.world + rank * self.band + (i % self.band)


def make_plan(width: int, rows_per_rank: int, world: int, band: int = 8) -> BandPlan:
    if world < 1 or rows_per_rank < 1 or width < 1:
        raise ValueError("width, rows_per_rank and world must be positive")
    if world > 1 and rows_per_rank % band:
        raise ValueError(f"rows_per_rank ({rows_per_rank}) must be a multiple of band ({band})")
    return BandPlan(width, rows_per_rank, world, band)


def unpermute(gathered, plan: BandPlan):
    """(world, rows_per_rank, W, 4) gathered shards -> (height, W, 4) image (torch or numpy)."""
    if plan.world == 1:
        return gathered[0]
    nb = plan.rows_per_rank // plan.band
    x = gathered.reshape(plan.world, nb, plan.band, plan.width, 4)
    if hasattr(x, "permute"):  # torch: one device copy
        return x.permute(1, 0, 2, 3, 4).reshape(plan.height, plan.width, 4)
    return x.transpose(1, 0, 2, 3, 4).reshape(plan.height, plan.width, 4)


def gather_frame(local, plan: BandPlan, rank: int, group=None):
    """Gathers every rank's shard to rank 0 (one collective; RCCL over xGMI with the nccl backend)
    and returns the assembled image on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    if plan.world == 1:
        return local
    bufs = [torch.empty_like(local) for _ in range(plan.world)] if rank == 0 else None
    dist.gather(local, gather_list=bufs, dst=0, group=group)
    if rank != 0:
        return None
    return unpermute(torch.stack(bufs), plan)
