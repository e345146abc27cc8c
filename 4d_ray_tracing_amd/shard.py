"""Pixel-band sharding of one frame over the GPUs of a node.

Every pixel is independent (the RNG depends only on the pixel's scr_coord bits, the seed and its own
call index: shader.frag:104-108; the whole texture is one draw: src/windows/windows.cpp:45), so a
frame splits into disjoint pixel sets with no exchange during rendering. Rows are dealt out in bands
of `band` rows, round-robin over ranks, so each rank gets the same mix of cheap sky rows and
expensive object rows. Any frame height splits over any number of ranks: the last band of the frame
may be short, ranks may own one band more than others (or none), and the gather pads every shard to
the largest one. Each rank renders its bands into a contiguous buffer (rt4_region band layout,
include/rt4.h); one gather to the root and one device-side row index assemble the image, which is
bit-identical to a 1-GPU render.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class BandPlan:
    width: int
    height: int  # rows of the whole frame
    world: int
    band: int

    @property
    def n_bands(self) -> int:
        return -(-self.height // self.band)

    def bands(self, rank: int) -> int:
        """Bands owned by `rank`: r, r + world, r + 2 world, ... below n_bands."""
        nb = self.n_bands
        return 0 if rank >= nb else (nb - rank + self.world - 1) // self.world

    def rows(self, rank: int) -> int:
        """Image rows owned by `rank` (its region height)."""
        k = self.bands(rank)
        if k == 0:
            return 0
        short = self.n_bands * self.band - self.height  # the frame's last band is this many rows short
        return k * self.band - (short if (self.n_bands - 1) % self.world == rank else 0)

    @property
    def rows_max(self) -> int:
        """Rows of the largest shard: every rank's buffer (and the gather) has this many rows."""
        return max(1, max(self.rows(r) for r in range(self.world)))

    def region_args(self, rank: int) -> dict:
        """Keyword arguments of rt4.region() for `rank` (local row i -> image row, include/rt4.h)."""
        if self.world == 1:
            return dict(w=self.width, h=self.height, x0=0, y0=0, band_rows=0, band_step=0)
        return dict(w=self.width, h=self.rows(rank), x0=0, y0=rank * self.band, band_rows=self.band,
                    band_step=self.band * self.world)

    def image_row(self, rank: int, i: int) -> int:
        if self.world == 1:
            return i
        return (i // self.band) * self.band * self.world + rank * self.band + (i % self.band)

    def owner(self, y: int) -> tuple[int, int]:
        """(rank, local row) of image row y."""
        b = y // self.band
        return b % self.world, (b // self.world) * self.band + y % self.band

    def gather_index(self):
        """numpy int64 (height,): image row y -> row of the flattened (world * rows_max) gather."""
        import numpy as np

        y = np.arange(self.height, dtype=np.int64)
        b = y // self.band
        return (b % self.world) * self.rows_max + (b // self.world) * self.band + y % self.band


def make_plan(width: int, *, height: int, world: int, band: int = 8) -> BandPlan:
    """Plan for a width x height frame over `world` ranks in bands of `band` rows. Any height >= 1
    works; a rank gets no rows when world exceeds the band count. `height` is the WHOLE frame's rows
    and keyword-only (round 1's make_plan took rows per rank there: an old positional call now fails
    instead of silently planning an N-times-smaller frame)."""
    if world < 1 or height < 1 or width < 1 or band < 1:
        raise ValueError("width, height, world and band must be positive")
    return BandPlan(width, height, world, band)


def weak_plan(width: int, *, rows_per_rank: int, world: int, band: int = 8) -> BandPlan:
    """Weak scaling: a frame of rows_per_rank * world rows, every rank the same number of rows when
    rows_per_rank is a multiple of band (otherwise the round-robin deal differs by at most one band)."""
    return make_plan(width, height=rows_per_rank * world, world=world, band=band)


def unpermute(gathered, plan: BandPlan):
    """(world, rows_max, W, C) gathered shards -> (height, W, C) image (torch or numpy): one row gather."""
    if plan.world == 1:
        return gathered[0][: plan.height]
    flat = gathered.reshape((plan.world * plan.rows_max,) + tuple(gathered.shape[2:]))
    if hasattr(flat, "index_select"):  # torch: one device copy, the row index uploaded once per plan and device
        return flat.index_select(0, _device_index(plan, flat.device))
    return flat[plan.gather_index()]


_INDEX_CACHE = {}
_RECV_CACHE = {}


def _device_index(plan: BandPlan, device):
    import torch

    key = (plan.width, plan.height, plan.world, plan.band, str(device))
    if key not in _INDEX_CACHE:
        _INDEX_CACHE[key] = torch.from_numpy(plan.gather_index()).to(device)
    return _INDEX_CACHE[key]


def gather_frame(local, plan: BandPlan, rank: int, group=None):
    """Gathers every rank's shard (rows_max rows each; rows past the rank's own are padding) to rank 0
    in one collective (RCCL over xGMI with the nccl backend) and returns the assembled image on rank
    0, None elsewhere."""
    import torch
    import torch.distributed as dist

    if plan.world == 1:
        return local
    if local.shape[0] != plan.rows_max:
        raise ValueError(f"shard has {local.shape[0]} rows, the plan gathers {plan.rows_max}")
    recv = None
    if rank == 0:  # one (world, rows_max, W, C) receive buffer, kept: the shards land in it without a stack copy
        key = (plan.world,) + tuple(local.shape) + (local.dtype, str(local.device))
        recv = _RECV_CACHE.get(key)
        if recv is None:
            recv = _RECV_CACHE[key] = torch.empty((plan.world,) + tuple(local.shape), dtype=local.dtype,
                                                  device=local.device)
    fail = os.environ.get("RT4_GATHER_FAIL_RANK")  # test hook: this rank's part of the gather fails
    if fail is not None and int(fail) == rank:
        raise GatherError(f"gather failure injected (RT4_GATHER_FAIL_RANK={rank})")
    dist.gather(local, gather_list=list(recv.unbind(0)) if recv is not None else None, dst=0, group=group)
    if rank != 0:
        return None
    return unpermute(recv, plan)


# ---- failure handling of the gather ------------------------------------------------------
# A rank whose part of a collective fails leaves its peers waiting inside theirs (RCCL: their gather kernels wait
# for its data; gloo: their receives). The failing rank posts its error to the process group's key-value store
# and exits; a peer learns of it either from its own collective failing (gloo sees the closed connection) or, on
# RCCL, while it waits for its stream with wait_or_failure, which polls the store instead of blocking, and then
# exits too. Every rank ends with status 1 and a message naming the failed rank, none hangs.
FAIL_KEY = "rt4/gather_failed"


class GatherError(RuntimeError):
    pass


def _store():
    try:
        import torch.distributed.distributed_c10d as c10d

        return c10d._get_default_store()
    except Exception:  # no process group, or a launcher without a store
        return None


def report_failure(rank: int, msg: str) -> None:
    """Posts `rank: msg` to the store (the first report is kept)."""
    st = _store()
    if st is not None:
        try:
            st.compare_set(FAIL_KEY, "", f"rank {rank}: {msg}")
        except Exception:
            pass


def failure(unreachable_is_failure: bool = False) -> str | None:
    """The failure a rank reported, or None. With unreachable_is_failure, a store that no longer answers is reported
    as a failure too: when the rank that hosts the store (rank 0 under plain env:// init, without torchrun's agent)
    has exited after a failure, its peers' gathers never complete and nothing else would end their wait."""
    st = _store()
    try:
        if st is not None and st.check([FAIL_KEY]):
            return st.get(FAIL_KEY).decode()
    except Exception as e:
        if unreachable_is_failure:
            return f"store unreachable ({type(e).__name__}: {e})"
    return None


def wait_or_failure(stream=None, check_s: float = 0.01) -> str | None:
    """Waits on the host for the work enqueued so far on `stream` (the gathers included), checking the store every
    check_s: None when the work completed, a failed rank's report when one arrived first (that rank's collective
    will never complete). The completion itself is polled without sleeping, so a timed region that ends with this
    wait ends within microseconds of the device work (the store's round trips only every check_s)."""
    import time

    import torch

    ev = torch.cuda.Event()
    ev.record(stream)
    next_check = time.perf_counter() + check_s
    while not ev.query():
        now = time.perf_counter()
        if now >= next_check:
            f = failure(unreachable_is_failure=True)
            if f is not None:
                return f
            next_check = now + check_s
    return None


def exit_failed(rank: int, msg: str, log=None) -> None:
    """Reports this rank's failure (or the one another rank reported first) and ends the process with status 1
    without waiting for collectives that will never complete (os._exit: no interpreter shutdown, which would
    join the process group's pending work)."""
    import sys

    report_failure(rank, msg)
    first = failure() or f"rank {rank}: {msg}"
    text = f"rank {rank}: stopping, the gather failed: {first}"
    (log or (lambda t: print(t, file=sys.stderr, flush=True)))(text)
    os._exit(1)
