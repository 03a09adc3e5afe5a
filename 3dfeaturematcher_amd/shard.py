"""Keypoint sharding over GPUs.

Every stage of the path is independent per query keypoint once frame B's
descriptors and both image pyramids are present on a device, so one frame pair
splits into contiguous query blocks, one per rank:

  rank r takes queries [lo_r, hi_r) of frame A against ALL of frame B, runs the
  whole path on its device (fm3d_pipeline_upload with queryOffset = lo_r, so
  queryIdx stays global), and the per-rank survivor records are all-gathered
  (count first, then fixed-capacity 64-byte records, all_gather_device) and
  concatenated in rank order (merge_gathered).  bench.py --gpus N runs exactly
  this on one 1M-keypoint frame pair (C5) with the record buffers on the GPUs.

Rank order x query order inside a shard == query order, so the merged list is
byte-identical to the single-GPU run.  The collective is torch.distributed's
all_gather (RCCL over xGMI with backend "nccl", or gloo on CPU for tests); no
other exchange is needed.  The reference has no distributed component to
mirror: main.cpp:91-155 runs the three stages in one process.
"""
from __future__ import annotations

import importlib
from typing import Callable

import numpy as np

RECORD_BYTES = 64


def partition(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of n queries for `rank` of `world` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_capacity(n: int, world: int) -> int:
    """Records per rank buffer: the largest block's query count (>= 1)."""
    return max(1, max(hi - lo for lo, hi in (partition(n, world, r) for r in range(world))))


def all_gather_device(rec_buf, n_kept: int, group=None):
    """The collective of one step: every rank's survivor count, then its fixed-capacity
    record buffer (rec_buf: (capacity, 64) uint8 tensor, records [0, n_kept) valid), all-
    gathered with all_gather_into_tensor (RCCL over xGMI for cuda tensors, gloo on CPU).
    Returns (gathered (world, capacity, 64) uint8, counts (world,) int32), on rec_buf's device."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    mine = torch.tensor([n_kept], dtype=torch.int32, device=rec_buf.device)
    counts = torch.empty(world, dtype=torch.int32, device=rec_buf.device)
    dist.all_gather_into_tensor(counts, mine, group=group)
    gathered = torch.empty((world,) + tuple(rec_buf.shape), dtype=torch.uint8, device=rec_buf.device)
    dist.all_gather_into_tensor(gathered.view(-1), rec_buf.reshape(-1), group=group)
    return gathered, counts


def merge_gathered(gathered, counts) -> np.ndarray:
    """Rank-order concatenation of the valid records of every rank's buffer: the single-
    device record list (rank order x query order inside a shard == query order)."""
    rec_dtype = importlib.import_module("3dfeaturematcher_amd").RECORD
    g = np.ascontiguousarray(gathered.cpu().numpy() if hasattr(gathered, "cpu") else gathered, dtype=np.uint8)
    c = np.asarray(counts.cpu().numpy() if hasattr(counts, "cpu") else counts).astype(np.int64)
    cap = g.shape[1]
    if g.ndim != 3 or g.shape[2] != RECORD_BYTES or (c < 0).any() or (c > cap).any():
        raise ValueError("gathered record buffers of an unexpected shape or count")
    parts = [g[r, : c[r]].reshape(-1).view(rec_dtype) for r in range(g.shape[0])]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=rec_dtype)


def gather_records(records: np.ndarray, capacity: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's survivor records (fm3d RECORD dtype) and merge them in
    rank order.  `capacity` = the largest shard's query count (fixed-size buffers)."""
    import torch
    import torch.distributed as dist

    rec_dtype = importlib.import_module("3dfeaturematcher_amd").RECORD
    world = dist.get_world_size(group)
    n = len(records)
    if n > capacity:
        raise ValueError("more records than the shard capacity")
    buf = np.zeros((capacity, RECORD_BYTES), dtype=np.uint8)
    buf[:n] = np.ascontiguousarray(records, dtype=rec_dtype).view(np.uint8).reshape(n, RECORD_BYTES)
    mine = torch.from_numpy(buf)
    if device is not None:
        mine = mine.to(device)
    gathered, counts = all_gather_device(mine, n, group=group)
    return merge_gathered(gathered, counts)


def run_shard(pair, settings, lo: int, hi: int, device: int = 0) -> np.ndarray:
    """This rank's block through the whole path on its GPU (libfm3d.so): records with
    global queryIdx.  Raises Fm3dError when the HIP library or the GPU is missing."""
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    ctx = fm3d.Context(settings, device=device)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1[lo:hi], pair.desc2, pair.kp1[lo:hi], pair.kp2, pair.img1, pair.img2, query_offset=lo)
        n, _ = pipe.run()
        return pipe.records(n)
    finally:
        ctx.close()


def run_sharded(pair, settings, group=None, device=None,
                shard_fn: Callable[..., np.ndarray] | None = None) -> np.ndarray:
    """One frame pair split over the ranks of `group`; every rank returns the merged
    records (identical to a single-device run).  `shard_fn(pair, settings, lo, hi)`
    computes one block; by default the GPU path (run_shard)."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n = len(pair.desc1)
    lo, hi = partition(n, world, rank)
    fn = shard_fn or (lambda p, s, a, b: run_shard(p, s, a, b, device=device.index if device is not None else 0))
    rec = fn(pair, settings, lo, hi)
    return gather_records(rec, shard_capacity(n, world), group=group, device=device)
