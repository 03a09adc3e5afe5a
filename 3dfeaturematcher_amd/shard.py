"""Keypoint sharding over GPUs.

Every stage of the path is independent per query keypoint once frame B's
descriptors and both image pyramids are present on a device, so one frame pair
splits into query blocks, one set per rank, each rank running the whole path on
its device against ALL of frame B:

  * block-cyclic (query_blocks, what bench.py --gpus N runs on C5's 1M-keypoint
    frame pair): blocks of BLOCK queries dealt round-robin, so every rank sees
    the same mix of queries.  The rank uploads its queries gathered into one
    array (queryIdx local), and the merge maps them back to global indices and
    orders the records by query.  Contiguous blocks left C5's last rank a fifth
    of the work of the others: the synthetic frame's last tenth are distractor
    descriptors without a match (profiles/r02_c5_balance_contiguous.json);
  * contiguous (partition): queries [lo_r, hi_r) with queryOffset = lo_r, so
    queryIdx stays global and the rank-order concatenation is already in query
    order.

The per-rank survivor records are all-gathered (count first, then fixed-capacity
64-byte records, all_gather_device) and merged (merge_gathered): either way the
merged list is byte-identical to the single-GPU run.  The collective is
torch.distributed's all_gather (RCCL over xGMI with backend "nccl", or gloo on
CPU for tests); no other exchange is needed.  The reference has no distributed
component to mirror: main.cpp:91-155 runs the three stages in one process.
"""
from __future__ import annotations

import importlib
from typing import Callable

import numpy as np

RECORD_BYTES = 64
BLOCK = 4096  # queries per block of the block-cyclic partition


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


def query_blocks(n: int, world: int, rank: int, block: int = BLOCK) -> np.ndarray:
    """Global indices of `rank`'s queries under the block-cyclic partition: blocks
    rank, rank + world, ... of `block` queries each, in increasing order."""
    if world <= 0 or not 0 <= rank < world or block <= 0:
        raise ValueError(f"bad rank {rank} of {world} (block {block})")
    starts = np.arange(rank * block, n, world * block, dtype=np.int64)
    if len(starts) == 0:
        return np.zeros(0, dtype=np.int64)
    idx = (starts[:, None] + np.arange(block, dtype=np.int64)[None, :]).reshape(-1)
    return idx[idx < n]


def blocks_capacity(n: int, world: int, block: int = BLOCK) -> int:
    """Records per rank buffer under the block-cyclic partition (>= 1)."""
    return max(1, max(len(query_blocks(n, world, r, block)) for r in range(world)))


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


def merge_gathered(gathered, counts, index_maps=None, by_query: bool = False) -> np.ndarray:
    """The valid records of every rank's buffer as the single-device record list.
    index_maps None: queryIdx is already global and the rank-order concatenation is in
    query order (contiguous blocks) -- unless by_query, which orders by queryIdx.
    index_maps[r]: rank r's records carry local query indices into index_maps[r] (the
    block-cyclic partition); they are mapped to global ones and ordered by query."""
    rec_dtype = importlib.import_module("3dfeaturematcher_amd").RECORD
    g, c = _host_gathered(gathered, counts)
    if index_maps is not None and len(index_maps) != g.shape[0]:
        raise ValueError("one index map per rank")
    parts = []
    for r in range(g.shape[0]):
        rec = g[r, : c[r]].reshape(-1).view(rec_dtype).copy()
        if index_maps is not None:
            m = np.asarray(index_maps[r])
            if len(rec) and (rec["queryIdx"].min() < 0 or rec["queryIdx"].max() >= len(m)):
                raise ValueError("a local query index outside the rank's index map")
            rec["queryIdx"] = m[rec["queryIdx"]]
        parts.append(rec)
    out = np.concatenate(parts) if parts else np.zeros(0, dtype=rec_dtype)
    if index_maps is not None or by_query:
        out = out[np.argsort(out["queryIdx"], kind="stable")]
    return out


def _host_gathered(gathered, counts):
    g = np.ascontiguousarray(gathered.cpu().numpy() if hasattr(gathered, "cpu") else gathered, dtype=np.uint8)
    c = np.asarray(counts.cpu().numpy() if hasattr(counts, "cpu") else counts).astype(np.int64).reshape(-1)
    if g.ndim != 3 or g.shape[2] != RECORD_BYTES or len(c) != g.shape[0] or (c < 0).any() or (c > g.shape[1]).any():
        raise ValueError("gathered record buffers of an unexpected shape or count")
    return g, c


def merge_gathered_shares(gathered, counts, n: int, block: int = BLOCK) -> np.ndarray:
    """The block-cyclic merge through the C++ merge of the C ABI (fm3d_merge_shares, the code
    fm3d_mgpu_pipeline_run runs after its RCCL all-gather): rank r's buffer holds its survivor
    records with local query indices of query_blocks(n, world, r, block)."""
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    g, c = _host_gathered(gathered, counts)
    parts = [g[r, : c[r]].reshape(-1).view(fm3d.RECORD) for r in range(g.shape[0])]
    return fm3d.merge_shares(parts, n, block)


def gather_records(records: np.ndarray, capacity: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's survivor records (fm3d RECORD dtype, global queryIdx) and
    merge them in query order.  `capacity` = the largest shard's query count (fixed-size
    buffers)."""
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
    return merge_gathered(gathered, counts, by_query=True)


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


def run_shard_queries(pair, settings, idx: np.ndarray, device: int = 0) -> np.ndarray:
    """The queries idx (global indices, increasing) through the whole path on this rank's
    GPU, uploaded as one gathered array: records with global queryIdx."""
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    idx = np.asarray(idx, dtype=np.int64)
    ctx = fm3d.Context(settings, device=device)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1[idx], pair.desc2, pair.kp1[idx], pair.kp2, pair.img1, pair.img2, query_offset=0)
        n, _ = pipe.run()
        rec = pipe.records(n)
        rec["queryIdx"] = idx[rec["queryIdx"]]
        return rec
    finally:
        ctx.close()


def run_sharded(pair, settings, group=None, device=None,
                shard_fn: Callable[..., np.ndarray] | None = None, block: int = BLOCK) -> np.ndarray:
    """One frame pair split block-cyclically over the ranks of `group`; every rank returns
    the merged records (identical to a single-device run).  `shard_fn(pair, settings, idx)`
    computes the queries idx with global queryIdx; by default the GPU path
    (run_shard_queries)."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n = len(pair.desc1)
    idx = query_blocks(n, world, rank, block)
    fn = shard_fn or (lambda p, s, q: run_shard_queries(p, s, q, device=device.index if device is not None else 0))
    rec = np.ascontiguousarray(fn(pair, settings, idx))
    # local query indices on the wire (as fm3d_mgpu exchanges them); the C++ merge maps them back
    rec["queryIdx"] = np.searchsorted(idx, rec["queryIdx"])
    cap = blocks_capacity(n, world, block)
    buf = np.zeros((cap, RECORD_BYTES), dtype=np.uint8)
    buf[:len(rec)] = rec.view(np.uint8).reshape(len(rec), RECORD_BYTES)
    import torch
    mine = torch.from_numpy(buf)
    if device is not None:
        mine = mine.to(device)
    gathered, counts = all_gather_device(mine, len(rec), group=group)
    return merge_gathered_shares(gathered, counts, n, block)
