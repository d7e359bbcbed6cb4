"""Data-parallel view sharding across the GPUs of a node (one process per GPU).

The reference is single-device and steps after every view (mtl_engine.mm:1085-1093). Here a
step renders one batch of V views, the views are sharded over the ranks, each rank runs
forward + backward for its views into a packed per-Gaussian gradient buffer (16 live floats,
64 B per Gaussian; include/gs_rasterizer.h gs_backward_packed) and ONE all-reduce (sum) over
RCCL (torch.distributed backend "nccl" on ROCm) combines them over xGMI. Density statistics are
non-linear per view, so each rank accumulates its own views' statistics locally before the
reduce; when densification runs (every 100 steps) the per-rank statistics are
summed once (`reduce_density_statistics`) so every replica applies the same prune/clone/split.
There is no other collective on the data path.

The helpers are backend-agnostic so the same code runs over gloo on the CPU in tests.
"""
from __future__ import annotations


def rank_views(num_views: int, rank: int, world: int) -> list[int]:
    """Views owned by `rank`: a contiguous block, sizes differing by at most one."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(num_views, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def reduce_gradients(packed, group=None) -> None:
    """Sum the packed per-Gaussian gradients of every rank, in place (one all-reduce)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)


def chunk_bounds(n: int, chunks: int) -> list[tuple[int, int]]:
    """[a, b) row ranges splitting n rows into `chunks` near-equal parts (multiples of 256)."""
    chunks = max(1, int(chunks))
    step = -(-n // chunks)
    step = -(-step // 256) * 256 if n > 256 else max(step, 1)
    return [(a, min(a + step, n)) for a in range(0, n, step)] or [(0, 0)]


def pipelined_reduce(packed, chunks: int, compute_chunk, finish_chunk=None, group=None) -> None:
    """The per-Gaussian chain and the gradient all-reduce, overlapped chunk by chunk.

    compute_chunk(a, b) must write rows [a, b) of `packed` (stream-ordered on the current stream);
    each chunk's all-reduce is issued as soon as it is enqueued (async, on the collective's own
    stream, ordered after the chunk), so chunk k is on the wire while chunk k + 1 computes.
    finish_chunk(a, b) is enqueued after chunk k's reduce has completed (a stream wait, not a host
    wait, under RCCL). Same sums as one all-reduce of the whole buffer: the collective reduces
    element-wise, so the split changes nothing in the result."""
    import torch.distributed as dist
    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    bounds = chunk_bounds(packed.shape[0], chunks)
    works = []
    for a, b in bounds:
        compute_chunk(a, b)
        works.append(dist.all_reduce(packed[a:b], op=dist.ReduceOp.SUM, group=group, async_op=True)
                     if distributed and b > a else None)
    for (a, b), w in zip(bounds, works):
        if w is not None:
            w.wait()
        if finish_chunk is not None and b > a:
            finish_chunk(a, b)


def accumulate_views(render_backward, views, packed_out) -> None:
    """packed_out = sum over `views` of render_backward(view, scratch) (per-rank, before reduce).

    render_backward(view, out) must write the packed gradients of one view into `out`."""
    import torch
    if len(views) == 0:
        packed_out.zero_()
        return
    render_backward(views[0], packed_out)
    if len(views) > 1:
        scratch = torch.empty_like(packed_out)
        for v in views[1:]:
            render_backward(v, scratch)
            packed_out.add_(scratch)


def reduce_density_statistics(read, write, group=None) -> None:
    """Sum the density accumulators over ranks before DensityController.apply.

    read() -> (accum f32[n], count i32[n], pos_accum f32[n, 3]) tensors of this rank's views;
    write(accum, count, pos_accum) stores the sums back. Three all-reduces, once per apply."""
    import torch.distributed as dist
    acc, cnt, pos = read()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        for t in (acc, cnt, pos):
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    write(acc, cnt, pos)
