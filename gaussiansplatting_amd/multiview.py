"""Data-parallel view sharding across the GPUs of a node (one process per GPU).

The reference is single-device and steps after every view (mtl_engine.mm:1085-1093). Here a
step renders one batch of V views, the views are sharded over the ranks, each rank runs
forward + backward for its views into per-Gaussian gradient rows (the 14 live fields a summed
gradient needs, 56 B per Gaussian; include/gs_rasterizer.h GS_GRAD_ROW_FLOATS) and ONE all-reduce
(sum) over RCCL (torch.distributed backend "nccl" on ROCm) combines them over xGMI. Density
statistics are non-linear per view, so each rank accumulates its own views' statistics locally
before the reduce from the per-view screen-space gradient, which therefore
travels in its own per-rank rows (2 floats per Gaussian) and is never reduced; when densification runs (every 100 steps) the per-rank statistics are
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


class CommTimer:
    """How long the step waits on its all-reduces (the exposed, not overlapped, communication).

    Around every chunk's wait in pipelined_reduce a mark is taken: on a GPU two events on the
    current stream (the wait is a stream wait under RCCL, so the gap between them is the time the
    stream stalled on the collective), on the CPU (gloo on host tensors: the wait blocks the host)
    the host clock. `exposed_ms()` sums the gaps of the last step; `steps()` the steps recorded
    since the last reset, `mean_exposed_ms()` their mean. Bytes are the all-reduced buffer's."""

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.reset()

    def reset(self) -> None:
        self._marks = []      # this step's (begin, end) pairs
        self._done = []       # exposed ms of finished steps (resolved lazily on the GPU)
        self.bytes_per_step = 0

    def _now(self):
        if self.cuda:
            import torch
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time
        return time.perf_counter()

    def begin_step(self) -> None:
        if self._marks:
            self._done.append(self._marks)
        self._marks = []
        self.bytes_per_step = 0

    def wait_begin(self):
        return self._now()

    def wait_end(self, begin, nbytes: int) -> None:
        self._marks.append((begin, self._now()))
        self.bytes_per_step += int(nbytes)

    @staticmethod
    def _gap_ms(a, b) -> float:
        return float(a.elapsed_time(b)) if hasattr(a, "elapsed_time") else 1e3 * (b - a)

    def _resolve(self, marks) -> float:
        return sum(self._gap_ms(a, b) for a, b in marks)

    def exposed_ms(self) -> float:
        if self.cuda:
            import torch
            torch.cuda.synchronize()
        return self._resolve(self._marks)

    def steps(self) -> int:
        return len(self._done) + (1 if self._marks else 0)

    def mean_exposed_ms(self) -> float:
        if self.cuda:
            import torch
            torch.cuda.synchronize()
        allm = self._done + ([self._marks] if self._marks else [])
        return sum(self._resolve(m) for m in allm) / max(1, len(allm))


def pipelined_reduce(packed, chunks: int, compute_chunk, finish_chunk=None, group=None,
                     timer: CommTimer | None = None, force: bool = False) -> None:
    """The per-Gaussian chain and the gradient all-reduce, overlapped chunk by chunk.

    compute_chunk(a, b) must write rows [a, b) of `packed` (stream-ordered on the current stream);
    each chunk's all-reduce is issued as soon as it is enqueued (async, on the collective's own
    stream, ordered after the chunk), so chunk k is on the wire while chunk k + 1 computes.
    finish_chunk(a, b) is enqueued after chunk k's reduce has completed (a stream wait, not a host
    wait, under RCCL). Same sums as one all-reduce of the whole buffer: the collective reduces
    element-wise, so the split changes nothing in the result. `timer` (CommTimer) records the time
    spent in each chunk's wait: the communication the chain did not hide. force: issue the
    collectives on a one-rank group too (bench.py --rccl-single-rank: RCCL's calls, stream hand-offs
    and waits exercised on a one-GPU box, where RCCL refuses two ranks on one device)."""
    import torch.distributed as dist
    distributed = dist.is_available() and dist.is_initialized() and (force or dist.get_world_size(group) > 1)
    bounds = chunk_bounds(packed.shape[0], chunks)
    works = []
    for a, b in bounds:
        compute_chunk(a, b)
        works.append(dist.all_reduce(packed[a:b], op=dist.ReduceOp.SUM, group=group, async_op=True)
                     if distributed and b > a else None)
    if timer is not None:
        timer.begin_step()
    for (a, b), w in zip(bounds, works):
        if w is not None:
            t0 = timer.wait_begin() if timer is not None else None
            w.wait()
            if timer is not None:
                timer.wait_end(t0, packed[a:b].numel() * packed.element_size())
        if finish_chunk is not None and b > a:
            finish_chunk(a, b)


def accumulate_views(render_backward, views, rows_out, on_view=None) -> None:
    """rows_out = sum over `views` of the gradient rows of each view (per-rank, before reduce).

    render_backward(view, rows, viewspace) must write the gradient rows of one view into `rows`
    ((N, 14)) and its screen-space gradient into `viewspace` ((N, 2)). on_view(view, rows,
    viewspace), if given, sees each view's own gradients before they are summed: that is where the
    non-linear per-view density statistics are accumulated (DensityController.accumulateGradients,
    density_control.mm:121-185: the norm of each view's screen-space gradient, so Σ|g| over views
    rather than |Σ g|; gs_density_accumulate_rows)."""
    import torch
    if len(views) == 0:
        rows_out.zero_()
        return
    vs = torch.empty((rows_out.shape[0], 2), dtype=rows_out.dtype, device=rows_out.device)
    render_backward(views[0], rows_out, vs)
    if on_view is not None:
        on_view(views[0], rows_out, vs)
    if len(views) > 1:
        scratch = torch.empty_like(rows_out)
        for v in views[1:]:
            render_backward(v, scratch, vs)
            if on_view is not None:
                on_view(v, scratch, vs)
            rows_out.add_(scratch)


class ViewStep:
    """One rank's share of a data-parallel step: forward + backward of one view per rank (the step
    bench.py times, and the GPU tests run through the same object).

      world == 1   compute(): gs_forward + gs_backward (GaussianGradients straight from the chain).
      world >  1   compute(): gs_forward + gs_backward_blend — everything before the collective,
                   capturable in one HIP graph; finish(): per chunk of Gaussians the chain into
                   56-B gradient rows (+ this rank's viewspace rows) and that chunk's all-reduce
                   (async, on the collective's stream), so chunk k is on the wire while chunk
                   k + 1 computes, then each chunk unpacked into GaussianGradients once its reduce
                   has landed (pipelined_reduce): summed gradients next to this rank's own
                   viewspace.

    Density statistics at world > 1: pass `density` (a rasterizer.DensityController). Each chunk's
    statistics are then accumulated from this rank's own rows between the chunk's chain and its
    all-reduce (gs_density_accumulate_rows_range), as density_control.mm:121-185 reads one view's
    gradients. Do NOT accumulate from `grad` after finish(): its position gradient is the sum over
    ranks, so pos_accum would carry every rank's views (and reduce_density_statistics would count
    them world times). At world == 1 `grad` is this view's own gradient and `density` accumulates
    from it after the backward.

    The arguments are the rasterizer (rasterizer.TiledRasterizer), the Gaussians (N, 28) device
    tensor, the view's uniforms (60 floats), the RGBA8 render target and ground truth ((H, W)
    int32), and the outputs: grad (N, 28) and, for world > 1, the rows (N, 14) float32 (the
    viewspace rows are allocated here)."""

    def __init__(self, rast, gaussians, uniforms, out, gt, grad, packed=None, world: int = 1,
                 chunks: int = 4, group=None, density=None, split: bool | None = None):
        import ctypes

        import numpy as np

        from . import _lib
        self.L = _lib.lib()
        self.check = _lib.check
        self.h = rast._h
        self.dg, self.out, self.gt, self.grad, self.packed = gaussians, out, gt, grad, packed
        self.n = int(gaussians.shape[0])
        self.h_px, self.w_px = int(out.shape[0]), int(out.shape[1])
        u = np.ascontiguousarray(np.asarray(uniforms, dtype=np.float32).reshape(-1))
        self.ubuf = (ctypes.c_float * 60).from_buffer_copy(u.tobytes())
        self.world, self.chunks, self.group = world, chunks, group
        # split: the world > 1 shape of the step (blend, then chunked chain + collectives) — also at
        # world 1 when asked (a one-rank RCCL rehearsal: the collectives are issued all the same)
        self.split = world > 1 if split is None else bool(split)
        if self.split and packed is None:
            raise ValueError("world > 1 needs the (N, 14) gradient-row buffer")
        self.viewspace = None
        if self.split:
            import torch
            self.viewspace = torch.empty((self.n, 2), dtype=torch.float32, device=gaussians.device)
        self.timer = None  # a CommTimer, set by the caller to record the exposed all-reduce time
        self.density = density  # a DensityController accumulating this rank's view, or None

    def _stream(self) -> int:
        from .rasterizer import _stream_ptr
        return _stream_ptr(None)

    def compute(self) -> None:
        st, L = self._stream(), self.L
        self.check(L.gs_forward(self.h, st, self.dg.data_ptr(), self.n, self.ubuf, self.w_px, self.h_px,
                                self.out.data_ptr(), None), "gs_forward")
        if not self.split:
            self.check(L.gs_backward(self.h, st, self.dg.data_ptr(), self.grad.data_ptr(), self.n, self.ubuf,
                                     self.out.data_ptr(), self.gt.data_ptr()), "gs_backward")
            if self.density is not None:
                self.density.accumulate_gradients(self.grad, self.n)
        else:
            self.check(L.gs_backward_blend(self.h, st, self.dg.data_ptr(), self.n, self.ubuf,
                                           self.out.data_ptr(), self.gt.data_ptr()), "gs_backward_blend")

    def finish(self) -> None:
        if not self.split:
            return
        L, st = self.L, self._stream()
        packed, grad = self.packed, self.grad

        vs = self.viewspace
        rb = packed.shape[1] * 4  # bytes per gradient row

        def chain(a, b):
            self.check(L.gs_backward_chain(self.h, st, self.dg.data_ptr(), None, packed.data_ptr(), vs.data_ptr(),
                                           self.n, self.ubuf, a, b - a), "gs_backward_chain")
            if self.density is not None:  # this rank's rows, stream-ordered before the chunk's reduce
                self.density.accumulate_rows_range(packed, vs, a, b - a, stream=st)

        def unpack(a, b):
            self.check(L.gs_unpack_gradients(st, packed.data_ptr() + a * rb, vs.data_ptr() + a * 8,
                                             grad.data_ptr() + a * 112, b - a), "gs_unpack_gradients")

        pipelined_reduce(packed, self.chunks, chain, unpack, self.group, self.timer, force=self.world == 1)

    def step(self) -> None:
        self.compute()
        self.finish()


def _staged(group, t) -> bool:
    """gloo moves host tensors: device tensors are staged through host memory (tests, rehearsals)."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _reduce_scatter(out, inp, group=None) -> None:
    import torch.distributed as dist
    if _staged(group, inp):
        o = out.cpu()
        dist.reduce_scatter_tensor(o, inp.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(o)
    else:
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def _all_gather(out, part, group=None) -> None:
    import torch.distributed as dist
    if _staged(group, part):
        o = out.cpu()
        dist.all_gather_into_tensor(o, part.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, part, group=group)


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int, int]:
    """(first, count, shard) of `rank`'s rows when n rows are reduce-scattered over `world` ranks in
    equal shards of `shard` rows (the last ones padded past n)."""
    shard = -(-n // world) if world > 0 else n
    first = min(rank * shard, n)
    return first, max(0, min(shard, n - first)), shard


def sharded_adam_step(adam, gaussians, rows, n: int, lrs, group=None) -> None:
    """The data-parallel optimizer step as reduce-scatter -> Adam on this rank's shard -> all-gather.

    `rows` holds this rank's gradient rows for Gaussians [0, n); after the call `gaussians[:n]`
    holds the updated Gaussians on every rank and the rows past n of either tensor are untouched.
    The same bytes on the wire as one all-reduce of the rows (reduce-scatter + all-gather is what a
    ring all-reduce does), but each rank runs Adam on 1 / world of the Gaussians instead of all of
    them (config 5: 0.78 ms replicated), and each rank's moments are current for its own shard only
    (gather_adam_state before a density apply). The collectives need world equal shards of
    ceil(n / world) rows: when n is not a multiple of world, the rows are staged into a padded
    buffer (the padding rows are reduced and never read) and the gather lands in a temporary."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        adam.step_rows(gaussians, rows[:n], lrs, 0, n)
        return
    rank = dist.get_rank(group)
    first, count, shard = shard_bounds(n, rank, world)
    if rows.shape[0] < n or gaussians.shape[0] < n:
        raise ValueError("sharded_adam_step: rows / gaussians hold fewer than n rows")
    padded = world * shard
    src = rows[:padded]
    if padded > n:  # rows [n, padded) of the caller's buffer are not this step's: reduce zeros
        src = torch.zeros((padded, rows.shape[1]), dtype=rows.dtype, device=rows.device)
        src[:n].copy_(rows[:n])
    mine = torch.empty((shard, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    _reduce_scatter(mine, src, group)
    adam.begin_step()  # one timestep per optimizer step on every rank, whatever its shard
    if count:
        adam.step_rows_range(gaussians, mine[:count], lrs, first, count)
    part = torch.zeros((shard, gaussians.shape[1]), dtype=gaussians.dtype, device=gaussians.device)
    part[:count].copy_(gaussians[first:first + count])
    if padded == n:
        _all_gather(gaussians[:n], part, group)
    else:
        full = torch.empty((padded, gaussians.shape[1]), dtype=gaussians.dtype, device=gaussians.device)
        _all_gather(full, part, group)
        gaussians[:n].copy_(full[:n])


def gather_adam_state(adam, n: int, group=None) -> None:
    """Make every rank's Adam moments current for all n Gaussians after sharded_adam_step (each rank
    stepped its own shard): one all-gather of the 2 x 96-B moment records, once per density apply."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        return
    rank = dist.get_rank(group)
    _, _, shard = shard_bounds(n, rank, world)
    adam.resize_if_needed(world * shard)
    m, v = adam.state_tensors(world * shard)
    for t in (m, v):
        part = t[rank * shard:(rank + 1) * shard].clone()
        _all_gather(t, part, group)
    adam.set_state(m, v, n)


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
