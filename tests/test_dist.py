"""Multi-process (world_size 2, gloo, CPU) test of the view-sharded data-parallel path: each rank
computes its views' gradient rows, one all-reduce sums them; the result equals the sum over all
views computed in one process. Per-view gradients come from the CPU oracle here (the HIP path is
covered by the GPU tests); what is under test is the sharding + packing + reduction plumbing."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gaussiansplatting_amd import multiview, scene

W, H, N, SEED, VIEWS = 48, 40, 400, 5, 5
# gradient rows (include/gs_rasterizer.h GS_GRAD_ROW_FLOATS) <- GaussianGradients float offsets
PACK = scene.ROW_FIELDS
ROWS = scene.ROW_FLOATS


def _view_grads(view: int) -> np.ndarray:
    from oracle import oracle
    g = scene.synthetic_gaussians(N, SEED, W, H)
    u = scene.rig_uniforms(view, W, H)
    gt = scene.synthetic_ground_truth(SEED, view, W, H)
    f = oracle.forward(g, u, W, H, threads=1)
    gr, _, _ = oracle.backward(g, f, f.rgba8, gt, threads=1)
    return gr.astype(np.float32)


def _view_packed(view: int) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(_view_grads(view)[:, PACK]))


def _view_vs(view: int) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(_view_grads(view)[:, scene.VIEWSPACE_FIELDS]))


def _density_stats(views):
    """DensityController.accumulateGradients over `views` (oracle), as torch tensors."""
    from oracle import oracle
    acc = np.zeros(N, np.float32)
    cnt = np.zeros(N, np.uint32)
    pos = np.zeros((N, 3), np.float32)
    for v in views:
        oracle.density_accumulate(_view_grads(v), acc, cnt, pos)
    return torch.from_numpy(acc), torch.from_numpy(cnt.view(np.int32)), torch.from_numpy(pos)


def _apply(acc, cnt):
    from oracle import oracle
    g = scene.synthetic_gaussians(N, SEED, W, H)
    out, _, _ = oracle.density_apply(g, acc.numpy(), cnt.numpy().view(np.uint32), 600, 2.0,
                                     float(W), float(W), 6.0, seed=600)
    return out


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    views = multiview.rank_views(VIEWS, rank, world)
    packed = torch.empty((N, ROWS), dtype=torch.float32)

    def render_backward(v, out, vs):
        out.copy_(_view_packed(v))

    multiview.accumulate_views(render_backward, views, packed)
    multiview.reduce_gradients(packed)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), packed.numpy())
    # density statistics: per-rank accumulation of its own views, one reduce before apply
    stats = {}
    multiview.reduce_density_statistics(lambda: _density_stats(views),
                                        lambda a, c, p: stats.update(acc=a, cnt=c, pos=p))
    np.save(os.path.join(out_dir, f"acc{rank}.npy"), stats["acc"].numpy())
    np.save(os.path.join(out_dir, f"cnt{rank}.npy"), stats["cnt"].numpy())
    np.save(os.path.join(out_dir, f"dens{rank}.npy"), _apply(stats["acc"], stats["cnt"]))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_views_partition():
    for v in (1, 5, 8, 13):
        for world in (1, 2, 3, 8):
            got = [multiview.rank_views(v, r, world) for r in range(world)]
            flat = [x for part in got for x in part]
            assert flat == list(range(v))
            sizes = [len(p) for p in got]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_allreduce(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    want = sum(_view_packed(v) for v in range(VIEWS)).numpy()
    for r in range(2):
        got = np.load(tmp_path / f"rank{r}.npy")
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
    # both ranks hold bit-identical replicas after the reduce
    assert np.array_equal(np.load(tmp_path / "rank0.npy").view(np.uint32),
                          np.load(tmp_path / "rank1.npy").view(np.uint32))


def test_two_rank_density_statistics(tmp_path):
    """Each rank accumulates its own views' density statistics; one reduce makes them the sum over
    all views, and both replicas then densify to bit-identical Gaussians."""
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    acc, cnt, _ = _density_stats(range(VIEWS))
    for r in range(2):
        np.testing.assert_allclose(np.load(tmp_path / f"acc{r}.npy"), acc.numpy(), rtol=1e-5, atol=1e-7)
        assert np.array_equal(np.load(tmp_path / f"cnt{r}.npy"), cnt.numpy())
    d0, d1 = np.load(tmp_path / "dens0.npy"), np.load(tmp_path / "dens1.npy")
    assert d0.shape == d1.shape and np.array_equal(d0.view(np.uint32), d1.view(np.uint32))


def _pipelined_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    views = multiview.rank_views(VIEWS, rank, world)
    full = torch.zeros((N, ROWS), dtype=torch.float32)
    for v in views:
        full += _view_packed(v)
    packed = torch.full((N, ROWS), float("nan"), dtype=torch.float32)
    finished = torch.zeros(N, dtype=torch.int32)
    order = []

    def compute_chunk(a, b):  # the chain of rows [a, b) (here: copy this rank's sums)
        order.append((a, b))
        packed[a:b] = full[a:b]

    def finish_chunk(a, b):  # the unpack of rows [a, b), after their reduce
        finished[a:b] += 1

    multiview.pipelined_reduce(packed, 3, compute_chunk, finish_chunk)
    np.save(os.path.join(out_dir, f"pipe{rank}.npy"), packed.numpy())
    np.save(os.path.join(out_dir, f"fin{rank}.npy"), finished.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _one_rank_forced_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    issued = []
    real = dist.all_reduce

    def counting_all_reduce(t, *a, **k):  # the collectives pipelined_reduce issues
        issued.append(int(t.shape[0]))
        return real(t, *a, **k)

    dist.all_reduce = counting_all_reduce
    try:
        packed = torch.zeros((N, ROWS), dtype=torch.float32)
        want = _view_packed(0)

        def compute_chunk(a, b):
            packed[a:b] = want[a:b]

        multiview.pipelined_reduce(packed, 3, compute_chunk, None)  # one rank: nothing issued
        plain = list(issued)
        multiview.pipelined_reduce(packed, 3, compute_chunk, None, force=True)  # the rehearsal
        np.save(os.path.join(out_dir, "issued.npy"), np.array([len(plain), len(issued) - len(plain),
                                                                sum(issued)], dtype=np.int64))
        np.save(os.path.join(out_dir, "forced.npy"), packed.numpy())
    finally:
        dist.all_reduce = real
    dist.destroy_process_group()


def test_one_rank_forced_collectives(tmp_path):
    """bench.py --rccl-single-rank: the N > 1 step shape on a group of one issues every chunk's
    all-reduce (a one-rank sum: the rows unchanged); without force a one-rank group issues none."""
    mp.spawn(_one_rank_forced_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    plain, forced, rows = np.load(tmp_path / "issued.npy")
    assert plain == 0 and forced == len(multiview.chunk_bounds(N, 3)) and rows == N
    assert np.array_equal(np.load(tmp_path / "forced.npy"), _view_packed(0).numpy())


def test_chunk_bounds_cover():
    for n in (0, 1, 255, 256, 1000, 1_000_000):
        for k in (1, 2, 3, 4, 8):
            b = multiview.chunk_bounds(n, k)
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
            assert len(b) <= max(k, 1)


def test_two_rank_pipelined_reduce(tmp_path):
    """Chunked chain + per-chunk all-reduce (the N > 1 bench path) == one all-reduce of the whole
    buffer, and every row is finished exactly once after its reduce."""
    port = _free_port()
    mp.spawn(_pipelined_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    want = sum(_view_packed(v) for v in range(VIEWS)).numpy()
    for r in range(2):
        np.testing.assert_allclose(np.load(tmp_path / f"pipe{r}.npy"), want, rtol=1e-5, atol=1e-6)
        assert np.all(np.load(tmp_path / f"fin{r}.npy") == 1)
    assert np.array_equal(np.load(tmp_path / "pipe0.npy").view(np.uint32),
                          np.load(tmp_path / "pipe1.npy").view(np.uint32))


def _on_view_worker(rank, world, port, out_dir):
    """Two views per rank; the density statistics are accumulated per view inside
    accumulate_views' on_view callback (the INTEGRATION.md section 4 pattern)."""
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    views = multiview.rank_views(4, rank, world)
    assert len(views) == 2
    packed = torch.empty((N, ROWS), dtype=torch.float32)
    acc = np.zeros(N, np.float32)
    cnt = np.zeros(N, np.uint32)
    pos = np.zeros((N, 3), np.float32)
    seen = []

    def render_backward(v, out, vs):
        out.copy_(_view_packed(v))
        vs.copy_(_view_vs(v))

    def on_view(v, buf, vs):  # view v's own gradient rows and viewspace, before they are summed
        seen.append(v)
        full = np.zeros((N, 28), np.float32)
        full[:, PACK] = buf.numpy()
        full[:, scene.VIEWSPACE_FIELDS] = vs.numpy()
        oracle.density_accumulate(full, acc, cnt, pos)

    multiview.accumulate_views(render_backward, views, packed, on_view=on_view)
    np.save(os.path.join(out_dir, f"local_acc{rank}.npy"), acc)
    multiview.reduce_gradients(packed)
    stats = {}
    multiview.reduce_density_statistics(
        lambda: (torch.from_numpy(acc), torch.from_numpy(cnt.view(np.int32)), torch.from_numpy(pos)),
        lambda a, c, p: stats.update(acc=a, cnt=c))
    np.save(os.path.join(out_dir, f"seen{rank}.npy"), np.array(seen))
    np.save(os.path.join(out_dir, f"acc{rank}.npy"), stats["acc"].numpy())
    np.save(os.path.join(out_dir, f"cnt{rank}.npy"), stats["cnt"].numpy())
    np.save(os.path.join(out_dir, f"grad{rank}.npy"), packed.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_on_view_density_statistics(tmp_path):
    """accumulate_views(on_view=...) with two views per rank: the local statistics equal the
    per-view accumulation over the rank's own views bit for bit, the reduced statistics equal the
    per-view sum over all four views (sum of per-view norms, not the norm of the summed gradient),
    and the gradients are the sum over views."""
    port = _free_port()
    mp.spawn(_on_view_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        own = multiview.rank_views(4, r, 2)
        assert np.load(tmp_path / f"seen{r}.npy").tolist() == own
        la, _, _ = _density_stats(own)
        assert np.array_equal(np.load(tmp_path / f"local_acc{r}.npy").view(np.uint32), la.numpy().view(np.uint32))
    acc, cnt, _ = _density_stats(range(4))
    summed = sum(_view_packed(v) for v in range(4)).numpy()
    vs_sum = sum(_view_vs(v) for v in range(4)).numpy()
    norm_of_sum = np.hypot(vs_sum[:, 0], vs_sum[:, 1])
    for r in range(2):
        got = np.load(tmp_path / f"acc{r}.npy")
        np.testing.assert_allclose(got, acc.numpy(), rtol=1e-6, atol=1e-9)
        assert np.array_equal(np.load(tmp_path / f"cnt{r}.npy"), cnt.numpy())
        np.testing.assert_allclose(np.load(tmp_path / f"grad{r}.npy"), summed, rtol=1e-5, atol=1e-6)
    live = cnt.numpy() > 1
    assert live.any() and np.any(np.abs(acc.numpy()[live] - norm_of_sum[live]) > 1e-3 * acc.numpy()[live])


def _timed_worker(rank, world, port, out_dir):
    import json
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    packed = torch.full((N, ROWS), 1.0 + rank, dtype=torch.float32)
    timer = multiview.CommTimer(cuda=False)

    def compute_chunk(a, b):
        packed[a:b] = 1.0 + rank

    for _ in range(3):
        multiview.pipelined_reduce(packed, 2, compute_chunk, None, timer=timer)
    res = {"steps": timer.steps(), "exposed": timer.mean_exposed_ms(), "bytes": timer.bytes_per_step,
           "sum_ok": bool(torch.all(packed == 3.0))}
    with open(os.path.join(out_dir, f"timer{rank}.json"), "w") as fh:
        json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_comm_timer_and_bench_fields(tmp_path):
    """The N > 1 bench line's communication record: multiview.CommTimer measures the exposed wait
    of every chunk's all-reduce (gloo on host tensors here: a host wait), bytes per step are the
    packed buffer's, and bench.comm_fields derives the algorithm and ring bus bandwidths."""
    import json
    import sys
    port = _free_port()
    mp.spawn(_timed_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = json.load(open(tmp_path / f"timer{r}.json"))
        assert d["steps"] == 3 and d["exposed"] >= 0.0 and d["sum_ok"]
        assert d["bytes"] == N * ROWS * 4
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    c = bench.comm_fields(2, 64_000_000, 0.25, 1.0, 4, "gloo")
    for k in ("allreduce_exposed_ms", "allreduce_standalone_ms", "algo_gbs", "bus_gbs", "bytes_per_step"):
        assert k in c
    assert abs(c["algo_gbs"] - 64.0) < 1e-9 and abs(c["bus_gbs"] - 64.0) < 1e-9  # 2 (n-1)/n = 1 at n = 2
    assert abs(bench.comm_fields(8, 64_000_000, 0.0, 1.0, 4, "nccl")["bus_gbs"] - 112.0) < 1e-9


class _MockAdam:
    """Stands in for rasterizer.AdamOptimizer on the CPU: an elementwise moment update per row field
    (m = 0.5 m + row, g -= 0.01 m) with the same step_rows / state_tensors / set_state / resize
    interface, so the sharded step's plumbing is checked against the replicated one exactly."""

    def __init__(self, n):
        self.m = torch.zeros((n, 24), dtype=torch.float32)
        self.v = torch.zeros((n, 24), dtype=torch.float32)
        self.t = 0

    def step_rows(self, g, rows, lrs, first, count):
        self.begin_step()
        self.step_rows_range(g, rows, lrs, first, count)

    def begin_step(self):
        self.t += 1

    def step_rows_range(self, g, rows, lrs, first, count):
        cols = torch.tensor(scene.ROW_FIELDS[:11])  # position .. rotation: moment lanes == gradient offsets
        for k in range(count):
            i = first + k
            self.m[i, cols] = 0.5 * self.m[i, cols] + rows[k, :11]
            self.v[i, cols] = self.v[i, cols] + rows[k, :11] * rows[k, :11]
            g[i, :3] -= 0.01 * self.m[i, :3]

    def resize_if_needed(self, n):
        if n > self.m.shape[0]:
            self.m = torch.cat([self.m, torch.zeros((n - self.m.shape[0], 24))])
            self.v = torch.cat([self.v, torch.zeros((n - self.v.shape[0], 24))])

    def state_tensors(self, n):
        return self.m[:n].clone(), self.v[:n].clone()

    def set_state(self, m, v, n):
        self.m[:n] = m[:n]
        self.v[:n] = v[:n]


def _sharded_worker(rank, world, port, out_dir, n):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g0 = torch.from_numpy(scene.synthetic_gaussians(n + 3, SEED, W, H))
    rng = np.random.default_rng(100 + rank)
    ga, gb = g0.clone(), g0.clone()
    gc = g0[:n].clone()  # exactly n rows: no capacity past the live Gaussians
    tail = torch.full((3, 28), float(rank + 7))
    gb[n:] = tail  # rows past n belong to the caller: never written
    a_rep, a_sh, a_ex = _MockAdam(n), _MockAdam(n), _MockAdam(n)
    for step in range(3):
        rows = torch.from_numpy(rng.standard_normal((n, ROWS)).astype(np.float32))
        # replicated: all-reduce + every Gaussian's step on every rank
        r_all = rows.clone()
        multiview.reduce_gradients(r_all[:n])
        a_rep.step_rows(ga, r_all[:n], None, 0, n)
        # sharded: reduce-scatter + this rank's shard + all-gather of the Gaussians
        multiview.sharded_adam_step(a_sh, gb, rows.clone(), n, None)
        multiview.sharded_adam_step(a_ex, gc, rows.clone(), n, None)
    assert torch.equal(gb[n:], tail)
    assert torch.equal(gb[:n], gc)
    multiview.gather_adam_state(a_sh, n)
    np.save(os.path.join(out_dir, f"ga{rank}.npy"), ga[:n].numpy())
    np.save(os.path.join(out_dir, f"gb{rank}.npy"), gb[:n].numpy())
    np.save(os.path.join(out_dir, f"ma{rank}.npy"), a_rep.m[:n].numpy())
    np.save(os.path.join(out_dir, f"mb{rank}.npy"), a_sh.m[:n].numpy())
    np.save(os.path.join(out_dir, f"t{rank}.npy"), np.array([a_rep.t, a_sh.t]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [400, 401])
def test_two_rank_sharded_adam_equals_replicated(tmp_path, n):
    """reduce-scatter -> Adam on the rank's shard -> all-gather (bench_configs --sharded-adam) gives
    every rank the Gaussians the replicated all-reduce + full Adam gives, bit for bit at two ranks
    (a sum of two floats has one rounding whatever the order), and gather_adam_state the full
    moments; n not a multiple of the world size pads the last shard, exactly-sized (n, 28) and
    (n, 14) buffers work, and the rows of the Gaussian buffer past n are never written."""
    port = _free_port()
    mp.spawn(_sharded_worker, args=(2, port, str(tmp_path), n), nprocs=2, join=True)
    for r in range(2):
        for a, b in (("ga", "gb"), ("ma", "mb")):
            x, y = np.load(tmp_path / f"{a}{r}.npy"), np.load(tmp_path / f"{b}{r}.npy")
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (a, b, r)
        assert np.load(tmp_path / f"t{r}.npy").tolist() == [3, 3]
    assert np.array_equal(np.load(tmp_path / "gb0.npy").view(np.uint32), np.load(tmp_path / "gb1.npy").view(np.uint32))


def test_shard_bounds():
    for n in (0, 1, 7, 400, 401, 1_000_003):
        for world in (1, 2, 3, 8):
            parts = [multiview.shard_bounds(n, r, world) for r in range(world)]
            assert sum(c for _, c, _ in parts) == n
            assert all(f == min(r * parts[0][2], n) for r, (f, _, _) in enumerate(parts))
