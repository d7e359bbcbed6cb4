"""The bench scripts' own rank launcher (gaussiansplatting_amd/launch.py): `python
bench.py --gpus N` must run N ranks or fail, never one rank that reports N. CPU only: the ranks are
a stand-in script that does what bench.py does with its world (gloo all-reduce, rank 0 prints one
JSON line)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussiansplatting_amd import launch  # noqa: E402

RANK_SCRIPT = textwrap.dedent("""
    import argparse, json, os, sys
    sys.path.insert(0, {root!r})
    from gaussiansplatting_amd import launch
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--fail-rank", type=int, default=-1)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    rc = launch.maybe_spawn(os.path.abspath(__file__), sys.argv[1:], args.gpus)
    if rc is not None:
        sys.exit(rc)
    world = launch.check_world(args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    if rank == args.fail_rank:
        sys.exit(3)
    total = rank
    if world > 1:
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t)
        total = float(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({{"n_gpus": world, "sum": total, "tag": args.tag,
                          "addr": os.environ.get("MASTER_ADDR")}}), flush=True)
""")


def _script(tmp_path):
    p = tmp_path / "rank_script.py"
    p.write_text(RANK_SCRIPT.format(root=ROOT))
    return str(p)


def _clean_env():
    env = dict(os.environ)
    for k in launch.ENV_KEYS:
        env.pop(k, None)
    return env


def test_launch_command_shape():
    cmd = launch.launch_command("/x/bench.py", ["--gpus", "8", "--steps", "5"], 8, 29512, python="py")
    assert cmd == ["py", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                   "--master-addr=127.0.0.1", "--master-port=29512", "/x/bench.py",
                   "--gpus", "8", "--steps", "5"]
    with pytest.raises(ValueError):
        launch.launch_command("s", [], 0, 1)


def test_rank_process_detection_and_world_check():
    assert not launch.is_rank_process({})
    assert launch.is_rank_process({"WORLD_SIZE": "2"})
    assert launch.check_world(1, {}) == 1
    assert launch.check_world(4, {"WORLD_SIZE": "4"}) == 4
    with pytest.raises(SystemExit) as e:
        launch.check_world(8, {"WORLD_SIZE": "1"})
    assert "WORLD_SIZE=1" in str(e.value)
    with pytest.raises(SystemExit):
        launch.check_world(2, {})  # --gpus 2 in a process no launcher started: not a rank
    # a rank process (or N == 1) goes on as itself
    assert launch.maybe_spawn("s", [], 1, env={}) is None
    assert launch.maybe_spawn("s", [], 4, env={"WORLD_SIZE": "4"}) is None


@pytest.mark.timeout(180)
def test_spawns_two_ranks_and_relays_rank0_line(tmp_path):
    r = subprocess.run([sys.executable, _script(tmp_path), "--gpus", "2", "--tag", "x y"],
                       env=_clean_env(), capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line: rank 0's
    d = json.loads(lines[0])
    assert d == {"n_gpus": 2, "sum": 3.0, "tag": "x y", "addr": "127.0.0.1"}


@pytest.mark.timeout(180)
def test_failed_rank_fails_the_launch(tmp_path):
    r = subprocess.run([sys.executable, _script(tmp_path), "--gpus", "2", "--fail-rank", "1"],
                       env=_clean_env(), capture_output=True, text=True, timeout=170)
    assert r.returncode != 0


def test_mismatched_launcher_world_exits_nonzero(tmp_path):
    env = _clean_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, _script(tmp_path), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
    assert not r.stdout.strip()


def test_bench_scripts_use_the_launcher():
    # both bench entry points start their ranks before importing torch (no GPU state in the parent)
    for name in ("bench.py", "bench_configs.py"):
        src = open(os.path.join(ROOT, name)).read()
        body = src[src.index("def main()"):]
        assert body.index("launch.maybe_spawn(") < body.index("import torch")
        assert "launch.check_world(args.gpus)" in body
        assert "warning: --gpus" not in src


def test_stdout_to_stderr_keeps_the_json_line_alone(tmp_path):
    """A native library writing to file descriptor 1 inside the block (RCCL's version banner at
    communicator init) lands on stderr; stdout keeps only what is printed outside it."""
    code = textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        from gaussiansplatting_amd import launch
        with launch.stdout_to_stderr():
            os.write(1, b"RCCL version : banner\\n")
            print("python print inside")
        print('{{"metric": "m"}}')
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines() == ['{"metric": "m"}']
    assert "RCCL version" in r.stderr and "python print inside" in r.stderr
