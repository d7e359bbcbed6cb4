"""One process per GPU for the bench scripts.

`python bench.py --gpus N` on a node must run N ranks, not one: when no launcher has set
WORLD_SIZE, `spawn_ranks` starts `torch.distributed.run` with N processes on this script (rendezvous
on 127.0.0.1, a free port), lets the ranks' stdout through (rank 0 prints the JSON line) and
returns the launcher's exit status, which is non-zero when any rank failed. The parent never
initialises the GPU: it only builds a command line and waits, so no HIP state exists in the
process that starts the ranks.

When a launcher did set WORLD_SIZE, `check_world` refuses a mismatch with `--gpus` instead of
silently running a different number of ranks than the line would claim.

The reference has no multi-device path (`mtl_engine.mm:177`, one `MTL::Device`); its per-view
loop (`mtl_engine.mm:1085-1093`) is what the view sharding replaces.
"""
from __future__ import annotations

import contextlib
import os
import socket
import subprocess
import sys

ENV_KEYS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return int(s.getsockname()[1])


@contextlib.contextmanager
def stdout_to_stderr():
    """File descriptor 1 points at stderr inside the block, output of native libraries included:
    RCCL prints its version banner on stdout when a communicator comes up, and the bench scripts'
    stdout carries only their JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def is_rank_process(env=None) -> bool:
    """True inside a process a launcher started (torchrun sets WORLD_SIZE for every rank)."""
    env = os.environ if env is None else env
    return "WORLD_SIZE" in env


def launch_command(script: str, argv: list[str], nproc: int, port: int,
                   python: str | None = None) -> list[str]:
    """The torch.distributed.run command line that runs `script argv` as `nproc` local ranks."""
    if nproc < 1:
        raise ValueError(f"nproc must be >= 1, got {nproc}")
    return [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={port}",
            script, *argv]


def spawn_ranks(script: str, argv: list[str], nproc: int, timeout: float | None = None,
                env: dict | None = None) -> int:
    """Run `script argv` as `nproc` ranks and return the worst exit status (torchrun's)."""
    child_env = dict(os.environ if env is None else env)
    for k in ENV_KEYS:  # the ranks get theirs from the launcher
        child_env.pop(k, None)
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    cmd = launch_command(script, argv, nproc, free_port())
    print(f"launching {nproc} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    try:
        r = subprocess.run(cmd, env=child_env, timeout=timeout)
    except subprocess.TimeoutExpired:
        print(f"error: {nproc}-rank launch timed out after {timeout} s", file=sys.stderr)
        return 124
    return r.returncode


def check_world(gpus: int, env=None) -> int:
    """The world size a rank process runs with; raises SystemExit (status 2) when it is not the
    `--gpus` the line would report."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"error: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks; "
                         f"run `python {os.path.basename(sys.argv[0])} --gpus {world} ...` or launch "
                         f"{gpus} ranks")
    return world


def maybe_spawn(script: str, argv: list[str], gpus: int, env=None) -> int | None:
    """In a plain `python script --gpus N` process with N > 1: run the N ranks and return their
    exit status. In a rank process (or N == 1): None, and the caller goes on as that rank."""
    if gpus > 1 and not is_rank_process(env):
        return spawn_ranks(script, argv, gpus, env=env)
    return None
