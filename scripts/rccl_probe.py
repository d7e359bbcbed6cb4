"""Probe: does RCCL (torch.distributed backend "nccl") run on this box? Two ranks on the one GPU of a
gpurun lease (RCCL may refuse two ranks on one device), then one rank alone; each all-reduces a
56-MB buffer (the bench's gradient rows at 1M Gaussians) and prints the time and the result check.

  timeout -k 10 120 python scripts/rccl_probe.py [WORLD]
"""
import os
import socket
import sys
import time


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank: int, world: int, port: int) -> None:
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((1_000_000, 14), float(rank + 1), dtype=torch.float32, device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        work = dist.all_reduce(x, async_op=True)
        work.wait()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    expect = float(sum(range(1, world + 1))) * world ** 5  # (6 all-reduces of a sum)
    ok = bool(torch.all(x == expect).item())
    print(f"rank {rank}/{world}: all_reduce of {x.numel() * 4 / 1e6:.0f} MB {dt * 1e3:.3f} ms, result ok {ok}",
          flush=True)
    dist.destroy_process_group()


def main() -> int:
    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.spawn(worker, args=(world, _port()), nprocs=world, join=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
