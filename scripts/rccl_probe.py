"""Probe: can two ranks share ONE GPU through RCCL ("nccl" backend)?  If so, the
device (non-host-staged) branches of TorchDepthColl and DataParallelSPFF can run
on a 1-GPU box.  Prints one line per rank; exits non-zero on failure.

    python scripts/rccl_probe.py
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    ok = bool((t == world * (world + 1) / 2).all())
    peer = 1 - rank
    a = torch.full((256,), float(rank), device=dev)
    b = torch.empty(256, device=dev)
    ops = [dist.P2POp(dist.isend, a, peer), dist.P2POp(dist.irecv, b, peer)]
    for op in dist.batch_isend_irecv(ops):
        op.wait()
    torch.cuda.synchronize()
    ok = ok and bool((b == peer).all())
    print(f"rank {rank}: all_reduce + send/recv on one GPU over {dist.get_backend()}: "
          f"{'ok' if ok else 'WRONG'}", flush=True)
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    mp.spawn(_worker, args=(2, _free_port()), nprocs=2, join=True)
