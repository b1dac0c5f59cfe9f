"""Probe (GPU box, measurement tooling): can two RCCL ranks share one GPU here? Each of 2
processes joins an nccl (RCCL) process group on cuda:0 and all-reduces a tensor. If it works,
the routed bench's real multi-process path can run with --gpus 2 on a one-GPU box
(RL_BENCH_SAME_DEVICE=1)."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}/{world}: all_reduce -> {t.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
