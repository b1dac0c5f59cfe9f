"""PCIe probe for the host path (measurement tooling): per 1e6-descriptor batch the engine moves
~40.9 MB host->device in six copies (blob, offsets, rule, req_of, now, hits) and ~24 MB
device->host in two (statuses, throttles). Times, on pinned (hipHostMalloc via torch) buffers:
  h2d6   the six H2D copies per batch, back to back on one stream
  d2h2   the two D2H copies per batch on one stream
  both   h2d6 on one stream and d2h2 on another, the same number of batches each
  h2d1   one 40.9 MB H2D copy per batch
and prints ms per batch for each, so the host path's ms_per_batch can be read against what
the link does with the same copy shapes.

usage: python tools/pcie_probe.py [batches]"""
import json
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
sizes_in = [17_000_000 + 32, 4_000_004, 4_000_000, 4_000_000, 8_000_000, 4_000_000]
sizes_out = [20_000_000, 4_000_000]
hin = [torch.empty(s, dtype=torch.uint8).pin_memory() for s in sizes_in]
din = [torch.empty(s, dtype=torch.uint8, device=dev) for s in sizes_in]
hout = [torch.empty(s, dtype=torch.uint8).pin_memory() for s in sizes_out]
dout = [torch.empty(s, dtype=torch.uint8, device=dev) for s in sizes_out]
big_h = torch.empty(sum(sizes_in), dtype=torch.uint8).pin_memory()
big_d = torch.empty(sum(sizes_in), dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def timed(fn):
    fn(2)
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn(N)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / N * 1e3


def h2d6(n, st=None):
    with torch.cuda.stream(st or s1):
        for _ in range(n):
            for h, d in zip(hin, din):
                d.copy_(h, non_blocking=True)


def d2h2(n, st=None):
    with torch.cuda.stream(st or s2):
        for _ in range(n):
            for h, d in zip(hout, dout):
                h.copy_(d, non_blocking=True)


def both(n):
    for _ in range(n):
        h2d6(1, s1)
        d2h2(1, s2)


def h2d1(n):
    with torch.cuda.stream(s1):
        for _ in range(n):
            big_d.copy_(big_h, non_blocking=True)


res = {k: round(timed(f), 4) for k, f in (("h2d6", h2d6), ("d2h2", d2h2), ("both", both), ("h2d1", h2d1))}
res["bytes_in"] = sum(sizes_in)
res["bytes_out"] = sum(sizes_out)
res["h2d_GBps"] = round(res["bytes_in"] / res["h2d6"] / 1e6, 1)
res["d2h_GBps"] = round(res["bytes_out"] / res["d2h2"] / 1e6, 1)
print(json.dumps(res))
