"""One rank of tests/test_gpu_router_processes.py (not collected by pytest): a separate process
per rank, the C-ABI router's collective transport with its collectives through the host
exchange (RL_ROUTER_HOST_XCHG) over a torch.distributed gloo group — the code path the RCCL
transport runs, across processes, on one GPU (RCCL refuses two ranks on one device).

usage: python -m torch.distributed.run --nproc-per-node G tests/router_procs_worker.py OUT STEPS PER DEPTH
Writes OUT/rank<r>.npz: every step's statuses and ThrottleMillis of this rank's batch, and the
results of a rule agreement (rl_router_allgather_host)."""
import ctypes as C
import datetime
import os
import sys
import traceback
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "api-ratelimit_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
import hiprl  # noqa: E402
from test_gpu_combining import RULES, Bufs, engines, skew_batches  # noqa: E402
from test_gpu_emulated_router import skew_times  # noqa: E402


def main():
    out, steps, per, depth = Path(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
    rank, G = dist.get_rank(), dist.get_world_size()

    @hiprl.HOST_XCHG_FN
    def xchg(ctx, send, sc, sd, recv, rc, rd):
        try:
            cs, cr = [int(sc[j]) for j in range(G)], [int(rc[j]) for j in range(G)]
            ns, nr = sum(cs), sum(cr)
            inp = torch.from_numpy(np.frombuffer((C.c_uint8 * max(ns, 1)).from_address(send), np.uint8)[:ns].copy())
            o = torch.empty(nr, dtype=torch.uint8)
            dist.all_to_all_single(o, inp, cr, cs)
            if nr:
                C.memmove(recv, o.numpy().ctypes.data, nr)
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1

    all_steps = skew_times(skew_batches(G, steps, per, seed=900 + G), seed=901 + G)
    eng = engines(1, 3 * per * G)[0]
    r = hiprl.Router([eng], max_desc=3 * per, n_shards=G, rank=rank, host_xchg=xchg)
    res = {}
    bufs = [Bufs([row[rank]]) for row in all_steps]
    args = [b.args() for b in bufs]
    torch.cuda.synchronize()
    pend = []
    for s, (bs, outs, thrs) in enumerate(args):
        r.submit(bs, outs, thrs)
        pend.append(s)
        if len(pend) == depth:
            r.wait()
            pend.pop(0)
    while pend:
        r.wait()
        pend.pop(0)
    for s, b in enumerate(bufs):
        (st, thr), = b.results()
        res[f"st{s}"] = st.view(np.uint8)
        res[f"thr{s}"] = thr
    # the batchers' rule agreement: every rank's new limits, gathered in rank order
    mine = np.array([rank + 1, 7 * rank + 3, len(RULES)], np.uint32).tobytes()
    got = r.allgather_host(mine, G)
    res["agree"] = np.frombuffer(b"".join(got), np.uint32)
    res["stats_steps"] = np.array([r.stats()["steps"]], np.uint64)
    r.close()
    np.savez(out / f"rank{rank}.npz", **res)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
