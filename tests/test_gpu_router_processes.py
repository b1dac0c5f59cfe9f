"""The C-ABI router across PROCESSES: one process per rank, each with its
own engine on the one GPU, the collective transport's code path (counts, records and replies
exchanges, status folding, time ranges, hot-set all-gather, rl_router_allgather_host) with its
collectives carried by the host exchange over a gloo process group — RCCL refuses two ranks on
one device, so this is how the cross-process path runs on a one-GPU box. Every step's outputs on
every rank equal the serial oracle over the rank-order concatenation of the step's batches
(src/redis/fixed_cache_impl.go:31-123 against the owner's counter)."""
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import hiprl
from test_gpu_combining import check, new_oracle, skew_batches
from test_gpu_emulated_router import skew_times

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("G,depth", [(2, 2), (3, 3)])
def test_router_across_processes(G, depth, tmp_path):
    steps, per = 6, 700
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={G}", "--master-addr",
           "127.0.0.1", f"--master-port={port}", str(ROOT / "tests" / "router_procs_worker.py"), str(tmp_path),
           str(steps), str(per), str(depth)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    ranks = [np.load(tmp_path / f"rank{r}.npz") for r in range(G)]
    all_steps = skew_times(skew_batches(G, steps, per, seed=900 + G), seed=901 + G)
    o = new_oracle()
    for s, row in enumerate(all_steps):
        got = [(ranks[r][f"st{s}"].view(hiprl.STATUS_DTYPE), ranks[r][f"thr{s}"]) for r in range(G)]
        check(o, row, got, f"processes G={G} step={s}")
    want = np.concatenate([np.array([r + 1, 7 * r + 3, 0], np.uint32) for r in range(G)])
    for r in range(G):
        agree = ranks[r]["agree"].copy()
        agree[2::3] = 0
        assert np.array_equal(agree, want)
        assert int(ranks[r]["stats_steps"][0]) == steps
