"""The multi-GPU bench path (bench.py under torchrun, router.ShardRouter over RCCL) on one GPU.

The driver's scaling run launches `bench.py --gpus N` with one rank per GPU; every rank packs
its batch, exchanges records and replies with RCCL all-to-alls and decides as an owner. On a
one-GPU box the same code runs as one rank with --force-routed (a communicator of one rank:
every collective is real RCCL, every record goes to its own owner), through the C-ABI router
(the default) and through router.ShardRouter (--torch-router), so the routed step's
plumbing is exercised before the 8-GPU run. Bit-exactness of routed steps is covered by
tests/test_gpu_router.py (GPU, logical shards) and tests/test_router_cpu.py (gloo, 2-3 ranks).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", [[], ["--torch-router"]], ids=["c_abi_router", "torch_router"])
def test_routed_bench_one_rank(mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--force-routed", "--steps", "3", "--warmup", "1", "--prefill", "6", "--batches-per-second", "4",
           "--desc", "200000", "--log2-slots", "22", "--cpu-seconds", "0", "--no-kernel-times",
           "--no-roofline-probe", "--no-host-path"] + mode
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] > 0 and line["n_gpus"] == 1
    assert "RCCL all-to-all" in line["config"]["parallelism"], line["config"]
    assert ("C-ABI router" in line["config"]["parallelism"]) == (not mode), line["config"]


def test_pack_async_pairs_and_device_errors():
    """rl_route_pack_async: per owner (count, status) on the device — counts equal the
    synchronous pack's, and a malformed batch (unknown rule id) reports RL_EINVAL in every
    pair instead of failing the call."""
    import torch

    sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    import hiprl
    import router
    import streams

    dev = torch.device("cuda", 0)
    world = 4
    e = hiprl.Engine(max_batch_desc=1 << 14)
    e.load_rules(streams.RULES)
    sh = router.EngineShard(e, 1, world, dev, 1 << 14)
    reqs = streams.make_stream(5, 800, t0=1_700_000_000)
    db = router.DeviceBatch.from_host(hiprl.build_batch(reqs), dev)
    _, _, counts, _ = sh.pack(db)
    _, x, _ = sh.pack_async(db)
    xs = x.cpu().numpy()
    assert list(xs[0::2]) == counts and not xs[1::2].any()
    bad = hiprl.build_batch(reqs)
    bad.rule[3] = len(streams.RULES) + 5  # unknown rule id: found on the device
    dbb = router.DeviceBatch.from_host(bad, dev)
    _, x, _ = sh.pack_async(dbb)
    assert (x.cpu().numpy()[1::2] == -1).all()
    with pytest.raises(hiprl.RedisError):
        sh.pack(dbb)


@pytest.mark.parametrize("world,n_req", [(1, 3000), (4, 3000), (7, 60000), (16, 90000)])
def test_pack_strided_matches_pack(world, n_req):
    """rl_route_pack_strided (one kernel, decoupled look-back across blocks) places every owner's
    records exactly where the three-kernel pack puts them, shifted to owner * stride: same
    records in the same (stable) order, same counts, perm consistent. Up to ~350 blocks of
    look-back; bit-exact."""
    import numpy as np
    import torch

    sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    import hiprl
    import router
    import streams

    dev = torch.device("cuda", 0)
    reqs = streams.make_stream(11 + world, n_req, t0=1_700_000_000)
    hb = hiprl.build_batch(reqs)
    n = hb.n_desc
    e = hiprl.Engine(max_batch_desc=n + 16)
    e.load_rules(streams.RULES)
    sh = router.EngineShard(e, 2 % world, world, dev, n + 16)
    db = router.DeviceBatch.from_host(hb, dev)
    send, _, counts, perm = sh.pack(db)
    ref_send = send.cpu().numpy().reshape(-1, 32)
    ref_perm = perm.cpu().numpy().view(np.uint32)
    stride = n + 5
    ssend = torch.empty(world * stride * 32, dtype=torch.uint8, device=dev)
    x = torch.empty(2 * world, dtype=torch.int32, device=dev)
    sperm = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    e.route_pack_strided(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), 2 % world, world, stride,
                         ssend.data_ptr(), x.data_ptr(), sperm.data_ptr())
    torch.cuda.synchronize()
    xs = x.cpu().numpy()
    assert list(xs[0::2]) == counts and not xs[1::2].any()
    got = ssend.cpu().numpy().reshape(world, stride, 32)
    off = np.concatenate([[0], np.cumsum(counts)])
    for j in range(world):
        assert np.array_equal(got[j, :counts[j]], ref_send[off[j]:off[j + 1]]), f"owner {j}"
    sp = sperm.cpu().numpy().view(np.uint32)[:n]
    local = ref_perm == 0xFFFFFFFF
    assert np.array_equal(sp[local], ref_perm[local])
    own = np.searchsorted(off, ref_perm[~local], side="right") - 1
    assert np.array_equal(sp[~local], own * stride + ref_perm[~local] - off[own])
    bad = hiprl.build_batch(reqs)
    bad.rule[n // 2] = len(streams.RULES) + 3
    dbb = router.DeviceBatch.from_host(bad, dev)
    e.route_pack_strided(dbb.n_desc, dbb.n_req, dbb.blob_bytes(), dbb.ptrs(), 0, world, stride,
                         ssend.data_ptr(), x.data_ptr(), sperm.data_ptr())
    torch.cuda.synchronize()  # the engine runs on the shard's stream, not torch's current one
    assert (x.cpu().numpy()[1::2] == -1).all()
