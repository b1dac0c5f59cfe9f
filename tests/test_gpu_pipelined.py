"""Two or three batches in flight (rl_submit_pipelined): bit-exact against the oracle's serial
replay.

Batch k+1 is fingerprinted and tile-sorted on the engine's second stream while batch k is
decided; a batch the bucketed pipeline refuses poisons the one behind it, and both are
rerun on the LSD pipeline, in order, before anything later is submitted. These streams make
that happen in the first batch (no hot set yet) and in the middle of a stream, with the
local cache on and off, and check every status, stat delta and request throttle.
"""

import numpy as np
import pytest
import torch

import hiprl
import oracle
import router
import streams
import workload

pytestmark = pytest.mark.gpu

from streams import RULES  # noqa: E402


def _pipelined(e, host_batches, dev, depth=2):
    """Submit every batch with up to `depth` in flight (rl_wait completes the oldest)."""
    dbs = [router.DeviceBatch.from_host(hb, dev) for hb in host_batches]
    outs = [torch.zeros(max(1, db.n_desc) * 20, dtype=torch.uint8, device=dev) for db in dbs]
    thrs = [torch.zeros(max(1, db.n_req), dtype=torch.int32, device=dev) for db in dbs]
    torch.cuda.synchronize()

    def sub(k):
        db = dbs[k]
        e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[k].data_ptr(), thrs[k].data_ptr())

    pending = 0
    for k in range(len(dbs)):
        sub(k)
        pending += 1
        if pending == depth:
            e.wait()
            pending -= 1
    for _ in range(pending):
        e.wait()
    torch.cuda.synchronize()
    st = np.concatenate([outs[k][:db.n_desc * 20].cpu().numpy().view(hiprl.STATUS_DTYPE) for k, db in enumerate(dbs)])
    thr = np.concatenate([thrs[k][:db.n_req].cpu().numpy().view(np.uint32) for k, db in enumerate(dbs)])
    return st, thr


def _oracle(host_batches, rules, local_cache, ratio=0.8):
    o = oracle.Oracle(near_limit_ratio=ratio, local_cache=local_cache)
    o.load_rules(rules)
    sts, thrs = [], []
    for hb in host_batches:
        s, t = o.submit(hb)
        sts.append(s)
        thrs.append(t)
    return np.concatenate(sts), np.concatenate(thrs)


def _requests_batches(reqs, sizes):
    out, i = [], 0
    for bs in sizes:
        out.append(hiprl.build_batch(reqs[i:i + bs]))
        i += bs
    return out


@pytest.mark.parametrize("depth", [2, 3])
@pytest.mark.parametrize("local_cache", [False, True])
def test_pipelined_fallbacks_first_and_middle(local_cache, depth):
    """Batch 0: one key with 1500 descriptors (an MSD bucket over BUCKET_CAP, no hot set yet)
    -> refused, batch 1 poisoned. Batch 4: a new key with 1500 descriptors -> refused while
    batch 5 is in flight. The rest: a skewed stream so a hot set forms in between."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    now = 1_700_000_200
    reqs, sizes = [], []
    for k in range(10):
        t = now + k // 3  # at most two adjacent seconds per batch, rollover every 3 batches
        batch = []
        for i in range(4000):
            x = rng.random()
            rule = int(rng.integers(0, 3))
            if k == 0 and i < 1500:
                key, rule = "big0", 2
            elif k == 4 and i % 2 == 0 and i < 3000:
                key, rule = "big4", 2
            elif x < 0.3:
                h = int(rng.integers(0, 4))
                key, rule = f"hot{h}", h % 3  # one rule per hot key: it can join the hot set
            else:
                key = f"k{int(rng.integers(0, 5000))}"
            batch.append(("pl", [[("k", key)]], [rule], int(rng.integers(0, 4)), t))
        reqs += batch
        sizes.append(len(batch))
    hbs = _requests_batches(reqs, sizes)
    e = hiprl.Engine(near_limit_ratio=0.8, local_cache=local_cache, max_batch_desc=1 << 14, pipeline="v4")
    e.load_rules(RULES)
    got = _pipelined(e, hbs, dev, depth)
    ref = _oracle(hbs, RULES, local_cache)
    streams.assert_same(*ref, *got, f"pipelined fallbacks local={local_cache} depth={depth}")
    s = e.stats()
    assert s["lsd_fallbacks"] >= 3, s  # batch 0, the poisoned batch 1, batch 4 (and 5 if it was poisoned)
    assert s["batches"] == len(hbs)


@pytest.mark.parametrize("depth", [2, 3])
@pytest.mark.parametrize("local_cache", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_pipelined_differential_stream(local_cache, seed, depth):
    """The seeded differential streams of test_gpu_parity (domains, 1-4 entries, nil limits,
    collisions, overrides, rollover), cut into batches and submitted two in flight."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(100 + seed)
    reqs = streams.make_stream(seed, 6000, 1_700_000_000 + 1000 * seed)
    sizes = streams.batch_sizes(reqs, rng, 900)
    hbs = _requests_batches(reqs, sizes)
    e = hiprl.Engine(near_limit_ratio=0.8, local_cache=local_cache, max_batch_desc=1 << 14, pipeline="v4")
    e.load_rules(RULES)
    got = _pipelined(e, hbs, dev, depth)
    ref = _oracle(hbs, RULES, local_cache)
    streams.assert_same(*ref, *got, f"pipelined stream seed={seed} local={local_cache} depth={depth}")


@pytest.mark.parametrize("depth", [2, 3])
def test_pipelined_config3_sample(depth):
    """Config 3's Zipf stream (200k descriptors per batch, 12 batches): the hot set forms,
    the first batch falls back, and the steady state runs two batches in flight."""
    dev = torch.device("cuda", 0)
    hbs = [workload.config3_batch(b, d=200_000) for b in range(12)]
    e = hiprl.Engine(log2_slots=(20, 20, 21, 12), max_batch_desc=200_000, max_batch_req=200_000,
                     max_blob_bytes=max(int(hb.blob.shape[0]) for hb in hbs) + 64, pipeline="v4")
    e.load_rules(workload.CONFIG3_RULES)
    got = _pipelined(e, hbs, dev, depth)
    ref = _oracle(hbs, workload.CONFIG3_RULES, False)
    streams.assert_same(*ref, *got, "pipelined config3")
    assert e.stats()["hot_keys"] > 0


def test_pipelined_rejects_shared_outputs():
    dev = torch.device("cuda", 0)
    reqs = [("pl", [[("k", str(i))]], [0], 1, 1_700_000_000) for i in range(100)]
    db = router.DeviceBatch.from_host(hiprl.build_batch(reqs), dev)
    out = torch.zeros(100 * 20, dtype=torch.uint8, device=dev)
    thr = torch.zeros(100, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    e = hiprl.Engine(max_batch_desc=1 << 10, pipeline="v4")
    e.load_rules(RULES)
    e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), out.data_ptr(), thr.data_ptr())
    with pytest.raises(hiprl.RedisError):
        e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), out.data_ptr(), thr.data_ptr())
    e.wait()


def test_pipelined_depth_limit():
    """RL_MAX_IN_FLIGHT (3) batches may be in flight; one more is RL_ESTATE, and the engine
    keeps working after the refusal. The third batch shares no output with the first two."""
    dev = torch.device("cuda", 0)
    reqs = [("pl", [[("k", str(i % 7))]], [0], 1, 1_700_000_000) for i in range(100)]
    db = router.DeviceBatch.from_host(hiprl.build_batch(reqs), dev)
    outs = [torch.zeros(100 * 20, dtype=torch.uint8, device=dev) for _ in range(4)]
    thrs = [torch.zeros(100, dtype=torch.int32, device=dev) for _ in range(4)]
    torch.cuda.synchronize()
    e = hiprl.Engine(max_batch_desc=1 << 10, pipeline="v4")
    e.load_rules(RULES)
    for k in range(3):
        e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[k].data_ptr(), thrs[k].data_ptr())
    with pytest.raises(hiprl.RedisError):
        e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[3].data_ptr(), thrs[3].data_ptr())
    for _ in range(3):
        e.wait()
    torch.cuda.synchronize()
    o = oracle.Oracle(near_limit_ratio=0.8)
    o.load_rules(RULES)
    for k in range(3):
        st, thr = o.submit(hiprl.build_batch(reqs))
        streams.assert_same(st, thr, outs[k].cpu().numpy().view(hiprl.STATUS_DTYPE),
                            thrs[k].cpu().numpy().view(np.uint32), f"depth-limit batch {k}")
