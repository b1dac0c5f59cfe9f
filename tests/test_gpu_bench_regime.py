"""The regime bench.py measures, checked against the oracle.

BASELINE config 3 (1e8 keys, Zipf s = 1.1, SECOND / MINUTE / HOUR rules by rank % 3) in
batches of 1e6 descriptors, many batches per SECOND window (`now` advances once every 16
batches, so every window's keys see thousands of INCRBYs across batches), two batches in flight
through rl_submit_pipelined, 24 batches: after the first batches the hot set is live (hot
buckets decided in k4_place, deferred freezes impossible without the local cache) and no batch
falls back to the LSD pipeline. Bit-exact against oracle.submit(threads=16) — every status,
stat delta and request throttle. Reference: src/redis/fixed_cache_impl.go:31-123 at the
BASELINE §8(d) sizes.
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
DEV = torch.device("cuda", 0)


def _run(e, dbs, outs, thrs, first, last, depth=2):
    pend = 0
    for k in range(first, last):
        db = dbs[k]
        e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[k].data_ptr(), thrs[k].data_ptr())
        pend += 1
        if pend == depth:
            e.wait()
            pend -= 1
    for _ in range(pend):
        e.wait()


def test_config3_full_size_many_batches_per_window_two_in_flight():
    K, nb, d = 16, 24, 1_000_000
    hbs = [workload.config3_batch(b, d=d, batches_per_s=K, t0=1_700_000_020) for b in range(nb)]
    dbs = [router.DeviceBatch.from_host(hb, DEV) for hb in hbs]
    outs = [torch.zeros(d * 20, dtype=torch.uint8, device=DEV) for _ in range(nb)]
    thrs = [torch.zeros(d, dtype=torch.int32, device=DEV) for _ in range(nb)]
    torch.cuda.synchronize()
    e = hiprl.Engine(log2_slots=(24, 24, 24, 12), max_batch_desc=d, max_batch_req=d,
                     max_blob_bytes=max(int(hb.blob.shape[0]) for hb in hbs) + 64, pipeline="v4")
    e.load_rules(workload.CONFIG3_RULES)
    warm = 4
    _run(e, dbs, outs, thrs, 0, warm)
    fb_warm = e.stats()["lsd_fallbacks"]
    _run(e, dbs, outs, thrs, warm, nb)
    torch.cuda.synchronize()
    s = e.stats()
    assert s["hot_keys"] > 0, s
    assert s["lsd_fallbacks"] == fb_warm, s  # the steady state never falls back
    o = oracle.Oracle()
    o.load_rules(workload.CONFIG3_RULES)
    for k, hb in enumerate(hbs):
        est, ethr = o.submit(hb, threads=16)
        st = outs[k].cpu().numpy().view(hiprl.STATUS_DTYPE)
        thr = thrs[k].cpu().numpy().view(np.uint32)
        streams.assert_same(est, ethr, st, thr, f"config3 regime batch {k}")
    over = sum(int(((outs[k].cpu().numpy().view(hiprl.STATUS_DTYPE)["code_flags"] & 0xFF) == 2).sum())
               for k in range(nb))
    assert over > 0  # the hot keys pass their SECOND limit inside each window
