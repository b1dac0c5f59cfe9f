"""BASELINE configs 4 and 5 in the regimes bench.py --config 4 / --config 5 measure, at 1e5
descriptors per batch, against the oracles.

Config 4: 4-entry descriptors [("a", v1), ("b", v2), ("c", v3), ("d", v4)] of 1e9 Zipf keys,
resolved on the device by the config4_yaml tree (rl_resolve_device, GetLimit semantics
config_impl.go:274-323) straight into the batch's rule array, then decided with the local
over-limit cache on and every other rule in shadow mode; two batches in flight, the resolve of
batch k+1 running beside batch k's decisions. Checked: the device's rule ids against
config_oracle.get_limit (the first batches) and the host rl_resolve (all), every status and
ThrottleMillis against the decision oracle.

Config 5: 60 simulated seconds (two batches per second) of Zipf(1.1) keys over 1e8 with
SECOND / MINUTE / HOUR rules by rank % 3 and hits_addend ~ U{1..8}, crossing minute and hour
boundaries (window rollover and expiry), near-limit ratio 0.8: every status, stat delta and
ThrottleMillis against oracle.submit(threads=16).
"""
import numpy as np
import pytest
import torch

import config_oracle
import hiprl
import oracle
import rl_config
import router
import streams
import workload

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _dev_resolve(r4, db):
    """The Resolve4's arrays on the device, strings = the device batch's own prefix bytes."""
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(DEV)
    keep = [t(r4.domain), t(r4.entry_first), t(r4.entry)]
    s = hiprl.RlResolveBatch()
    s.n_desc, s.n_entries, s.bytes_len, s.reserved = r4.n_desc, r4.n_entries, r4.bytes_len, 0
    s.bytes, s.domain, s.entry_first, s.entry = db.blob.data_ptr(), keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr()
    s.override_rule = None
    return s, keep


def test_config4_regime_resolved_on_device_two_in_flight():
    d, nb = 100_000, 8
    y = workload.config4_yaml(4)
    cfg = rl_config.RateLimitConfig([("c4.yaml", y)])
    orc_cfg = config_oracle.Config([("c4.yaml", y)])
    e = hiprl.Engine(local_cache=True, max_batch_desc=d, max_batch_req=d, max_blob_bytes=d * 32 + 64,
                     log2_slots=(22, 22, 22, 12))
    cfg.install(e)
    rules = [(r[0], r[1], k % 2 == 0) for k, r in enumerate(cfg.rule_table())]
    e.load_rules(rules)
    o = oracle.Oracle(local_cache=True)
    o.load_rules(rules)
    hbs = [workload.config4_batch(b, d=d, batches_per_s=2, t0=1_700_000_000 - 3, hits_max=4) for b in range(nb)]
    dbs = [router.DeviceBatch.from_host(hb, DEV) for hb, _ in hbs]
    res = [_dev_resolve(r4, db) for (_, r4), db in zip(hbs, dbs)]
    outs = [torch.zeros(d * 20, dtype=torch.uint8, device=DEV) for _ in range(nb)]
    thrs = [torch.zeros(d, dtype=torch.int32, device=DEV) for _ in range(nb)]
    torch.cuda.synchronize()
    pend = 0
    for k, db in enumerate(dbs):
        e.resolve_device(res[k][0], db.rule.data_ptr())
        e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[k].data_ptr(), thrs[k].data_ptr())
        pend += 1
        if pend == 2:
            e.wait()
            pend -= 1
    for _ in range(pend):
        e.wait()
    torch.cuda.synchronize()
    n_sh = n_lc = 0
    for k, ((hb, r4), db) in enumerate(zip(hbs, dbs)):
        rid = db.rule.cpu().numpy().view(np.uint32)
        host = e.resolve(r4)
        assert np.array_equal(rid, host), k
        if k < 2:  # the device walk against the config oracle (GetLimit)
            want = [orc_cfg.get_limit(dm, en) for dm, en in r4.descriptors()]
            have = [None if x == hiprl.NIL_RULE else (cfg.rules[int(x)].requests_per_unit, cfg.rules[int(x)].unit)
                    for x in rid]
            assert have == [None if w is None else (w.requests_per_unit, w.unit) for w in want], k
        b = hiprl.Batch(hb.blob, hb.off, rid.copy(), hb.req_of, hb.now, hb.hits)
        est, ethr = o.submit(b, threads=16)
        gst = outs[k].cpu().numpy().view(hiprl.STATUS_DTYPE)
        gthr = thrs[k].cpu().numpy().view(np.uint32)
        streams.assert_same(gst, gthr, est, ethr, f"config4 batch {k}")
        n_sh += int(((gst["code_flags"] >> 8) & hiprl.FLAG_SHADOW).astype(bool).sum())
        n_lc += int(((gst["code_flags"] >> 8) & hiprl.FLAG_LOCAL_CACHE_HIT).astype(bool).sum())
    assert n_sh > 0 and n_lc > 0, (n_sh, n_lc)


def test_config5_regime_sixty_seconds():
    d, K, secs = 100_000, 2, 60
    nb = K * secs
    e = hiprl.Engine(max_batch_desc=d, max_batch_req=d, max_blob_bytes=d * 24 + 64, log2_slots=(22, 22, 22, 12))
    e.load_rules(workload.CONFIG5_RULES)
    o = oracle.Oracle(near_limit_ratio=0.8)
    o.load_rules(workload.CONFIG5_RULES)
    near = 0
    chunk = 12
    for c0 in range(0, nb, chunk):
        hbs = [workload.config5_batch(b, d=d, N=100_000_000, batches_per_s=K) for b in range(c0, min(nb, c0 + chunk))]
        dbs = [router.DeviceBatch.from_host(hb, DEV) for hb in hbs]
        outs = [torch.zeros(d * 20, dtype=torch.uint8, device=DEV) for _ in hbs]
        thrs = [torch.zeros(d, dtype=torch.int32, device=DEV) for _ in hbs]
        torch.cuda.synchronize()
        pend = 0
        for k, db in enumerate(dbs):
            e.submit_pipelined(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[k].data_ptr(), thrs[k].data_ptr())
            pend += 1
            if pend == 2:
                e.wait()
                pend -= 1
        for _ in range(pend):
            e.wait()
        torch.cuda.synchronize()
        for k, hb in enumerate(hbs):
            est, ethr = o.submit(hb, threads=16)
            gst = outs[k].cpu().numpy().view(hiprl.STATUS_DTYPE)
            streams.assert_same(gst, thrs[k].cpu().numpy().view(np.uint32), est, ethr, f"config5 batch {c0 + k}")
            near += int(gst["near_limit_delta"].astype(np.int64).sum())
    assert near > 0
    assert e.stats()["hot_keys"] > 0
