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


def _uniform_prefill(e, units, per_unit, d, now, seed=77):
    """per_unit batches of d distinct-looking keys "bench_k_<k>_" (k uniform below ~4e9, made on
    the device by tools/gen/libworkload_gen.so) for each rule id in `units`, all at `now`: the
    regions of those home units fill with ≈ per_unit·d live strings each."""
    import ctypes as C
    import math
    from pathlib import Path

    lib = C.CDLL(str(Path(__file__).resolve().parents[1] / "tools" / "gen" / "libworkload_gen.so"))
    vp, u32, u64, dbl = C.c_void_p, C.c_uint32, C.c_uint64, C.c_double
    lib.rlw_keys.argtypes = [C.c_int, u64, dbl, dbl, dbl, dbl, u64, u64, u64, u32, vp, vp, vp, vp]
    lib.rlw_bytes.argtypes = [u32, vp, vp, vp, vp, vp]
    N = 4_000_000_000
    mult = 2654435761
    while math.gcd(mult, N) != 1:
        mult += 2
    key = torch.empty(d, dtype=torch.int64, device=DEV)
    ln = torch.empty(d, dtype=torch.int32, device=DEV)
    db = router.DeviceBatch(torch.zeros(d * 20 + 64, dtype=torch.uint8, device=DEV),
                            torch.zeros(d + 1, dtype=torch.int32, device=DEV), torch.empty(d, dtype=torch.int32, device=DEV),
                            torch.empty(d, dtype=torch.int32, device=DEV), torch.full((d,), now, dtype=torch.int64, device=DEV),
                            torch.ones(d, dtype=torch.int32, device=DEV))
    out = torch.empty(d * 20, dtype=torch.uint8, device=DEV)
    thr = torch.empty(d, dtype=torch.int32, device=DEV)
    st = torch.cuda.current_stream(DEV).cuda_stream
    b = 0
    for rid in units:
        for _ in range(per_unit):
            rc = lib.rlw_keys(1, N, 0.0, 0.0, 0.0, 0.0, seed, 1_000 + b, mult, d, key.data_ptr(), db.rule.data_ptr(),
                              ln.data_ptr(), st)
            torch.cumsum(ln, 0, dtype=torch.int32, out=db.off[1:])
            rc |= lib.rlw_bytes(d, key.data_ptr(), db.off.data_ptr(), db.blob.data_ptr(), db.req_of.data_ptr(), st)
            assert rc == 0
            db.rule.fill_(rid)
            db.nbytes = -1
            torch.cuda.synchronize()
            e.submit_device_async(d, d, db.blob_bytes(), db.ptrs(), out.data_ptr(), thr.data_ptr())
            e.wait()
            b += 1


def test_bench_table_state_long_probe_chains():
    """the bench's table state — 2^27-slot regions taken past 20 % load in the
    SECOND, MINUTE and HOUR regions of one window (long probe chains, claims among 2.7e7 live
    strings per region) — then 120 batches of config-3 traffic in that one SECOND window, two in
    flight, hot set live. The checked keys ("chk_k_...") are disjoint from the prefill's, so their
    answers depend on the prefill only through the table's shape (probe chains, occupancy, claims):
    every status and throttle of the 120 batches must equal the serial oracle of those batches."""
    now = 1_700_000_001  # not a multiple of 60: SECOND / MINUTE / HOUR home regions
    lg = 27
    e = hiprl.Engine(log2_slots=(lg, lg, lg, 14), max_batch_desc=1 << 20, max_batch_req=1 << 20,
                     max_blob_bytes=(1 << 20) * 24, pipeline="v4")
    rules = workload.CONFIG3_RULES
    e.load_rules(rules)
    per_unit, d = 27, 1 << 20  # 2.83e7 strings per region: 21 % of 2^27
    _uniform_prefill(e, [0, 1, 2], per_unit, d, now)
    occ = e.occupancy()
    live = sorted(occ["live"], reverse=True)[:3]
    assert min(live) >= 0.2 * (1 << lg), occ
    nb, dc = 120, 40_000
    z = workload.Zipf(100_000_000, 1.1)
    hbs = []
    for b in range(nb):
        rank = z.sample(3, b, dc) - 1
        kk = workload.permute(rank, 100_000_000)
        blob, off = workload.prefix_blob([b"chk_k_", kk, b"_"])
        hbs.append(hiprl.Batch(blob, off, (rank % 3).astype(np.uint32), np.arange(dc, dtype=np.uint32),
                               np.full(dc, now, np.int64), np.ones(dc, np.uint32)))
    dbs = [router.DeviceBatch.from_host(hb, DEV) for hb in hbs]
    outs = [torch.zeros(dc * 20, dtype=torch.uint8, device=DEV) for _ in range(nb)]
    thrs = [torch.zeros(dc, dtype=torch.int32, device=DEV) for _ in range(nb)]
    torch.cuda.synchronize()
    _run(e, dbs, outs, thrs, 0, nb)
    torch.cuda.synchronize()
    s = e.stats()
    assert s["hot_keys"] > 0, s
    o = oracle.Oracle()
    o.load_rules(rules)
    for k, hb in enumerate(hbs):
        est, ethr = o.submit(hb, threads=16)
        st = outs[k].cpu().numpy().view(hiprl.STATUS_DTYPE)
        thr = thrs[k].cpu().numpy().view(np.uint32)
        streams.assert_same(est, ethr, st, thr, f"prefilled regime batch {k}")
    occ2 = e.occupancy()
    assert sum(occ2["live"]) > sum(occ["live"]), (occ, occ2)  # the checked keys claimed slots among the prefill's
