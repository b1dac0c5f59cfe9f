"""The compact host wire format (rl_hip.h rl_batch_c): prefix bytes + one word per descriptor +
one per request (+ req_of when requests hold several descriptors) in, 8-B raw replies out, the
status made on the host by rl_decide_raw (GetResponseDescriptorStatus, base_limiter.go:70-195).
Bit-exact against the serial oracle and against the full rl_submit path.

Reference: src/redis/fixed_cache_impl.go:91-123 (DoLimit reads the INCRBY replies of its pipeline
and makes every status from them), src/limiter/base_limiter.go:57-66 (local-cache lookup)."""
import numpy as np
import pytest

import hiprl
import streams
import workload
from test_gpu_pipelined import _oracle

pytestmark = pytest.mark.gpu


def _stream_batches(seed, n_req, max_bs, t0=1_700_000_000 - 40):
    reqs = streams.make_stream(seed, n_req, t0=t0)
    sizes = streams.batch_sizes(reqs, np.random.default_rng(seed + 1), max_bs)
    out, i = [], 0
    for n in sizes:
        out.append(hiprl.build_batch(reqs[i:i + n]))
        i += n
    return out


def _stage(e, cb):
    sl = e.host_acquire_c()
    nb = int(cb.blob.shape[0])
    sl["blob"][:nb] = cb.blob
    sl["desc_word"][:cb.n_desc] = cb.desc_word
    sl["req_word"][:cb.n_req] = cb.req_word
    if cb.req_of is not None:
        sl["req_of"][:cb.n_desc] = cb.req_of
    e.submit_c_staged(cb.n_desc, cb.n_req, nb, cb.now_base, sl, one_per_req=cb.req_of is None)


@pytest.mark.parametrize("local_cache", [False, True])
def test_compact_three_in_flight_multi_descriptor_requests(local_cache):
    """Requests of 1-5 descriptors (req_of on the wire), nil limits, colliding key strings,
    hits_addend 0-8, three batches in flight, every fourth built in place in the slot; raw
    replies by view and by copy; statuses by rl_decide_raw."""
    hbs = _stream_batches(31, 9000, 1200)
    e = hiprl.Engine(local_cache=local_cache, max_batch_desc=1 << 14)
    e.load_rules(streams.RULES)
    cbs = [hiprl.compact_batch(b) for b in hbs]
    assert any(cb.req_of is not None for cb in cbs)
    got, pend = [], []

    def collect(k):
        cb = pend.pop(0)
        raw = e.wait_raw_view(cb.n_desc).copy() if k % 2 else e.wait_raw_into(cb.n_desc)
        got.append(e.decide_raw(cb, raw))
    for k, cb in enumerate(cbs):
        if k % 4 == 3:
            _stage(e, cb)
        else:
            e.submit_c(cb)
        pend.append(cb)
        if len(pend) == hiprl.MAX_IN_FLIGHT:
            collect(k)
    while pend:
        collect(len(pend))
    want = _oracle(hbs, streams.RULES, local_cache)
    streams.assert_same(*want, np.concatenate([g[0] for g in got]), np.concatenate([g[1] for g in got]), "compact")
    assert e.stats()["host_batches"] == len(hbs)


def test_compact_config3_one_per_request_and_fallback():
    """Config 3 shape (one descriptor per request: no req_of on the wire), 25 B per descriptor
    H2D at ~17-B prefixes; the first batch runs on the LSD pipeline (no hot set yet), so raw
    replies come from both pipelines. Equal to the full-format engine and to the oracle."""
    d = 60_000
    bs = [workload.config3_batch(b, d=d, N=2_000_000, batches_per_s=4) for b in range(6)]
    e = hiprl.Engine(max_batch_desc=1 << 17, log2_slots=(18, 18, 18, 14))
    e.load_rules(workload.CONFIG3_RULES)
    f = hiprl.Engine(max_batch_desc=1 << 17, log2_slots=(18, 18, 18, 14))
    f.load_rules(workload.CONFIG3_RULES)
    wire = 0
    for k, b in enumerate(bs):
        cb = hiprl.compact_batch(b)
        assert cb.req_of is None
        wire += cb.wire_bytes()
        st, thr = e.submit_compact(b)
        fst, fthr = f.submit(b)
        streams.assert_same(fst, fthr, st, thr, f"config3 compact batch {k}")
    assert wire / (len(bs) * d) <= 28.0, wire / (len(bs) * d)
    assert e.stats()["lsd_fallbacks"] >= 1
    want = _oracle(bs, workload.CONFIG3_RULES, False)
    # (the engine f already matched batch by batch; the oracle pins both)
    o_st, o_thr = want
    assert np.array_equal(o_st[-d:], st) and np.array_equal(o_thr[-d:], thr)


def test_compact_lsd_pipeline_raw_replies():
    """The LSD pipeline writes raw replies for descriptor batches (nil limits as RL_RAW_NIL)."""
    hbs = _stream_batches(41, 3000, 900)
    e = hiprl.Engine(local_cache=True, pipeline="lsd", max_batch_desc=1 << 13)
    e.load_rules(streams.RULES)
    got = [e.submit_compact(b) for b in hbs]
    want = _oracle(hbs, streams.RULES, True)
    streams.assert_same(*want, np.concatenate([g[0] for g in got]), np.concatenate([g[1] for g in got]), "lsd compact")


def test_decide_raw_ranges_split_anywhere():
    """rl_decide_raw over ranges cut inside requests equals one call over the batch: a request's
    ThrottleMillis is written by the call that holds all of its descriptors."""
    b = _stream_batches(51, 1500, 1500)[0]
    e = hiprl.Engine(max_batch_desc=1 << 13)
    e.load_rules(streams.RULES)
    cb = hiprl.compact_batch(b)
    e.submit_c(cb)
    raw = e.wait_raw_into(cb.n_desc)
    whole_st, whole_thr = e.decide_raw(cb, raw)
    # split at request boundaries only: every ThrottleMillis written exactly once
    req_starts = np.flatnonzero(np.r_[True, np.diff(b.req_of) != 0])
    cuts = sorted(set([0, cb.n_desc] + list(np.random.default_rng(5).choice(req_starts, 7))))
    st = np.zeros(cb.n_desc, hiprl.STATUS_DTYPE)
    thr = np.full(cb.n_req, 0xDEADBEEF, np.uint32)
    for a, z in zip(cuts[:-1], cuts[1:]):
        e.decide_raw(cb, raw, int(a), int(z), st, thr)
    assert np.array_equal(st, whole_st) and np.array_equal(thr, whole_thr)
    # a cut inside a request leaves that request's word to neither side
    multi = np.flatnonzero(np.bincount(b.req_of) > 1)
    q = int(multi[0])
    inside = int(np.searchsorted(b.req_of, q, "left")) + 1
    thr2 = np.full(cb.n_req, 0xDEADBEEF, np.uint32)
    e.decide_raw(cb, raw, 0, inside, np.zeros(cb.n_desc, hiprl.STATUS_DTYPE), thr2)
    e.decide_raw(cb, raw, inside, cb.n_desc, np.zeros(cb.n_desc, hiprl.STATUS_DTYPE), thr2)
    assert thr2[q] == 0xDEADBEEF
    thr2[q] = whole_thr[q]
    assert np.array_equal(thr2, whole_thr)


def test_compact_refusals():
    """Waits of the wrong form are refused without completing anything; a compact batch with an
    unknown rule id is RL_EINVAL at its wait, like rl_submit's."""
    b = _stream_batches(61, 400, 400)[0]
    e = hiprl.Engine(max_batch_desc=1 << 12)
    e.load_rules(streams.RULES)
    cb = hiprl.compact_batch(b)
    e.submit_c(cb)
    with pytest.raises(hiprl.RedisError) as ei:
        e.wait_view(cb.n_desc, cb.n_req)
    assert ei.value.code == -5
    with pytest.raises(hiprl.RedisError) as ei:
        e.wait_into(cb.n_desc, cb.n_req)
    assert ei.value.code == -5
    e.wait_raw_into(cb.n_desc)
    e.submit_host_async(b)
    with pytest.raises(hiprl.RedisError) as ei:
        e.wait_raw_into(b.n_desc)
    assert ei.value.code == -5
    e.wait_into(b.n_desc, b.n_req)
    bad = hiprl.CompactBatch(cb.blob, cb.desc_word.copy(), cb.req_word, cb.req_of, cb.now_base)
    k = int(np.flatnonzero((bad.desc_word >> 16) != hiprl.NIL_RULE16)[0])
    bad.desc_word[k] = (bad.desc_word[k] & 0xFFFF) | (len(streams.RULES) << 16)
    e.submit_c(bad)
    with pytest.raises(hiprl.RedisError) as ei:
        e.wait_raw_into(bad.n_desc)
    assert ei.value.code == -1
    with pytest.raises(ValueError):
        hiprl.compact_batch(hiprl.Batch(b.blob, b.off, b.rule, b.req_of, b.now, np.full(b.n_req, 1 << 24, np.uint32)))


def test_decide_raw_refuses_request_index_out_of_range():
    """a compact batch whose trailing nil-limit descriptors carry req_of >= n_req
    passes the device (nil descriptors never look at their request), but rl_decide_raw must not
    read req_word or write ThrottleMillis past the caller's arrays: RL_EINVAL, nothing written.
    A decreasing request index is refused the same way."""
    e = hiprl.Engine(max_batch_desc=1024)
    e.load_rules([(5, hiprl.SECOND)])
    reqs = [("oob", [[("k", str(i))]], [0], 1, 1_700_000_001) for i in range(8)]
    cb = hiprl.compact_batch(hiprl.build_batch(reqs))
    n = cb.n_desc
    # two nil descriptors past the last request, claiming requests 8 and 9 of 8
    dw = np.concatenate([cb.desc_word, np.array([hiprl.NIL_RULE16 << 16] * 2, np.uint32)])
    req_of = np.concatenate([np.arange(n, dtype=np.uint32), np.array([8, 9], np.uint32)])
    bad = hiprl.CompactBatch(cb.blob, dw, cb.req_word, req_of, cb.now_base)
    raw = np.zeros(n + 2, hiprl.RAW_DTYPE)
    raw["flags"][n:] = hiprl.RAW_NIL
    st = np.zeros(n + 2, hiprl.STATUS_DTYPE)
    thr = np.full(bad.n_req + 4, 0xABCD, np.uint32)  # guard words past n_req
    with pytest.raises(hiprl.RedisError) as ei:
        e.decide_raw(bad, raw, 0, n + 2, st, thr)
    assert ei.value.code == -1
    assert np.all(thr == 0xABCD) and not st.view(np.uint32).any()
    dec = req_of.copy()
    dec[3], dec[4] = 4, 3
    with pytest.raises(hiprl.RedisError):
        e.decide_raw(hiprl.CompactBatch(cb.blob, dw, cb.req_word, dec, cb.now_base), raw, 0, n + 2, st, thr)
    # the in-range part of the same batch is fine
    e.decide_raw(bad, raw, 0, n, st, thr)
    assert np.all(thr[bad.n_req:] == 0xABCD)
