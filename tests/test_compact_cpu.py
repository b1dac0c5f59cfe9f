"""The compact host wire format's encoder (hiprl.compact_batch, rl_hip.h rl_batch_c) on the CPU:
decoding the words gives back the batch, and the wire is <= 28 B per descriptor at config 3."""
import numpy as np
import pytest

import hiprl
import streams
import workload


def decode(cb):
    lens = (cb.desc_word & 0xFFFF).astype(np.int64)
    off = np.r_[0, np.cumsum(lens)].astype(np.uint32)
    r16 = cb.desc_word >> 16
    rule = np.where(r16 == hiprl.NIL_RULE16, hiprl.NIL_RULE, r16).astype(np.uint32)
    req_of = np.arange(cb.n_desc, dtype=np.uint32) if cb.req_of is None else cb.req_of
    now = cb.now_base + (cb.req_word >> 24).astype(np.int64)
    hits = (cb.req_word & 0xFFFFFF).astype(np.uint32)
    return hiprl.Batch(cb.blob, off, rule, req_of, now, hits)


def test_roundtrip_stream_batches():
    reqs = streams.make_stream(7, 2000, t0=1_700_000_000)
    sizes = streams.batch_sizes(reqs, np.random.default_rng(8), 500)
    i = 0
    for n in sizes:
        b = hiprl.build_batch(reqs[i:i + n])
        i += n
        cb = hiprl.compact_batch(b)
        d = decode(cb)
        for f in ("blob", "off", "rule", "req_of", "now", "hits"):
            assert np.array_equal(getattr(d, f), getattr(b, f)), f


def test_config3_wire_bytes():
    b = workload.config3_batch(0, d=100_000)
    cb = hiprl.compact_batch(b)
    assert cb.req_of is None and cb.flags == hiprl.BC_ONE_PER_REQ
    full = int(b.blob.shape[0]) + 4 * (b.n_desc + 1) + 8 * b.n_desc + 12 * b.n_req
    per = cb.wire_bytes() / b.n_desc
    assert per <= 28.0 and per < 0.65 * full / b.n_desc, (per, full / b.n_desc)


def test_out_of_range_batches_are_refused():
    b = workload.config3_batch(0, d=1000)
    with pytest.raises(ValueError):
        hiprl.compact_batch(hiprl.Batch(b.blob, b.off, b.rule, b.req_of, b.now, np.full(b.n_req, 1 << 24, np.uint32)))
    now = b.now.copy()
    now[-1] += 256
    with pytest.raises(ValueError):
        hiprl.compact_batch(hiprl.Batch(b.blob, b.off, b.rule, b.req_of, now, b.hits))
    rule = b.rule.copy()
    rule[0] = 0xFFFF
    with pytest.raises(ValueError):
        hiprl.compact_batch(hiprl.Batch(b.blob, b.off, rule, b.req_of, b.now, b.hits))
