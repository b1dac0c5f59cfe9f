"""RESP replay: the exact INCRBY/EXPIRE command stream of the reference's
Redis backend, rebuilt from decided batches and replayed into a Redis stand-in.

Encoding is pinned by the reference's mock expectations (test/redis/fixed_cache_impl_test.go:
60-61, 78-80, 106-111: command, key string and argument values) framed as radix v3.5.1 FlatCmd
writes them (RESP arrays of bulk strings). Decisions are checked reply-by-reply against
GetResponseDescriptorStatus (resp.check_replies). A live redis-server is used only when
RL_REDIS_ADDR=host:port is set; none exists in this image or on the GPU box, so that leg is
parity unpinned here."""
import os

import numpy as np
import pytest

import hiprl
import oracle
import resp
from streams import RULES, batch_sizes, make_stream


def test_flat_cmd_reference_vectors():
    # fixed_cache_impl_test.go:60-61 (10/SECOND @1234) and :78-80 (10/MINUTE @1234)
    assert resp.flat_cmd("INCRBY", b"domain_key_value_1234", 1) == \
        b"*3\r\n$6\r\nINCRBY\r\n$21\r\ndomain_key_value_1234\r\n$1\r\n1\r\n"
    assert resp.flat_cmd("EXPIRE", b"domain_key_value_1234", 1) == \
        b"*3\r\n$6\r\nEXPIRE\r\n$21\r\ndomain_key_value_1234\r\n$1\r\n1\r\n"
    k2 = b"domain_key2_value2_subkey2_subvalue2_1200"
    assert resp.cache_key(hiprl.cache_key_prefix("domain", [("key2", "value2"), ("subkey2", "subvalue2")]),
                          hiprl.MINUTE, 1234) == k2
    assert resp.flat_cmd("EXPIRE", k2, 60) == b"*3\r\n$6\r\nEXPIRE\r\n$%d\r\n%s\r\n$2\r\n60\r\n" % (len(k2), k2)
    # :106-111 (HOUR and DAY windows at now = 1e6)
    assert resp.cache_key(b"domain_key3_value3_", hiprl.HOUR, 1000000) == b"domain_key3_value3_997200"
    assert resp.cache_key(b"domain_key3_value3_subkey3_subvalue3_", hiprl.DAY, 1000000) == \
        b"domain_key3_value3_subkey3_subvalue3_950400"


def test_reference_redis_scenario_commands():
    # TestRedis :55-137 as one stream: nil + 10/MINUTE descriptor, then HOUR and DAY limits
    rules = [(10, hiprl.SECOND), (10, hiprl.MINUTE), (10, hiprl.HOUR), (10, hiprl.DAY)]
    reqs = [("domain", [[("key", "value")]], [0], 1, 1234),
            ("domain", [[("key2", "value2")], [("key2", "value2"), ("subkey2", "subvalue2")]],
             [hiprl.NIL_RULE, 1], 1, 1234)]
    b = hiprl.build_batch(reqs)
    o = oracle.Oracle()
    o.load_rules(rules)
    st, _ = o.submit(b)
    cmds = resp.commands(b, rules, st)
    assert [(c.desc, c.key, c.hits, c.ttl) for c in cmds] == [
        (0, b"domain_key_value_1234", 1, 1), (2, b"domain_key2_value2_subkey2_subvalue2_1200", 1, 60)]
    main, ps = resp.encode(cmds)
    assert ps == b"" and main.count(b"INCRBY") == 2 and main.count(b"EXPIRE") == 2
    assert resp.parse_replies(resp.RespStore().execute(main)) == [1, 1, 1, 1]


def test_parse_error_reply_raises_redis_error():
    with pytest.raises(hiprl.RedisError):
        resp.parse_replies(b":1\r\n-ERR wrong number of arguments\r\n")


def _replay_stream(backend_factory, local_cache, per_second_split, seed):
    rng = np.random.default_rng(seed)
    reqs = make_stream(seed, 600, 1_700_000_000, keyspace=12, dt_max=70)
    sizes = batch_sizes(reqs, rng, 64)
    be = backend_factory(local_cache)
    be.load_rules(RULES)
    o = oracle.Oracle(local_cache=local_cache, per_second_split=per_second_split)
    o.load_rules(RULES)
    store, ps_store = resp.RespStore(), (resp.RespStore() if per_second_split else None)
    i = n_cmds = 0
    for bs in sizes:
        b = hiprl.build_batch(reqs[i:i + bs])
        i += bs
        st, _ = be.submit(b)
        o.submit(b)
        n_cmds += len(resp.replay_local(store, ps_store, b, RULES, st, per_second_split))
    # the stand-in's final counters are the oracle's Redis stand-in's
    for k, v in store.counters.items():
        assert o.counter(k, per_second=False) == v, k
    if ps_store is not None:
        for k, v in ps_store.counters.items():
            assert o.counter(k, per_second=True) == v, k
    assert n_cmds > 300


@pytest.mark.parametrize("local_cache", [False, True])
@pytest.mark.parametrize("per_second_split", [False, True])
def test_oracle_decisions_match_replayed_redis_stream(local_cache, per_second_split):
    _replay_stream(lambda lc: oracle.Oracle(local_cache=lc, per_second_split=per_second_split),
                   local_cache, per_second_split, seed=11 + 2 * local_cache + per_second_split)


@pytest.mark.gpu
@pytest.mark.parametrize("local_cache", [False, True])
def test_gpu_decisions_match_replayed_redis_stream(local_cache):
    _replay_stream(lambda lc: hiprl.Engine(local_cache=lc), local_cache, False, seed=21 + local_cache)


@pytest.mark.skipif(not os.environ.get("RL_REDIS_ADDR"), reason="no redis-server (set RL_REDIS_ADDR=host:port of a scratch server; its keys get incremented)")
def test_live_redis_replay():
    host, port = os.environ["RL_REDIS_ADDR"].rsplit(":", 1)
    reqs = make_stream(5, 200, 1_700_000_000, keyspace=8)
    b = hiprl.build_batch(reqs)
    o = oracle.Oracle()
    o.load_rules(RULES)
    st, _ = o.submit(b)
    cmds = resp.commands(b, RULES, st)
    main, _ = resp.encode(cmds)
    replies = resp.parse_replies(resp.replay_to_redis(main, host, int(port), 2 * len(cmds)))
    resp.check_replies(b, RULES, st, cmds, resp.incr_replies(cmds, replies, []))
