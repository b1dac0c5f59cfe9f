"""Writes tests/golden/reference_vectors.json.

Every vector below is transcribed by hand from an assertion in the reference's own tests
(kentik/api-ratelimit @ v2; the file:line is in each vector's "src"). The reference is Go
and cannot be built or run in this environment (no Go toolchain, no redis-server), so
these transcribed known answers are what pins the oracle (tests/test_oracle_golden.py)
and, through the same vectors replayed on the device, the HIP path
(tests/test_gpu_golden.py).

Vector kinds
  decide : GetResponseDescriptorStatus inputs (L, unit, now, hits, INCRBY post-value
           `after`, optional explicit `before`, local-cache hit) -> status + stat deltas +
           throttle. The Redis mock in fixed_cache_impl_test.go injects `after` via
           PipeAppend(...).SetArg(1, uint32(after)).
  key    : GenerateCacheKey(domain, entries, unit, now) -> exact key string.
  stream : request sequences with per-request expected statuses and cumulative stats
           (integration_test.go against a real Redis).
Run:  python tests/golden/make_golden.py
"""
import json
from pathlib import Path

S, M, H, D = 1, 2, 3, 4
OK, OVER = 1, 2
FT = "test/redis/fixed_cache_impl_test.go"
BT = "test/limiter/base_limiter_test.go"
IT = "test/integration/integration_test.go"


def dv(src, L, unit, now, hits, after, code, remaining, reset, over=0, near=0, throttle=0, local_hit=False,
       before=None, has_limit=True):
    return dict(src=src, L=L, unit=unit, now=now, hits=hits, after=after, before=before, local_hit=local_hit,
                has_limit=has_limit,
                expect=dict(code=code, remaining=remaining, reset=reset, over=over, near=near, throttle=throttle))


DECIDE = [
    # TestRedis (ratio 0.8)
    dv(f"{FT}:60-74", 10, S, 1234, 1, 5, OK, 5, 1),
    dv(f"{FT}:78-102", 10, M, 1234, 1, 11, OVER, 0, 26, over=1),
    dv(f"{FT}:105-135", 10, H, 1000000, 1, 11, OVER, 0, 800, over=1),
    dv(f"{FT}:109-129", 10, D, 1000000, 1, 13, OVER, 0, 36800, over=1),
    # TestNearLimit
    dv(f"{FT}:286-304", 15, H, 1000000, 1, 11, OK, 4, 800),
    dv(f"{FT}:307-322", 15, H, 1000000, 1, 13, OK, 2, 800, near=1, throttle=400000),
    dv(f"{FT}:326-339", 15, H, 1000000, 1, 16, OVER, 0, 800, over=1),
    dv(f"{FT}:343-356", 20, S, 1234, 3, 5, OK, 15, 1),
    dv(f"{FT}:359-375", 8, S, 1234, 2, 7, OK, 1, 1, near=1, throttle=1000),
    dv(f"{FT}:378-394", 20, S, 1234, 3, 19, OK, 1, 1, near=3, throttle=1000),
    dv(f"{FT}:397-412", 20, S, 1234, 3, 22, OVER, 0, 1, over=2, near=1),
    dv(f"{FT}:415-430", 20, S, 1234, 7, 22, OVER, 0, 1, over=2, near=4),
    dv(f"{FT}:433-448", 10, S, 1234, 3, 30, OVER, 0, 1, over=3),
    # TestRedisWithJitter (jitter only changes EXPIRE)
    dv(f"{FT}:462-478", 10, S, 1234, 1, 5, OK, 5, 1),
    # TestOverLimitWithLocalCache: 4th call is a local-cache hit (no INCRBY)
    dv(f"{FT}:256-269", 15, H, 1000000, 1, 0, OVER, 0, 800, over=1, local_hit=True),
    # base_limiter_test.go (LimitInfo constructed directly)
    dv(f"{BT}:69-86", 5, S, 1234, 2, 6, OVER, 0, 1, over=2, local_hit=True, before=2),
    dv(f"{BT}:88-108", 5, S, 1234, 1, 7, OVER, 0, 1, over=2, near=1, before=2),
    dv(f"{BT}:110-125", 10, S, 1234, 1, 6, OK, 4, 1, before=2),
    dv(f"{BT}:59-67", 0, S, 1234, 1, 0, OK, 0, 0, has_limit=False),
]

KEYS = [
    dict(src=f"{FT}:60; {BT}:31", domain="domain", entries=[["key", "value"]], unit=S, now=1234,
         key="domain_key_value_1234"),
    dict(src=f"{FT}:78", domain="domain", entries=[["key2", "value2"], ["subkey2", "subvalue2"]], unit=M, now=1234,
         key="domain_key2_value2_subkey2_subvalue2_1200"),
    dict(src=f"{FT}:106", domain="domain", entries=[["key3", "value3"]], unit=H, now=1000000,
         key="domain_key3_value3_997200"),
    dict(src=f"{FT}:109", domain="domain", entries=[["key3", "value3"], ["subkey3", "subvalue3"]], unit=D,
         now=1000000, key="domain_key3_value3_subkey3_subvalue3_950400"),
    dict(src=f"{FT}:190", domain="domain", entries=[["key4", "value4"]], unit=H, now=1000000,
         key="domain_key4_value4_997200"),
    dict(src=f"{FT}:344", domain="domain", entries=[["key5", "value5"]], unit=S, now=1234,
         key="domain_key5_value5_1234"),
]


def integration_streams():
    """integration_test.go testBasicBaseConfig, with and without the local cache.
    Rules (test/integration/runtime/current/ratelimit/config/*.yaml): basic.key1 SECOND 50,
    another.key2 MINUTE 20, another.key3 HOUR 10. Time is fixed inside one minute."""
    out = []
    now = 1_700_000_000 - (1_700_000_000 % 3600) + 5  # early in an hour, so the minute does not roll
    for local in (False, True):
        rules = [[50, S], [20, M], [10, H]]
        stat_keys = ["basic.key1", "another.key2", "another.key3"]
        reqs, expects = [], []
        # :282-290 unknown key -> {OK, nil, 0}
        reqs.append(dict(domain="foo", descriptors=[[["hello", "world"]]], rules=[None], hits=1, now=now))
        expects.append(dict(src=f"{IT}:282-290", statuses=[[OK, 0, False]], stats={}))
        # :294-312 basic key1 -> OK 49
        reqs.append(dict(domain="basic", descriptors=[[["key1", "foo"]]], rules=[0], hits=1, now=now))
        expects.append(dict(src=f"{IT}:294-312", statuses=[[OK, 49, True]],
                            stats={"basic.key1": dict(total_hits=1)}))
        # :331-390 25 requests on one fresh key2 value, MINUTE 20
        for i in range(25):
            reqs.append(dict(domain="another", descriptors=[[["key2", "7070707"]]], rules=[1], hits=1, now=now))
            over = i >= 20
            st = dict(total_hits=i + 1, over_limit=(i - 19) if over else 0,
                      over_limit_with_local_cache=(i - 20) if (local and over) else 0)
            expects.append(dict(src=f"{IT}:331-390 i={i}", statuses=[[OVER if over else OK, 0 if over else 19 - i,
                                                                     True]], stats={"another.key2": st}))
        # :392-474 15 requests, two descriptors (fresh key2 value + key3 HOUR 10)
        for i in range(15):
            reqs.append(dict(domain="another", descriptors=[[["key2", "8080808"]], [["key3", "8080808"]]],
                             rules=[1, 2], hits=1, now=now))
            over3 = i >= 10
            st2 = dict(total_hits=i + 26, over_limit=5, over_limit_with_local_cache=4 if local else 0)
            st3 = dict(total_hits=i + 1, over_limit=(i - 9) if over3 else 0,
                       over_limit_with_local_cache=(i - 10) if (local and over3) else 0)
            expects.append(dict(src=f"{IT}:392-474 i={i}",
                                statuses=[[OK, 19 - i, True], [OVER if over3 else OK, 0 if over3 else 9 - i, True]],
                                stats={"another.key2": st2, "another.key3": st3}))
        out.append(dict(name=f"integration_basic_local{int(local)}", local_cache=local, rules=rules,
                        stat_keys=stat_keys, requests=reqs, expect=expects))
    return out


def local_cache_stream():
    """TestOverLimitWithLocalCache as a stream: 15/HOUR; the mock injects INCRBY replies
    11, 13, 16 and then expects a local-cache hit. Replayed on a real counter by warm-up
    requests that bring the counter to 10, 12 and 14 first; only the four checked
    requests carry expectations (per-request deltas)."""
    now = 1000000
    reqs, checks = [], []

    def add(check=None):
        reqs.append(dict(domain="domain", descriptors=[[["key4", "value4"]]], rules=[0], hits=1, now=now))
        checks.append(check)

    for _ in range(10):
        add()
    add(dict(src=f"{FT}:200-209", status=[OK, 4], delta=dict(over=0, near=0, olwlc=0), throttle=0))
    add()
    add(dict(src=f"{FT}:221-230", status=[OK, 2], delta=dict(over=0, near=1, olwlc=0), throttle=400000))
    add()
    add()
    add(dict(src=f"{FT}:242-251", status=[OVER, 0], delta=dict(over=1, near=0, olwlc=0), throttle=0))
    add(dict(src=f"{FT}:261-269", status=[OVER, 0], delta=dict(over=1, near=0, olwlc=1), throttle=0))
    return dict(name="local_cache_key4", local_cache=True, rules=[[15, H]], requests=reqs, checks=checks)


def main():
    doc = dict(
        about="Known answers transcribed from kentik/api-ratelimit tests; see make_golden.py docstring.",
        near_limit_ratio=0.8,
        decide=DECIDE,
        keys=KEYS,
        streams=integration_streams(),
        check_streams=[local_cache_stream()],
    )
    p = Path(__file__).with_name("reference_vectors.json")
    p.write_text(json.dumps(doc, indent=1) + "\n")
    print(f"wrote {p} ({len(DECIDE)} decide, {len(KEYS)} key, 2+1 streams)")


if __name__ == "__main__":
    main()
