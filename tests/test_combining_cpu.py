"""The combining router's protocol on the CPU (no GPU): the arithmetic the device kernels
implement (csrc/rl_route.hip k_route_pack2 / k_route_hot_scan / k_route_unpack_raw), checked
against the serial oracle.

Per step, each origin sends each cold descriptor as one record and each hot prefix group (one
key string: one request time, one rule) as ONE record carrying its sum of hits_addend; each
owner applies its records in origin order (here: the oracle keyed by the records' prefix lanes,
one INCRBY per record) and answers with the raw post-value of each record's INCRBY; the origin
rebuilds every descriptor's post-value — the record's reply, or inside a group
reply - sum + its inclusive prefix of h — and decides it (GetResponseDescriptorStatus,
src/limiter/base_limiter.go:70-177). The result must equal one oracle replaying the origins'
batches in rank order (src/redis/fixed_cache_impl.go:31-123), local cache off. TEST
INFRASTRUCTURE ONLY.
"""
import numpy as np

import hiprl
import oracle
import routing
import streams

SEED = 0x5EE7AB1E5EED


def _batches(G, steps, per, seed):
    rng = np.random.default_rng(seed)
    hot_rule = [int(rng.integers(0, len(streams.RULES))) for _ in range(5)]
    out = []
    for s in range(steps):
        row = []
        for _ in range(G):
            reqs = []
            for _ in range(per):
                nd = 1 + int(rng.random() < 0.25)
                descs, rules = [], []
                for _ in range(nd):
                    if rng.random() < 0.6:
                        k = int(rng.integers(0, 5))
                        descs.append([("hot", f"h{k}")])
                        rules.append(hot_rule[k])
                    else:
                        k = int(rng.integers(0, 300))
                        descs.append([("c", str(k))])
                        rules.append(k % len(streams.RULES) if rng.random() < 0.95 else hiprl.NIL_RULE)
                reqs.append(("cpu", descs, rules, int(rng.integers(0, 9)), 1_700_000_000 + s))
            row.append(hiprl.build_batch(reqs))
        out.append(row)
    return out


def _routed_step(G, batches, owners, ratio=0.8):
    """One combining step over the CPU owners; returns per-origin (status, throttle)."""
    lanes_of, recs = [], [[] for _ in range(G)]  # recs[owner] = [(origin, key lanes, now, rule, h, members)]
    n_groups = 0
    for i, b in enumerate(batches):
        lanes = [oracle.prefix_lanes(b.prefix(d), SEED) if b.rule[d] != hiprl.NIL_RULE else None
                 for d in range(b.n_desc)]
        lanes_of.append(lanes)
        groups = {}  # prefix lanes -> descriptor indices (arrival order)
        for d in range(b.n_desc):
            if lanes[d] is not None:
                groups.setdefault(lanes[d], []).append(d)
        per_owner = [[] for _ in range(G)]
        for ln, ds in groups.items():
            q = [int(b.req_of[d]) for d in ds]
            one_key = len({int(b.now[x]) for x in q}) == 1 and len({int(b.rule[d]) for d in ds}) == 1
            own = oracle.route_owner(ln[0], ln[1], G)
            if len(ds) >= 3 and one_key:  # a hot group: one record with the sum of h
                hs = [max(1, int(b.hits[x])) for x in q]
                per_owner[own].append((ds[0], (i, ln, int(b.now[q[0]]), int(b.rule[ds[0]]), sum(hs), ds)))
                n_groups += 1
            else:
                for d in ds:
                    x = int(b.req_of[d])
                    per_owner[own].append((d, (i, ln, int(b.now[x]), int(b.rule[d]), max(1, int(b.hits[x])), [d])))
        for j in range(G):  # an origin's records for owner j in arrival order of their first descriptor
            recs[j] += [r for _, r in sorted(per_owner[j], key=lambda t: t[0])]
    replies = {}
    gid = 0
    for j in range(G):
        o = owners[j]
        for (i, ln, now, rule, h, ds) in recs[j]:
            gid += 1
            blob = np.frombuffer(np.array(ln, np.uint64).tobytes(), np.uint8).copy()
            o.submit(hiprl.Batch(blob, np.array([0, 16], np.uint32), np.array([rule], np.uint32),
                                 np.array([0], np.uint32), np.array([now], np.int64), np.array([h], np.uint32)))
            unit = streams.RULES[rule][1]
            after = o.counter(oracle.cache_key(blob.tobytes(), unit, now), now)
            assert after > 0
            for d in ds:
                replies[(i, d)] = (after & 0xFFFFFFFF, h, gid)
    got = []
    for i, b in enumerate(batches):
        st = np.zeros(b.n_desc, hiprl.STATUS_DTYPE)
        thr = np.zeros(b.n_req, np.uint32)
        prefix = {}  # group -> running prefix of h
        for d in range(b.n_desc):
            r = int(b.rule[d])
            if r == hiprl.NIL_RULE:
                st[d] = (hiprl.CODE_OK, 0, 0, 0, 0)
                continue
            q = int(b.req_of[d])
            h = max(1, int(b.hits[q]))
            rec_after, rec_sum, g = replies[(i, d)]
            prefix[g] = prefix.get(g, 0) + h  # inclusive prefix of h inside the record's group
            after = (rec_after - rec_sum + prefix[g]) & 0xFFFFFFFF  # = rec_after for a single record
            L, unit = streams.RULES[r]
            s, t = oracle.decide(L, unit, ratio, int(b.now[q]), h, after)
            st[d] = s
            thr[q] = max(int(thr[q]), t)
        got.append((st, thr))
    return got, n_groups


def test_combining_protocol_matches_serial_oracle():
    G = 3
    owners = []
    for _ in range(G):
        o = oracle.Oracle()
        o.load_rules(streams.RULES)
        owners.append(o)
    ref = oracle.Oracle()
    ref.load_rules(streams.RULES)
    combined = 0
    for s, batches in enumerate(_batches(G, 3, 120, seed=5)):
        got, n_groups = _routed_step(G, batches, owners)
        combined += n_groups
        est, ethr = ref.submit(routing.concat_batches(batches))
        d0 = r0 = 0
        for i, (b, (st, thr)) in enumerate(zip(batches, got)):
            streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], st, thr, f"step {s} origin {i}")
            d0 += b.n_desc
            r0 += b.n_req
    assert combined >= 3 * G * 4  # the hot prefixes travelled combined on every origin
