// rl_oracle.cpp — CPU restatement of the reference DoLimit hot path.
// TEST INFRASTRUCTURE ONLY: see rl_oracle.h. Never part of the product path.
//
// Every function cites the reference file:line it restates (paths relative to the
// kentik/api-ratelimit tree). The Redis stand-in is a string-keyed map whose
// INCRBY returns the post-increment int64 (Redis semantics; pinned by
// test/redis/driver_impl_test.go:121-133, miniredis v2.11.4: INCRBY -> 1 then 2).
// EXPIRE follows Redis: every INCRBY is followed by `EXPIRE key ttl` (fixed_cache_impl.go:
// 26-29), ttl = UnitToDivider(unit) + jitter (:69-72: JitterRand.Int63n(jitterMax) per INCRBY;
// the draws are an input here, one per descriptor, as the host batcher draws them — 0 when the
// caller passes none), the key is alive while now < expiry and
// an expired key reads as missing (INCRBY starts from 0). Keys are exact strings, so a
// MINUTE key "p_3600" and an HOUR key "p_3600" are one Redis key (one store) and one
// freecache entry, whose TTL is the unit divider of the Set (base_limiter.go:102).
// Time is integer seconds: a TTL that ends exactly at `now` has expired.
#include "rl_oracle.h"

#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

// utils.UnitToDivider — src/utils/utilities.go:19-32. Other units panic there; we
// report them as bad input (-2) before touching state.
int64_t unit_to_divider(uint32_t unit) {
  switch (unit) {
    case RLO_UNIT_SECOND: return 1;
    case RLO_UNIT_MINUTE: return 60;
    case RLO_UNIT_HOUR: return 60 * 60;
    case RLO_UNIT_DAY: return 60 * 60 * 24;
  }
  return 0;
}

// utils.Max — src/utils/utilities.go:40-45
inline uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// Go's int64 division truncates toward zero, like C++.
inline int64_t window_start(int64_t now, int64_t div) { return (now / div) * div; }

// strconv.FormatInt(v, 10)
void append_dec(std::string& s, int64_t v) {
  char buf[24];
  int n = snprintf(buf, sizeof buf, "%lld", (long long)v);
  s.append(buf, (size_t)n);
}

}  // namespace

// A Redis key: INCRBY counter and EXPIRE deadline (unix seconds; alive while now < exp).
struct RKey {
  int64_t count;
  int64_t exp;
};

struct rlo_engine {
  float near_ratio;
  bool local_cache;       // localCache != nil (base_limiter.go:58, :94)
  bool per_second_split;  // perSecondClient != nil (fixed_cache_impl.go:75)
  std::vector<rlo_rule> rules;
  std::vector<uint32_t> near_thr;  // per rule, base_limiter.go:86
  std::vector<char> shadow;        // per rule: RLO_RULE_SHADOW (extension, do_limit)
  // Redis stand-ins: main client and per-second client (fixed_cache_impl.go:74-85).
  std::unordered_map<std::string, RKey> redis[2];
  // freecache stand-in: over-limit keys and their expiry (base_limiter.go:94-106; freecache
  // v1.1.0 Get misses once now >= expireAt).
  std::unordered_map<std::string, int64_t> lcache;
  uint64_t lc_hit = 0, lc_miss = 0;
  // rlo_submit_mt: the state lives in key shards between multi-threaded calls
  std::vector<rlo_engine*> shards;
};

namespace {
// Move the key shards' state back into the engine (before any serial use of it).
void merge_shards(rlo_engine* e) {
  for (rlo_engine* sh : e->shards) {
    for (int s = 0; s < 2; ++s) e->redis[s].insert(sh->redis[s].begin(), sh->redis[s].end());
    e->lcache.insert(sh->lcache.begin(), sh->lcache.end());
    e->lc_hit += sh->lc_hit;
    e->lc_miss += sh->lc_miss;
    delete sh;
  }
  e->shards.clear();
}
}  // namespace

// C linkage comes from the declarations in rl_oracle.h.

rlo_engine* rlo_create(float near_limit_ratio, int local_cache, int per_second_split) {
  auto* e = new rlo_engine();
  e->near_ratio = near_limit_ratio;
  e->local_cache = local_cache != 0;
  e->per_second_split = per_second_split != 0;
  return e;
}

void rlo_destroy(rlo_engine* e) {
  merge_shards(e);
  delete e;
}

int rlo_load_rules(rlo_engine* e, const rlo_rule* rules, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (unit_to_divider(rules[i].unit & ~RLO_RULE_SHADOW) == 0) return -2;
  e->rules.assign(rules, rules + n);
  e->near_thr.resize(n);
  e->shadow.resize(n);
  for (uint32_t i = 0; i < n; ++i) {
    e->shadow[i] = (rules[i].unit & RLO_RULE_SHADOW) != 0;
    e->rules[i].unit &= ~RLO_RULE_SHADOW;
    // nearLimitThreshold = uint32(math.Floor(float64(float32(L) * ratio)))  base_limiter.go:86
    float p = (float)rules[i].requests_per_unit * e->near_ratio;  // float32 * float32
    e->near_thr[i] = (uint32_t)std::floor((double)p);
  }
  return 0;
}

uint32_t rlo_cache_key(const uint8_t* prefix, uint32_t len, uint32_t unit, int64_t now, char* out, uint32_t cap) {
  // GenerateCacheKey: domain '_' (key '_' value '_')* FormatInt((now/div)*div)  cache_key.go:57-68
  std::string k((const char*)prefix, len);
  append_dec(k, window_start(now, unit_to_divider(unit)));
  uint32_t n = (uint32_t)k.size();
  memcpy(out, k.data(), n < cap ? n : cap);
  return n;
}

// GetResponseDescriptorStatus + checkOverLimitThreshold + checkNearLimitThreshold +
// generateResponseDescriptorStatus + CalculateReset.
//   base_limiter.go:70-115 (status), :129-145 (over), :154-177 (near), :179-195 (reset),
//   utilities.go:34-38 (DurationUntilReset = div - now % div).
// `after` is the uint32 INCRBY reply (fixed_cache_impl.go:51,109); before = after - h
// with uint32 wraparound (:110). The local-cache Set on OVER_LIMIT is done by the caller.
static void decide(uint32_t L, uint32_t near, int64_t div, int64_t now, uint32_t h, uint32_t before,
                   uint32_t after, bool local_hit, bool has_limit, rlo_status* o, uint32_t* throttle) {
  *throttle = 0;
  o->over_limit_delta = 0;
  o->near_limit_delta = 0;
  if (!has_limit) {  // key == "" -> {OK, nil, 0} without reset  :72-75, :189-193
    o->code_flags = RLO_CODE_OK;
    o->limit_remaining = 0;
    o->reset_s = 0;
    return;
  }
  const uint32_t reset = (uint32_t)(div - now % div);
  if (local_hit) {  // :76-81
    o->code_flags = RLO_CODE_OVER_LIMIT | ((RLO_FLAG_HAS_LIMIT | RLO_FLAG_LOCAL_CACHE_HIT) << 8);
    o->limit_remaining = 0;
    o->reset_s = reset;
    o->over_limit_delta = h;  // OverLimit.Add(h) and OverLimitWithLocalCache.Add(h)
    return;
  }
  o->reset_s = reset;
  if (after > L) {  // :88
    o->code_flags = RLO_CODE_OVER_LIMIT | (RLO_FLAG_HAS_LIMIT << 8);
    o->limit_remaining = 0;
    // checkOverLimitThreshold :129-145
    if (before >= L) {
      o->over_limit_delta = h;
    } else {
      o->over_limit_delta = after - L;
      o->near_limit_delta = L - umax(near, before);
    }
  } else {
    o->code_flags = RLO_CODE_OK | (RLO_FLAG_HAS_LIMIT << 8);
    o->limit_remaining = L - after;  // :108-109
    // checkNearLimitThreshold :154-177
    if (after > near) {
      const int64_t end = window_start(now, div) + div;
      const uint32_t millis = (uint32_t)(end - now) * 1000u;
      const uint32_t calls = umax(L - after, 1u);
      *throttle = millis / calls;
      o->near_limit_delta = (before >= near) ? h : after - near;
    }
  }
}

void rlo_decide(uint32_t requests_per_unit, uint32_t unit, float near_limit_ratio, int64_t now, uint32_t hits,
                uint32_t before, uint32_t after, int local_cache_hit, int has_limit, rlo_status* out,
                uint32_t* throttle_ms) {
  const float p = (float)requests_per_unit * near_limit_ratio;
  const uint32_t near = (uint32_t)std::floor((double)p);
  int64_t div = unit_to_divider(unit);
  if (div == 0) div = 1;
  decide(requests_per_unit, near, div, now, hits, before, after, local_cache_hit != 0, has_limit != 0, out,
         throttle_ms);
}

namespace {

struct Desc {
  uint32_t i;
  std::string key;
  bool per_second;
};

// Validate one batch; returns 0 or a negative error.
int validate(const rlo_engine* e, uint32_t n_desc, const uint32_t* prefix_off, const uint32_t* rule_id,
             const uint32_t* req_of, uint32_t n_req) {
  for (uint32_t i = 0; i < n_desc; ++i) {
    if (prefix_off[i + 1] < prefix_off[i]) return -1;
    if (req_of[i] >= n_req) return -1;
    if (i && req_of[i] < req_of[i - 1]) return -1;
    if (rule_id[i] != RLO_NIL_RULE && rule_id[i] >= e->rules.size()) return -1;
  }
  return 0;
}

// The cache keys of descriptors [d0, d1) of one request (GenerateCacheKeys, one `now` per
// request, base_limiter.go:39-54; GenerateCacheKey, cache_key.go:43-73).
void build_keys(const rlo_engine* e, uint32_t d0, uint32_t d1, const uint8_t* blob, const uint32_t* off,
                const uint32_t* rule_id, int64_t now, std::vector<Desc>& keys) {
  for (uint32_t i = d0; i < d1; ++i) {
    Desc d{i, std::string(), false};
    const uint32_t r = rule_id[i];
    if (r != RLO_NIL_RULE) {  // nil limit -> "" key (cache_key.go:46-51)
      const rlo_rule& rule = e->rules[r];
      d.key.assign((const char*)blob + off[i], off[i + 1] - off[i]);
      append_dec(d.key, window_start(now, unit_to_divider(rule.unit)));
      d.per_second = rule.unit == RLO_UNIT_SECOND;  // cache_key.go:33-35,70-72
    }
    keys.push_back(std::move(d));
  }
}

// One request: fixedRateLimitCacheImpl.DoLimit, fixed_cache_impl.go:31-123, over the given
// descriptors of the request (all of them, or one key shard's). Returns the request's
// ThrottleMillis contribution.
uint32_t do_limit(rlo_engine* e, const std::vector<Desc>& keys, const uint32_t* rule_id, int64_t now,
                  uint32_t hits_addend, const uint16_t* jitter, rlo_status* out) {
  // hitsAddend := utils.Max(1, request.HitsAddend)  :39
  const uint32_t h = umax(1u, hits_addend);
  // HOT LOOP 1 :55-86 — local-cache lookups for every descriptor precede any Set.
  std::vector<char> local_hit(keys.size(), 0);
  std::vector<uint32_t> results(keys.size(), 0);
  for (size_t k = 0; k < keys.size(); ++k) {
    if (keys[k].key.empty()) continue;
    if (e->local_cache) {  // IsOverLimitWithLocalCache base_limiter.go:57-66
      auto it = e->lcache.find(keys[k].key);
      if (it != e->lcache.end() && now < it->second) { ++e->lc_hit; local_hit[k] = 1; continue; }
      ++e->lc_miss;
    }
  }
  // PipeDo of the main pipeline, then of the per-second one (:91-102): INCRBY key h (post value,
  // a missing or expired key counts as 0) into results[i] as uint32, then EXPIRE key div.
  for (int pass = 0; pass < 2; ++pass) {
    for (size_t k = 0; k < keys.size(); ++k) {
      if (local_hit[k] || keys[k].key.empty()) continue;
      const int store = (e->per_second_split && keys[k].per_second) ? 1 : 0;
      if (store != pass) continue;
      RKey& c = e->redis[store][keys[k].key];  // a new key is {0, 0}: expired
      if (now >= c.exp) c.count = 0;
      c.count += (int64_t)h;
      // EXPIRE key UnitToDivider(unit) + JitterRand.Int63n(max)  fixed_cache_impl.go:69-72
      c.exp = now + unit_to_divider(e->rules[rule_id[keys[k].i]].unit) + (jitter ? jitter[keys[k].i] : 0);
      results[k] = (uint32_t)c.count;
    }
  }
  // HOT LOOP 2 :108-117
  uint32_t throttle_max = 0;
  for (size_t k = 0; k < keys.size(); ++k) {
    const uint32_t i = keys[k].i;
    const uint32_t r = rule_id[i];
    const bool has = !keys[k].key.empty();
    uint32_t L = 0, near = 0;
    int64_t div = 1;
    if (has) {
      L = e->rules[r].requests_per_unit;
      near = e->near_thr[r];
      div = unit_to_divider(e->rules[r].unit);
    }
    uint32_t thr = 0;
    // limitBeforeIncrease := limitAfterIncrease - hitsAddend (uint32 wrap)  fixed_cache_impl.go:109-110
    decide(L, near, div, now, h, results[k] - h, results[k], local_hit[k] != 0, has, &out[i], &thr);
    // Shadow mode — an extension: this fork has none (config_impl.go:49-59 rejects the key).
    // Restated from envoyproxy/ratelimit's later GetResponseDescriptorStatus: an OVER_LIMIT
    // decision (from Redis or the local cache) is answered OK and counted in Stats.ShadowMode;
    // the INCRBY, the local-cache Set below and the over/near stats are unchanged. Parity
    // unpinned (no reference fixture).
    if (has && e->shadow[r] && (out[i].code_flags & 0xFFu) == RLO_CODE_OVER_LIMIT)
      out[i].code_flags = (out[i].code_flags & ~0xFFu) | RLO_CODE_OK | (RLO_FLAG_SHADOW << 8);
    // response.ThrottleMillis = max(...)  base_limiter.go:163-165
    if (thr > throttle_max) throttle_max = thr;
    // localCache.Set(key, TTL = UnitToDivider(unit)) on OVER_LIMIT from Redis  base_limiter.go:94-106
    if (has && !local_hit[k] && e->local_cache && results[k] > L) e->lcache[keys[k].key] = now + div;
  }
  return throttle_max;
}

}  // namespace

int rlo_submit(rlo_engine* e, uint32_t n_desc, const uint8_t* prefix_blob, const uint32_t* prefix_off,
               const uint32_t* rule_id, const uint32_t* req_of, uint32_t n_req, const int64_t* now,
               const uint32_t* hits_addend, const uint16_t* ttl_jitter, rlo_status* out, uint32_t* req_throttle_ms) {
  int rc = validate(e, n_desc, prefix_off, rule_id, req_of, n_req);
  if (rc) return rc;
  merge_shards(e);
  std::vector<Desc> keys;
  uint32_t d = 0;
  for (uint32_t r = 0; r < n_req; ++r) {
    uint32_t d1 = d;
    while (d1 < n_desc && req_of[d1] == r) ++d1;
    keys.clear();
    build_keys(e, d, d1, prefix_blob, prefix_off, rule_id, now[r], keys);
    req_throttle_ms[r] = do_limit(e, keys, rule_id, now[r], hits_addend[r], ttl_jitter, out);
    d = d1;
  }
  return 0;
}

// Key-sharded over n_threads host threads (the N-core CPU baseline): (1) threads build the
// key strings of contiguous request ranges and partition the descriptors by key shard,
// (2) each shard's thread applies its descriptors request by request in serial order with its
// own Redis / local-cache shard. Per-key serial order is kept (a key lives in one shard), so the
// outputs equal rlo_submit's.
int rlo_submit_mt(rlo_engine* e, int n_threads, uint32_t n_desc, const uint8_t* prefix_blob,
                  const uint32_t* prefix_off, const uint32_t* rule_id, const uint32_t* req_of, uint32_t n_req,
                  const int64_t* now, const uint32_t* hits_addend, const uint16_t* ttl_jitter, rlo_status* out,
                  uint32_t* req_throttle_ms) {
  if (n_threads <= 1)
    return rlo_submit(e, n_desc, prefix_blob, prefix_off, rule_id, req_of, n_req, now, hits_addend, ttl_jitter, out,
                      req_throttle_ms);
  int rc = validate(e, n_desc, prefix_off, rule_id, req_of, n_req);
  if (rc) return rc;
  const int T = n_threads;
  std::hash<std::string> H;
  // key k lives in shard H(k) % T; the shards persist across calls with the same T
  if ((int)e->shards.size() != T) {
    merge_shards(e);
    e->shards.resize(T);
    for (int t = 0; t < T; ++t) {
      e->shards[t] = new rlo_engine();
      e->shards[t]->near_ratio = e->near_ratio;
      e->shards[t]->local_cache = e->local_cache;
      e->shards[t]->per_second_split = e->per_second_split;
    }
    for (int s = 0; s < 2; ++s)
      for (auto& kv : e->redis[s]) e->shards[H(kv.first) % T]->redis[s].emplace(kv.first, kv.second);
    for (auto& kv : e->lcache) e->shards[H(kv.first) % T]->lcache.emplace(kv.first, kv.second);
    e->redis[0].clear();
    e->redis[1].clear();
    e->lcache.clear();
  }
  std::vector<rlo_engine*>& shard = e->shards;
  for (int t = 0; t < T; ++t) {
    shard[t]->rules = e->rules;
    shard[t]->near_thr = e->near_thr;
    shard[t]->shadow = e->shadow;
  }
  // (1) keys and shard lists per request range
  struct Item { uint32_t req; Desc d; };
  std::vector<std::vector<std::vector<Item>>> lists(T, std::vector<std::vector<Item>>(T));
  std::vector<uint32_t> r_lo(T + 1);
  for (int t = 0; t <= T; ++t) r_lo[t] = (uint32_t)((uint64_t)n_req * t / T);
  std::vector<uint32_t> d_lo(T + 1, n_desc);
  {
    uint32_t d = 0;
    for (int t = 0; t < T; ++t) {
      while (d < n_desc && req_of[d] < r_lo[t]) ++d;
      d_lo[t] = d;
    }
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      std::vector<Desc> keys;
      uint32_t d = d_lo[t];
      for (uint32_t r = r_lo[t]; r < r_lo[t + 1]; ++r) {
        uint32_t d1 = d;
        while (d1 < n_desc && req_of[d1] == r) ++d1;
        keys.clear();
        build_keys(e, d, d1, prefix_blob, prefix_off, rule_id, now[r], keys);
        for (auto& k : keys) {
          const int o = k.key.empty() ? 0 : (int)(H(k.key) % T);  // nil-limit descriptors go to shard 0
          lists[t][o].push_back(Item{r, std::move(k)});
        }
        d = d1;
      }
    });
  }
  for (auto& x : th) x.join();
  th.clear();
  // (2) every shard applies its descriptors, request by request, in serial order; each records
  // (request, ThrottleMillis) for the requests it saw, merged by max below
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> thr(T);
  for (int o = 0; o < T; ++o) {
    th.emplace_back([&, o] {
      std::vector<Desc> keys;
      for (int t = 0; t < T; ++t) {
        auto& L = lists[t][o];
        for (size_t a = 0; a < L.size();) {
          size_t b = a;
          keys.clear();
          while (b < L.size() && L[b].req == L[a].req) keys.push_back(std::move(L[b++].d));
          const uint32_t r = L[a].req;
          thr[o].emplace_back(r, do_limit(shard[o], keys, rule_id, now[r], hits_addend[r], ttl_jitter, out));
          a = b;
        }
      }
    });
  }
  for (auto& x : th) x.join();
  if (n_req) memset(req_throttle_ms, 0, (size_t)n_req * 4);
  for (int t = 0; t < T; ++t)
    for (const auto& x : thr[t]) req_throttle_ms[x.first] = std::max(req_throttle_ms[x.first], x.second);
  return 0;
}

int64_t rlo_counter(rlo_engine* e, const char* key, uint32_t len, int per_second, int64_t now) {
  merge_shards(e);
  const int s = (e->per_second_split && per_second) ? 1 : 0;
  auto it = e->redis[s].find(std::string(key, len));
  if (it == e->redis[s].end() || now >= it->second.exp) return -1;
  return it->second.count;
}

int rlo_local_cached(rlo_engine* e, const char* key, uint32_t len, int64_t now) {
  merge_shards(e);
  auto it = e->lcache.find(std::string(key, len));
  return (it != e->lcache.end() && now < it->second) ? 1 : 0;
}

uint64_t rlo_num_keys(rlo_engine* e) { merge_shards(e); return e->redis[0].size() + e->redis[1].size(); }

uint64_t rlo_num_strings(rlo_engine* e) {
  merge_shards(e);
  std::unordered_set<std::string> u;
  for (int s = 0; s < 2; ++s)
    for (auto& kv : e->redis[s]) u.insert(kv.first);
  for (auto& kv : e->lcache) u.insert(kv.first);
  return u.size();
}

void rlo_local_cache_stats(rlo_engine* e, uint64_t* hit, uint64_t* miss, uint64_t* lookup, uint64_t* entries) {
  merge_shards(e);
  *hit = e->lc_hit;
  *miss = e->lc_miss;
  *lookup = e->lc_hit + e->lc_miss;
  *entries = e->lcache.size();
}
