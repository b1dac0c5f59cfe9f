// rl_cache_shim.cpp — test access to the C++ host-side mirror of the reference's
// RateLimitCache contract (api-ratelimit_amd/csrc/rl_cache.hpp, HipRateLimitCache), whose entry
// points are C++ classes that ctypes cannot reach. Test infrastructure only: tests/
// test_gpu_cache_mirror.py drives it with the reference's integration streams.
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rl_cache.hpp"

using namespace ratelimit;

namespace {
class FixedTime : public TimeSource {
 public:
  std::atomic<int64_t> t{0};
  int64_t UnixNow() override { return t.load(); }
};
struct Shim {
  std::shared_ptr<FixedTime> ts = std::make_shared<FixedTime>();
  StatsStore store;
  std::vector<std::shared_ptr<RateLimit>> rules;
  std::unique_ptr<RateLimitCache> cache;
  HipRateLimitCache* single = nullptr;
  HipRoutedRateLimitCache* routed = nullptr;
  std::string err;
  // serial-order trace (rlc_trace_on): tag of each request in flight, and (tag, seq, pos) per call
  std::mutex tmu;
  std::map<const RateLimitRequest*, uint64_t> tags;
  std::vector<uint64_t> trace;
  void on_trace(const RateLimitRequest* r, uint64_t seq, uint32_t pos) {
    std::lock_guard<std::mutex> g(tmu);
    auto it = tags.find(r);
    trace.push_back(it == tags.end() ? ~0ull : it->second);
    trace.push_back(seq);
    trace.push_back(pos);
  }
};

// The tests' jitter source (EXPIRATION_JITTER_MAX_SECONDS): draw k = splitmix64(seed + k) mod n,
// so a test can replay the k-th draw of a batcher (they are made in its enqueue order).
uint64_t splitmix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
int64_t g_jitter_max = 0;
uint64_t g_jitter_seed = 0;
void set_jitter(HipSettings& hs) {
  hs.expiration_jitter_max_seconds = g_jitter_max;
  if (g_jitter_max > 0) {
    auto k = std::make_shared<std::atomic<uint64_t>>(0);
    const uint64_t seed = g_jitter_seed;
    hs.jitter_rand = [k, seed](int64_t n) { return (int64_t)(splitmix(seed + k->fetch_add(1)) % (uint64_t)n); };
  }
}
}  // namespace

extern "C" {

// The jitter settings of the caches created next (0 = none).
void rlc_next_jitter(int64_t max_seconds, uint64_t seed) {
  g_jitter_max = max_seconds;
  g_jitter_seed = seed;
}

// flags: bit 0 = per-second split (REDIS_PERSECOND), bit 1 = no early answers (HIP_BATCH_ANSWER_EARLY=false),
// bit 2 = batches of at most 4 descriptors (HIP_BATCH_LIMIT=4: with several callers queued, every
// batch is formed and submitted while the one before it is still in flight)
void* rlc_create(int local_cache, float near_ratio, int flags, uint32_t window_us) {
  auto* s = new Shim();
  HipSettings hs;
  set_jitter(hs);
  hs.local_cache = local_cache != 0;
  hs.near_limit_ratio = near_ratio;
  hs.per_second_split = (flags & 1) != 0;
  hs.answer_early = (flags & 2) == 0;
  hs.batch_window_us = window_us;
  hs.batch_limit = (flags & 4) ? 4u : 1u << 14;
  try {
    auto c = std::make_unique<HipRateLimitCache>(hs, s->ts);
    s->single = c.get();
    s->cache = std::move(c);
  } catch (const std::exception& e) {
    delete s;
    return nullptr;
  }
  return s;
}

// HIP_LOCAL_CACHE=freecache: the single-engine batcher with the host's bounded local cache of
// `bytes` (LOCAL_CACHE_SIZE_IN_BYTES; freecache's 512-KiB floor applies).
void* rlc_create_fc(int64_t bytes, float near_ratio, int flags, uint32_t window_us) {
  auto* s = new Shim();
  HipSettings hs;
  set_jitter(hs);
  hs.local_cache = true;
  hs.local_cache_freecache = true;
  hs.local_cache_bytes = bytes;
  hs.near_limit_ratio = near_ratio;
  hs.per_second_split = (flags & 1) != 0;
  hs.answer_early = (flags & 2) == 0;
  hs.batch_window_us = window_us;
  hs.batch_limit = 1u << 14;
  try {
    auto c = std::make_unique<HipRateLimitCache>(hs, s->ts);
    s->single = c.get();
    s->cache = std::move(c);
  } catch (const std::exception& e) {
    delete s;
    return nullptr;
  }
  return s;
}
// hits, misses, lookups, entries, evicted, expired of the batcher's freecache model
void rlc_local_cache_stats(void* p, uint64_t* out) { static_cast<Shim*>(p)->single->local_cache_stats(out); }

// One rank of the multi-GPU batcher (HipRoutedRateLimitCache). id: RL_ROUTER_ID_BYTES from
// rl_router_unique_id or rl_router_emu_world (emulated != 0). Collective: every rank's create runs
// at the same time (one thread per rank). Destroy (rlc_destroy) is collective too.
void* rlc_create_routed(uint32_t n_shards, uint32_t rank, const uint8_t* id, int emulated, int local_cache,
                        uint32_t step_us, uint32_t rule_sync_every, uint32_t batch_limit) {
  auto* s = new Shim();
  HipSettings hs;
  set_jitter(hs);
  hs.local_cache = local_cache != 0;
  hs.batch_limit = batch_limit;
  hs.log2_slots[0] = hs.log2_slots[1] = hs.log2_slots[2] = 16;
  hs.log2_slots[3] = 14;
  HipRoutedSettings rs;
  rs.n_shards = n_shards;
  rs.rank = rank;
  rs.id.assign(id, id + RL_ROUTER_ID_BYTES);
  rs.emulated = emulated != 0;
  rs.step_us = step_us;
  rs.rule_sync_every = rule_sync_every;
  try {
    auto c = std::make_unique<HipRoutedRateLimitCache>(hs, rs, s->ts);
    s->routed = c.get();
    s->cache = std::move(c);
  } catch (const std::exception& e) {
    delete s;
    return nullptr;
  }
  return s;
}

// Routed batcher counters: steps, empty steps, rule agreements, agreed rules, calls held for one.
void rlc_routed_stats(void* p, uint64_t* out) {
  const auto* r = static_cast<Shim*>(p)->routed;
  const auto s = r ? r->routed_stats() : HipRoutedRateLimitCache::RoutedStats{0, 0, 0, 0, 0};
  out[0] = s.steps;
  out[1] = s.empty_steps;
  out[2] = s.rule_syncs;
  out[3] = s.rules;
  out[4] = s.held_calls;
}

void rlc_destroy(void* p) { delete static_cast<Shim*>(p); }

void rlc_set_time(void* p, int64_t now) { static_cast<Shim*>(p)->ts->t.store(now); }

// config.NewRateLimit(rpu, unit, key, scope): the rule's index, for rlc_do_limit / rlc_stats;
// unit | RL_RULE_SHADOW sets RateLimit.ShadowMode (extension)
int rlc_add_rule(void* p, uint32_t rpu, uint32_t unit, const char* key) {
  auto* s = static_cast<Shim*>(p);
  s->rules.push_back(NewRateLimit(rpu, (Unit)(unit & ~RL_RULE_SHADOW), key, s->store, false, false));
  s->rules.back()->ShadowMode = (unit & RL_RULE_SHADOW) != 0;
  return (int)s->rules.size() - 1;
}

// One DoLimit. Descriptor i has n_entries[i] entries taken in order from keys / values, and
// limit rule[i] (an rlc_add_rule index, -1 = nil). out[4 * i ..]: code, LimitRemaining,
// CurrentLimit != nil, DurationUntilReset seconds. Returns 0, or -1 with rlc_error set
// (a RedisError from the backend).
int rlc_do_limit_tagged(void* p, uint64_t tag, const char* domain, uint32_t n_desc, const uint32_t* n_entries,
                        const char* const* keys, const char* const* values, const int32_t* rule, uint32_t hits,
                        uint32_t* out, uint32_t* throttle);
int rlc_do_limit(void* p, const char* domain, uint32_t n_desc, const uint32_t* n_entries, const char* const* keys,
                 const char* const* values, const int32_t* rule, uint32_t hits, uint32_t* out, uint32_t* throttle) {
  return rlc_do_limit_tagged(p, ~0ull, domain, n_desc, n_entries, keys, values, rule, hits, out, throttle);
}

// rlc_do_limit with a caller's tag: the trace (rlc_trace_on) names the call by it.
int rlc_do_limit_tagged(void* p, uint64_t tag, const char* domain, uint32_t n_desc, const uint32_t* n_entries,
                        const char* const* keys, const char* const* values, const int32_t* rule, uint32_t hits,
                        uint32_t* out, uint32_t* throttle) {
  auto* s = static_cast<Shim*>(p);
  RateLimitRequest req;
  struct Tagged {
    Shim* s;
    const RateLimitRequest* r;
    Tagged(Shim* s_, const RateLimitRequest* r_, uint64_t t) : s(s_), r(r_) {
      std::lock_guard<std::mutex> g(s->tmu);
      s->tags[r] = t;
    }
    ~Tagged() {
      std::lock_guard<std::mutex> g(s->tmu);
      s->tags.erase(r);
    }
  } tagged(s, &req, tag);
  req.Domain = domain;
  req.HitsAddend = hits;
  std::vector<std::shared_ptr<RateLimit>> limits(n_desc);
  size_t k = 0;
  for (uint32_t i = 0; i < n_desc; ++i) {
    RateLimitDescriptor d;
    for (uint32_t e = 0; e < n_entries[i]; ++e, ++k) d.Entries.push_back(DescriptorEntry{keys[k], values[k]});
    req.Descriptors.push_back(std::move(d));
    if (rule[i] >= 0) limits[i] = s->rules[rule[i]];
  }
  try {
    DoLimitResponse r = s->cache->DoLimit(req, limits);
    for (uint32_t i = 0; i < n_desc; ++i) {
      const DescriptorStatus& d = r.DescriptorStatuses[i];
      out[4 * i] = (uint32_t)d.code;
      out[4 * i + 1] = d.LimitRemaining;
      out[4 * i + 2] = d.CurrentLimit != nullptr;
      out[4 * i + 3] = (uint32_t)d.DurationUntilResetSeconds;
    }
    *throttle = r.ThrottleMillis;
  } catch (const RedisError& e) {
    s->err = e.what();
    return -1;
  }
  return 0;
}

// Stats of a rule: TotalHits, OverLimit, NearLimit, OverLimitWithLocalCache.
void rlc_stats(void* p, int rule, uint64_t* out) {
  const auto& st = *static_cast<Shim*>(p)->rules[rule]->Stats;
  out[0] = st.TotalHits.Value();
  out[1] = st.OverLimit.Value();
  out[2] = st.NearLimit.Value();
  out[3] = st.OverLimitWithLocalCache.Value();
  out[4] = st.ShadowMode.Value();
}

const char* rlc_error(void* p) { return static_cast<Shim*>(p)->err.c_str(); }

// Record every call's place in the serial order (HipRateLimitCache / HipRoutedRateLimitCache
// set_trace): before the first DoLimit.
void rlc_trace_on(void* p) {
  auto* s = static_cast<Shim*>(p);
  TraceFn f = [s](const RateLimitRequest* r, uint64_t seq, uint32_t pos) { s->on_trace(r, seq, pos); };
  if (s->single) s->single->set_trace(f);
  if (s->routed) s->routed->set_trace(f);
}
// The trace so far: up to max (tag, seq, pos) triples into out; returns how many there are.
uint32_t rlc_trace(void* p, uint64_t* out, uint32_t max) {
  auto* s = static_cast<Shim*>(p);
  std::lock_guard<std::mutex> g(s->tmu);
  const uint32_t n = (uint32_t)(s->trace.size() / 3);
  for (uint32_t i = 0; i < n && i < max; ++i)
    for (int k = 0; k < 3; ++k) out[3 * i + k] = s->trace[3 * i + k];
  return n;
}

void rlc_flush(void* p) { static_cast<Shim*>(p)->cache->Flush(); }

// Batcher counters (5 words): batches, rule loads, rule loads made while a batch was in flight,
// drains (batches in flight completed early for a load / submit the engine refused with them in
// flight), batches sent in the compact wire format.
void rlc_batcher_stats(void* p, uint64_t* out) {
  const auto s = static_cast<Shim*>(p)->single->batcher_stats();
  out[0] = s.batches;
  out[1] = s.rule_loads;
  out[2] = s.rule_loads_in_flight;
  out[3] = s.drains;
  out[4] = s.compact_batches;
}

}  // extern "C"
