// rl_cache.hpp — C++ mirror of the reference's backend plugin interface, implemented on
// the HIP engine (include/rl_hip.h).
//
// The reference host code is Go; its toolchain is absent here, so this is the host side
// above the C ABI, with the same names, argument meaning and error behaviour:
//   limiter.RateLimitCache{DoLimit, Flush}            src/limiter/cache.go:15-33
//   limiter.DoLimitResponse                            src/limiter/cache.go:9-12
//   config.RateLimit / config.RateLimitStats           src/config/config.go:18-32
//   redis.RedisError (thrown, Go panics)               src/redis/driver.go:6-10
//   utils.TimeSource                                   src/utils/utilities.go:10-14
//   redis.NewFixedRateLimitCacheImpl (constructor)     src/redis/fixed_cache_impl.go:128-135
// DoLimit may be called concurrently from many threads (as grpc-go does); calls are
// micro-batched by one submitter thread (REDIS_PIPELINE_WINDOW / _LIMIT analogue,
// src/settings/settings.go:32-33), and the batch order is the serial order.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "rl_freecache.hpp"
#include "rl_hip.h"

namespace ratelimit {

// pb.RateLimitResponse_RateLimit_Unit / _Code
enum class Unit : uint32_t { UNKNOWN = 0, SECOND = 1, MINUTE = 2, HOUR = 3, DAY = 4 };
enum class Code : uint32_t { UNKNOWN = 0, OK = 1, OVER_LIMIT = 2 };

// gostats counter (additive only)
class Counter {
 public:
  void Add(uint64_t d) { v_.fetch_add(d, std::memory_order_relaxed); }
  uint64_t Value() const { return v_.load(std::memory_order_relaxed); }

 private:
  std::atomic<uint64_t> v_{0};
};

// config.RateLimitStats  src/config/config.go:18-23
struct RateLimitStats {
  Counter TotalHits, OverLimit, NearLimit, OverLimitWithLocalCache;
  Counter ShadowMode;  // extension (rl_hip.h RL_RULE_SHADOW): over-limit decisions reported as OK
};

// Stats scope: counters are shared by name (`<FullKey>.total_hits` ...), like
// statsScope.NewCounter returning the existing counter (config_impl.go:64-71,281-289).
class StatsStore {
 public:
  std::shared_ptr<RateLimitStats> Get(const std::string& key);

 private:
  std::mutex mu_;
  std::unordered_map<std::string, std::shared_ptr<RateLimitStats>> m_;
};

// pb.RateLimitResponse_RateLimit
struct RateLimitLimit {
  uint32_t RequestsPerUnit = 0;
  Unit unit = Unit::UNKNOWN;
};

// config.RateLimit  src/config/config.go:26-32
struct RateLimit {
  std::string FullKey;
  std::shared_ptr<RateLimitStats> Stats;
  RateLimitLimit Limit;
  bool SleepOnThrottle = false;
  bool ReportDetails = false;
  bool ShadowMode = false;  // extension (rl_hip.h RL_RULE_SHADOW); the fork's config has no shadow_mode key
};
// config.NewRateLimit  src/config/config_impl.go:79-89
std::shared_ptr<RateLimit> NewRateLimit(uint32_t requests_per_unit, Unit unit, const std::string& key,
                                        StatsStore& scope, bool sleep_on_throttle, bool report_details);

struct DescriptorEntry {
  std::string Key, Value;
};
struct RateLimitDescriptor {
  std::vector<DescriptorEntry> Entries;
};
// pb.RateLimitRequest
struct RateLimitRequest {
  std::string Domain;
  std::vector<RateLimitDescriptor> Descriptors;
  uint32_t HitsAddend = 0;
};

// pb.RateLimitResponse_DescriptorStatus
struct DescriptorStatus {
  Code code = Code::UNKNOWN;
  const RateLimitLimit* CurrentLimit = nullptr;  // nil when no limit applies
  uint32_t LimitRemaining = 0;
  bool HasDurationUntilReset = false;
  int64_t DurationUntilResetSeconds = 0;
  bool operator==(const DescriptorStatus& o) const;
};

// limiter.DoLimitResponse  src/limiter/cache.go:9-12
struct DoLimitResponse {
  std::vector<DescriptorStatus> DescriptorStatuses;
  uint32_t ThrottleMillis = 0;
};

// redis.RedisError — the only backend failure the service recovers
// (src/service/ratelimit.go:276-281).
class RedisError : public std::runtime_error {
 public:
  explicit RedisError(const std::string& m) : std::runtime_error(m) {}
};

// utils.TimeSource
class TimeSource {
 public:
  virtual ~TimeSource() = default;
  virtual int64_t UnixNow() = 0;
};
class SystemTimeSource : public TimeSource {
 public:
  int64_t UnixNow() override;
};

// limiter.RateLimitCache  src/limiter/cache.go:15-33
class RateLimitCache {
 public:
  virtual ~RateLimitCache() = default;
  virtual DoLimitResponse DoLimit(const RateLimitRequest& request,
                                  const std::vector<std::shared_ptr<RateLimit>>& limits) = 0;
  virtual void Flush() = 0;
};

// One DoLimit call waiting in a micro-batcher (rl_cache.cpp).
struct PendingCall;

// Test hook of both batchers: every call's place in the serial order as it is put in a batch —
// (the batch's / step's sequence number, the call's request position in it). The serial order
// of one engine is (batch, position); of a routed deployment (step, rank, position).
using TraceFn = std::function<void(const RateLimitRequest* request, uint64_t seq, uint32_t pos)>;

// HIP_* settings (BACKEND_TYPE=hip)
struct HipSettings {
  int device = 0;                         // HIP_DEVICES
  uint32_t log2_slots[4] = {20, 20, 20, 18};  // HIP_TABLE_SLOTS per unit
  float near_limit_ratio = 0.8f;          // NEAR_LIMIT_RATIO
  bool local_cache = false;               // LOCAL_CACHE_SIZE_IN_BYTES > 0
  // HIP_LOCAL_CACHE=freecache (single-engine batcher): the local cache is a host-side model of
  // freecache holding LOCAL_CACHE_SIZE_IN_BYTES bytes (rl_freecache.hpp: it evicts, as the
  // reference's does under a small size; parity-unpinned), looked up when a call is enqueued and
  // Set when its batch is decided, instead of the device's cache (which never evicts)
  bool local_cache_freecache = false;
  int64_t local_cache_bytes = 0;
  bool per_second_split = false;          // REDIS_PERSECOND
  uint32_t batch_window_us = 75;          // HIP_BATCH_WINDOW
  uint32_t batch_limit = 1u << 16;        // HIP_BATCH_LIMIT (descriptors)
  uint64_t hash_seed = 0x5ee7ab1e5eedull;  // HIP_HASH_SEED: the same in every process of a deployment
  uint32_t max_load_permille = 750;        // HIP_TABLE_MAX_LOAD: refuse a batch past this region load
  bool answer_early = true;                // HIP_BATCH_ANSWER_EARLY: while gathering, answer the batch in
                                           // flight as soon as the device is done with it (rl_query)
  // EXPIRATION_JITTER_MAX_SECONDS (settings.go:43, default 300; at most 65536 here): every INCRBY's
  // EXPIRE gets JitterRand.Int63n(max) more seconds (fixed_cache_impl.go:69-72). The batcher draws
  // one value per descriptor with a limit, in enqueue order, from jitter_rand (a seeded Int63n
  // source by default; the reference's NewFixedRateLimitCacheImpl takes its jitterRand too).
  int64_t expiration_jitter_max_seconds = 0;
  std::function<int64_t(int64_t)> jitter_rand;  // Int63n(n): uniform in [0, n)
};

// The HIP backend. Equivalent of redis.NewFixedRateLimitCacheImpl + fixedRateLimitCacheImpl.
class HipRateLimitCache : public RateLimitCache {
 public:
  HipRateLimitCache(const HipSettings& s, std::shared_ptr<TimeSource> time_source);
  ~HipRateLimitCache() override;
  DoLimitResponse DoLimit(const RateLimitRequest& request,
                          const std::vector<std::shared_ptr<RateLimit>>& limits) override;
  // Flush() is a no-op for the Redis backend (fixed_cache_impl.go:125-126); here it
  // waits until every enqueued call has been decided.
  void Flush() override;

  // Batcher counters (tests): batches submitted, rule-table loads, and loads made while an
  // earlier batch was still in flight (append-only rule table, rl_hip.h rl_load_rules).
  // drains: times the batches in flight were completed early so that a rule-table load or a
  // submit the engine refused with them in flight (RL_ESTATE) could be made.
  // compact_batches: batches sent in the compact wire format (rl_submit_c); the others went as
  // rl_batch (a rule id past 0xFFFE, a prefix past 65535 bytes or hits_addend past 2^24 - 1).
  struct BatcherStats {
    uint64_t batches, rule_loads, rule_loads_in_flight, drains, compact_batches;
  };
  BatcherStats batcher_stats() const {
    return {n_batches_.load(), n_loads_.load(), n_loads_inflight_.load(), n_drains_.load(), n_compact_.load()};
  }
  // (tests) set before the first DoLimit
  void set_trace(TraceFn f) { trace_ = std::move(f); }
  // HIP_LOCAL_CACHE=freecache: hits, misses, lookups, entries, evicted, expired (zeros otherwise)
  void local_cache_stats(uint64_t* out);

 private:
  struct Staged;
  void submitter();
  uint32_t rule_id(const RateLimitLimit& l, bool shadow);
  bool fits(const Staged& st, const PendingCall& c) const;
  bool compactable(const PendingCall& c) const;
  void add(Staged& st, const std::shared_ptr<PendingCall>& c);
  void submit(Staged& st, std::deque<Staged>& inflight);
  void finish(Staged& st);
  void fail(std::vector<std::shared_ptr<PendingCall>>& calls);
  void done_calls(size_t n);

  HipSettings s_;
  std::shared_ptr<TimeSource> ts_;
  rl_engine* eng_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::deque<std::shared_ptr<PendingCall>> q_;
  size_t inflight_ = 0;  // calls enqueued and not yet answered
  bool stop_ = false;
  std::thread thr_;
  // rule registry (submitter thread only): append-only, so ids keep their meaning while
  // batches that use them are in flight
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> rule_ids_;
  std::vector<rl_rule> rules_;
  bool rules_dirty_ = false;
  std::atomic<uint64_t> n_batches_{0}, n_loads_{0}, n_loads_inflight_{0}, n_drains_{0}, n_compact_{0};
  // statuses of a compact batch made on the host from its raw replies (rl_decide_raw)
  std::vector<rl_status> dec_out_;
  std::vector<uint32_t> dec_thr_;
  TraceFn trace_;
  bool jitter_ = false;
  uint64_t staged_seq_ = 0;  // batches gathered (= submitted, in order)
  std::unique_ptr<FreeCacheModel> fc_;  // HIP_LOCAL_CACHE=freecache
  std::mutex fc_mu_;                    // (freecache's segment locks)
};

// ---- Multi-GPU deployment ------------------------------------------------
// One HipRoutedRateLimitCache per GPU: one process per GPU over RCCL (rl_router_unique_id made by
// rank 0 and handed to the others out of band), or one thread per rank of this process over the
// emulated collectives (rl_router_emu_world; tests). Each rank's DoLimit callers enqueue on its
// own batcher; every rank steps on a fixed cadence (step_us) — gathering what its callers queued
// during the step into the router's pinned slot, or an EMPTY batch when its queue is idle — so the
// ranks' collectives always pair up (rl_hip.h: every rank makes the same sequence of router
// calls). Two steps are in flight. Rule ids must mean one limit on every owner: a new (L, unit)
// is agreed at the next rule-sync step (every rule_sync_every steps, with nothing in flight, by
// rl_router_allgather_host: every rank appends every rank's new rules in rank order), and a call
// that needs it waits for that step. A stop is agreed the same way: a rank leaves only when every
// rank asked to stop with nothing queued. Serial order: each step, rank 0's batch, rank 1's, ...
// The reference's equivalent is the radix cluster client sending each key's commands to the node
// that owns it, pipelined (src/redis/driver_impl.go:84-110); DoLimit stays synchronous for its
// caller (src/limiter/cache.go:15-33).
struct HipRoutedSettings {
  uint32_t n_shards = 1;
  uint32_t rank = 0;
  std::vector<uint8_t> id;        // RL_ROUTER_ID_BYTES: rl_router_unique_id, or rl_router_emu_world
  bool emulated = false;          // id is an emulated world (one thread per rank in this process)
  uint32_t step_us = 200;         // step cadence (HIP_STEP_US)
  uint32_t rule_sync_every = 16;  // steps between rule / stop agreements
};

class HipRoutedRateLimitCache : public RateLimitCache {
 public:
  // Collective: every rank constructs at the same time (rl_router_create agrees configurations).
  HipRoutedRateLimitCache(const HipSettings& s, const HipRoutedSettings& r, std::shared_ptr<TimeSource> time_source);
  // Collective too: returns once every rank has asked to stop and nothing is queued anywhere.
  ~HipRoutedRateLimitCache() override;
  DoLimitResponse DoLimit(const RateLimitRequest& request,
                          const std::vector<std::shared_ptr<RateLimit>>& limits) override;
  void Flush() override;

  struct RoutedStats {
    uint64_t steps, empty_steps, rule_syncs, rules, held_calls;
  };
  RoutedStats routed_stats() const {
    return {n_steps_.load(), n_empty_.load(), n_syncs_.load(), n_rules_.load(), n_held_.load()};
  }
  // (tests) set before the first DoLimit
  void set_trace(TraceFn f) { trace_ = std::move(f); }

 private:
  struct Step;
  void submitter();
  bool known(const PendingCall& c);
  bool sync(bool want_stop);
  void fail(std::vector<std::shared_ptr<PendingCall>>& calls, const std::string& msg);
  void done_calls(size_t n);

  HipSettings s_;
  HipRoutedSettings r_;
  std::shared_ptr<TimeSource> ts_;
  rl_engine* eng_ = nullptr;
  rl_router* rt_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::deque<std::shared_ptr<PendingCall>> q_;
  size_t inflight_ = 0;
  bool stop_ = false;
  bool broken_ = false;  // the router's communicator is gone: every call fails
  std::string broken_msg_;
  std::thread thr_;
  // agreed rule registry (submitter thread): identical on every rank after each sync
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> ids_;
  std::vector<rl_rule> rules_;
  std::vector<rl_rule> pending_;  // new limits seen here, not agreed yet
  std::set<std::pair<uint32_t, uint32_t>> pending_set_;
  std::atomic<uint64_t> n_steps_{0}, n_empty_{0}, n_syncs_{0}, n_rules_{0}, n_held_{0};
  TraceFn trace_;
  bool jitter_ = false;
};

}  // namespace ratelimit
