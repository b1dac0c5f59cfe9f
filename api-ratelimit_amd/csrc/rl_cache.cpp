// rl_cache.cpp — HipRateLimitCache: the reference's RateLimitCache contract on the HIP engine.
#include "rl_cache.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>

namespace ratelimit {

std::shared_ptr<RateLimitStats> StatsStore::Get(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto& p = m_[key];
  if (!p) p = std::make_shared<RateLimitStats>();
  return p;
}

std::shared_ptr<RateLimit> NewRateLimit(uint32_t requests_per_unit, Unit unit, const std::string& key,
                                        StatsStore& scope, bool sleep_on_throttle, bool report_details) {
  auto r = std::make_shared<RateLimit>();
  r->FullKey = key;
  r->Stats = scope.Get(key);
  r->Limit.RequestsPerUnit = requests_per_unit;
  r->Limit.unit = unit;
  r->SleepOnThrottle = sleep_on_throttle;
  r->ReportDetails = report_details;
  return r;
}

bool DescriptorStatus::operator==(const DescriptorStatus& o) const {
  if (code != o.code || LimitRemaining != o.LimitRemaining) return false;
  if ((CurrentLimit == nullptr) != (o.CurrentLimit == nullptr)) return false;
  if (CurrentLimit && (CurrentLimit->RequestsPerUnit != o.CurrentLimit->RequestsPerUnit ||
                       CurrentLimit->unit != o.CurrentLimit->unit))
    return false;
  if (HasDurationUntilReset != o.HasDurationUntilReset) return false;
  return !HasDurationUntilReset || DurationUntilResetSeconds == o.DurationUntilResetSeconds;
}

int64_t SystemTimeSource::UnixNow() {
  return std::chrono::duration_cast<std::chrono::seconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

struct HipRateLimitCache::Call {
  const RateLimitRequest* req = nullptr;
  const std::vector<std::shared_ptr<RateLimit>>* limits = nullptr;
  int64_t now = 0;
  uint32_t hits = 1;
  std::vector<std::string> prefix;  // per descriptor ("" = nil limit)
  size_t blob_bytes = 0;
  DoLimitResponse resp;
  std::promise<void> done;
};

HipRateLimitCache::HipRateLimitCache(const HipSettings& s, std::shared_ptr<TimeSource> ts)
    : s_(s), ts_(std::move(ts)) {
  rl_config c;
  memset(&c, 0, sizeof c);
  c.struct_size = sizeof c;
  c.device = s.device;
  for (int u = 0; u < 4; ++u) c.log2_slots[u] = s.log2_slots[u];
  c.near_limit_ratio = s.near_limit_ratio;
  c.local_cache = s.local_cache ? 1 : 0;
  c.per_second_split = s.per_second_split ? 1 : 0;
  c.max_batch_desc = s.batch_limit + 4096;
  c.max_batch_req = s.batch_limit + 4096;
  c.max_blob_bytes = (s.batch_limit + 4096) * 128u;
  c.hash_seed = s.hash_seed;
  c.max_load_permille = s.max_load_permille;
  int rc = rl_create(&c, &eng_);
  if (rc) throw RedisError("rl_create failed: " + std::to_string(rc));
  thr_ = std::thread([this] { submitter(); });
}

HipRateLimitCache::~HipRateLimitCache() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  thr_.join();
  rl_destroy(eng_);
}

void HipRateLimitCache::Flush() {
  std::unique_lock<std::mutex> g(mu_);
  idle_cv_.wait(g, [&] { return inflight_ == 0; });
}

DoLimitResponse HipRateLimitCache::DoLimit(const RateLimitRequest& request,
                                           const std::vector<std::shared_ptr<RateLimit>>& limits) {
  // assert.Assert(len(request.Descriptors) == len(limits))  base_limiter.go:41
  if (request.Descriptors.size() != limits.size())
    throw std::logic_error("assert: len(request.Descriptors) == len(limits)");
  auto call = std::make_shared<Call>();
  call->req = &request;
  call->limits = &limits;
  call->now = ts_->UnixNow();                                   // base_limiter.go:43
  call->hits = request.HitsAddend > 1 ? request.HitsAddend : 1;  // fixed_cache_impl.go:39
  call->prefix.resize(limits.size());
  for (size_t i = 0; i < limits.size(); ++i) {
    if (!limits[i]) continue;
    // GenerateCacheKey prefix: domain '_' (key '_' value '_')*   cache_key.go:57-65
    std::string& p = call->prefix[i];
    p = request.Domain;
    p += '_';
    for (const auto& e : request.Descriptors[i].Entries) {
      p += e.Key;
      p += '_';
      p += e.Value;
      p += '_';
    }
    call->blob_bytes += p.size();
    // Stats.TotalHits.Add(hitsAddend) for every non-nil limit  base_limiter.go:49-51
    limits[i]->Stats->TotalHits.Add(call->hits);
  }
  std::future<void> f = call->done.get_future();
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(call);
    ++inflight_;  // until its batch is decided (Flush waits for 0)
  }
  cv_.notify_one();
  f.get();  // rethrows RedisError
  return std::move(call->resp);
}

uint32_t HipRateLimitCache::rule_id(const RateLimitLimit& l, bool shadow) {
  auto k = std::make_pair(l.RequestsPerUnit, (uint32_t)l.unit | (shadow ? RL_RULE_SHADOW : 0u));
  auto it = rule_ids_.find(k);
  if (it != rule_ids_.end()) return it->second;
  const uint32_t id = (uint32_t)rules_.size();
  rules_.push_back(rl_rule{l.RequestsPerUnit, k.second});
  rule_ids_.emplace(k, id);
  rules_dirty_ = true;
  return id;
}

// The batch being built in one of the engine's pinned staging slots (rl_host_acquire): calls
// are written straight into C memory, the way the Go batcher does.
struct HipRateLimitCache::Staged {
  std::vector<std::shared_ptr<Call>> calls;
  rl_host_batch hb{};
  uint32_t nd = 0, nr = 0, nb = 0;
  int64_t tmin = 0, tmax = 0;
  bool failed = false;  // refused at submit: its callers already have the error
};

bool HipRateLimitCache::fits(const Staged& st, const Call& c) const {
  if (st.calls.empty()) return true;
  const int64_t lo = c.now < st.tmin ? c.now : st.tmin, hi = c.now > st.tmax ? c.now : st.tmax;
  // A batch may straddle at most one window boundary of a unit (rl_submit refuses a SECOND key
  // spanning three windows), so it is cut before a request 2 s or more from the others; and
  // before one the slot cannot hold, or past HIP_BATCH_LIMIT descriptors.
  return hi - lo < 2 && st.nd + c.prefix.size() <= s_.batch_limit && st.nd + c.prefix.size() <= st.hb.max_desc &&
         st.nr + 1 <= st.hb.max_req && st.nb + c.blob_bytes <= st.hb.max_blob;
}

// One request into the slot: GenerateCacheKey's bytes before the timestamp per descriptor with
// a limit (cache_key.go:57-65), the rule id, the request index; now and the raw HitsAddend.
void HipRateLimitCache::add(Staged& st, const std::shared_ptr<Call>& cp) {
  Call& c = *cp;
  if (st.calls.empty()) st.tmin = st.tmax = c.now;
  st.tmin = c.now < st.tmin ? c.now : st.tmin;
  st.tmax = c.now > st.tmax ? c.now : st.tmax;
  const uint32_t r = st.nr++;
  st.hb.now[r] = c.now;
  st.hb.hits_addend[r] = c.req->HitsAddend;
  st.hb.prefix_off[0] = 0;
  for (size_t i = 0; i < c.prefix.size(); ++i) {
    const auto& lim = (*c.limits)[i];
    memcpy(st.hb.prefix_blob + st.nb, c.prefix[i].data(), c.prefix[i].size());
    st.nb += (uint32_t)c.prefix[i].size();
    st.hb.rule_id[st.nd] = lim ? rule_id(lim->Limit, lim->ShadowMode) : RL_NIL_RULE;
    st.hb.req_of[st.nd] = r;
    ++st.nd;
    st.hb.prefix_off[st.nd] = st.nb;
  }
  st.calls.push_back(cp);
}

void HipRateLimitCache::fail(std::vector<std::shared_ptr<Call>>& calls) {
  // checkError -> panic(RedisError(...))  src/redis/driver_impl.go:50-54
  const std::string msg = std::string("hip backend: ") + rl_last_error(eng_);
  for (auto& c : calls) c->done.set_exception(std::make_exception_ptr(RedisError(msg)));
  done_calls(calls.size());
  calls.clear();
}

void HipRateLimitCache::done_calls(size_t n) {
  {
    std::lock_guard<std::mutex> g(mu_);
    inflight_ -= n;
  }
  idle_cv_.notify_all();
}

// Hand the slot's batch to the engine. New (L, unit) rules are appended to the device table
// first: that is allowed while the previous batch is in flight (rule ids keep their meaning,
// rl_hip.h rl_load_rules). Two things need nothing in flight (RL_ESTATE otherwise): a rule
// table that crosses V4_MAX_RULES or outgrows its allocation, and a second batch in flight once
// the engine runs the LSD pipeline (more than 32768 rules). Then the batches in flight are
// completed first (their callers answered) and the load / submit is made again; any other
// refusal fails this batch's calls, keeping the table dirty.
void HipRateLimitCache::submit(Staged& st, std::deque<Staged>& inflight) {
  for (int attempt = 0;; ++attempt) {
    int rc = 0;
    if (rules_dirty_) {
      rc = rl_load_rules(eng_, rules_.data(), (uint32_t)rules_.size());
      if (!rc) {
        rules_dirty_ = false;
        n_loads_ += 1;
        if (!inflight.empty()) n_loads_inflight_ += 1;
      }
    }
    if (!rc) {
      rl_batch b;
      memset(&b, 0, sizeof b);
      b.n_desc = st.nd;
      b.n_req = st.nr;
      b.blob_bytes = st.nb;
      b.prefix_blob = st.hb.prefix_blob;  // the slot's own arrays: rl_submit does not copy them
      b.prefix_off = st.hb.prefix_off;
      b.rule_id = st.hb.rule_id;
      b.req_of = st.hb.req_of;
      b.now = st.hb.now;
      b.hits_addend = st.hb.hits_addend;
      rc = rl_submit(eng_, &b, nullptr, nullptr);  // results stay in the slot until rl_wait_view
      if (!rc) n_batches_ += 1;
    }
    if (rc == RL_ESTATE && attempt == 0 && !inflight.empty()) {
      // the slot acquired for this batch stays this batch's: completing the others submits nothing
      while (!inflight.empty()) {
        finish(inflight.front());
        inflight.pop_front();
      }
      n_drains_ += 1;
      continue;
    }
    if (rc) {
      fail(st.calls);
      st.failed = true;
    }
    return;
  }
}

// Collect the oldest batch in flight: rl_wait_view hands out its results in the slot's pinned
// memory (no copy), read here before the next submit reuses the slot.
void HipRateLimitCache::finish(Staged& st) {
  if (st.failed) return;
  const rl_status* out = nullptr;
  const uint32_t* thr = nullptr;
  if (rl_wait_view(eng_, &out, &thr)) {
    fail(st.calls);
    return;
  }
  size_t d = 0;
  for (size_t r = 0; r < st.calls.size(); ++r) {
    Call& c = *st.calls[r];
    c.resp.DescriptorStatuses.resize(c.prefix.size());
    c.resp.ThrottleMillis = thr[r];
    for (size_t i = 0; i < c.prefix.size(); ++i, ++d) {
      const auto& lim = (*c.limits)[i];
      const rl_status& s = out[d];
      DescriptorStatus& o = c.resp.DescriptorStatuses[i];
      o.code = (Code)(s.code_flags & 0xFF);
      o.LimitRemaining = s.limit_remaining;
      const uint32_t fl = s.code_flags >> 8;
      if (lim && (fl & RL_FLAG_HAS_LIMIT)) {
        o.CurrentLimit = &lim->Limit;
        o.HasDurationUntilReset = true;
        o.DurationUntilResetSeconds = s.reset_s;
        // Stats adds of GetResponseDescriptorStatus (base_limiter.go:77-78,129-177)
        if (s.over_limit_delta) lim->Stats->OverLimit.Add(s.over_limit_delta);
        if (fl & RL_FLAG_LOCAL_CACHE_HIT) lim->Stats->OverLimitWithLocalCache.Add(s.over_limit_delta);
        if (s.near_limit_delta) lim->Stats->NearLimit.Add(s.near_limit_delta);
        if (fl & RL_FLAG_SHADOW) lim->Stats->ShadowMode.Add(1);
      }
    }
    c.done.set_value();
  }
  done_calls(st.calls.size());
}

// The submitter thread owns the engine (rl_hip.h: one thread per engine) and keeps two batches
// in flight, as the Go batcher does: batch k+1 is gathered, built in its
// pinned slot and submitted (its H2D copy and fingerprint overlap batch k's kernels) before
// batch k's results are collected; with nothing queued it finishes what is in flight instead
// of waiting. Gathering lasts up to batch_window_us (implicit pipelining analogue,
// src/redis/driver_impl.go:84-89).
void HipRateLimitCache::submitter() {
  std::deque<Staged> inflight;
  std::shared_ptr<Call> carry;
  for (;;) {
    std::shared_ptr<Call> first = std::move(carry);
    carry.reset();
    if (!first) {
      std::unique_lock<std::mutex> g(mu_);
      if (!inflight.empty() && q_.empty()) {
        g.unlock();
        finish(inflight.front());
        inflight.pop_front();
        continue;
      }
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) break;  // stopping
      first = q_.front();
      q_.pop_front();
    }
    Staged st;
    if (rl_host_acquire(eng_, &st.hb)) {
      std::vector<std::shared_ptr<Call>> one{first};
      fail(one);
      continue;
    }
    if (first->prefix.size() > st.hb.max_desc || first->blob_bytes > st.hb.max_blob) {
      first->done.set_exception(std::make_exception_ptr(RedisError("hip backend: request larger than a batch")));
      done_calls(1);
      continue;
    }
    add(st, first);
    {
      std::unique_lock<std::mutex> g(mu_);
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(s_.batch_window_us);
      for (;;) {
        while (!q_.empty()) {
          std::shared_ptr<Call> c = q_.front();
          q_.pop_front();
          if (!fits(st, *c)) {
            carry = std::move(c);  // starts the next batch
            goto full;
          }
          add(st, c);
        }
        if (stop_ || st.nd >= s_.batch_limit) break;
        if (!inflight.empty()) {
          // while gathering, answer the batch in flight as soon as the device is done with it
          // (rl_query), not when this window closes: under light load a caller's latency is then
          // its batch's own, not that plus the next batch's window
          g.unlock();
          const int qr = rl_query(eng_);
          if (qr == 1) {
            finish(inflight.front());
            inflight.pop_front();
          }
          g.lock();
          if (qr == 1) continue;
          const auto slice = std::min(deadline, std::chrono::steady_clock::now() + std::chrono::microseconds(10));
          cv_.wait_until(g, slice);
        } else if (cv_.wait_until(g, deadline) == std::cv_status::timeout && q_.empty()) {
          break;
        }
        if (std::chrono::steady_clock::now() >= deadline) break;
      }
    full:;
    }
    submit(st, inflight);
    inflight.push_back(std::move(st));
    if (inflight.size() == 2) {
      finish(inflight.front());
      inflight.pop_front();
    }
  }
  for (auto& st : inflight) finish(st);
}

}  // namespace ratelimit
