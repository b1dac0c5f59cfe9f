// rl_cache.cpp — HipRateLimitCache: the reference's RateLimitCache contract on the HIP engine.
#include "rl_cache.hpp"

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
  idle_cv_.wait(g, [&] { return q_.empty() && inflight_ == 0; });
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

void HipRateLimitCache::submitter() {
  const size_t cap_desc = s_.batch_limit + 4096, cap_blob = (size_t)(s_.batch_limit + 4096) * 128u;
  for (;;) {
    std::vector<std::shared_ptr<Call>> batch;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (stop_ && q_.empty()) return;
      // Gather for up to batch_window_us or batch_limit descriptors (implicit pipelining
      // analogue, src/redis/driver_impl.go:84-89). A batch may straddle at most one window
      // boundary of a unit, so it is cut when request times are 2 s or more apart.
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(s_.batch_window_us);
      size_t nd = 0, nb = 0;
      int64_t tmin = 0, tmax = 0;
      for (;;) {
        while (!q_.empty()) {
          auto& c = q_.front();
          const size_t d = c->prefix.size();
          if (!batch.empty()) {
            const int64_t lo = c->now < tmin ? c->now : tmin, hi = c->now > tmax ? c->now : tmax;
            if (nd + d > s_.batch_limit || nd + d > cap_desc || nb + c->blob_bytes > cap_blob || hi - lo >= 2)
              goto full;
          }
          if (batch.empty()) tmin = tmax = c->now;
          tmin = c->now < tmin ? c->now : tmin;
          tmax = c->now > tmax ? c->now : tmax;
          nd += d;
          nb += c->blob_bytes;
          batch.push_back(c);
          q_.pop_front();
        }
        if (stop_ || nd >= s_.batch_limit) break;
        if (cv_.wait_until(g, deadline) == std::cv_status::timeout && q_.empty()) break;
        if (std::chrono::steady_clock::now() >= deadline) break;
      }
    full:
      inflight_ += batch.size();
    }
    run_batch(batch);
    {
      std::lock_guard<std::mutex> g(mu_);
      inflight_ -= batch.size();
    }
    idle_cv_.notify_all();
  }
}

void HipRateLimitCache::run_batch(std::vector<std::shared_ptr<Call>>& calls) {
  std::vector<uint8_t> blob;
  std::vector<uint32_t> off{0}, rule, req_of, hits;
  std::vector<int64_t> now;
  for (size_t r = 0; r < calls.size(); ++r) {
    Call& c = *calls[r];
    now.push_back(c.now);
    hits.push_back(c.hits);
    for (size_t i = 0; i < c.prefix.size(); ++i) {
      const auto& lim = (*c.limits)[i];
      blob.insert(blob.end(), c.prefix[i].begin(), c.prefix[i].end());
      off.push_back((uint32_t)blob.size());
      rule.push_back(lim ? rule_id(lim->Limit, lim->ShadowMode) : RL_NIL_RULE);
      req_of.push_back((uint32_t)r);
    }
  }
  std::vector<rl_status> st(rule.size());
  std::vector<uint32_t> thr(calls.size());
  int rc = 0;
  if (rules_dirty_) {
    rc = rl_load_rules(eng_, rules_.data(), (uint32_t)rules_.size());
    rules_dirty_ = rc != 0;
  }
  if (!rc) {
    rl_batch b;
    memset(&b, 0, sizeof b);
    b.n_desc = (uint32_t)rule.size();
    b.n_req = (uint32_t)calls.size();
    b.blob_bytes = (uint32_t)blob.size();
    b.prefix_blob = blob.data();
    b.prefix_off = off.data();
    b.rule_id = rule.data();
    b.req_of = req_of.data();
    b.now = now.data();
    b.hits_addend = hits.data();
    rc = rl_submit(eng_, &b, st.data(), thr.data());
    if (!rc) rc = rl_wait(eng_);
  }
  if (rc) {
    // checkError -> panic(RedisError(...))  src/redis/driver_impl.go:50-54
    const std::string msg = std::string("hip backend: ") + rl_last_error(eng_);
    for (auto& c : calls) c->done.set_exception(std::make_exception_ptr(RedisError(msg)));
    return;
  }
  size_t d = 0;
  for (size_t r = 0; r < calls.size(); ++r) {
    Call& c = *calls[r];
    c.resp.DescriptorStatuses.resize(c.prefix.size());
    c.resp.ThrottleMillis = thr[r];
    for (size_t i = 0; i < c.prefix.size(); ++i, ++d) {
      const auto& lim = (*c.limits)[i];
      const rl_status& s = st[d];
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
}

}  // namespace ratelimit
