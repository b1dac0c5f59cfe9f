// rl_cache.cpp — HipRateLimitCache: the reference's RateLimitCache contract on the HIP engine.
#include "rl_cache.hpp"

#include "rl_common.h"  // decide_status (a local-cache hit's status, as the device makes it)

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

struct PendingCall {
  const RateLimitRequest* req = nullptr;
  const std::vector<std::shared_ptr<RateLimit>>* limits = nullptr;
  int64_t now = 0;
  uint32_t hits = 1;
  std::vector<std::string> prefix;  // per descriptor ("" = nil limit)
  // HIP_LOCAL_CACHE=freecache: per descriptor, a hit of the lookup made at enqueue (no INCRBY)
  // and the full cache key (GenerateCacheKey, cache_key.go:57-68) it was looked up / is Set by
  std::vector<uint8_t> lhit;
  std::vector<std::string> fkey;
  size_t blob_bytes = 0;
  DoLimitResponse resp;
  std::promise<void> done;
};

namespace {

// The caller's side of DoLimit, shared by both batchers: GenerateCacheKeys' prefix bytes per
// descriptor with a limit (cache_key.go:57-65), one time per request (base_limiter.go:43), the
// hits (fixed_cache_impl.go:39), Stats.TotalHits (base_limiter.go:49-51).
std::shared_ptr<PendingCall> make_call(const RateLimitRequest& request,
                                       const std::vector<std::shared_ptr<RateLimit>>& limits, TimeSource& ts) {
  // assert.Assert(len(request.Descriptors) == len(limits))  base_limiter.go:41
  if (request.Descriptors.size() != limits.size())
    throw std::logic_error("assert: len(request.Descriptors) == len(limits)");
  auto call = std::make_shared<PendingCall>();
  call->req = &request;
  call->limits = &limits;
  call->now = ts.UnixNow();                                     // base_limiter.go:43
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
  return call;
}

// A call's DescriptorStatuses and stat adds from its statuses (GetResponseDescriptorStatus's
// outputs, base_limiter.go:70-115,129-177), then the caller is released.
uint32_t unit_divider(Unit u) {  // utils.UnitToDivider
  return u == Unit::SECOND ? 1u : u == Unit::MINUTE ? 60u : u == Unit::HOUR ? 3600u : u == Unit::DAY ? 86400u : 0u;
}

void answer(PendingCall& c, const rl_status* out, uint32_t thr) {
  c.resp.DescriptorStatuses.resize(c.prefix.size());
  c.resp.ThrottleMillis = thr;
  for (size_t i = 0; i < c.prefix.size(); ++i) {
    const auto& lim = (*c.limits)[i];
    rl_status hit_st;
    if (!c.lhit.empty() && c.lhit[i]) {
      // IsOverLimitWithLocalCache: OVER_LIMIT, nothing remaining, OverLimit and
      // OverLimitWithLocalCache += hits (base_limiter.go:76-81); no ThrottleMillis
      rlhip::DevRule R{};
      R.L = lim->Limit.RequestsPerUnit;
      R.div = unit_divider(lim->Limit.unit);
      R.unit = (uint32_t)lim->Limit.unit;
      R.shadow = lim->ShadowMode ? 1u : 0u;
      rlhip::decide_status(0, true, c.hits, (uint32_t)(c.now % R.div), R, hit_st);
    }
    const rl_status& s = (!c.lhit.empty() && c.lhit[i]) ? hit_st : out[i];
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

// EXPIRATION_JITTER_MAX_SECONDS: the settings' jitter source, or a seeded Int63n one (the
// reference seeds its lockedSource with the start time, runner.go / utils.NewLockedSource).
bool setup_jitter(HipSettings& s) {
  if (s.expiration_jitter_max_seconds <= 0) return false;
  if (s.expiration_jitter_max_seconds > 65536)
    throw RedisError("EXPIRATION_JITTER_MAX_SECONDS above 65536 (rl_batch.ttl_jitter is 16-bit)");
  if (!s.jitter_rand) {
    auto state = std::make_shared<std::pair<std::mutex, uint64_t>>();
    state->second = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    s.jitter_rand = [state](int64_t n) {
      std::lock_guard<std::mutex> g(state->first);
      uint64_t z = (state->second += 0x9E3779B97F4A7C15ull);  // splitmix64
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      return (int64_t)(z % (uint64_t)n);
    };
  }
  return true;
}
// One draw: expirationSeconds += JitterRand.Int63n(max)  fixed_cache_impl.go:69-72
uint16_t draw_jitter(const HipSettings& s) { return (uint16_t)s.jitter_rand(s.expiration_jitter_max_seconds); }

}  // namespace

HipRateLimitCache::HipRateLimitCache(const HipSettings& s, std::shared_ptr<TimeSource> ts)
    : s_(s), ts_(std::move(ts)) {
  jitter_ = setup_jitter(s_);
  rl_config c;
  memset(&c, 0, sizeof c);
  c.struct_size = sizeof c;
  c.device = s.device;
  for (int u = 0; u < 4; ++u) c.log2_slots[u] = s.log2_slots[u];
  c.near_limit_ratio = s.near_limit_ratio;
  // HIP_LOCAL_CACHE=freecache: the host's bounded model is the local cache, the device keeps none
  if (s.local_cache && s.local_cache_freecache) fc_ = std::make_unique<FreeCacheModel>(s.local_cache_bytes);
  c.local_cache = s.local_cache && !fc_ ? 1 : 0;
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
  auto call = make_call(request, limits, *ts_);
  if (fc_) {
    // every lookup of the request before any of its INCRBYs (fixed_cache_impl.go:55-66)
    PendingCall& c = *call;
    c.lhit.assign(c.prefix.size(), 0);
    c.fkey.resize(c.prefix.size());
    std::lock_guard<std::mutex> g(fc_mu_);
    for (size_t i = 0; i < c.prefix.size(); ++i) {
      if (!limits[i]) continue;  // "" keys are skipped
      const int64_t div = unit_divider(limits[i]->Limit.unit);
      if (!div) continue;
      c.fkey[i] = c.prefix[i] + std::to_string(c.now / div * div);
      c.lhit[i] = fc_->Get(c.fkey[i], (uint32_t)c.now) ? 1 : 0;
    }
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

// The batch being built in one of the engine's pinned staging slots (rl_host_acquire_c, or
// rl_host_acquire for the full format): calls are written straight into C memory, the way the Go
// batcher does. The compact wire format (rl_batch_c) is the default; a batch
// whose first call does not fit it goes as rl_batch.
struct HipRateLimitCache::Staged {
  std::vector<std::shared_ptr<PendingCall>> calls;
  bool compact = true;
  rl_host_batch hb{};      // full format
  rl_host_batch_c hc{};    // compact format
  uint32_t nd = 0, nr = 0, nb = 0;
  uint32_t max_desc = 0, max_req = 0, max_blob = 0;
  int64_t tmin = 0, tmax = 0;
  bool one_per_req = true;  // compact: every request so far holds one descriptor (req_of implicit)
  bool failed = false;      // refused at submit: its callers already have the error
  uint64_t seq = 0;         // gathered (and submitted) in this order
};

static int64_t compact_base(int64_t first_now) { return first_now > 0 ? first_now - 1 : 0; }

// A call the compact form can carry: prefixes of at most 65535 bytes, hits_addend below 2^24 and
// rule ids (those it has and those it would be given) below 0xFFFF.
bool HipRateLimitCache::compactable(const PendingCall& c) const {
  if (c.req->HitsAddend > 0xFFFFFFu) return false;
  size_t fresh = 0;
  for (size_t i = 0; i < c.prefix.size(); ++i) {
    if (c.prefix[i].size() > 0xFFFFu) return false;
    const auto& lim = (*c.limits)[i];
    if (!lim) continue;
    auto it = rule_ids_.find({lim->Limit.RequestsPerUnit, (uint32_t)lim->Limit.unit | (lim->ShadowMode ? RL_RULE_SHADOW : 0u)});
    if (it == rule_ids_.end()) ++fresh;
    else if (it->second >= RL_NIL_RULE16) return false;
  }
  return rules_.size() + fresh < RL_NIL_RULE16;
}

bool HipRateLimitCache::fits(const Staged& st, const PendingCall& c) const {
  if (st.calls.empty()) return true;
  if (st.compact && !compactable(c)) return false;  // starts a full-format batch
  const int64_t lo = c.now < st.tmin ? c.now : st.tmin, hi = c.now > st.tmax ? c.now : st.tmax;
  // A batch may straddle at most one window boundary of a unit (rl_submit refuses a SECOND key
  // spanning three windows), so it is cut before a request 2 s or more from the others; and
  // before one the slot cannot hold, or past HIP_BATCH_LIMIT descriptors.
  return hi - lo < 2 && st.nd + c.prefix.size() <= s_.batch_limit && st.nd + c.prefix.size() <= st.max_desc &&
         st.nr + 1 <= st.max_req && st.nb + c.blob_bytes <= st.max_blob;
}

// One request into the slot: GenerateCacheKey's bytes before the timestamp per descriptor with
// a limit (cache_key.go:57-65), the rule id, the request index; now and the raw HitsAddend.
void HipRateLimitCache::add(Staged& st, const std::shared_ptr<PendingCall>& cp) {
  PendingCall& c = *cp;
  if (st.calls.empty()) st.tmin = st.tmax = c.now;
  st.tmin = c.now < st.tmin ? c.now : st.tmin;
  st.tmax = c.now > st.tmax ? c.now : st.tmax;
  const uint32_t r = st.nr++;
  if (trace_) trace_(c.req, st.seq, r);
  if (st.compact) {
    // one word per request: hits_addend | (now - now_base) << 24, now_base = the batch's first
    // time minus one (the batch spans < 2 s, so the delta is 0..2)
    const int64_t base = compact_base(st.calls.empty() ? c.now : st.calls[0]->now);
    st.hc.req_word[r] = c.req->HitsAddend | (uint32_t)(c.now - base) << 24;
    if (c.prefix.size() != 1) st.one_per_req = false;
    for (size_t i = 0; i < c.prefix.size(); ++i) {
      const auto& lim = (*c.limits)[i];
      memcpy(st.hc.prefix_blob + st.nb, c.prefix[i].data(), c.prefix[i].size());
      st.nb += (uint32_t)c.prefix[i].size();
      // a local-cache hit goes as a nil descriptor: no INCRBY, and no jitter draw (:61-65)
      const bool inc = lim && (c.lhit.empty() || !c.lhit[i]);
      const uint32_t rid = inc ? rule_id(lim->Limit, lim->ShadowMode) : RL_NIL_RULE16;
      st.hc.desc_word[st.nd] = (uint32_t)c.prefix[i].size() | rid << 16;
      st.hc.req_of[st.nd] = r;  // (sent only when some request holds several descriptors)
      if (jitter_) st.hc.ttl_jitter[st.nd] = inc ? draw_jitter(s_) : 0;
      ++st.nd;
    }
    st.calls.push_back(cp);
    return;
  }
  st.hb.now[r] = c.now;
  st.hb.hits_addend[r] = c.req->HitsAddend;
  st.hb.prefix_off[0] = 0;
  for (size_t i = 0; i < c.prefix.size(); ++i) {
    const auto& lim = (*c.limits)[i];
    memcpy(st.hb.prefix_blob + st.nb, c.prefix[i].data(), c.prefix[i].size());
    st.nb += (uint32_t)c.prefix[i].size();
    const bool inc = lim && (c.lhit.empty() || !c.lhit[i]);
    st.hb.rule_id[st.nd] = inc ? rule_id(lim->Limit, lim->ShadowMode) : RL_NIL_RULE;
    st.hb.req_of[st.nd] = r;
    if (jitter_) st.hb.ttl_jitter[st.nd] = inc ? draw_jitter(s_) : 0;
    ++st.nd;
    st.hb.prefix_off[st.nd] = st.nb;
  }
  st.calls.push_back(cp);
}

void HipRateLimitCache::fail(std::vector<std::shared_ptr<PendingCall>>& calls) {
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
    if (!rc && st.compact) {
      rl_batch_c b;
      memset(&b, 0, sizeof b);
      b.n_desc = st.nd;
      b.n_req = st.nr;
      b.blob_bytes = st.nb;
      b.flags = st.one_per_req ? RL_BC_ONE_PER_REQ : 0u;
      b.now_base = compact_base(st.calls[0]->now);
      b.prefix_blob = st.hc.prefix_blob;  // the slot's own arrays: rl_submit_c does not copy them
      b.desc_word = st.hc.desc_word;
      b.req_word = st.hc.req_word;
      b.req_of = st.one_per_req ? nullptr : st.hc.req_of;
      b.ttl_jitter = jitter_ ? st.hc.ttl_jitter : nullptr;
      rc = rl_submit_c(eng_, &b);  // raw replies stay in the slot until rl_wait_raw_view
      if (!rc) n_batches_ += 1, n_compact_ += 1;
    } else if (!rc) {
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
      b.ttl_jitter = jitter_ ? st.hb.ttl_jitter : nullptr;
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
  if (st.compact) {
    // raw replies (the INCRBY post-values, fixed_cache_impl.go:91-102) -> statuses on the host:
    // GetResponseDescriptorStatus (base_limiter.go:70-195) by rl_decide_raw
    const rl_raw_reply* raw = nullptr;
    rl_batch_c b;
    memset(&b, 0, sizeof b);
    b.n_desc = st.nd;
    b.n_req = st.nr;
    b.blob_bytes = st.nb;
    b.flags = st.one_per_req ? RL_BC_ONE_PER_REQ : 0u;
    b.now_base = compact_base(st.calls[0]->now);
    b.prefix_blob = st.hc.prefix_blob;
    b.desc_word = st.hc.desc_word;  // the slot's inputs stay until it is acquired again
    b.req_word = st.hc.req_word;
    b.req_of = st.one_per_req ? nullptr : st.hc.req_of;
    if (dec_out_.size() < st.nd) dec_out_.resize(st.nd);
    if (dec_thr_.size() < st.nr) dec_thr_.resize(st.nr);
    if (rl_wait_raw_view(eng_, &raw) || rl_decide_raw(eng_, &b, raw, 0, st.nd, dec_out_.data(), dec_thr_.data())) {
      fail(st.calls);
      return;
    }
    out = dec_out_.data();
    thr = dec_thr_.data();
  } else if (rl_wait_view(eng_, &out, &thr)) {
    fail(st.calls);
    return;
  }
  size_t d = 0;
  for (size_t r = 0; r < st.calls.size(); ++r) {
    PendingCall& c = *st.calls[r];
    if (fc_) {
      // a reply past the limit Sets the key with TTL = the unit's divider (base_limiter.go:94-106),
      // shadow rules included (the limiter does not know them), before the caller is released
      std::lock_guard<std::mutex> g(fc_mu_);
      for (size_t i = 0; i < c.prefix.size(); ++i) {
        const auto& lim = (*c.limits)[i];
        if (!lim || c.lhit[i]) continue;
        const uint32_t cf = out[d + i].code_flags;
        if ((cf & 0xFFu) == RL_CODE_OVER_LIMIT || ((cf >> 8) & RL_FLAG_SHADOW))
          fc_->Set(c.fkey[i], unit_divider(lim->Limit.unit), (uint32_t)c.now);
      }
    }
    answer(c, out + d, thr[r]);
    d += c.prefix.size();
  }
  done_calls(st.calls.size());
}

void HipRateLimitCache::local_cache_stats(uint64_t* out) {
  for (int k = 0; k < 6; ++k) out[k] = 0;
  std::lock_guard<std::mutex> g(fc_mu_);
  if (fc_) fc_->stats(out);
}

// The submitter thread owns the engine (rl_hip.h: one thread per engine) and keeps two batches
// in flight, as the Go batcher does: batch k+1 is gathered, built in its
// pinned slot and submitted (its H2D copy and fingerprint overlap batch k's kernels) before
// batch k's results are collected; with nothing queued it finishes what is in flight instead
// of waiting. Gathering lasts up to batch_window_us (implicit pipelining analogue,
// src/redis/driver_impl.go:84-89).
void HipRateLimitCache::submitter() {
  std::deque<Staged> inflight;
  std::shared_ptr<PendingCall> carry;
  for (;;) {
    std::shared_ptr<PendingCall> first = std::move(carry);
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
    st.seq = staged_seq_++;
    st.compact = compactable(*first);
    if (st.compact ? rl_host_acquire_c(eng_, &st.hc) : rl_host_acquire(eng_, &st.hb)) {
      std::vector<std::shared_ptr<PendingCall>> one{first};
      fail(one);
      continue;
    }
    st.max_desc = st.compact ? st.hc.max_desc : st.hb.max_desc;
    st.max_req = st.compact ? st.hc.max_req : st.hb.max_req;
    st.max_blob = st.compact ? st.hc.max_blob : st.hb.max_blob;
    if (first->prefix.size() > st.max_desc || first->blob_bytes > st.max_blob) {
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
          std::shared_ptr<PendingCall> c = q_.front();
          q_.pop_front();
          if (!fits(st, *c)) {
            carry = std::move(c);  // starts the next batch
            goto full;
          }
          add(st, c);
        }
        if (stop_ || st.nd >= s_.batch_limit) break;
        if (!inflight.empty() && s_.answer_early) {
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

// ---- HipRoutedRateLimitCache ------------------------------------------------------------
struct HipRoutedRateLimitCache::Step {
  std::vector<std::shared_ptr<PendingCall>> calls;
  uint32_t nd = 0, nr = 0, nb = 0;
  int64_t tmin = 0, tmax = 0;
};

namespace {
// One rank's words in a rule / stop agreement (rl_router_allgather_host, RL_ROUTER_AG_MAX bytes).
constexpr uint32_t SYNC_RULES = (RL_ROUTER_AG_MAX - 8) / sizeof(rl_rule);
struct SyncWords {
  uint32_t stop, n;
  rl_rule rules[SYNC_RULES];
};
static_assert(sizeof(SyncWords) <= RL_ROUTER_AG_MAX, "sync words");
std::pair<uint32_t, uint32_t> limit_key(const RateLimit& r) {
  return {r.Limit.RequestsPerUnit, (uint32_t)r.Limit.unit | (r.ShadowMode ? RL_RULE_SHADOW : 0u)};
}
}  // namespace

HipRoutedRateLimitCache::HipRoutedRateLimitCache(const HipSettings& s, const HipRoutedSettings& r,
                                                 std::shared_ptr<TimeSource> ts)
    : s_(s), r_(r), ts_(std::move(ts)) {
  jitter_ = setup_jitter(s_);
  if (r.id.size() != RL_ROUTER_ID_BYTES) throw RedisError("routed cache: id must hold RL_ROUTER_ID_BYTES bytes");
  if (s.local_cache && s.local_cache_freecache)
    throw RedisError("routed cache: HIP_LOCAL_CACHE=freecache is single-engine only (the device cache is the routed one)");
  rl_config c;
  memset(&c, 0, sizeof c);
  c.struct_size = sizeof c;
  c.device = s.device;
  for (int u = 0; u < 4; ++u) c.log2_slots[u] = s.log2_slots[u];
  c.near_limit_ratio = s.near_limit_ratio;
  c.local_cache = s.local_cache ? 1 : 0;
  c.per_second_split = s.per_second_split ? 1 : 0;
  // an owner may receive every origin's whole batch (a key hot everywhere)
  c.max_batch_desc = s.batch_limit * r.n_shards;
  c.max_batch_req = s.batch_limit * r.n_shards;
  c.max_blob_bytes = s.batch_limit * 128u;
  c.hash_seed = s.hash_seed;
  c.max_load_permille = s.max_load_permille;
  int rc = rl_create(&c, &eng_);
  if (rc) throw RedisError("rl_create failed: " + std::to_string(rc) + ": " + rl_last_error(nullptr));
  rl_router_config rc2;
  memset(&rc2, 0, sizeof rc2);
  rc2.struct_size = sizeof rc2;
  rc2.n_shards = r.n_shards;
  rc2.rank = r.rank;
  rc2.max_desc = s.batch_limit;
  rc2.rccl_id = r.id.data();
  rc2.flags = RL_ROUTER_HOST | (r.emulated ? RL_ROUTER_EMULATED : 0u);
  rc2.max_blob_bytes = s.batch_limit * 128u;
  rl_engine* es[1] = {eng_};
  rc = rl_router_create(&rc2, es, &rt_);
  if (rc) {
    rl_destroy(eng_);
    throw RedisError("rl_router_create failed: " + std::to_string(rc));
  }
  thr_ = std::thread([this] { submitter(); });
}

HipRoutedRateLimitCache::~HipRoutedRateLimitCache() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  thr_.join();
  rl_router_destroy(rt_);
  rl_destroy(eng_);
}

void HipRoutedRateLimitCache::Flush() {
  std::unique_lock<std::mutex> g(mu_);
  idle_cv_.wait(g, [&] { return inflight_ == 0; });
}

DoLimitResponse HipRoutedRateLimitCache::DoLimit(const RateLimitRequest& request,
                                                 const std::vector<std::shared_ptr<RateLimit>>& limits) {
  auto call = make_call(request, limits, *ts_);
  std::future<void> f = call->done.get_future();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (broken_) throw RedisError("hip backend: " + broken_msg_);
    q_.push_back(call);
    ++inflight_;
  }
  cv_.notify_one();
  f.get();  // rethrows RedisError
  return std::move(call->resp);
}

void HipRoutedRateLimitCache::done_calls(size_t n) {
  {
    std::lock_guard<std::mutex> g(mu_);
    inflight_ -= n;
  }
  idle_cv_.notify_all();
}

void HipRoutedRateLimitCache::fail(std::vector<std::shared_ptr<PendingCall>>& calls, const std::string& msg) {
  for (auto& c : calls) c->done.set_exception(std::make_exception_ptr(RedisError("hip backend: " + msg)));
  done_calls(calls.size());
  calls.clear();
}

// Every limit of the call has an agreed id; otherwise its new limits are queued for the next sync.
bool HipRoutedRateLimitCache::known(const PendingCall& c) {
  bool ok = true;
  for (const auto& lim : *c.limits) {
    if (!lim) continue;
    const auto k = limit_key(*lim);
    if (ids_.count(k)) continue;
    ok = false;
    if (pending_set_.insert(k).second) pending_.push_back(rl_rule{k.first, k.second});
  }
  return ok;
}

// The rule / stop agreement (nothing in flight on any rank): every rank's new limits appended to
// every rank's table in rank order (the first occurrence keeps its id), loaded into the engine.
// Returns true when every rank asked to stop.
bool HipRoutedRateLimitCache::sync(bool want_stop) {
  SyncWords mine;
  memset(&mine, 0, sizeof mine);
  mine.stop = want_stop ? 1u : 0u;
  mine.n = (uint32_t)std::min<size_t>(pending_.size(), SYNC_RULES);
  std::copy(pending_.begin(), pending_.begin() + mine.n, mine.rules);
  std::vector<SyncWords> all(r_.n_shards);
  int rc = rl_router_allgather_host(rt_, &mine, sizeof mine, all.data());
  if (rc) throw RedisError(std::string("rule agreement: ") + rl_router_last_error(rt_));
  n_syncs_ += 1;
  bool all_stop = true;
  const size_t before = rules_.size();
  for (const SyncWords& w : all) {
    all_stop &= w.stop != 0;
    for (uint32_t i = 0; i < w.n; ++i) {
      const auto k = std::make_pair(w.rules[i].requests_per_unit, w.rules[i].unit);
      if (ids_.emplace(k, (uint32_t)rules_.size()).second) rules_.push_back(w.rules[i]);
    }
  }
  for (uint32_t i = 0; i < mine.n; ++i)
    pending_set_.erase(std::make_pair(pending_[i].requests_per_unit, pending_[i].unit));
  pending_.erase(pending_.begin(), pending_.begin() + mine.n);
  if (rules_.size() != before) {
    rc = rl_load_rules(eng_, rules_.data(), (uint32_t)rules_.size());
    if (rc) throw RedisError(std::string("rl_load_rules: ") + rl_last_error(eng_));
    n_rules_ = rules_.size();
  }
  return all_stop;
}

// The rank's step loop: rule / stop agreement every rule_sync_every steps (nothing in flight),
// otherwise gather for one step period, submit (an empty batch when idle), two steps in flight.
void HipRoutedRateLimitCache::submitter() {
  std::deque<Step> fl;
  std::deque<std::shared_ptr<PendingCall>> held;  // calls waiting for a rule agreement
  std::vector<rl_status> out;
  std::vector<uint32_t> thr;
  uint64_t seq = 0;
  auto finish_one = [&] {
    Step st = std::move(fl.front());
    fl.pop_front();
    out.resize(std::max<size_t>(1, st.nd));
    thr.resize(std::max<size_t>(1, st.nr));
    rl_status* o[1] = {out.data()};
    uint32_t* t[1] = {thr.data()};
    const int rc = rl_router_wait_into(rt_, o, t);
    if (rc) {
      if (rc == RL_ECOMM) {
        std::lock_guard<std::mutex> g(mu_);
        broken_ = true;
        broken_msg_ = rl_router_last_error(rt_);
      }
      fail(st.calls, rl_router_last_error(rt_));
      return;
    }
    size_t d = 0;
    for (size_t r = 0; r < st.calls.size(); ++r) {
      PendingCall& c = *st.calls[r];
      answer(c, out.data() + d, thr[r]);
      d += c.prefix.size();
    }
    done_calls(st.calls.size());
  };
  auto fail_all = [&](const std::string& msg) {
    while (!fl.empty()) {
      fail(fl.front().calls, msg);
      fl.pop_front();
    }
    std::vector<std::shared_ptr<PendingCall>> rest(held.begin(), held.end());
    held.clear();
    {
      std::lock_guard<std::mutex> g(mu_);
      broken_ = true;
      broken_msg_ = msg;
      rest.insert(rest.end(), q_.begin(), q_.end());
      q_.clear();
    }
    fail(rest, msg);
  };
  try {
    for (;;) {
      if (broken_) break;
      if (seq % r_.rule_sync_every == 0) {
        while (!fl.empty()) finish_one();
        bool want_stop;
        {
          std::lock_guard<std::mutex> g(mu_);
          want_stop = stop_ && q_.empty() && held.empty();
        }
        if (sync(want_stop)) break;  // every rank stops here
        if (!held.empty()) {  // calls whose limits are agreed now go back to the front, in order
          std::lock_guard<std::mutex> g(mu_);
          for (auto it = held.rbegin(); it != held.rend(); ++it) q_.push_front(*it);
          held.clear();
        }
      }
      Step st;
      rl_host_batch hb;
      if (rl_router_host_acquire(rt_, 0, &hb)) throw RedisError(rl_router_last_error(rt_));
      {
        std::unique_lock<std::mutex> g(mu_);
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(r_.step_us);
        for (;;) {
          while (!q_.empty()) {
            std::shared_ptr<PendingCall> cp = q_.front();
            PendingCall& c = *cp;
            if (!known(c)) {  // waits for the next agreement
              held.push_back(cp);
              q_.pop_front();
              n_held_ += 1;
              continue;
            }
            const int64_t lo = st.calls.empty() ? c.now : std::min(st.tmin, c.now);
            const int64_t hi = st.calls.empty() ? c.now : std::max(st.tmax, c.now);
            // one batch straddles at most one window boundary (hi - lo < 2), and fits the slot
            if (hi - lo >= 2 || st.nd + c.prefix.size() > s_.batch_limit || st.nd + c.prefix.size() > hb.max_desc ||
                st.nr + 1 > hb.max_req || st.nb + c.blob_bytes > hb.max_blob)
              goto full;
            q_.pop_front();
            st.tmin = lo;
            st.tmax = hi;
            const uint32_t rq = st.nr++;
            if (trace_) trace_(c.req, seq, rq);
            hb.now[rq] = c.now;
            hb.hits_addend[rq] = c.req->HitsAddend;
            hb.prefix_off[0] = 0;
            for (size_t i = 0; i < c.prefix.size(); ++i) {
              const auto& lim = (*c.limits)[i];
              memcpy(hb.prefix_blob + st.nb, c.prefix[i].data(), c.prefix[i].size());
              st.nb += (uint32_t)c.prefix[i].size();
              hb.rule_id[st.nd] = lim ? ids_.at(limit_key(*lim)) : RL_NIL_RULE;
              hb.req_of[st.nd] = rq;
              if (jitter_) hb.ttl_jitter[st.nd] = lim ? draw_jitter(s_) : 0;
              ++st.nd;
              hb.prefix_off[st.nd] = st.nb;
            }
            st.calls.push_back(cp);
          }
          if (st.nd >= s_.batch_limit) break;
          if (cv_.wait_until(g, deadline) == std::cv_status::timeout) break;
          if (std::chrono::steady_clock::now() >= deadline) break;
        }
      full:;
      }
      rl_batch b;
      memset(&b, 0, sizeof b);
      b.n_desc = st.nd;
      b.n_req = st.nr;
      b.blob_bytes = st.nb;
      if (st.nd || st.nr) {
        b.prefix_blob = hb.prefix_blob;  // the router's pinned slot: staged without a copy
        b.prefix_off = hb.prefix_off;
        b.rule_id = hb.rule_id;
        b.req_of = hb.req_of;
        b.now = hb.now;
        b.hits_addend = hb.hits_addend;
        b.ttl_jitter = jitter_ ? hb.ttl_jitter : nullptr;
      } else {
        n_empty_ += 1;  // an idle rank still takes part in the step's collectives
      }
      const int rc = rl_router_submit_host(rt_, &b);
      ++seq;
      n_steps_ += 1;
      if (rc) {  // refused before its collectives (a broken communicator): this rank cannot step on
        const std::string msg = rl_router_last_error(rt_);
        fail(st.calls, msg);
        throw RedisError(msg);
      }
      fl.push_back(std::move(st));
      if (fl.size() == 2) finish_one();
    }
  } catch (const RedisError& e) {
    fail_all(e.what());
  }
  while (!fl.empty()) finish_one();
}

}  // namespace ratelimit
