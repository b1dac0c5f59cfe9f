// rl_router.cpp — the routed DoLimit step behind the C ABI (include/rl_hip.h
// "Router object").
//
// The reference sends each key's INCRBY to the Redis server that holds it and pipelines the
// commands of a request (src/redis/fixed_cache_impl.go:66-80, src/redis/driver_impl.go:84-110).
// Here GPU s owns the keys whose prefix fingerprint maps to s (route_owner). One step:
//   origin   pack its batch by owner into a strided send buffer: one record per descriptor,
//            except hot prefixes (the shard's route hot set), whose descriptors travel as ONE
//            combined record per prefix carrying their sum of hits_addend (rl_route.hip)
//   exchange per-owner (count, status) pairs, then the records (all-to-all)
//   owner    decide the records received from every origin, in origin order, answering each
//            with its raw INCRBY post-value (rl_submit_routed_async, RL_ROUTED_RAW)
//   exchange the owners' statuses and the raw replies (reverse all-to-all)
//   origin   every descriptor's post-value from its record's reply (and, inside a combined
//            record, its prefix of hits_addend), then its decision (k_route_unpack_raw)
//
// Transports: RCCL (one process per GPU, ncclAllToAll / ncclAllToAllv / ncclAllGather on a
// stream the router owns) or local (n_shards engines in one process, device copies). Status
// words ride in the counts exchange (pack) and the reply exchange (decide, and any local HIP
// failure after the counts), so every shard completes every collective of a step and all of
// them fail together.
//
// Two steps may be in flight (rl_router_submit / rl_router_wait): step k+1's pack, counts and
// record exchange run on the origin and exchange streams while step k's owner batch is decided
// on the engine's streams (the engine pipelines routed batches like rl_submit_pipelined).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include "rl_common.h"
#include "rl_hip.h"
#include "rl_internal.h"

using namespace rlhip;

namespace {

constexpr uint32_t REC = sizeof(RRec);
constexpr uint32_t RAWB = sizeof(RawReply);
constexpr uint32_t MAXS = RL_ROUTE_MAX_SHARDS;
constexpr int NSLOT = 2;                   // steps in flight
constexpr uint64_t ROUTE_HOT_EVERY = 8;    // route hot set refresh period (steps)
constexpr uint32_t ROUTE_HOT_KEEP = 64;    // a group stays while its origin sends it >= this sum of hits per step
static_assert(REC == RL_ROUTE_RECORD_BYTES && RAWB == sizeof(rl_raw_reply), "record layouts");
constexpr uint32_t HX_HOT = 8 * MAXS;      // pinned mirror: hot sums, then the control words

// Host wait for an event by polling: a blocking stream synchronize sleeps and wakes 10-20 us
// after the GPU is done, on the routed step's critical path between exchanges.
hipError_t poll_event(hipEvent_t ev) {
  for (int k = 0; k < (1 << 20); ++k) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
  }
  return hipEventSynchronize(ev);
}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Fault injection for the tests (RL_ROUTER_FAULT="phase:shard", read at create, fires once):
// the shard behaves as if a HIP call of that phase failed.
enum Phase { PH_NONE = 0, PH_PACK, PH_RECORDS, PH_DECIDE, PH_REPLIES, PH_UNPACK };

// One hot-set entry as exchanged between ranks (32 B): an owner's hot prefix.
struct AgEntry {
  uint64_t a, b;
  uint32_t unit, rule, count, pad;
};
static_assert(sizeof(AgEntry) == 32, "allgather entry");

// Pinned + device staging of one shard's host batch (RL_ROUTER_HOST), the engine's layout.
struct HostStage {
  uint8_t* h_in = nullptr;
  uint8_t* d_in = nullptr;
  rl_status* d_out = nullptr;
  rl_status* h_out = nullptr;
  uint32_t* d_thr = nullptr;
  uint32_t* h_thr = nullptr;
};

// One shard's part of one step in flight.
struct ShardStep {
  RoutePackBufs pb{};
  uint8_t* zero = nullptr;    // look-back areas + control words: clear before every pack
  size_t zero_bytes = 0;
  bool zeroed = true;         // the unpack cleared them (else the next pack memsets first)
  RRec* recv = nullptr;       // owner: records from every origin
  RawReply* reply = nullptr;  // owner: one raw reply per received record
  RawReply* back = nullptr;   // origin: replies to its records, strided like send
  int32_t* d_x = nullptr;     // [2G] pairs sent | [2G] received | [G] statuses sent | [G] received
  int32_t* h_x = nullptr;     // pinned mirror; at HX_HOT the hot sums, then the control words
  HostStage hs;
  rl_batch b{};               // the origin batch (device pointers)
  rl_status* out = nullptr;
  uint32_t* thr = nullptr;
  uint32_t cnt[MAXS] = {};    // records this origin sends each owner
  uint32_t rcv[MAXS] = {};    // records this owner receives from each origin
  uint32_t n_in = 0;
  int rc_pack = 0, rc_dec = 0, rc_local = 0;
  std::string msg;
  const char* phase = "";     // where msg comes from: pack, records, decide, replies, unpack
  bool submitted = false;     // owner batch handed to the engine (rl_wait pending)
  bool combined = false;
};

struct Shard {
  rl_engine* e = nullptr;
  EngineView v{};
  hipStream_t os = nullptr;   // origin work: staging copies, pack, hot scan, unpack
  hipEvent_t ev = nullptr;    // os -> exchange stream
  ShardStep st[NSLOT];
  // route hot set (this shard as origin)
  std::vector<HotKey> hot;
  HotEntry* d_hot = nullptr;
  HotEntry* h_hot = nullptr;
  hipEvent_t ev_hot = nullptr;
  uint32_t last_tot[HOT_MAX] = {};  // sums of hits per group, last step that combined
  bool last_valid = false;
  bool repacked = false;            // since the last refresh
};

struct StepSlot {
  bool busy = false;
  bool host = false;
  bool counts_failed = false;  // every shard left after the counts exchange
  double t0 = 0;
  int32_t status[MAXS] = {};   // per shard (RCCL: as received from every origin / owner)
};

}  // namespace

struct rl_router {
  rl_router_config cfg{};
  bool rccl = false, broken = false;
  ncclComm_t comm = nullptr;
  hipStream_t rs = nullptr;  // exchanges
  hipEvent_t ev_rs = nullptr;
  hipEvent_t ev_cnt = nullptr;  // the counts' host copy
  hipEvent_t ev_end = nullptr;  // the reply exchange (rs) and the unpack (os) of the step
  std::vector<Shard> sh;
  StepSlot slot[NSLOT];
  uint64_t seq = 0, done = 0;
  double t_pack0 = 0;        // start of the current submit's packs (host clock)
  size_t in_bytes = 0, o_off = 0, o_rule = 0, o_req = 0, o_now = 0, o_hits = 0;  // host staging layout
  AgEntry* d_ag = nullptr;   // RCCL hot-set allgather: [HOT_MAX] send | [G * HOT_MAX] receive
  AgEntry* h_ag = nullptr;
  int fault_phase = PH_NONE;
  uint32_t fault_shard = 0;
  rl_router_stats st{};
  std::string err;

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  // RCCL failure: abort the communicator (its peers' collectives return), every later call fails
  int nccl_fail(ncclResult_t nr, const char* what) {
    if (comm) (void)ncclCommAbort(comm);
    comm = nullptr;
    broken = true;
    return fail(RL_ECOMM, "%s: %s (communicator aborted)", what, ncclGetErrorString(nr));
  }
  bool fault(int phase, uint32_t s) {
    if (fault_phase != phase || fault_shard != s) return false;
    fault_phase = PH_NONE;
    return true;
  }
  uint32_t n_local() const { return (uint32_t)sh.size(); }
  uint32_t shard_id(uint32_t s) const { return rccl ? cfg.rank : s; }

  int alloc_shard(Shard& s);
  void free_all();
  int validate(const rl_batch& b) const;
  int stage_host(uint32_t s, uint32_t k, const rl_batch& hb, rl_batch& db);
  void pack(uint32_t s, uint32_t k);
  void note_combine(uint32_t s, uint32_t k);
  void refresh_hot();
  int submit(const rl_batch* batches, rl_status* const* out, uint32_t* const* thr, bool host);
  int wait(rl_status* const* out, uint32_t* const* thr, bool into);
  int submit_rccl(uint32_t k);
  int submit_local(uint32_t k);
  void wait_rccl(uint32_t k);
  void wait_local(uint32_t k);
  int step_result(uint32_t k);
};

void rl_router::free_all() {
  for (Shard& s : sh) {
    for (ShardStep& t : s.st) {
      for (void* p : {(void*)t.pb.send, (void*)t.pb.perm, (void*)t.pb.bhs, (void*)t.pb.bstat, (void*)t.zero,
                      (void*)t.pb.hot_pos, (void*)t.recv, (void*)t.reply, (void*)t.back, (void*)t.d_x,
                      (void*)t.hs.d_in, (void*)t.hs.d_out, (void*)t.hs.d_thr})
        if (p) (void)hipFree(p);
      for (void* p : {(void*)t.h_x, (void*)t.hs.h_in, (void*)t.hs.h_out, (void*)t.hs.h_thr})
        if (p) (void)hipHostFree(p);
    }
    if (s.d_hot) (void)hipFree(s.d_hot);
    if (s.h_hot) (void)hipHostFree(s.h_hot);
    if (s.ev_hot) (void)hipEventDestroy(s.ev_hot);
    if (s.ev) (void)hipEventDestroy(s.ev);
    if (s.os) (void)hipStreamDestroy(s.os);
  }
  sh.clear();
  if (d_ag) (void)hipFree(d_ag);
  if (h_ag) (void)hipHostFree(h_ag);
  if (comm) (void)ncclCommDestroy(comm);
  for (hipEvent_t e : {ev_rs, ev_cnt, ev_end})
    if (e) (void)hipEventDestroy(e);
  if (rs) (void)hipStreamDestroy(rs);
  d_ag = nullptr;
  h_ag = nullptr;
  comm = nullptr;
  ev_rs = ev_cnt = ev_end = nullptr;
  rs = nullptr;
}

int rl_router::alloc_shard(Shard& s) {
  const uint32_t G = cfg.n_shards;
  const size_t D = cfg.max_desc;
  hipError_t he = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && he == hipSuccess) he = x; };
  chk(hipStreamCreateWithFlags(&s.os, hipStreamNonBlocking));
  chk(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
  chk(hipEventCreateWithFlags(&s.ev_hot, hipEventDisableTiming));
  chk(hipMalloc(&s.d_hot, sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX)));
  chk(hipHostMalloc(&s.h_hot, sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX), hipHostMallocDefault));
  if (he == hipSuccess) chk(hipEventRecord(s.ev_hot, s.os));
  const size_t lbw = route2_lb_words((uint32_t)D);
  for (ShardStep& t : s.st) {
    chk(hipMalloc(&t.pb.send, D * G * REC));
    chk(hipMalloc(&t.pb.perm, D * 4 + 64));
    chk(hipMalloc(&t.pb.bhs, route2_bhs_words((uint32_t)D) * 4 + 64));
    chk(hipMalloc(&t.pb.bstat, (size_t)route2_blocks((uint32_t)D) * 16 + 64));
    chk(hipMalloc(&t.pb.hot_pos, (size_t)HOT_MAX * 8));  // hot_pos | hot_tot
    t.pb.hot_tot = t.pb.hot_pos + HOT_MAX;
    // zeroed per step: two look-back areas and the control words; the hot scan's u64 sums follow
    t.zero_bytes = (2 * lbw + 16 + route2_hot_lb_words()) * 4;
    chk(hipMalloc(&t.zero, t.zero_bytes + (size_t)HOT_MAX * 8 + 64));
    t.pb.lb = reinterpret_cast<uint32_t*>(t.zero);
    t.pb.rctl = t.pb.lb + 2 * lbw;
    t.pb.zero_words = (uint32_t)(t.zero_bytes / 4);
    if (he == hipSuccess) chk(hipMemset(t.zero, 0, t.zero_bytes));
    t.zeroed = true;
    chk(hipMalloc(&t.recv, D * G * REC));
    chk(hipMalloc(&t.reply, D * G * RAWB));
    chk(hipMalloc(&t.back, D * G * RAWB));
    chk(hipMalloc(&t.d_x, 8 * MAXS * 4));
    chk(hipHostMalloc(&t.h_x, (HX_HOT + HOT_MAX + 16) * 4, hipHostMallocDefault));
    t.pb.x = reinterpret_cast<uint32_t*>(t.d_x);
    t.pb.h_hot = reinterpret_cast<uint32_t*>(t.h_x + HX_HOT);
    if (cfg.flags & RL_ROUTER_HOST) {
      chk(hipMalloc(&t.hs.d_in, in_bytes));
      chk(hipHostMalloc(&t.hs.h_in, in_bytes, hipHostMallocDefault));
      chk(hipMalloc(&t.hs.d_out, D * sizeof(rl_status) + 64));
      chk(hipHostMalloc(&t.hs.h_out, D * sizeof(rl_status) + 64, hipHostMallocDefault));
      chk(hipMalloc(&t.hs.d_thr, D * 4 + 64));
      chk(hipHostMalloc(&t.hs.h_thr, D * 4 + 64, hipHostMallocDefault));
    }
  }
  return he == hipSuccess ? 0 : fail(RL_EHIP, "router allocation: %s", hipGetErrorString(he));
}

int rl_router::validate(const rl_batch& b) const {
  if (b.n_desc > cfg.max_desc) return RL_ECAPACITY;
  if (b.reserved || b.n_req > RL_ROUTE_MAX_REQ || (b.n_desc && !b.n_req)) return RL_EINVAL;
  if (b.n_desc && (!b.prefix_blob || !b.prefix_off || !b.rule_id || !b.req_of)) return RL_EINVAL;
  if (b.n_req && (!b.now || !b.hits_addend)) return RL_EINVAL;
  return 0;
}

// Host batch -> the slot's pinned staging (unless the caller built it there) -> device, on the
// shard's origin stream ahead of its pack.
int rl_router::stage_host(uint32_t s, uint32_t k, const rl_batch& b, rl_batch& d) {
  ShardStep& t = sh[s].st[k];
  uint8_t* h = t.hs.h_in;
  if ((size_t)b.blob_bytes + RL_BLOB_SLACK > o_off || b.n_desc > cfg.max_desc || b.n_req > cfg.max_desc)
    return RL_ECAPACITY;
  struct Arr { const void* src; size_t o, n; } arrs[] = {
      {b.prefix_blob, 0, b.blob_bytes}, {b.prefix_off, o_off, b.n_desc ? ((size_t)b.n_desc + 1) * 4 : 0},
      {b.rule_id, o_rule, (size_t)b.n_desc * 4}, {b.req_of, o_req, (size_t)b.n_desc * 4},
      {b.now, o_now, (size_t)b.n_req * 8}, {b.hits_addend, o_hits, (size_t)b.n_req * 4}};
  for (auto& a : arrs)
    if (a.n && a.src != h + a.o) memcpy(h + a.o, a.src, a.n);
  memset(h + b.blob_bytes, 0, RL_BLOB_SLACK);  // the device reads prefixes in 16-B words
  const size_t ext[] = {(size_t)b.blob_bytes + RL_BLOB_SLACK, arrs[1].n, arrs[2].n, arrs[3].n, arrs[4].n, arrs[5].n};
  hipError_t he = hipSuccess;
  for (int q = 0; q < 6 && he == hipSuccess; ++q)
    if (ext[q]) he = hipMemcpyAsync(t.hs.d_in + arrs[q].o, h + arrs[q].o, ext[q], hipMemcpyHostToDevice, sh[s].os);
  if (he != hipSuccess) return RL_EHIP;
  d = b;
  d.prefix_blob = t.hs.d_in;
  d.prefix_off = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_off);
  d.rule_id = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_rule);
  d.req_of = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_req);
  d.now = reinterpret_cast<const int64_t*>(t.hs.d_in + o_now);
  d.hits_addend = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_hits);
  return 0;
}

// Origin pack of shard s for slot k on its origin stream: the (count, status) pairs land in
// d_x[0, 2G) and, with combining, the groups' sums and the control words in the pinned mirror.
void rl_router::pack(uint32_t s, uint32_t k) {
  Shard& S = sh[s];
  ShardStep& t = S.st[k];
  const uint32_t G = cfg.n_shards;
  t.combined = false;
  auto send_status = [&](int32_t rc) {  // pairs (0, rc) to every owner
    for (uint32_t j = 0; j < G; ++j) {
      t.h_x[2 * j] = 0;
      t.h_x[2 * j + 1] = rc;
    }
    (void)hipMemcpyAsync(t.d_x, t.h_x, 8 * G, hipMemcpyHostToDevice, S.os);
  };
  if (t.rc_pack || !t.b.n_desc) {
    if (!t.rc_pack && t.b.n_req && t.thr) (void)hipMemsetAsync(t.thr, 0, (size_t)t.b.n_req * 4, S.os);
    send_status(t.rc_pack);
    return;
  }
  const bool combine = !(cfg.flags & RL_ROUTER_NO_COMBINE) && !S.v.local_cache && !S.hot.empty();
  if (!t.zeroed) (void)hipMemsetAsync(t.zero, 0, t.zero_bytes, S.os);  // (the slot's last step had no unpack)
  t.pb.thr = t.thr;  // zeroed by the pack
  // the hot scan writes the group sums and its verdict straight into the pinned mirror
  launch_route_pack2(S.os, t.b, S.v.rules, S.v.n_rules, S.v.seed, shard_id(s), G, cfg.max_desc,
                     combine ? S.d_hot : nullptr, t.pb);
  t.zeroed = false;
  t.combined = combine;
  const hipError_t he = hipGetLastError();
  if (he != hipSuccess || fault(PH_PACK, s)) {  // the pack cannot be trusted: fail the step everywhere
    t.rc_pack = RL_EHIP;
    t.msg = he != hipSuccess ? std::string("route pack: ") + hipGetErrorString(he) : "injected fault (pack)";
    t.phase = "pack";
    t.combined = false;
    send_status(RL_EHIP);
  }
}

// After the counts: did shard s's pack combine (its groups' sums keep the route hot set), or
// did its batch need the repack (a hot group was not one key string)?
void rl_router::note_combine(uint32_t s, uint32_t k) {
  ShardStep& t = sh[s].st[k];
  if (!t.combined) return;
  const uint32_t* ctl = reinterpret_cast<const uint32_t*>(t.h_x + HX_HOT + HOT_MAX);  // k_route_hot_scan
  if (ctl[0] || !ctl[1]) {
    if (s == 0) ++st.repacks;
    sh[s].repacked = true;
    t.combined = false;
  } else {
    memcpy(sh[s].last_tot, t.h_x + HX_HOT, sizeof sh[s].last_tot);
    sh[s].last_valid = true;
    if (s == 0) ++st.combined_steps;
  }
}

// Route hot set refresh (every ROUTE_HOT_EVERY steps, at the same step on every shard): keep the
// groups this origin still sends with >= ROUTE_HOT_KEEP hits per step, add the owners' hot keys
// (each engine's own hot set: prefixes that reach it with many records per batch; over RCCL
// gathered from every rank), up to HOT_MAX. A shard that had to repack starts over.
void rl_router::refresh_hot() {
  std::vector<HotKey> cand;
  if (rccl) {
    std::vector<HotKey> mine;
    rlx_engine_hot(sh[0].e, mine);
    for (uint32_t i = 0; i < HOT_MAX; ++i) {
      AgEntry& a = h_ag[i];
      memset(&a, 0, sizeof a);
      if (i < mine.size()) a = AgEntry{mine[i].a, mine[i].b, mine[i].unit, mine[i].rule, std::max(1u, mine[i].count), 0};
    }
    const size_t n = HOT_MAX * sizeof(AgEntry);
    hipError_t he = hipMemcpyAsync(d_ag, h_ag, n, hipMemcpyHostToDevice, rs);
    const ncclResult_t nr = ncclAllGather(d_ag, d_ag + HOT_MAX, n, ncclUint8, comm, rs);
    if (nr != ncclSuccess) {
      nccl_fail(nr, "ncclAllGather(hot sets)");
      return;
    }
    if (he == hipSuccess) he = hipMemcpyAsync(h_ag + HOT_MAX, d_ag + HOT_MAX, n * cfg.n_shards, hipMemcpyDeviceToHost, rs);
    if (he == hipSuccess) he = hipStreamSynchronize(rs);
    if (he != hipSuccess) return;  // keep the current sets (decisions do not depend on them)
    for (uint32_t i = 0; i < HOT_MAX * cfg.n_shards; ++i) {
      const AgEntry& a = h_ag[HOT_MAX + i];
      if (a.count) cand.push_back(HotKey{a.a, a.b, a.unit, a.rule, a.count});
    }
  } else {
    for (Shard& s : sh) {
      std::vector<HotKey> h;
      rlx_engine_hot(s.e, h);
      cand.insert(cand.end(), h.begin(), h.end());
    }
  }
  std::stable_sort(cand.begin(), cand.end(), [](const HotKey& x, const HotKey& y) { return x.count > y.count; });
  for (Shard& s : sh) {
    std::vector<HotKey> next;
    std::unordered_set<uint64_t> seen;
    if (!s.repacked && s.last_valid)
      for (size_t i = 0; i < s.hot.size(); ++i)
        if (s.last_tot[i] >= ROUTE_HOT_KEEP) {
          HotKey k = s.hot[i];
          k.count = s.last_tot[i];
          seen.insert(k.a);
          next.push_back(k);
        }
    for (const HotKey& c : cand) {
      if (next.size() >= (size_t)HOT_MAX) break;
      if (!seen.insert(c.a).second) continue;  // (a prefix seen with a second rule: the pack repacks)
      next.push_back(c);
    }
    s.repacked = false;
    bool same = next.size() == s.hot.size();
    for (size_t i = 0; same && i < next.size(); ++i)
      same = next[i].a == s.hot[i].a && next[i].b == s.hot[i].b && next[i].rule == s.hot[i].rule;
    if (same) continue;
    std::vector<HotEntry> t;
    build_hot_table(next, t);
    // the staging's previous copy is done; the next pack is ordered behind this copy on os
    if (hipEventSynchronize(s.ev_hot) != hipSuccess) continue;
    memcpy(s.h_hot, t.data(), sizeof(HotEntry) * t.size());
    if (hipMemcpyAsync(s.d_hot, s.h_hot, sizeof(HotEntry) * t.size(), hipMemcpyHostToDevice, s.os) != hipSuccess)
      continue;
    (void)hipEventRecord(s.ev_hot, s.os);
    s.hot = std::move(next);
    s.last_valid = false;
  }
}

// RCCL: counts (+ pack statuses), then records; the owner batch is handed to the engine.
int rl_router::submit_rccl(uint32_t k) {
  const uint32_t G = cfg.n_shards, me = cfg.rank;
  Shard& S = sh[0];
  ShardStep& t = S.st[k];
  const double t0 = t_pack0;
  hipError_t he = hipEventRecord(S.ev, S.os);
  if (he == hipSuccess) he = hipStreamWaitEvent(rs, S.ev, 0);
  ncclResult_t nr = ncclAllToAll(t.d_x, t.d_x + 2 * G, 2, ncclInt32, comm, rs);
  if (nr != ncclSuccess) return nccl_fail(nr, "ncclAllToAll(counts)");
  if (he == hipSuccess) he = hipMemcpyAsync(t.h_x, t.d_x, 16 * G, hipMemcpyDeviceToHost, rs);
  if (he == hipSuccess) he = hipEventRecord(ev_cnt, rs);
  if (he == hipSuccess) he = poll_event(ev_cnt);
  if (he != hipSuccess) {  // the counts are unknown: nobody can take part in the record exchange
    broken = true;
    if (comm) (void)ncclCommAbort(comm);
    comm = nullptr;
    return fail(RL_ECOMM, "counts exchange: %s (communicator aborted)", hipGetErrorString(he));
  }
  const int32_t* hs = t.h_x;
  const int32_t* hr = t.h_x + 2 * G;
  if (!t.rc_pack && hs[1]) {  // the device refused the pack (one status in every owner's pair)
    t.rc_pack = hs[1];
    t.msg = t.rc_pack == RL_EDEVICE ? "route pack: the device's look-back spin limit expired (device fault)"
                                    : "route pack: batch references an unknown rule id or request index, malformed "
                                      "prefix offsets, or a time outside [0, 0xFFFD0000]";
    t.phase = "pack";
  }
  st.pack_us = now_us() - t0;
  bool any = false;
  for (uint32_t j = 0; j < G; ++j) {
    t.cnt[j] = t.rc_pack ? 0u : (uint32_t)hs[2 * j];
    t.rcv[j] = (uint32_t)hr[2 * j];
    slot[k].status[j] = hr[2 * j + 1];
    any |= hr[2 * j + 1] != 0;
  }
  if (any) {  // every rank saw the same status words: all leave after this exchange
    slot[k].counts_failed = true;
    return 0;
  }
  note_combine(0, k);
  // records: to owner j this origin's section j (stride D); from origin j its count, compact
  const size_t D = cfg.max_desc;
  std::vector<size_t> sc(G), sd(G), rc(G), rd(G);
  uint64_t ro = 0;
  for (uint32_t j = 0; j < G; ++j) {
    sc[j] = (size_t)t.cnt[j] * REC;
    sd[j] = j * D * REC;
    rc[j] = (size_t)t.rcv[j] * REC;
    rd[j] = ro;
    ro += rc[j];
    st.sent[j] = t.cnt[j];
  }
  t.n_in = (uint32_t)(ro / REC);
  for (uint32_t j = 0; j < G; ++j) st.recv[j] = j == me ? t.n_in : 0;
  nr = ncclAllToAllv(t.pb.send, sc.data(), sd.data(), t.recv, rc.data(), rd.data(), ncclUint8, comm, rs);
  if (nr != ncclSuccess) return nccl_fail(nr, "ncclAllToAllv(records)");
  const double t1 = now_us();
  he = hipEventRecord(ev_rs, rs);
  if (fault(PH_RECORDS, 0)) he = hipErrorUnknown;
  if (he != hipSuccess) {  // keep going: the failure travels in the reply exchange
    t.rc_local = RL_EHIP;
    t.msg = std::string("record exchange: ") + (he == hipErrorUnknown ? "injected fault (records)" : hipGetErrorString(he));
    t.phase = "records";
  } else if (t.n_in) {
    ShardStep& prev = S.st[k ^ 1u];
    t.rc_dec = rl_submit_routed_async(S.e, t.recv, t.n_in, t.reply, RL_ROUTED_RAW, ev_rs);
    if (t.rc_dec == RL_ESTATE && prev.submitted) {
      // an engine that cannot pipeline (LSD only): finish the previous owner batch first
      const int rp = rl_wait(S.e);
      if (rp) {
        prev.rc_dec = rp;
        prev.msg = rl_last_error(S.e);
        prev.phase = "decide";
      }
      prev.submitted = false;
      t.rc_dec = rl_submit_routed_async(S.e, t.recv, t.n_in, t.reply, RL_ROUTED_RAW, ev_rs);
    }
    if (t.rc_dec) {
      t.msg = rl_last_error(S.e);
      t.phase = "decide";
    }
    t.submitted = t.rc_dec == 0;
  }
  st.exchange_us = now_us() - t1;
  return 0;
}

// Local transport: every shard's counts on the host, records by device copies; the owners
// decide one after another, each timed alone (each models one GPU: decide_max_us is the step's
// critical path on G real GPUs).
int rl_router::submit_local(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  const double t0 = t_pack0;
  for (uint32_t s = 0; s < G; ++s) {
    ShardStep& t = sh[s].st[k];
    hipError_t he = hipMemcpyAsync(t.h_x, t.d_x, 8 * G, hipMemcpyDeviceToHost, sh[s].os);
    if (he == hipSuccess) he = hipStreamSynchronize(sh[s].os);
    if (he != hipSuccess && !t.rc_pack) {
      t.rc_pack = RL_EHIP;
      t.msg = std::string("counts: ") + hipGetErrorString(he);
      t.phase = "pack";
    }
    if (!t.rc_pack && t.h_x[1]) {
      t.rc_pack = t.h_x[1];
      t.msg = t.rc_pack == RL_EDEVICE ? "route pack: the device's look-back spin limit expired (device fault)"
                                      : "route pack: batch references an unknown rule id or request index, malformed "
                                        "prefix offsets, or a time outside [0, 0xFFFD0000]";
      t.phase = "pack";
    }
    slot[k].status[s] = t.rc_pack;
  }
  st.pack_us = now_us() - t0;
  bool any = false;
  for (uint32_t s = 0; s < G; ++s) any |= sh[s].st[k].rc_pack != 0;
  if (any) {
    slot[k].counts_failed = true;
    return 0;
  }
  for (uint32_t s = 0; s < G; ++s) {
    ShardStep& t = sh[s].st[k];
    for (uint32_t j = 0; j < G; ++j) t.cnt[j] = (uint32_t)t.h_x[2 * j];
    note_combine(s, k);
  }
  for (uint32_t j = 0; j < G; ++j) st.sent[j] = sh[0].st[k].cnt[j];
  const size_t D = cfg.max_desc;
  hipError_t he = hipSuccess;
  for (uint32_t j = 0; j < G; ++j) {  // owner j: origin 0's section j, then origin 1's, ...
    uint64_t o = 0;
    for (uint32_t i = 0; i < G; ++i) {
      const uint32_t c = sh[i].st[k].cnt[j];
      sh[j].st[k].rcv[i] = c;
      if (c && he == hipSuccess)
        he = hipMemcpyAsync(sh[j].st[k].recv + o, sh[i].st[k].pb.send + j * D, (size_t)c * REC,
                            hipMemcpyDeviceToDevice, rs);
      o += c;
    }
    sh[j].st[k].n_in = (uint32_t)o;
    st.recv[j] = (uint32_t)o;
  }
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  const double t1 = now_us();
  st.exchange_us = t1 - t0 - st.pack_us;
  st.decide_max_us = 0;
  for (uint32_t j = 0; j < G; ++j) {
    ShardStep& t = sh[j].st[k];
    if (he != hipSuccess || fault(PH_RECORDS, j)) {
      t.rc_local = RL_EHIP;
      t.msg = he != hipSuccess ? std::string("record exchange: ") + hipGetErrorString(he) : "injected fault (records)";
      t.phase = "records";
      continue;
    }
    const double a = now_us();
    if (t.n_in) {
      t.rc_dec = rl_submit_routed_async(sh[j].e, t.recv, t.n_in, t.reply, RL_ROUTED_RAW, nullptr);
      if (!t.rc_dec) t.rc_dec = rl_wait(sh[j].e);
      if (t.rc_dec) {
        t.msg = rl_last_error(sh[j].e);
        t.phase = "decide";
      }
    }
    st.decide_max_us = std::max(st.decide_max_us, now_us() - a);
  }
  st.decide_us = now_us() - t1;
  return 0;
}

int rl_router::submit(const rl_batch* batches, rl_status* const* out, uint32_t* const* thr, bool host) {
  if (broken) return fail(RL_ECOMM, "the router's communicator was aborted after a transport failure");
  const uint32_t k = (uint32_t)(seq % NSLOT);
  if (slot[k].busy) return fail(RL_ESTATE, "two routed steps in flight: call rl_router_wait");
  if (host && !(cfg.flags & RL_ROUTER_HOST)) return fail(RL_EINVAL, "router created without RL_ROUTER_HOST");
  const uint32_t G = cfg.n_shards, nl = n_local();
  if (!rccl)  // the local transport refuses a bad batch before anything moves (RCCL: in the counts exchange)
    for (uint32_t s = 0; s < G; ++s)
      if (batches[s].n_desc > cfg.max_desc)
        return fail(RL_ECAPACITY, "shard %u: batch of %u descriptors exceeds the router's max_desc %u", s,
                    batches[s].n_desc, cfg.max_desc);
  for (uint32_t j = 0; j < MAXS; ++j) st.recv[j] = 0, st.sent[j] = 0, slot[k].status[j] = 0;
  slot[k].t0 = now_us();
  t_pack0 = slot[k].t0;
  slot[k].host = host;
  slot[k].counts_failed = false;
  if (seq % ROUTE_HOT_EVERY == 0) {
    refresh_hot();
    if (broken) return RL_ECOMM;
  }
  for (uint32_t s = 0; s < nl; ++s) {
    Shard& S = sh[s];
    ShardStep& t = S.st[k];
    t.rc_pack = t.rc_dec = t.rc_local = 0;
    t.msg.clear();
    t.phase = "";
    t.submitted = false;
    t.n_in = 0;
    t.rc_pack = validate(batches[s]);
    if (t.rc_pack) {
      t.msg = "bad origin batch (capacity, reserved, request count or null arrays)";
      t.phase = "pack";
    }
    if (host) {
      t.out = t.hs.d_out;
      t.thr = t.hs.d_thr;
      if (!t.rc_pack) {
        t.rc_pack = stage_host(s, k, batches[s], t.b);
        if (t.rc_pack) {
          t.msg = "host staging (capacity)";
          t.phase = "pack";
        }
      }
      if (t.rc_pack) t.b = rl_batch{};
    } else {
      t.b = batches[s];
      t.out = out[s];
      t.thr = thr[s];
      if (t.rc_pack) t.b = rl_batch{};
    }
    const int rc = rlx_engine_view(S.e, &S.v);  // (rules may have been appended since)
    if (rc && !t.rc_pack) {
      t.rc_pack = rc;
      t.msg = rl_last_error(S.e);
      t.phase = "pack";
    }
    pack(s, k);
    // local transport (logical shards on one device): one origin's pack at a time, so
    // pack_us / G is one origin's pack (as on G GPUs)
    if (!rccl) (void)hipStreamSynchronize(S.os);
  }
  slot[k].busy = true;
  ++seq;
  return rccl ? submit_rccl(k) : submit_local(k);
}

// The step's outcome from each shard's status: the first failing shard's code on that shard
// (local transport: returned), RL_EPEER on the others.
int rl_router::step_result(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  for (uint32_t j = 0; j < MAXS; ++j) st.status[j] = j < G ? slot[k].status[j] : 0;
  int bad = -1;
  for (uint32_t j = 0; j < G && bad < 0; ++j)
    if (st.status[j]) bad = (int)j;
  if (bad < 0) return 0;
  const int code = st.status[bad];
  for (uint32_t j = 0; j < G; ++j)
    if (st.status[j] == 0) st.status[j] = RL_EPEER;
  if (rccl && (uint32_t)bad != cfg.rank) {
    const int32_t own = st.status[cfg.rank];
    const ShardStep& t = sh[0].st[k];
    if (own != RL_EPEER) return fail(own, "shard %u (%s): %s", cfg.rank, t.phase, t.msg.c_str());
    return fail(RL_EPEER, "shard %d failed this step with %d (see rl_router_stats.status)", bad, code);
  }
  const ShardStep& t = sh[rccl ? 0 : bad].st[k];
  return fail(code, "shard %d (%s): %s", bad, t.phase, t.msg.c_str());
}

void rl_router::wait_rccl(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  Shard& S = sh[0];
  ShardStep& t = S.st[k];
  const double t0 = now_us();
  if (t.submitted) {
    const int rc = rl_wait(S.e);
    if (rc) {
      t.rc_dec = rc;
      t.msg = rl_last_error(S.e);
      t.phase = "decide";
    }
    t.submitted = false;
  }
  if (!t.rc_dec && !t.rc_local && fault(PH_DECIDE, 0)) {
    t.rc_dec = RL_EHIP;
    t.msg = "injected fault (decide)";
    t.phase = "decide";
  }
  st.decide_us = st.decide_max_us = now_us() - t0;
  const double t1 = now_us();
  int32_t* hs = t.h_x + 4 * G;  // statuses sent | received
  int32_t mine = t.rc_dec ? t.rc_dec : t.rc_local;
  if (!mine && fault(PH_REPLIES, 0)) {
    mine = t.rc_local = RL_EHIP;
    t.msg = "injected fault (replies)";
    t.phase = "replies";
  }
  for (uint32_t j = 0; j < G; ++j) hs[j] = mine;
  hipError_t he = hipMemcpyAsync(t.d_x + 4 * G, hs, 4 * G, hipMemcpyHostToDevice, rs);
  // replies: to origin j the replies to its records (compact), into its back buffer at my section
  const size_t D = cfg.max_desc;
  std::vector<size_t> sc(G), sd(G), rc(G), rd(G);
  uint64_t so = 0;
  for (uint32_t j = 0; j < G; ++j) {
    sc[j] = (size_t)t.rcv[j] * RAWB;
    sd[j] = so;
    so += sc[j];
    rc[j] = (size_t)t.cnt[j] * RAWB;
    rd[j] = j * D * RAWB;  // perm = owner * D + position
  }
  ncclResult_t nr = ncclGroupStart();
  if (nr == ncclSuccess) nr = ncclAllToAll(t.d_x + 4 * G, t.d_x + 5 * G, 1, ncclInt32, comm, rs);
  if (nr == ncclSuccess)
    nr = ncclAllToAllv(t.reply, sc.data(), sd.data(), t.back, rc.data(), rd.data(), ncclUint8, comm, rs);
  const ncclResult_t ne = ncclGroupEnd();
  if (nr != ncclSuccess || ne != ncclSuccess) {
    nccl_fail(nr != ncclSuccess ? nr : ne, "ncclAllToAll(replies)");
    return;
  }
  if (he == hipSuccess) he = hipMemcpyAsync(t.h_x + 5 * G, t.d_x + 5 * G, 4 * G, hipMemcpyDeviceToHost, rs);
  if (he == hipSuccess) he = hipEventRecord(ev_rs, rs);
  if (he == hipSuccess) he = hipStreamWaitEvent(S.os, ev_rs, 0);
  st.reply_us = now_us() - t1;
  const double t2 = now_us();
  if (he == hipSuccess) {  // (the owners' statuses arrived with the replies, d_x[5G, 6G); thr zeroed by the pack)
    launch_route_unpack_raw(S.os, t.b, S.v.rules, t.pb, t.back, t.d_x + 5 * G, cfg.max_desc, t.out, t.thr);
    he = hipGetLastError();
    t.zeroed = he == hipSuccess && t.b.n_desc;
  }
  if (he == hipSuccess && slot[k].host) {
    if (t.b.n_desc)
      he = hipMemcpyAsync(t.hs.h_out, t.out, (size_t)t.b.n_desc * sizeof(rl_status), hipMemcpyDeviceToHost, S.os);
    if (he == hipSuccess && t.b.n_req) he = hipMemcpyAsync(t.hs.h_thr, t.thr, (size_t)t.b.n_req * 4, hipMemcpyDeviceToHost, S.os);
  }
  // the unpack waited for the reply exchange (ev_rs), so one event on os covers both streams;
  // after a failure to enqueue, drain both streams
  hipError_t h2;
  if (he == hipSuccess && hipEventRecord(ev_end, S.os) == hipSuccess) {
    h2 = poll_event(ev_end);
    he = h2;
  } else {
    h2 = hipStreamSynchronize(rs);
    if (he == hipSuccess) he = h2;
    if (he == hipSuccess) he = hipStreamSynchronize(S.os);
  }
  if (he == hipSuccess && fault(PH_UNPACK, 0)) he = hipErrorUnknown;
  st.unpack_us = now_us() - t2;
  for (uint32_t j = 0; j < G; ++j) slot[k].status[j] = h2 == hipSuccess ? t.h_x[5 * G + j] : RL_EHIP;
  if (he != hipSuccess) {  // after the last collective: only this shard's results are lost
    slot[k].status[cfg.rank] = RL_EHIP;
    t.msg = std::string("reply exchange / unpack: ") +
            (he == hipErrorUnknown ? "injected fault (unpack)" : hipGetErrorString(he));
    t.phase = "unpack";
  }
}

void rl_router::wait_local(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  const size_t D = cfg.max_desc;
  const double t0 = now_us();
  for (uint32_t j = 0; j < G; ++j) {
    ShardStep& t = sh[j].st[k];
    if (!t.rc_dec && !t.rc_local && fault(PH_DECIDE, j)) {
      t.rc_dec = RL_EHIP;
      t.msg = "injected fault (decide)";
      t.phase = "decide";
    }
    if (!t.rc_dec && !t.rc_local && fault(PH_REPLIES, j)) {
      t.rc_local = RL_EHIP;
      t.msg = "injected fault (replies)";
      t.phase = "replies";
    }
    slot[k].status[j] = t.rc_dec ? t.rc_dec : t.rc_local;
  }
  hipError_t he = hipSuccess;
  for (uint32_t j = 0; j < G; ++j) {  // owner j's replies, origin-major, into each origin's section j
    uint64_t o = 0;
    for (uint32_t i = 0; i < G; ++i) {
      const uint32_t c = sh[j].st[k].rcv[i];
      if (c && he == hipSuccess)
        he = hipMemcpyAsync(sh[i].st[k].back + j * D, sh[j].st[k].reply + o, (size_t)c * RAWB, hipMemcpyDeviceToDevice,
                            rs);
      o += c;
    }
  }
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  st.reply_us = now_us() - t0;
  const double t1 = now_us();
  for (uint32_t i = 0; i < G; ++i) {
    Shard& S = sh[i];
    ShardStep& t = S.st[k];
    hipError_t hu = he;
    // every owner's decide status into this origin's device words (as the RCCL reply exchange
    // delivers them)
    for (uint32_t j = 0; j < G; ++j) t.h_x[5 * G + j] = slot[k].status[j];
    if (hu == hipSuccess) hu = hipMemcpyAsync(t.d_x + 5 * G, t.h_x + 5 * G, 4 * G, hipMemcpyHostToDevice, S.os);
    if (hu == hipSuccess) {  // (thr zeroed by the pack)
      launch_route_unpack_raw(S.os, t.b, S.v.rules, t.pb, t.back, t.d_x + 5 * G, cfg.max_desc, t.out, t.thr);
      hu = hipGetLastError();
      t.zeroed = hu == hipSuccess && t.b.n_desc;
    }
    if (hu == hipSuccess && slot[k].host) {
      if (t.b.n_desc)
        hu = hipMemcpyAsync(t.hs.h_out, t.out, (size_t)t.b.n_desc * sizeof(rl_status), hipMemcpyDeviceToHost, S.os);
      if (hu == hipSuccess && t.b.n_req)
        hu = hipMemcpyAsync(t.hs.h_thr, t.thr, (size_t)t.b.n_req * 4, hipMemcpyDeviceToHost, S.os);
    }
    if (hu == hipSuccess) hu = hipStreamSynchronize(S.os);
    if (hu == hipSuccess && fault(PH_UNPACK, i)) hu = hipErrorUnknown;
    if (hu != hipSuccess && !slot[k].status[i]) {
      slot[k].status[i] = RL_EHIP;
      t.msg = std::string("reply exchange / unpack: ") +
              (hu == hipErrorUnknown ? "injected fault (unpack)" : hipGetErrorString(hu));
      t.phase = "unpack";
    }
  }
  st.unpack_us = now_us() - t1;
}

int rl_router::wait(rl_status* const* out, uint32_t* const* thr, bool into) {
  if (broken) return fail(RL_ECOMM, "the router's communicator was aborted after a transport failure");
  const uint32_t k = (uint32_t)(done % NSLOT);
  if (!slot[k].busy) return fail(RL_ESTATE, "rl_router_wait without a routed step in flight");
  if (!slot[k].counts_failed) {
    if (rccl) wait_rccl(k);
    else wait_local(k);
  }
  slot[k].busy = false;
  ++done;
  if (broken) return RL_ECOMM;
  const int rc = step_result(k);
  const ShardStep& t0s = sh[0].st[k];
  st.hot_groups = (uint32_t)sh[0].hot.size();
  st.combined = 0;
  if (t0s.combined)
    for (uint32_t i = 0; i < HOT_MAX; ++i) st.combined += t0s.h_x[HX_HOT + i] != 0 ? 1u : 0u;
  if (into && !rc && slot[k].host)
    for (uint32_t s = 0; s < n_local(); ++s) {
      const ShardStep& t = sh[s].st[k];
      if (out && out[s] && t.b.n_desc) memcpy(out[s], t.hs.h_out, (size_t)t.b.n_desc * sizeof(rl_status));
      if (thr && thr[s] && t.b.n_req) memcpy(thr[s], t.hs.h_thr, (size_t)t.b.n_req * 4);
    }
  st.step_us = now_us() - slot[k].t0;
  ++st.steps;
  return rc;
}

extern "C" {

int rl_router_unique_id(uint8_t* id_out) {
  if (!id_out) return RL_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RL_ECOMM;
  memcpy(id_out, &id, RL_ROUTER_ID_BYTES);
  return 0;
}

int rl_router_create(const rl_router_config* cfg, rl_engine* const* engines, rl_router** out) {
  if (!cfg || !engines || !out) return RL_EINVAL;
  *out = nullptr;
  if (cfg->struct_size != sizeof(rl_router_config)) return RL_EINVAL;
  const uint32_t G = cfg->n_shards;
  if (G == 0 || G > MAXS || cfg->max_desc == 0 || cfg->max_desc > (1u << 27)) return RL_EINVAL;
  if (cfg->flags & ~(uint32_t)(RL_ROUTER_NO_COMBINE | RL_ROUTER_HOST)) return RL_EINVAL;
  const bool rccl = cfg->rccl_id != nullptr;
  if (rccl && cfg->rank >= G) return RL_EINVAL;
  const uint32_t n_eng = rccl ? 1u : G;
  for (uint32_t s = 0; s < n_eng; ++s)
    if (!engines[s]) return RL_EINVAL;
  rl_router* r = new rl_router();
  r->cfg = *cfg;
  r->cfg.rccl_id = nullptr;
  r->rccl = rccl;
  r->st.n_shards = G;
  {
    const size_t N = cfg->max_desc, B = cfg->max_blob_bytes ? cfg->max_blob_bytes : (size_t)cfg->max_desc * 64;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    r->o_off = al(B + RL_BLOB_SLACK);
    r->o_rule = r->o_off + al((N + 1) * 4);
    r->o_req = r->o_rule + al(N * 4);
    r->o_now = r->o_req + al(N * 4);
    r->o_hits = r->o_now + al(N * 8);
    r->in_bytes = r->o_hits + al(N * 4);
  }
  if (const char* f = getenv("RL_ROUTER_FAULT")) {  // tests: "phase:shard"
    static const char* const names[] = {"", "pack", "records", "decide", "replies", "unpack"};
    char ph[32] = {0};
    unsigned s = 0;
    if (sscanf(f, "%31[a-z]:%u", ph, &s) == 2)
      for (int p = 1; p <= PH_UNPACK; ++p)
        if (!strcmp(ph, names[p])) {
          r->fault_phase = p;
          r->fault_shard = rccl ? (s == cfg->rank ? 0u : 0xFFFFFFFFu) : s;
        }
  }
  auto bail = [&](int code) {
    r->free_all();
    delete r;
    return code;
  };
  if (hipStreamCreateWithFlags(&r->rs, hipStreamNonBlocking) != hipSuccess) return bail(RL_EHIP);
  if (hipEventCreateWithFlags(&r->ev_rs, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&r->ev_cnt, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&r->ev_end, hipEventDisableTiming) != hipSuccess)
    return bail(RL_EHIP);
  r->sh.resize(n_eng);
  for (uint32_t s = 0; s < n_eng; ++s) {
    r->sh[s].e = engines[s];
    if (rlx_engine_view(engines[s], &r->sh[s].v)) return bail(RL_EINVAL);
    if (r->alloc_shard(r->sh[s])) return bail(RL_EHIP);
  }
  if (rccl) {
    if (hipMalloc(&r->d_ag, sizeof(AgEntry) * HOT_MAX * (G + 1)) != hipSuccess ||
        hipHostMalloc(&r->h_ag, sizeof(AgEntry) * HOT_MAX * (G + 1), hipHostMallocDefault) != hipSuccess)
      return bail(RL_EHIP);
    ncclUniqueId id;
    memcpy(&id, cfg->rccl_id, RL_ROUTER_ID_BYTES);
    if (ncclCommInitRank(&r->comm, (int)G, id, (int)cfg->rank) != ncclSuccess) {
      r->comm = nullptr;
      return bail(RL_ECOMM);
    }
  }
  *out = r;
  return 0;
}

int rl_router_submit(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_thr) {
  if (!r || !batches || !d_out || !d_thr) return RL_EINVAL;
  return r->submit(batches, d_out, d_thr, false);
}

int rl_router_wait(rl_router* r) {
  if (!r) return RL_EINVAL;
  return r->wait(nullptr, nullptr, false);
}

int rl_router_step(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_thr) {
  const int rc = rl_router_submit(r, batches, d_out, d_thr);
  if (rc) return rc;
  return rl_router_wait(r);
}

int rl_router_host_acquire(rl_router* r, uint32_t shard, rl_host_batch* out) {
  if (!r || !out) return RL_EINVAL;
  if (!(r->cfg.flags & RL_ROUTER_HOST)) return r->fail(RL_EINVAL, "router created without RL_ROUTER_HOST");
  if (shard >= r->n_local()) return r->fail(RL_EINVAL, "shard %u out of range", shard);
  const uint32_t k = (uint32_t)(r->seq % NSLOT);
  if (r->slot[k].busy) return r->fail(RL_ESTATE, "two routed steps in flight: call rl_router_wait_into");
  uint8_t* h = r->sh[shard].st[k].hs.h_in;
  out->prefix_blob = h;
  out->prefix_off = reinterpret_cast<uint32_t*>(h + r->o_off);
  out->rule_id = reinterpret_cast<uint32_t*>(h + r->o_rule);
  out->req_of = reinterpret_cast<uint32_t*>(h + r->o_req);
  out->now = reinterpret_cast<int64_t*>(h + r->o_now);
  out->hits_addend = reinterpret_cast<uint32_t*>(h + r->o_hits);
  out->max_desc = r->cfg.max_desc;
  out->max_req = r->cfg.max_desc;
  out->max_blob = (uint32_t)(r->o_off - RL_BLOB_SLACK);
  out->reserved = 0;
  return 0;
}

int rl_router_submit_host(rl_router* r, const rl_batch* host_batches) {
  if (!r || !host_batches) return RL_EINVAL;
  return r->submit(host_batches, nullptr, nullptr, true);
}

int rl_router_wait_into(rl_router* r, rl_status* const* out, uint32_t* const* thr) {
  if (!r) return RL_EINVAL;
  return r->wait(out, thr, true);
}

int rl_router_get_stats(const rl_router* r, rl_router_stats* out) {
  if (!r || !out) return RL_EINVAL;
  *out = r->st;
  return 0;
}

const char* rl_router_last_error(const rl_router* r) { return r ? r->err.c_str() : "null router"; }

void rl_router_destroy(rl_router* r) {
  if (!r) return;
  // steps still in flight: complete them (every rank issued their collectives)
  while (!r->broken && r->done < r->seq) (void)r->wait(nullptr, nullptr, false);
  for (Shard& s : r->sh) (void)hipStreamSynchronize(s.os);
  if (r->rs) (void)hipStreamSynchronize(r->rs);
  r->free_all();
  delete r;
}

}  // extern "C"
