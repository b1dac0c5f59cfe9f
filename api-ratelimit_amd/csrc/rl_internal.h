// rl_internal.h — host-side pieces shared by the engine (rl_engine.cpp) and the router
// (rl_router.cpp) inside libratelimit_hip.so; not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "rl_common.h"
#include "rl_hip.h"

namespace rlhip {

// A hot key prefix (host side): fingerprint lanes after the prefix bytes, its unit and rule,
// and how many descriptors carried it in the batch it was counted on.
struct HotKey {
  uint64_t a, b;
  uint32_t unit, rule, count;
};

// The device hot-set table (rl_common.h HOT_TAGS): open-addressed tag words (home =
// hot_home(a), word = hot_tag(a) | index + 1) followed by the entries in index order.
inline void build_hot_table(const std::vector<HotKey>& hot, std::vector<HotEntry>& t) {
  t.assign(HOT_SLOTS + HOT_MAX, HotEntry{});
  for (auto& x : t) x.idx = 0xFFFFFFFFu;
  std::vector<uint32_t> tags(HOT_TAGS, 0u);
  static_assert(HOT_MAX < 512 && (size_t)HOT_TAGS * 4 == HOT_SLOTS * sizeof(HotEntry), "hot tag words");
  for (size_t i = 0; i < hot.size() && i < (size_t)HOT_MAX; ++i) {
    HotEntry he{};
    he.a = hot[i].a;
    he.b = hot[i].b;
    he.unit = hot[i].unit;
    he.rule = hot[i].rule;
    he.idx = (uint32_t)i;
    uint32_t s = hot_home(he.a);
    while (tags[s]) s = (s + 1) & (HOT_TAGS - 1);
    tags[s] = hot_tag(he.a) | (uint32_t)(i + 1);
    t[HOT_SLOTS + i] = he;
  }
  memcpy(t.data(), tags.data(), (size_t)HOT_TAGS * 4);
}

// What the router needs from an engine (rl_engine.cpp).
struct EngineView {
  const DevRule* rules;
  uint32_t n_rules;
  uint64_t seed;
  int local_cache;
  int device;
  uint32_t max_batch_desc;
};
int rlx_engine_view(rl_engine* e, EngineView* v);
// A router's engine keeps SECOND key strings findable up to 3 s behind its newest time
// (TableDesc.lag, rl_common.h slot_free_for). Set by rl_router_create once the router exists
// (dry: only the check); RL_ESTATE for an engine that decided batches without it.
int rlx_engine_set_lag(rl_engine* e, bool dry);
// The engine's current hot set (keys it owns that arrive with many descriptors per batch).
void rlx_engine_hot(rl_engine* e, std::vector<HotKey>& out);

// ---- combining route kernels (rl_route.hip) ----------------------------------------------
// Per origin batch of a routed step: records grouped by owner in a strided send buffer
// (owner j at [j * stride, ...)), cold descriptors one record each in arrival order, then one
// combined record per hot prefix group (the hot set's prefixes, when combining is on and the
// batch's hot descriptors share one request time); per owner (count, status) pairs in x.
struct RoutePackBufs {
  RRec* send;          // n_shards * stride records
  uint32_t* perm;      // per descriptor: record position | PERM_HOT group code | RL_ROUTE_LOCAL
  uint32_t* x;         // [xs * n_shards]: (count, status[, tmin, tmax]) per owner
  uint32_t* lb;        // look-back words + error word, two areas (pack, repack), zeroed by the caller
  uint32_t* bhs;       // [blocks][HOT_MAX] hot h sums per block -> exclusive prefixes over blocks
  uint32_t* bstat;     // [blocks][4] per block: ~min now, max now, flags of its hot descriptors
  uint32_t* rctl;      // [16] step words: [0] repack (combining refused), [1] combined records, [2] done ctr;
                       // then the hot scan's look-back words (route2_hot_lb_words), then its u64 sums
  uint32_t* hot_pos;   // [HOT_MAX] record position of each hot group's combined record
  uint32_t* hot_tot;   // [HOT_MAX] its sum of hits_addend
  uint32_t* h_hot;     // pinned host [HOT_MAX + 2]: group sums, repack flag, applied flag (k_route_hot_scan)
  uint32_t* thr;       // the origin's ThrottleMillis output: zeroed by the pack (nullable)
  uint32_t zero_words; // lb / rctl words the unpack clears for the slot's next step (from lb)
  uint32_t xs;         // words per owner in x: 2 = (count, status); 4 = (count, status, tmin, tmax)
  uint32_t* tr;        // [8][64] zeroed: the pack blocks' request-time range words (xs = 4)
};
uint32_t route2_blocks(uint32_t n);
size_t route2_lb_words(uint32_t n);     // one area
size_t route2_bhs_words(uint32_t n);
size_t route2_hot_lb_words();          // the hot scan's look-back words (after rctl[16], zeroed with it)
// hot == nullptr: no combining
void launch_route_pack2(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                        uint32_t origin, uint32_t n_shards, uint32_t stride, const HotEntry* hot,
                        const RoutePackBufs& o);
// Origin: raw replies (back, strided like send) -> statuses and ThrottleMillis (the decisions).
// owner_status: per owner its decide status (device; nonzero: that owner applied nothing and its
// descriptors come out RL_CODE_UNKNOWN); stride: the owners' section size in back. h_status
// (pinned host words, may be null): the n_shards owner statuses copied there by the kernel.
// Launches nothing for an empty batch.
// Test fault (RL_ROUTER_FAULT=stall): holds the stream until *release becomes non-zero (pinned
// host word) or 20 s pass.
void launch_router_stall(hipStream_t st, const uint32_t* release);
void launch_route_unpack_raw(hipStream_t st, const rl_batch& b, const DevRule* rules, const RoutePackBufs& o,
                             const RawReply* back, const int32_t* owner_status, uint32_t stride, rl_status* out,
                             uint32_t* thr, int32_t* h_status = nullptr, uint32_t n_shards = 0);
constexpr uint32_t ROUTE2_BLOCK = 1024;  // descriptors per pack block
constexpr uint32_t PERM_HOT = 0x80000000u;
constexpr int PERM_HOT_PRE_BITS = 22;

}  // namespace rlhip
