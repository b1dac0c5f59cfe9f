// rl_common.h — shared device/host definitions of the HIP rate-limit pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_hip.h"

namespace rlhip {

// ---------------------------------------------------------------------------
// Key identity. A Redis key is the exact byte string of
// GenerateCacheKey (src/limiter/cache_key.go:57-68) = prefix || decimal(window_start).
// The prefix always ends in '_' and the decimal has none, so (prefix bytes,
// window_start) <-> key string is a bijection; the fingerprint hashes exactly those two
// parts and nothing else: a MINUTE key "p_3600" and an HOUR key "p_3600" are one string,
// hence one table slot, exactly as they are one freecache entry (base_limiter.go:57-66)
// and — without REDIS_PERSECOND, or for MINUTE/HOUR/DAY always — one Redis counter
// (fixed_cache_impl.go:74-85). The slot holds both stores' counters.
// Two 64-bit lanes over 8-byte little-endian words (tail zero-padded, length folded in).
// Each lane step is a bijection of the lane state for a fixed word, so two equal-length
// prefixes that differ anywhere give different lane-a states.
// ---------------------------------------------------------------------------
constexpr uint64_t K0 = 0x9E3779B97F4A7C15ull;
constexpr uint64_t K1 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t K2 = 0x165667B19E3779F9ull;
constexpr uint64_t K3 = 0xD6E8FEB86659FD93ull;
constexpr uint64_t K4 = 0xFF51AFD7ED558CCDull;
constexpr uint64_t K5 = 0xC4CEB9FE1A85EC53ull;

__host__ __device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t x) {
  x ^= x >> 33; x *= K4; x ^= x >> 33; x *= K5; x ^= x >> 33;
  return x;
}
struct FpState { uint64_t a, b; };
__host__ __device__ __forceinline__ FpState fp_init(uint32_t len, uint64_t seed) {
  return FpState{seed ^ K0, (seed + K1) ^ ((uint64_t)len << 32)};
}
__host__ __device__ __forceinline__ void fp_word(FpState& s, uint64_t w) {
  s.a = rotl64((s.a ^ w) * K2, 31);
  s.b = (s.b + w) * K3;
  s.b ^= s.b >> 29;
}
// Identity = (sort key: region | hi >> 3, lo & 0xFFFFFFFF): 93 bits.
__host__ __device__ __forceinline__ void fp_final(FpState s, uint64_t window_start, uint64_t& hi, uint64_t& lo) {
  s.a ^= window_start * K1;
  s.b = (s.b ^ window_start) * K2;
  hi = fmix64(s.a + rotl64(s.b, 23));
  lo = fmix64(s.b ^ (s.a * K5)) & 0xFFFFFFFFull;
}

// Units (rl_hip.h RL_UNIT_*): divider = utils.UnitToDivider (src/utils/utilities.go:19-32)
__host__ __device__ __forceinline__ uint32_t unit_div(uint32_t unit) {
  return unit == RL_UNIT_SECOND ? 1u : unit == RL_UNIT_MINUTE ? 60u : unit == RL_UNIT_HOUR ? 3600u : 86400u;
}

// Home unit of a key string: the largest unit whose divider divides its window start.
// Every unit that can produce the string divides it, so all of them are <= home, and every
// touch of the string happens inside the home unit's window [ws, ws + div(home)).
__host__ __device__ __forceinline__ uint32_t home_unit(uint32_t ws) {
  return ws % 86400u == 0 ? (uint32_t)RL_UNIT_DAY
         : ws % 3600u == 0 ? (uint32_t)RL_UNIT_HOUR
         : ws % 60u == 0   ? (uint32_t)RL_UNIT_MINUTE
                           : (uint32_t)RL_UNIT_SECOND;
}
// Table region (home unit x window parity) and window generation (home window index + 1)
// of a key string.
struct Place { uint32_t region, gen; };
__host__ __device__ __forceinline__ Place place_of(uint32_t ws) {
  const uint32_t H = home_unit(ws);
  const uint32_t w = ws / unit_div(H);
  return Place{(H - 1u) * 2u + (w & 1u), w + 1u};
}
// Window start of every key of (region, gen).
__host__ __device__ __forceinline__ uint32_t region_ws(uint32_t region, uint32_t gen) {
  return (gen - 1u) * unit_div(region / 2u + 1u);
}
// Latest admissible request time: ws + div and t + div stay below 2^32.
constexpr int64_t MAX_NOW = 0xFFFD0000ll;

// Sort key: [region:3 | fingerprint.hi >> 3]. ~0 marks nil-limit descriptors, which sort
// last and are decided without the table.
constexpr uint64_t NIL_KEY = ~0ull;
__host__ __device__ __forceinline__ uint64_t make_sort_key(uint32_t region, uint64_t hi) {
  uint64_t k = ((uint64_t)region << 61) | (hi >> 3);
  return k == NIL_KEY ? NIL_KEY - 1 : k;
}
__host__ __device__ __forceinline__ uint32_t key_region(uint64_t k) { return (uint32_t)(k >> 61); }

// Per-descriptor record written by the LSD fingerprint kernel in arrival order (32 B).
struct __attribute__((aligned(16))) ItemRec {
  uint64_t fp_lo;    // low fingerprint lane (identity = (sort key, fp_lo))
  uint32_t rule;     // rule id or RL_NIL_RULE
  uint32_t req;      // request index
  uint32_t h;        // max(1, hits_addend)
  int32_t now_mod;   // now - window_start (CalculateReset: div - now % div)
  uint32_t gen;      // home window index + 1 (0 = never-used slot)
  uint32_t jit;      // EXPIRE jitter, seconds (rl_batch.ttl_jitter / the routed record's)
};

// Per-descriptor record in sorted order written by the LSD scan kernel (32 B).
struct __attribute__((aligned(16))) SortedRec {
  uint64_t P;        // inclusive prefix sum of h within the key's segment (exotic keys: the
                     // leader overwrites it with the INCRBY reply | local-hit << 32)
  uint32_t head;     // sorted position of the segment head; bit31: rule changes within segment so far
  uint32_t idx;      // arrival index
  uint32_t rule;
  uint32_t req;
  uint32_t h;
  int32_t now_mod;
};
constexpr uint32_t HEAD_MIXED_RULE = 0x80000000u;

// Per-segment decision state written by the leader at the segment head (16 B).
struct __attribute__((aligned(16))) SegInfo {
  uint64_t base;     // counter before this batch (INCRBY post-value = base + P)
  uint32_t freeze;   // SEG_NO_FREEZE, SEG_FROZEN_BEFORE, SEG_EXOTIC, or the request R* that froze the key
  uint32_t pad;
};
constexpr uint32_t SEG_NO_FREEZE = 0xFFFFFFFFu;
constexpr uint32_t SEG_FROZEN_BEFORE = 0xFFFFFFFEu;
constexpr uint32_t SEG_EXOTIC = 0xFFFFFFFDu;  // per-descriptor replies (P = reply | local-hit << 32)
constexpr uint64_t P_LOCAL_HIT = 1ull << 32;

// Counter-table slot (32 B): one Redis key string. word0 = gen | tag << 32 is the claim word.
//   count/exp: the main store's counter (int64 in Redis, observed as uint32: fixed_cache_impl.go:51)
//              and its expiry second (alive while now < exp; 0 = absent);
//   pcount:    the per-second store's counter (REDIS_PERSECOND; only SECOND keys use it, all at
//              now == window start, so its TTL never decides an outcome);
//   frz:       the local over-limit cache entry of the string (freecache TTL = div of the rule
//              that went over, base_limiter.go:102): frozen while now < frz; 0 = none.
struct __attribute__((aligned(32))) Slot {
  uint64_t ctrl;     // gen (low 32) | tag = (uint32)fp_lo (high 32)
  uint64_t key;      // sort key (region | fp.hi >> 3)
  uint32_t count;
  uint32_t exp;
  uint32_t pcount;
  uint32_t frz;
};
static_assert(sizeof(Slot) == 32, "Slot is 32 B");

// Rule table entry on the device.
struct __attribute__((aligned(16))) DevRule {
  uint32_t L;        // requests_per_unit
  uint32_t near;     // uint32(floor(float64(float32(L) * ratio)))  base_limiter.go:86
  uint32_t div;      // UnitToDivider
  uint32_t unit;
  uint32_t shadow;   // 1: RL_RULE_SHADOW (OVER_LIMIT reported as OK + RL_FLAG_SHADOW)
  uint32_t pad[3];
};

// Shadow mode (rl_hip.h RL_RULE_SHADOW): an OVER_LIMIT code becomes OK with RL_FLAG_SHADOW.
__host__ __device__ inline uint32_t shadow_code(uint32_t code_flags, uint32_t shadow) {
  return (shadow && (code_flags & 0xFFu) == RL_CODE_OVER_LIMIT)
             ? ((code_flags & ~0xFFu) | RL_CODE_OK | (RL_FLAG_SHADOW << 8))
             : code_flags;
}

// The decision from the INCRBY reply (after) or a local-cache hit: GetResponseDescriptorStatus
// + checkOverLimitThreshold + checkNearLimitThreshold + CalculateReset (base_limiter.go:70-195,
// utilities.go:34-38). Returns the ThrottleMillis contribution (0 = none). Host and device share
// it: the device decides every status form, the host a compact batch's raw replies (rl_decide_raw).
__host__ __device__ inline uint32_t decide_status(uint32_t after, bool local_hit, uint32_t h, uint32_t now_mod, const DevRule& R,
                              rl_status& st) {
  const uint32_t reset = R.div - now_mod;  // div - now % div
  st.reset_s = reset;
  st.over_limit_delta = 0;
  st.near_limit_delta = 0;
  uint32_t throttle = 0;
  if (local_hit) {
    st.code_flags = RL_CODE_OVER_LIMIT | ((RL_FLAG_HAS_LIMIT | RL_FLAG_LOCAL_CACHE_HIT) << 8);
    st.limit_remaining = 0;
    st.over_limit_delta = h;
  } else {
    const uint32_t before = after - h;
    const uint32_t L = R.L, near = R.near;
    if (after > L) {
      st.code_flags = RL_CODE_OVER_LIMIT | (RL_FLAG_HAS_LIMIT << 8);
      st.limit_remaining = 0;
      if (before >= L) {
        st.over_limit_delta = h;
      } else {
        st.over_limit_delta = after - L;
        st.near_limit_delta = L - (near > before ? near : before);
      }
    } else {
      st.code_flags = RL_CODE_OK | (RL_FLAG_HAS_LIMIT << 8);
      st.limit_remaining = L - after;
      if (after > near) {
        const uint32_t millis = reset * 1000u;  // uint32(end - now) * 1000
        const uint32_t calls = (L - after) > 1u ? (L - after) : 1u;
        throttle = millis / calls;
        st.near_limit_delta = before >= near ? h : after - near;
      }
    }
  }
  st.code_flags = shadow_code(st.code_flags, R.shadow);
  return throttle;
}

// Device error flags (bitmask in EngineCtl.err).
enum : uint32_t {
  ERR_TABLE_FULL = 1u,    // a region would pass its load limit: refused before any table write
  ERR_SPIN = 2u,
  ERR_NEED_RESORT = 4u,   // a sort-prefix run holds two different fingerprints
  ERR_BAD_TIME = 8u,
  ERR_BAD_INPUT = 16u,    // rule id or request index out of range
  ERR_WINDOW_SPAN = 32u,  // a region saw window generations more than one apart in one batch
  ERR_FALLBACK = 64u,     // the bucketed pipeline cannot take this batch: rerun it on the LSD pipeline
};

// Small device control block, zeroed per batch. Same-line atomics serialise at the L2
// (~9 ns each on MI355X, measured), so every word that more than one block writes is
// either written once by a single reducer block or lives on a 256-B line of its own.
struct EngineCtl {
  uint32_t err;          // atomicOr, only on an error
  uint32_t n_nil;        // nil-limit descriptors (sorted to the tail)
  uint32_t n_segments;   // unique keys in the batch (U)
  uint32_t n_inserted;   // new table slots of the batch (all regions)
  uint32_t gen_min[8];   // per region: min window generation in the batch
  uint32_t gen_max[8];   // per region: max window generation in the batch
  uint32_t ins[8];       // per region: new table slots of the batch
  uint32_t pad0[64 - 28];
  uint32_t tile_ctr[32][64];  // dynamic tile tickets / hand-off counters, one 256-B line each
};
static_assert(sizeof(EngineCtl) == 256 + 32 * 256, "EngineCtl layout");
// tile_ctr rows 16..23: per-region new-slot counters of the LSD leader (row INS_CTR0 + region)
constexpr int INS_CTR0 = 16;
constexpr int INS_LINES = 8;

// Per-block fingerprint partials: ~min / max home generation per region, nil count,
// max unit window + 1 per (unit, window parity) (hot keys), descriptors per region.
constexpr int FP_GMIN = 0, FP_GMAX = 8, FP_NIL = 16, FP_UW = 17, FP_CNT = 25;
constexpr int FP_PART_WORDS = 33;
__host__ __device__ __forceinline__ bool fp_is_max(int w) { return w < FP_NIL || (w >= FP_UW && w < FP_CNT); }

// Counter table: 8 regions (home unit x window parity), region r has 2^region_log2[r] slots.
struct TableDesc {
  Slot* slots;
  uint64_t region_base[8];  // slot offset of each region
  uint32_t region_log2[8];
  uint32_t split;           // REDIS_PERSECOND: SECOND rules count in the per-second store
  uint32_t local_cache;     // local over-limit cache on
  uint32_t lag;             // SECOND-home regions keep the previous generation live (routers' engines)
};
__host__ __device__ __forceinline__ bool per_second_store(const TableDesc& t, uint32_t unit) {
  return t.split && unit == RL_UNIT_SECOND;
}

// Per-region occupancy kept across batches (capacity check before any table write).
struct RegionOcc {
  uint32_t gen;    // window generation the count belongs to
  uint32_t live;   // slots claimed for that generation
  uint32_t limit;  // load limit (slots)
  uint32_t prev;   // SECOND-home regions: slots of the region's previous generation (gen - 2), still live
};

// Slot reuse (window expiry). A slot of an older window generation is free for a key of
// generation G. Engines driven by a router (rl_router_create sets TableDesc.lag) keep, in the
// two SECOND-home regions (a key string lives one second there), the region's previous
// generation live too — a slot is free only when its generation g satisfies g + 2 < G — so a
// request may come up to 3 s behind the newest time the table has seen (requests of several
// origins in rank order, a multi-GPU step whose origins' clocks or batch cuts differ,
// DESIGN.md §5c) and still find its key string. That costs the SECOND-home regions up to twice
// the live slots against the same load limit, so a lone engine (one batcher, times in enqueue
// order) runs without it. MINUTE/HOUR/DAY strings live a minute or more per generation: there
// the previous generation is already that far back.
__host__ __device__ __forceinline__ bool lazy_region(uint32_t lag, uint32_t region) { return lag && region < 2u; }
__host__ __device__ __forceinline__ bool slot_free_for(uint32_t g, uint32_t G, bool lazy) {
  return lazy ? (g == 0u || g + 2u < G) : g < G;
}
// Slots of a region that a key of generation `gen` cannot take (capacity check).
__host__ __device__ __forceinline__ uint32_t region_live(const RegionOcc& o, bool lazy, uint32_t gen) {
  if (!lazy) return o.gen < gen ? 0u : o.live;
  uint32_t v = 0;
  if (o.gen + 2u >= gen) v += o.live;  // generation o.gen >= gen - 2
  if (o.gen >= gen) v += o.prev;       // generation o.gen - 2 >= gen - 2
  return v;
}
// After a batch: its new slots `ins` of generation gm in a region (gm = 0: untouched).
__host__ __device__ __forceinline__ void occ_advance(RegionOcc& o, bool lazy, uint32_t gm, uint32_t ins) {
  if (!gm) return;
  if (o.gen < gm) {
    o.prev = (lazy && o.gen + 2u == gm) ? o.live : 0u;
    o.gen = gm;
    o.live = ins;
  } else if (lazy && o.gen == gm + 2u) {
    o.prev += ins;  // a batch behind the region's newest generation (its slots are generation gm)
  } else {
    o.live += ins;
  }
}

// Hot-key set entry: a key prefix seen with many descriptors per batch. (a, b) is the
// fingerprint lane state after the prefix bytes (length folded in), i.e. a 128-bit hash of
// the prefix bytes; the window is not part of it.
struct __attribute__((aligned(32))) HotEntry {
  uint64_t a, b;
  uint32_t unit;
  uint32_t rule;   // the rule id every descriptor of the prefix must carry (else the batch falls back)
  uint32_t idx;    // hot index 0..HOT_MAX-1; 0xFFFFFFFF = empty slot
  uint32_t pad;
};
constexpr int HOT_MAX = 256;              // hot prefixes per batch
// Hot-set table (device + LDS copy in k4_hist): HOT_TAGS u32 tag words (open addressing from
// the prefix state's low bits, load <= 1/8), in the space of HOT_SLOTS HotEntry units, then
// the HOT_MAX entries by hot index. Tag word = (a >> 32) with its low 9 bits replaced by
// hot index + 1 (0 = empty); a tag match is confirmed on the entry's full (a, b).
constexpr int HOT_SLOTS = 256;
constexpr int HOT_TAGS = HOT_SLOTS * 32 / 4;
constexpr uint32_t HOT_TAG_MASK = ~0x1FFu;
__host__ __device__ __forceinline__ uint32_t hot_tag(uint64_t a) { return (uint32_t)(a >> 32) & HOT_TAG_MASK; }
__host__ __device__ __forceinline__ uint32_t hot_home(uint64_t a) { return (uint32_t)a & (HOT_TAGS - 1); }
constexpr int HOT_BUCKETS = 2 * HOT_MAX;  // hot prefix x window parity
constexpr int MSD_BITS = 11;
constexpr int MSD_BUCKETS = 1 << MSD_BITS;   // 11 fingerprint bits below the region bits
constexpr int NBUCKETS = HOT_BUCKETS + MSD_BUCKETS + 1;
constexpr uint32_t NIL_BUCKET = NBUCKETS - 1;
constexpr int BUCKET_CAP = 1024;          // max descriptors in one MSD bucket on the fast path
constexpr uint32_t HOT_MIN_SEG = 128;     // a new key joins the hot set with at least this many descriptors
constexpr uint32_t HOT_CAND_MIN = 64;     // segments at least this long are reported (hot keys stay hot)
constexpr int CAND_MAX = 1024;
constexpr int CAND_CTR = 30;  // EngineCtl::tile_ctr[CAND_CTR][0] counts hot candidates (own line)

struct __attribute__((aligned(16))) HotCand {
  uint64_t a, b;
  uint32_t unit, rule, count, first_idx;  // first_idx ~0: (a, b, unit) already filled in
};

// ---------------------------------------------------------------------------
// v4 pipeline (rl_kernels_v4.hip)
// ---------------------------------------------------------------------------
constexpr int V4_TILE = 2048;             // k4_hist / k4_place arrival tile
constexpr int V4_THREADS = 512;  // k4_hist / k4_place threads per tile (1024 measured slower: DESIGN.md §6)
constexpr int V4_ROW16 = (NBUCKETS + 7) / 8 * 8;  // tile row of u16 bucket starts
constexpr int V4_RULE_BITS = 15;          // MRec.rn = rule | now_mod << 15 (now_mod < 86400 < 2^17)
constexpr uint32_t V4_MAX_RULES = 1u << V4_RULE_BITS;
constexpr int DFR_CTR = 29;               // EngineCtl::tile_ctr[DFR_CTR][0] counts deferred hot descriptors

// Multi-GPU: a descriptor routed to the GPU that owns its key (32 B). The owner needs the
// key identity before the window (prefix lanes), the request time, the rule, hits_addend and
// a request id that orders requests across origins: origin << ROUTE_REQ_BITS | request.
struct __attribute__((aligned(16))) RRec {
  uint64_t a, b;     // fingerprint lane state after the key-prefix bytes
  uint32_t now;      // request time, unix seconds (<= MAX_NOW, checked at the origin)
  uint32_t rule;     // rule id (< 0xFFFF; every shard loads the same rule table) | EXPIRE jitter << 16
  uint32_t h;        // max(1, hits_addend)
  uint32_t greq;     // global request id
};
__host__ __device__ __forceinline__ uint32_t rrec_rule(uint32_t w) { return w == 0xFFFFFFFFu ? w : (w & 0xFFFFu); }
__host__ __device__ __forceinline__ uint32_t rrec_jit(uint32_t w) { return w == 0xFFFFFFFFu ? 0u : (w >> 16); }
constexpr uint32_t RREC_MAX_RULE = 0xFFFFu;  // routed rule ids stay below it (the jitter shares the word)
// Owner shard of a key: a mix of the prefix lanes, so every window of a key (and every
// origin) maps to the same GPU. Multiply-shift keeps it uniform for any shard count.
__host__ __device__ __forceinline__ uint32_t route_owner(uint64_t a, uint64_t b, uint32_t n_shards) {
  const uint64_t x = fmix64(a ^ rotl64(b, 29));
  return (uint32_t)(((x >> 32) * (uint64_t)n_shards) >> 32);
}
// Reply of an owner to an origin, one per routed record (24 B): the DescriptorStatus and the
// record's ThrottleMillis contribution.
struct RReply {
  rl_status st;
  uint32_t thr;
};
static_assert(sizeof(RReply) == 24, "RReply is 6 words");
// Raw reply of an owner to an origin (8 B, the combining router): the INCRBY
// post-value the record's key saw (Redis' reply to the record's INCRBY, uint32 as
// fixed_cache_impl.go:51 decodes it) or a local-cache hit; the origin makes the decisions.
struct RawReply {
  uint32_t after;
  uint32_t flags;  // RAW_*
};
constexpr uint32_t RAW_LOCAL_HIT = 1u;  // the key was in the local over-limit cache: no INCRBY
constexpr uint32_t RAW_NIL = 2u;        // a record without a limit (never sent by rl_route_pack)
// How a pipeline writes its decisions: per descriptor statuses (+ ThrottleMillis per request),
// routed statuses (+ ThrottleMillis per record), or raw replies (RawReply per record).
constexpr int OUT_STATUS = 0, OUT_ROUTED = 1, OUT_RAW = 2;
constexpr int ROUTE_REQ_BITS = 27;
constexpr uint32_t ROUTE_MAX_SHARDS = 16;
constexpr uint8_t ROUTE_LOCAL = 0xFF;  // descriptor decided at the origin (nil limit)
// rl_batch.reserved bit: prefix_blob holds RRec records (rl_submit_routed), n_req = n_desc and
// every record has its own ThrottleMillis slot.
constexpr uint32_t RL_BATCH_ROUTED = 1u;
constexpr uint32_t RL_BATCH_RAW = 2u;  // raw replies (RawReply per descriptor / record) instead of statuses

// MSD descriptor record (32 B): tile-sorted (k4_hist) and in bucket order (k4_place,
// grouped by k4_group). A hot record carries its in-tile INCRBY prefix in `key` and its hot
// bucket in `fp_lo`. The high half of fp_lo carries the descriptor's EXPIRE jitter (MREC_JIT):
// a key's identity is the sort key and the low 32 bits of fp_lo (the table's tag).
struct __attribute__((aligned(16))) MRec {
  uint64_t key;      // sort key (region | fp.hi >> 3)
  uint64_t fp_lo;    // tag (or hot bucket) | jitter << 32
  uint32_t idx;      // arrival index
  uint32_t req;      // request index
  uint32_t h;        // max(1, hits_addend)
  uint32_t rn;       // rule | now_mod << V4_RULE_BITS
};

// Per-batch state of one hot bucket (one key). k4_scan fills it (table claim, counter before
// the batch, h total); k4_place records the freezing request and the times the last INCRBY
// happened at (exact EXPIRE / freecache TTLs, finalised by k4_group's last block).
struct __attribute__((aligned(16))) HotBucket {
  uint64_t key;
  uint64_t fp_lo;
  uint64_t base;    // counter before this batch
  uint64_t slot;    // Slot* of the key; 0 = bucket empty (or batch rejected)
  uint64_t total;   // sum of h over the bucket's descriptors
  uint32_t rule;
  uint32_t flags;   // HB_FROZEN_PRE | HB_PS
  uint32_t rstar;   // request that froze the key in this batch (local cache), ~0 = none yet
  uint32_t ws;      // window start of the key string
  uint32_t t_all;   // time of the key's last descriptor of the batch (P == total)
  uint32_t t_rstar; // time of the freezing request
};
constexpr uint32_t HB_FROZEN_PRE = 1u;  // the local cache holds the key for the whole batch
constexpr uint32_t HB_PS = 2u;          // counts in the per-second store
// Behind the HOT_BUCKETS buckets (one allocation): per bucket, index << 32 | jitter of the
// freezing request's last INCRBY of the key (atomicMax; local cache only). Derived from the
// bucket array rather than passed, since k4_group is at its scalar-register limit.
__host__ __device__ __forceinline__ unsigned long long* hot_exp(const HotBucket* hb) {
  return reinterpret_cast<unsigned long long*>(const_cast<HotBucket*>(hb) + HOT_BUCKETS);
}

// A hot descriptor whose decision needs the freezing request of an earlier tile (k4_group).
struct __attribute__((aligned(16))) Deferred {
  uint64_t P;        // INCRBY prefix of the key up to and including this descriptor
  uint32_t idx, bucket, req, h, rule, now_mod;  // bucket | EXPIRE jitter << 16
};
__host__ __device__ __forceinline__ uint32_t mrec_jit(uint64_t fp_lo) { return (uint32_t)(fp_lo >> 32); }

constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;
constexpr int MAX_PASSES = 16;

}  // namespace rlhip
