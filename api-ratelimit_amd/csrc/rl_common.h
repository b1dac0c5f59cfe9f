// rl_common.h — shared device/host definitions of the HIP rate-limit pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_hip.h"

namespace rlhip {

// ---------------------------------------------------------------------------
// Key fingerprint. A key is the exact byte string of
// GenerateCacheKey (src/limiter/cache_key.go:57-68) = prefix || decimal(window_start).
// The prefix always ends in '_' and the decimal has none, so (prefix bytes,
// window_start) <-> key string is a bijection; the fingerprint hashes exactly those
// two parts, plus the unit (each unit has its own key space).
// Two 64-bit lanes over 8-byte little-endian words (tail zero-padded, length folded
// in). Each lane step is a bijection of the lane state for a fixed word, so two
// equal-length prefixes that differ anywhere give different lane-a states.
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
__host__ __device__ __forceinline__ FpState fp_init(uint32_t len, uint32_t unit, uint64_t seed) {
  return FpState{seed ^ K0, (seed + K1) ^ ((uint64_t)len << 32) ^ (uint64_t)unit};
}
__host__ __device__ __forceinline__ void fp_word(FpState& s, uint64_t w) {
  s.a = rotl64((s.a ^ w) * K2, 31);
  s.b = (s.b + w) * K3;
  s.b ^= s.b >> 29;
}
__host__ __device__ __forceinline__ void fp_final(FpState s, uint64_t window_start, uint64_t& hi, uint64_t& lo) {
  s.a ^= window_start * K1;
  s.b = (s.b ^ window_start) * K2;
  hi = fmix64(s.a + rotl64(s.b, 23));
  lo = fmix64(s.b ^ (s.a * K5));
}

// Units (rl_hip.h RL_UNIT_*): divider = utils.UnitToDivider (src/utils/utilities.go:19-32)
__host__ __device__ __forceinline__ uint32_t unit_div(uint32_t unit) {
  return unit == RL_UNIT_SECOND ? 1u : unit == RL_UNIT_MINUTE ? 60u : unit == RL_UNIT_HOUR ? 3600u : 86400u;
}

// Sort key: [region:3 | fingerprint.hi >> 3]. region = (unit-1)*2 + (window_index & 1):
// every (unit, window parity) owns one region of the counter table. ~0 marks nil-limit
// descriptors, which sort last and are decided without the table.
constexpr uint64_t NIL_KEY = ~0ull;
__host__ __device__ __forceinline__ uint64_t make_sort_key(uint32_t region, uint64_t hi) {
  uint64_t k = ((uint64_t)region << 61) | (hi >> 3);
  return k == NIL_KEY ? NIL_KEY - 1 : k;
}
__host__ __device__ __forceinline__ uint32_t key_region(uint64_t k) { return (uint32_t)(k >> 61); }

// Per-descriptor record written by the fingerprint kernel in arrival order (32 B).
struct __attribute__((aligned(16))) ItemRec {
  uint64_t fp_lo;    // low fingerprint lane (identity = (sort key, fp_lo))
  uint32_t rule;     // rule id or RL_NIL_RULE
  uint32_t req;      // request index
  uint32_t h;        // max(1, hits_addend)
  int32_t now_mod;   // now - window_start (CalculateReset: div - now % div)
  uint32_t gen;      // window_index + 1 (0 = never-used slot)
  uint32_t pad;
};

// Per-descriptor record in sorted order written by the scan kernel (32 B).
struct __attribute__((aligned(16))) SortedRec {
  uint64_t P;        // inclusive prefix sum of h within the key's segment
  uint32_t head;     // sorted position of the segment head; bit31: rule changes within segment so far
  uint32_t idx;      // arrival index
  uint32_t rule;
  uint32_t req;
  uint32_t h;
  int32_t now_mod;
};
constexpr uint32_t HEAD_MIXED_RULE = 0x80000000u;

// Per-segment decision state written by the leader kernel at the segment head (16 B).
struct __attribute__((aligned(16))) SegInfo {
  uint64_t base;     // counter before this batch (INCRBY post-value = base + P)
  uint32_t freeze;   // SEG_NO_FREEZE, SEG_FROZEN_BEFORE, or the request index R* that froze the key
  uint32_t pad;
};
constexpr uint32_t SEG_NO_FREEZE = 0xFFFFFFFFu;
constexpr uint32_t SEG_FROZEN_BEFORE = 0xFFFFFFFEu;

// Counter-table slot (32 B). word0 = gen | (fp_lo low 32 bits) << 32 is the claim word.
struct __attribute__((aligned(32))) Slot {
  uint64_t ctrl;     // gen (low 32) | tag = (uint32)fp_lo (high 32)
  uint64_t key;      // sort key (region | fp.hi >> 3)
  uint32_t fp_lo_hi; // fp_lo >> 32
  uint32_t flags;    // SLOT_FROZEN: local over-limit cache holds this key
  uint64_t count;    // Redis counter value (INCRBY semantics, int64 in Redis)
};
constexpr uint32_t SLOT_FROZEN = 1u;

// Rule table entry on the device.
struct __attribute__((aligned(16))) DevRule {
  uint32_t L;        // requests_per_unit
  uint32_t near;     // uint32(floor(float64(float32(L) * ratio)))  base_limiter.go:86
  uint32_t div;      // UnitToDivider
  uint32_t unit;
};

// Device error flags (bitmask in EngineCtl.err).
enum : uint32_t {
  ERR_TABLE_FULL = 1u,
  ERR_SPIN = 2u,
  ERR_NEED_RESORT = 4u,  // a sort-prefix run holds two different fingerprints
  ERR_BAD_TIME = 8u,
  ERR_BAD_INPUT = 16u,    // rule id or request index out of range
  ERR_WINDOW_SPAN = 32u,  // a region saw window generations more than one apart in one batch
  ERR_V2_FALLBACK = 64u,  // the bucketed pipeline cannot take this batch: rerun it on the LSD pipeline
};

// Small device control block, zeroed per batch. Same-line atomics serialise at the L2
// (~9 ns each on MI355X, measured), so every word that more than one block writes is
// either written once by a single reducer block or lives on a 256-B line of its own.
struct EngineCtl {
  uint32_t err;          // atomicOr, only on an error
  uint32_t n_nil;        // nil-limit descriptors (sorted to the tail); written by k_hist_scan
  uint32_t n_segments;   // unique keys in the batch (U); written by k_leader block 0
  uint32_t n_inserted;   // unused (new keys are counted in tile_ctr[INS_CTR0..])
  uint32_t gen_min[8];   // per region: min window generation in the batch (k_hist_scan)
  uint32_t gen_max[8];   // per region: max window generation in the batch (k_hist_scan)
  uint32_t pad0[64 - 20];
  uint32_t tile_ctr[32][64];  // dynamic tile tickets, one 256-B line each
};
static_assert(sizeof(EngineCtl) == 256 + 32 * 256, "EngineCtl layout");
// tile_ctr rows 16..23: per-batch new-key counters (k_leader, one row per wave id mod 8)
constexpr int INS_CTR0 = 16;
constexpr int INS_LINES = 8;
constexpr int FP_PART_WORDS = 17;  // per fingerprint block: 8 x ~min gen, 8 x max gen, nil count

// Counter table: 8 regions (unit x window parity), region r has 2^region_log2[r] slots.
struct TableDesc {
  Slot* slots;
  uint64_t region_base[8];  // slot offset of each region
  uint32_t region_log2[8];
};

// Hot-key set entry (v2 pipeline): a key prefix seen with many descriptors per batch.
// (a, b) is the fingerprint lane state after the prefix bytes (length and unit folded in),
// i.e. a 128-bit hash of (prefix bytes, unit); the window is not part of it.
struct __attribute__((aligned(32))) HotEntry {
  uint64_t a, b;
  uint32_t unit;
  uint32_t rule;   // the rule id every hot descriptor must carry (else the batch falls back)
  uint32_t idx;    // hot index 0..HOT_MAX-1; 0xFFFFFFFF = empty slot
  uint32_t pad;
};
constexpr int HOT_MAX = 256;              // hot prefixes per batch
constexpr int HOT_SLOTS = 512;            // open-addressing table of HotEntry (device + LDS copy)
constexpr int HOT_BUCKETS = 2 * HOT_MAX;  // hot prefix x window parity
constexpr int MSD_BITS = 11;
constexpr int MSD_BUCKETS = 1 << MSD_BITS;   // 11 fingerprint bits below the region bits
constexpr int NBUCKETS = HOT_BUCKETS + MSD_BUCKETS + 1;
constexpr uint32_t NIL_BUCKET = NBUCKETS - 1;
constexpr int BUCKET_CAP = 1024;          // max descriptors in one MSD bucket on the fast path
constexpr int BG_RANGE = 1024;            // k_bgroup: MSD buckets whose start lies in one 1024-window
constexpr int BG_MAX = BG_RANGE + BUCKET_CAP;
constexpr int V2_TILE = 4096;             // k_fp2 / k_bscatter arrival tile
constexpr int HOT_CHUNK = 4096;           // k_bgroup hot-region chunk
constexpr uint32_t HOT_MIN_SEG = 128;     // a new key joins the hot set with at least this many descriptors
constexpr uint32_t HOT_CAND_MIN = 64;     // segments at least this long are reported (hot keys stay hot)
constexpr int CAND_MAX = 1024;
constexpr int CAND_CTR = 30;  // EngineCtl::tile_ctr[CAND_CTR][0] counts hot candidates (own line)

struct __attribute__((aligned(16))) HotCand {
  uint64_t a, b;
  uint32_t unit, rule, count, first_idx;  // first_idx ~0: (a, b, unit) already filled in
};

// Per-batch state of one hot bucket (one key): identity from k_fp2, table slot and base
// from k_bscan, first over-limit position from k_bscatter; k_bgroup decides from it.
struct __attribute__((aligned(16))) HotBucket {
  uint64_t key;    // sort key (identical writes from every tile that sees the bucket)
  uint64_t fp_lo;
  uint64_t base;   // counter before this batch
  uint64_t slot;   // Slot* of the key; 0 = no table update (empty bucket or error)
  uint32_t gen;    // window generation
  uint32_t flags;  // HB_FROZEN_PRE: the local cache already holds the key
  uint32_t jpos;   // first bucket position whose INCRBY reply exceeds the limit (~0: none)
  uint32_t pad;
};
constexpr uint32_t HB_FROZEN_PRE = 1u;

// ---------------------------------------------------------------------------
// v3 pipeline (rl_kernels_v3.hip)
// ---------------------------------------------------------------------------
constexpr int V3_TILE = 2048;             // k3_hist / k3_place arrival tile
constexpr int V3_THREADS = 512;
constexpr int V3_ROW16 = (NBUCKETS + 7) / 8 * 8;  // tile histogram row (u16 counts)
constexpr int V3_SCAN_BUCKETS = HOT_BUCKETS + MSD_BUCKETS;  // buckets k3_scan scans (not NIL)
#ifndef RL_V3_GRANGE
#define RL_V3_GRANGE 256
#endif
constexpr int V3_GRANGE = RL_V3_GRANGE;            // k3_group: MSD buckets whose start lies in one 256-window
constexpr int V3_GCAP = 768;              // k3_group: records staged in LDS (larger ranges run in place)
constexpr int V3_GHASH = 1024;            // k3_group: LDS hash slots (power of two, > V3_GCAP)
constexpr int V3_RULE_BITS = 15;          // MRec.rn = rule | now_mod << 15 (now_mod < 86400 < 2^17)
constexpr uint32_t V3_MAX_RULES = 1u << V3_RULE_BITS;
constexpr int DFR_CTR = 29;               // EngineCtl::tile_ctr[DFR_CTR][0] counts deferred hot descriptors
constexpr int SCAN_CTR = 28;              // EngineCtl::tile_ctr[SCAN_CTR][0]: k3_scan blocks done

// Multi-GPU: a descriptor routed to the GPU that owns its key (32 B). The owner needs the
// key identity before the window (prefix lanes), the request time, the rule, hits_addend and
// a request id that orders requests across origins: origin << ROUTE_REQ_BITS | request.
struct __attribute__((aligned(16))) RRec {
  uint64_t a, b;     // fingerprint lane state after the key-prefix bytes (unit folded in)
  uint32_t now;      // request time, unix seconds (< 2^32, checked at the origin)
  uint32_t rule;     // rule id (every shard loads the same rule table)
  uint32_t h;        // max(1, hits_addend)
  uint32_t greq;     // global request id
};
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
constexpr int ROUTE_REQ_BITS = 27;
constexpr uint32_t ROUTE_MAX_SHARDS = 16;
constexpr uint8_t ROUTE_LOCAL = 0xFF;  // descriptor decided at the origin (nil limit)
// rl_batch.reserved bit: prefix_blob holds RRec records (rl_submit_routed), n_req = n_desc and
// every record has its own ThrottleMillis slot.
constexpr uint32_t RL_BATCH_ROUTED = 1u;

// Per-descriptor record in arrival order (32 B), written by k3_hist, read by k3_place.
struct __attribute__((aligned(16))) ARec {
  uint64_t kp;       // MSD: sort key; hot: INCRBY prefix of the key inside the tile (inclusive)
  uint64_t lo;       // fp_lo
  uint32_t req;      // request index
  uint32_t h;        // max(1, hits_addend)
  uint32_t rn;       // rule | now_mod << V3_RULE_BITS
  uint16_t bucket;   // hot / MSD / NIL_BUCKET
  uint16_t rank;     // MSD: position inside (tile, bucket)
};

// MSD descriptor in bucket order (32 B), written by k3_place, grouped by k3_group.
struct __attribute__((aligned(16))) MRec {
  uint64_t key;      // sort key (region | fp.hi >> 3)
  uint64_t fp_lo;
  uint32_t idx;      // arrival index
  uint32_t req;      // request index
  uint32_t h;        // max(1, hits_addend)
  uint32_t rn;       // rule | now_mod << V3_RULE_BITS
};

// Per-batch state of one hot bucket (one key) in the v3 pipeline. k3_scan fills it (table
// claim, counter before the batch, h total); k3_place records the freezing request.
struct __attribute__((aligned(16))) HotBucket3 {
  uint64_t key;
  uint64_t fp_lo;
  uint64_t base;    // counter before this batch
  uint64_t slot;    // Slot* of the key; 0 = bucket empty (or batch rejected)
  uint64_t total;   // sum of h over the bucket's descriptors
  uint32_t rule;
  uint32_t flags;   // HB_FROZEN_PRE
  uint32_t rstar;   // request that froze the key in this batch (local cache), ~0 = none yet
  uint32_t pad[3];
};

// Global scratch of k3_group for ranges too large for LDS (indexed by bucket-order position;
// slot/cnt/base hold 4 words per position; base holds each key's list end).
struct V3GroupScratch {
  uint64_t* key;
  uint64_t* lo;
  uint4* pay;
  uint64_t* P;
  uint32_t* slot;
  uint32_t* cnt;
  uint32_t* base;
  uint32_t* list;
  uint32_t* grp;
  uint32_t* rank;
  uint32_t* tail;
  uint32_t* cursor;  // one word per k3_group workgroup
};

// A hot descriptor whose decision needs the freezing request of an earlier tile (k3_group).
struct __attribute__((aligned(16))) Deferred {
  uint64_t P;        // INCRBY prefix of the key up to and including this descriptor
  uint32_t idx, bucket, req, h, rule, now_mod;
};

constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;
constexpr int MAX_PASSES = 16;

}  // namespace rlhip
