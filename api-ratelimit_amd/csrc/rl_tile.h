// rl_tile.h — device helpers of the bucketed (v4) decision pipeline: descriptor loading +
// fingerprint, hot-set lookup, LDS tile sort, segmented scan element, decisions of hot /
// local-cache-hit descriptors. Included by rl_kernels_v4.hip only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"
#include "rl_decide.h"
#include "rl_device.h"

namespace rlhip {
#ifdef RL_STAMPS
__device__ uint64_t g_st4[4096][8];  // diagnostic phase stamps (rl_kernels_v4.hip)
#endif
#ifdef RL_HIST_FINE
#define HSTF(k) do { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
  if (threadIdx.x == 0 && blockIdx.x < 1024) g_st4[1024 + blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define HSTF(k) do { } while (0)
#endif
namespace tile {

constexpr int T = V4_TILE;
constexpr int NT = V4_THREADS;
constexpr int R = T / NT;      // descriptors per thread
constexpr int W = NT / 64;     // waves per tile block
constexpr int PRE_DW = PREFIX_PRE_DW;  // blob dwords preloaded per descriptor (rl_device.h)
constexpr uint32_t BKT_NONE = 4095;  // past the end of the batch (sorts last in 12 bits)
static_assert(NBUCKETS <= 4095, "bucket ids are 12-bit");
static_assert(T <= 65536, "u16 tile offsets");


RL_DEV uint32_t msd_bucket(uint64_t key) { return (uint32_t)((key << 3) >> (64 - MSD_BITS)); }
RL_DEV uint32_t rule_of(uint32_t rn) { return rn & (V4_MAX_RULES - 1u); }

// Hot entry of a key prefix (any unit: one prefix, one hot bucket pair), or ~0. sh_hot = the
// table (rl_common.h HOT_TAGS): u32 tag words, then the entries by hot index. With at most
// 256 keys in 2048 words a miss ends after ~1.1 probes of one LDS word each; the per-slot
// 32-B entry probe it replaces walked clusters at load 1/2 (7 us of k4_hist at config 3).
RL_DEV uint32_t hot_lookup(const HotEntry* sh_hot, uint64_t a, uint64_t b, uint32_t& rule) {
  const uint32_t* tags = reinterpret_cast<const uint32_t*>(sh_hot);
  const HotEntry* list = sh_hot + HOT_SLOTS;
  const uint32_t t = hot_tag(a);
  uint32_t s = hot_home(a);
  for (int probe = 0; probe < HOT_TAGS; ++probe) {
    const uint32_t w = tags[s];
    if (w == 0u) return 0xFFFFFFFFu;
    if ((w & HOT_TAG_MASK) == t) {
      const HotEntry& e = list[(w & ~HOT_TAG_MASK) - 1u];
      if (e.a == a && e.b == b) {
        rule = e.rule;
        return e.idx;
      }
    }
    s = (s + 1) & (HOT_TAGS - 1);
  }
  return 0xFFFFFFFFu;
}

template <class V>
RL_DEV V wave_sum(V x) {
  if constexpr (sizeof(V) == 4) {
    return (V)wave_sum_u32((uint32_t)x);
  } else {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
  }
}

template <class V>
RL_DEV V wave_incl_scan(V x) {
  if constexpr (sizeof(V) == 4) return (V)wave_incl_scan_u32((uint32_t)x);
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const V y = __shfl_up(x, s, 64);
    if (lane >= (uint32_t)s) x += y;
  }
  return x;
}

// Exclusive scan over a block of NTH threads (one value each); sh_w holds NTH/64 words.
template <int NTH>
RL_DEV uint32_t block_excl_scan(uint32_t v, uint32_t* sh_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan<uint32_t>(v);
  if (lane == 63) sh_w[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < NTH / 64; ++w) {
    const uint32_t x = sh_w[w];
    before += (uint32_t)w < wave ? x : 0u;
    total += x;
  }
  __syncthreads();
  return before + incl - v;
}

// ---------------------------------------------------------------------------
// Per-descriptor input: load + fingerprint. The loads of a thread's R descriptors are
// issued together in two dependent levels: (rule, request, prefix offsets), then (now,
// hits_addend, rule entry, prefix bytes as 16-B loads).
// ---------------------------------------------------------------------------
struct D3 {
  uint64_t key, lo;
  uint32_t req, rule, h, now_mod, bucket, gen;
  uint32_t uw;   // unit window slot (unit - 1) * 2 + parity, 8 = none
  uint32_t uwv;  // unit window index + 1
};

// Words of a prefix beyond the preloaded dwords. p[0] = d0 is the dword holding the first
// remaining byte at byte offset sh; only dwords that overlap the prefix are read.
RL_DEV void hash_tail(const uint32_t* p, uint32_t d0, uint32_t sh, uint32_t rem, FpState& s) {
  for (uint32_t k = 0; rem > 0; ++k) {
    const uint32_t d1 = sh + rem > 4 ? p[2 * k + 1] : 0u;
    const uint32_t d2 = sh + rem > 8 ? p[2 * k + 2] : 0u;
    const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint64_t w = ((uint64_t)hi << 32) | lo;
    if (rem < 8) w &= (~0ull) >> (64 - 8 * rem);
    fp_word(s, w);
    d0 = d2;
    rem = rem > 8 ? rem - 8 : 0;
  }
}

// Prefix state (lanes a, b) of a byte string, reading only dwords that overlap it.
RL_DEV FpState prefix_state(const uint8_t* blob, uint32_t off, uint32_t len, uint64_t seed) {
  FpState s = fp_init(len, seed);
  if (len) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(blob + (off & ~3u));
    hash_tail(p, p[0], off & 3u, len, s);
  }
  return s;
}

// Window, sort key, table place and bucket of one valid descriptor from its prefix state.
// The key is the Redis key string (prefix, window start): its region and generation come
// from the string's home unit, not the descriptor's (rl_common.h place_of).
RL_DEV void key_of(D3& x, const FpState& s, int64_t now, const DevRule& rr, const HotEntry* sh_hot, uint32_t& err) {
  const uint32_t unit = rr.unit;
  // now / divider for now in [0, MAX_NOW] (checked by the caller): 32-bit multiply-high by the
  // divider's magic number, branch-free across lanes of different units (exact for every
  // 32-bit now: 60 -> 0x88888889 >> 37, 3600 -> 0x91A2B3C5 >> 43, 86400 = 2^7 * 675 ->
  // 0xC22E4507 >> 41 on now >> 7)
  const uint32_t n32 = (uint32_t)now;
  const uint32_t q60 = __umulhi(n32, 0x88888889u) >> 5, q3600 = __umulhi(n32, 0x91A2B3C5u) >> 11,
                 q86400 = __umulhi(n32 >> 7, 0xC22E4507u) >> 9;
  const uint32_t widx = unit == RL_UNIT_SECOND ? n32
                        : unit == RL_UNIT_MINUTE ? q60
                        : unit == RL_UNIT_HOUR   ? q3600
                                                 : q86400;
  const uint32_t ws = widx * rr.div;  // (now/divider)*divider  cache_key.go:66-68
  uint32_t hot_rule = 0;
  const uint32_t hidx = hot_lookup(sh_hot, s.a, s.b, hot_rule);
  uint64_t hi, lo;
  fp_final(s, (uint64_t)ws, hi, lo);
  const Place pl = place_of(ws);
  x.key = make_sort_key(pl.region, hi);
  x.lo = lo;
  x.gen = pl.gen;
  x.now_mod = n32 - ws;
  x.uw = (unit - 1u) * 2u + (widx & 1u);
  x.uwv = widx + 1u;
  if (hidx != 0xFFFFFFFFu) {
    // a hot prefix takes every descriptor of the prefix under one rule, so a key string
    // never splits between a hot bucket and an MSD bucket
    if (hot_rule != x.rule) err |= ERR_FALLBACK;
    x.bucket = hidx * 2u + (widx & 1u);
  } else {
    x.bucket = HOT_BUCKETS + msd_bucket(x.key);
  }
}

RL_DEV void load_descs(const DevBatch& in, const DevRule* __restrict__ rules, uint32_t n_rules, uint64_t seed,
                       const HotEntry* sh_hot, uint32_t t0, D3 (&d)[R], uint32_t& err) {
  // Every load is unconditional at a clamped index, so each of the two dependent levels (the
  // descriptor arrays; then now / hits / the rule / the prefix's first 32 bytes) issues as one
  // run of loads and waits once. A load behind a per-lane condition made the compiler wait
  // after each one. Clamped reads stay inside the arrays (n_desc >= 1 here: a tile exists only
  // for a non-empty batch; n_req >= 1 and the rule table holds >= 1 entry, both host-checked)
  // and inside the blob's 32 readable bytes of slack (rl_hip.h, rl_batch.prefix_blob).
  const uint32_t tid = threadIdx.x;
  const uint32_t last = in.n_desc - 1u;
  uint32_t rl[R], q[R], qp[R], oa[R], ob[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = min(t0 + r * NT + tid, last);
    rl[r] = in.rule[i];
    q[r] = in.req_of[i];
    qp[r] = in.req_of[i ? i - 1u : 0u];
    oa[r] = in.off[i];
    ob[r] = in.off[i + 1u];
  }
  HSTF(2);
  uint32_t o0[R], len[R];
  bool ok[R];
  int64_t now[R];
  uint32_t ha[R];
  DevRule rr[R];
  u32x4 w0[R], w1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bool v = t0 + r * NT + tid < in.n_desc;
    // batch layout checks (the device validates every submit form): prefix offsets in order
    // and inside the blob, request indices non-decreasing and in range, known rule ids
    const bool lay = oa[r] <= ob[r] && ob[r] <= in.blob_bytes && qp[r] <= q[r];
    const bool q_ok = q[r] < in.n_req, rule_ok = rl[r] < n_rules, nil = rl[r] == RL_NIL_RULE;
    if (v && (!lay || (!nil && (!rule_ok || !q_ok)))) err |= ERR_BAD_INPUT;
    ok[r] = v && !nil && rule_ok && q_ok && lay;
    o0[r] = ok[r] ? oa[r] : 0u;
    len[r] = ok[r] ? ob[r] - oa[r] : 0u;
    const uint32_t qc = q_ok ? q[r] : 0u;
    now[r] = in.now[qc];
    ha[r] = in.hits[qc];
    rr[r] = rules[rule_ok ? rl[r] : 0u];
    const u32x4* p = reinterpret_cast<const u32x4*>(in.blob + (o0[r] & ~3u));
    w0[r] = p[0];
    w1[r] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint32_t*>(p) + 4);
  }
  HSTF(3);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = t0 + r * NT + tid;
    D3& x = d[r];
    x.req = i < in.n_desc ? q[r] : 0u;
    x.rule = i < in.n_desc ? rl[r] : RL_NIL_RULE;
    // utils.Max(1, request.HitsAddend)  fixed_cache_impl.go:39
    x.h = i < in.n_desc && q[r] < in.n_req && ha[r] > 1u ? ha[r] : 1u;
    x.now_mod = 0;
    x.gen = 0;
    x.uw = 8;
    x.uwv = 0;
    x.key = NIL_KEY;
    x.lo = 0;
    x.bucket = i < in.n_desc ? NIL_BUCKET : BKT_NONE;
    if (!ok[r]) continue;
    if (now[r] < 0 || now[r] > MAX_NOW) {
      err |= ERR_BAD_TIME;
      continue;
    }
    const FpState s = prefix_state_pre(w0[r], w1[r], in.blob, o0[r], len[r], seed);
    key_of(x, s, now[r], rr[r], sh_hot, err);
  }
}

// Routed batch (owner side of the multi-GPU router): each record already carries the
// prefix state of its key, its rule, now and hits (one 32-B load per descriptor).
RL_DEV void load_routed(const DevBatch& in, const DevRule* __restrict__ rules, uint32_t n_rules,
                        const HotEntry* sh_hot, uint32_t t0, D3 (&d)[R], uint32_t& err) {
  const uint32_t tid = threadIdx.x;
  RRec rc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = t0 + r * NT + tid;
    if (i < in.n_desc) {
      rc[r] = in.recs[i];
    } else {
      rc[r].a = rc[r].b = 0;
      rc[r].now = rc[r].h = rc[r].greq = 0;
      rc[r].rule = RL_NIL_RULE;
    }
  }
  DevRule rr[R];
  bool ok[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    ok[r] = rrec_rule(rc[r].rule) < n_rules;
    if (ok[r]) rr[r] = rules[rrec_rule(rc[r].rule)];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = t0 + r * NT + tid;
    D3& x = d[r];
    x.req = rc[r].greq;
    x.rule = rrec_rule(rc[r].rule);
    x.h = rc[r].h > 1u ? rc[r].h : 1u;
    x.now_mod = 0;
    x.gen = 0;
    x.uw = 8;
    x.uwv = 0;
    x.key = NIL_KEY;
    x.lo = 0;
    x.bucket = i < in.n_desc ? NIL_BUCKET : BKT_NONE;
    if (!ok[r]) {
      if (i < in.n_desc && rc[r].rule != RL_NIL_RULE) err |= ERR_BAD_INPUT;
      continue;
    }
    if ((int64_t)rc[r].now > MAX_NOW) {
      err |= ERR_BAD_TIME;
      continue;
    }
    key_of(x, FpState{rc[r].a, rc[r].b}, (int64_t)rc[r].now, rr[r], sh_hot, err);
    // the record's EXPIRE jitter rides in lo's high half (the key's identity uses the low half):
    // no register of its own across the tile (k4_hist's VGPR count decides what of k4_group can
    // run beside it)
    x.lo = (uint32_t)x.lo | ((uint64_t)rrec_jit(rc[r].rule) << 32);
  }
}

RL_DEV void load_hot_table(const HotEntry* __restrict__ hot, HotEntry* sh_hot) {
  for (int k = threadIdx.x; k < HOT_SLOTS + HOT_MAX; k += blockDim.x) sh_hot[k] = hot[k];
}

// One stable LDS counting pass over 64 digits of the tile: src -> dst by (s_d[x] >> shift) & 63.
RL_DEV void tile_digit_pass(const uint16_t* s_d, const uint16_t* src, uint16_t* dst, int shift, uint32_t (*s_cnt)[64],
                            uint32_t* sh_w) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < W * 64; i += NT) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = lanemask_lt();
  uint32_t dg[R], rk[R], sv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t p = wave * (T / W) + r * 64 + lane;
    const uint32_t o = src[p];
    const uint32_t dd = ((uint32_t)s_d[o] >> shift) & 63u;
    uint64_t m = ~0ull;
#pragma unroll
    for (int bt = 0; bt < 6; ++bt) {
      const bool bit = (dd >> bt) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    const uint32_t before = s_cnt[wave][dd];
    __builtin_amdgcn_wave_barrier();
    if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_cnt[wave][dd] = before + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
    dg[r] = dd;
    rk[r] = before + (uint32_t)__popcll(m & lt);
    sv[r] = o;
  }
  __syncthreads();
  {  // digit-major exclusive offsets: entry (digit, wave) = tid
    static_assert(W * 64 == NT, "one (digit, wave) entry per thread");
    const uint32_t dd = tid / W, w = tid % W;
    const uint32_t v = s_cnt[w][dd];
    uint32_t total;
    const uint32_t off = block_excl_scan<NT>(v, sh_w, total);
    s_cnt[w][dd] = off;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) dst[s_cnt[wave][dg[r]] + rk[r]] = (uint16_t)sv[r];
  __syncthreads();
}

struct SegEl {
  uint32_t f, hp;
  unsigned long long s;
};
RL_DEV SegEl seg_op(const SegEl a, const SegEl b) {
  if (b.f) return b;
  return SegEl{a.f, a.hp, a.s + b.s};
}


RL_DEV rl_status local_hit_status(uint32_t h, uint32_t reset, uint32_t shadow) {
  // base_limiter.go:76-81: OVER_LIMIT from the local cache, no INCRBY
  rl_status st;
  st.code_flags = shadow_code(RL_CODE_OVER_LIMIT | ((RL_FLAG_HAS_LIMIT | RL_FLAG_LOCAL_CACHE_HIT) << 8), shadow);
  st.limit_remaining = 0;
  st.reset_s = reset;
  st.over_limit_delta = h;
  st.near_limit_delta = 0;
  return st;
}

// Decision of a descriptor whose INCRBY post-value is base + P (decide_one in rl_decide.h).
// routed (OUT_*): a routed record's ThrottleMillis slot is its own position (idx), not its
// request; OUT_RAW writes the raw reply instead.
RL_DEV void decide_at(uint32_t idx, uint32_t req, uint32_t rule, uint32_t h, uint32_t now_mod, uint64_t base,
                      uint64_t P, uint32_t freeze, const DevRule* __restrict__ rules, rl_status* __restrict__ out,
                      uint32_t* __restrict__ req_thr, int routed) {
  SortedRec o;
  o.P = P;
  o.head = 0;
  o.idx = idx;
  o.rule = rule;
  o.req = req;
  o.h = h;
  o.now_mod = (int32_t)now_mod;
  SegInfo si;
  si.base = base;
  si.freeze = freeze;
  si.pad = 0;
  decide_one(o, si, rules[rule], out, req_thr, routed ? idx : req, routed);
}

// A local-cache hit (base_limiter.go:76-81), as a status or a raw reply (mode OUT_*).
RL_DEV void emit_local_hit(rl_status* __restrict__ out, uint32_t i, uint32_t h, uint32_t reset, uint32_t shadow,
                           int mode) {
  if (mode == OUT_RAW)
    emit_raw(out, i, 0u, RAW_LOCAL_HIT);
  else
    out[i] = local_hit_status(h, reset, shadow);
}

}  // namespace tile
}  // namespace rlhip
