// rl_kernels_v2.hip — the bucketed decision pipeline (default path).
//
// Same contract and outputs as the LSD pipeline in rl_kernels.hip (which stays as the
// fallback), with two global passes over the batch instead of six radix passes:
//
//   k_fp2       per descriptor: fingerprint, sort key, arrival record, hot-set lookup,
//               bucket id; per 4096-descriptor tile: bucket histogram and hot h-sums
//   k_bscan     per bucket: exclusive scan over tiles (counts; h-sums for hot buckets);
//               oversized MSD bucket -> ERR_V2_FALLBACK before anything touches the table
//   k_bscatter  stable counting scatter of (key, index) into bucket order; for hot
//               descriptors also the INCRBY prefix P (tile prefix + in-tile ordered prefix)
//   k_bgroup    MSD buckets: LDS-resident stable grouping by full fingerprint, segmented
//               prefix of hits_addend, sorted records; hot buckets (one key each, already in
//               arrival order): sorted records straight from the scatter
//   k_leader, k_decide (rl_kernels.hip) then run unchanged on the sorted records.
//
// Buckets: [0, HOT_BUCKETS) hot prefix x window parity, then MSD buckets = the 11 fingerprint
// bits below the region bits (msd_bucket), then one NIL bucket (nil limits).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"
#include "rl_device.h"
#include "rl_decide.h"

namespace rlhip {

#ifdef RL_STAMPS
// Diagnostic build only: per-block phase timestamps of k_bgroup (s_memrealtime, 100 MHz).
__device__ uint64_t g_bg_stamps[2048][10];
#define BSTAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 2048) g_bg_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define BSTAMPV(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 2048) g_bg_stamps[blockIdx.x][k] = (v); } while (0)
#else
#define BSTAMP(k) do { } while (0)
#define BSTAMPV(k, v) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// k_fp2
// ---------------------------------------------------------------------------
// MSD bucket: the top MSD_BITS fingerprint bits below the region bits, so the batch spreads
// over every bucket whatever its unit mix; within a bucket the probe positions of all
// regions share the same 1/2^MSD_BITS slice of their region (L2 locality for k_leader).
RL_DEV uint32_t msd_bucket(uint64_t key) { return (uint32_t)((key << 3) >> (64 - MSD_BITS)); }
// Bits grouped inside a bucket workgroup: key bits [GK_SHIFT, 61) (bucket bits included).
constexpr int GK_SHIFT = 61 - MSD_BITS - 24;
RL_DEV uint64_t gkey(uint64_t key) { return (key << 3) >> (GK_SHIFT + 3); }

RL_DEV uint32_t hot_lookup(const HotEntry* sh_hot, uint64_t a, uint64_t b, uint32_t unit, uint32_t& rule) {
  uint32_t s = (uint32_t)(a >> 40) & (HOT_SLOTS - 1);
  for (int probe = 0; probe < HOT_SLOTS; ++probe) {
    const HotEntry& e = sh_hot[s];
    if (e.idx == 0xFFFFFFFFu) return 0xFFFFFFFFu;
    if (e.a == a && e.b == b && e.unit == unit) {
      rule = e.rule;
      return e.idx;
    }
    s = (s + 1) & (HOT_SLOTS - 1);
  }
  return 0xFFFFFFFFu;
}

constexpr int V2_THREADS = 1024;                 // k_fp2 / k_bscatter: 16 waves per tile
constexpr int V2_WAVES = V2_THREADS / 64;
constexpr int V2_ROUNDS = V2_TILE / V2_THREADS;  // 4 rounds of 64 per wave
constexpr uint32_t BKT_SENTINEL = 4095;          // past-the-end items (sorts last in 12 bits)

// Lanes of this wave holding the same 12-bit value (among `valid` lanes).
RL_DEV uint64_t match12(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 12; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

template <class T>
RL_DEV T wave_incl_scan(T x) {
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const T y = __shfl_up(x, s, 64);
    if (lane >= (uint32_t)s) x += y;
  }
  return x;
}

// Exclusive scan over a block of NT threads (one value each); sh_w holds NT/64 words.
template <int NT>
RL_DEV uint32_t block_excl_scan(uint32_t v, uint32_t* sh_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan<uint32_t>(v);
  if (lane == 63) sh_w[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint32_t x = sh_w[w];
    before += (uint32_t)w < wave ? x : 0u;
    total += x;
  }
  __syncthreads();
  return before + incl - v;
}

// Global bucket bases (exclusive scan of the NBUCKETS totals) into LDS, by NT threads.
template <int NT>
RL_DEV void bucket_bases(const uint32_t* __restrict__ btotal, uint32_t* s_base, uint32_t* sh_w) {
  constexpr int PER = (NBUCKETS + NT - 1) / NT;
  const uint32_t tid = threadIdx.x;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t b = tid * PER + k;
    v[k] = b < (uint32_t)NBUCKETS ? btotal[b] : 0u;
    sum += v[k];
  }
  uint32_t total;
  uint32_t run = block_excl_scan<NT>(sum, sh_w, total);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t b = tid * PER + k;
    if (b < (uint32_t)NBUCKETS) s_base[b] = run;
    run += v[k];
  }
  if (tid == 0) s_base[NBUCKETS] = total;
  __syncthreads();
}

// Tile histograms are stored bucket-major: [bucket][tile].
__global__ __launch_bounds__(V2_THREADS) void k_fp2(DevBatch in, const DevRule* __restrict__ rules,
                                                    uint32_t n_rules, uint64_t seed,
                                                    const HotEntry* __restrict__ hot,
                                                    uint64_t* __restrict__ keys_orig, ItemRec* __restrict__ recs,
                                                    uint16_t* __restrict__ bkt, uint32_t* __restrict__ hbuf,
                                                    rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                                                    uint32_t* __restrict__ fpart, uint32_t ntiles,
                                                    uint32_t* __restrict__ tcount,
                                                    unsigned long long* __restrict__ thsum,
                                                    HotBucket* __restrict__ hb, EngineCtl* ctl) {
  __shared__ HotEntry sh_hot[HOT_SLOTS];
  __shared__ uint32_t sh_cnt[NBUCKETS];
  __shared__ unsigned long long sh_hs[HOT_BUCKETS];
  __shared__ uint32_t sh_nil, sh_err;
  __shared__ uint32_t sh_gmin[8], sh_gmax[8];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < HOT_SLOTS; i += V2_THREADS) sh_hot[i] = hot[i];
  for (int i = tid; i < NBUCKETS; i += V2_THREADS) sh_cnt[i] = 0;
  for (int i = tid; i < HOT_BUCKETS; i += V2_THREADS) sh_hs[i] = 0;
  if (tid < 8) { sh_gmin[tid] = 0; sh_gmax[tid] = 0; }
  if (tid == 0) { sh_nil = 0; sh_err = 0; }
  __syncthreads();

  const uint32_t tile = blockIdx.x;
  uint32_t err = 0, nil_cnt = 0;
  uint32_t gmin[8], gmax[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) { gmin[r] = 0xFFFFFFFFu; gmax[r] = 0; }
  for (int k = 0; k < V2_ROUNDS; ++k) {
    const uint32_t i = tile * V2_TILE + wave * (V2_TILE / V2_WAVES) + k * 64 + lane;
    const bool valid = i < in.n_desc;
    uint32_t bucket = NIL_BUCKET, hh = 1;
    uint64_t hkey = 0, hlo = 0;
    uint32_t hgen = 0;
    if (valid) {
      const uint32_t r = in.rule[i];
      const uint32_t q = in.req_of[i];
      const bool q_ok = q < in.n_req;
      const int64_t now = q_ok ? in.now[q] : 0;
      const uint32_t ha = q_ok ? in.hits[q] : 1u;
      if (q_ok) {  // zero the ThrottleMillis of the requests this descriptor opens
        const uint32_t pq = i == 0 ? 0u : in.req_of[i - 1];
        const uint32_t first = i == 0 ? 0u : (pq < q ? pq + 1u : q + 1u);
        for (uint32_t rr = first; rr <= q; ++rr) req_thr[rr] = 0;
        if (i + 1 == in.n_desc)
          for (uint32_t rr = q + 1; rr < in.n_req; ++rr) req_thr[rr] = 0;
      }
      ItemRec rec;
      rec.rule = r;
      rec.req = q;
      rec.h = ha > 1u ? ha : 1u;  // utils.Max(1, request.HitsAddend)  fixed_cache_impl.go:39
      rec.fp_lo = 0;
      rec.now_mod = 0;
      rec.gen = 0;
      rec.pad = 0;
      uint64_t key = NIL_KEY;
      if (r != RL_NIL_RULE && (r >= n_rules || !q_ok)) err |= ERR_BAD_INPUT;
      if (r != RL_NIL_RULE && r < n_rules && q_ok) {
        if (now < 0 || now > 0xFFFFFFF0ll) {
          err |= ERR_BAD_TIME;
        } else {
          const DevRule R = rules[r];
          const int64_t widx = div_const(now, R.unit);
          const int64_t ws = widx * (int64_t)R.div;  // (now/divider)*divider  cache_key.go:66-68
          const uint32_t o0 = in.off[i], o1 = in.off[i + 1];
          FpState s = fp_init(o1 - o0, R.unit, seed);
          hash_prefix(in.blob, o0, o1 - o0, s);
          uint32_t hot_rule = 0;
          const uint32_t hidx = hot_lookup(sh_hot, s.a, s.b, R.unit, hot_rule);
          uint64_t hi, lo;
          fp_final(s, (uint64_t)ws, hi, lo);
          const uint32_t region = (R.unit - 1u) * 2u + (uint32_t)(widx & 1);
          key = make_sort_key(region, hi);
          rec.fp_lo = lo;
          rec.now_mod = (int32_t)(now - ws);
          rec.gen = (uint32_t)widx + 1u;
#pragma unroll
          for (int rg = 0; rg < 8; ++rg)  // static register indexing
            if ((uint32_t)rg == region) {
              gmin[rg] = rec.gen < gmin[rg] ? rec.gen : gmin[rg];
              gmax[rg] = rec.gen > gmax[rg] ? rec.gen : gmax[rg];
            }
          if (hidx != 0xFFFFFFFFu) {
            // a hot prefix must keep one rule in the batch (its bucket is one key)
            if (hot_rule != r) err |= ERR_V2_FALLBACK;
            bucket = hidx * 2u + (uint32_t)(widx & 1);
          } else {
            bucket = HOT_BUCKETS + msd_bucket(key);
          }
        }
      }
      recs[i] = rec;
      keys_orig[i] = key;
      hkey = key;
      hlo = rec.fp_lo;
      hgen = rec.gen;
      bkt[i] = (uint16_t)bucket;
      hbuf[i] = rec.h;
      hh = rec.h;
      if (bucket == NIL_BUCKET) {
        // GetResponseDescriptorStatus("" key) -> {OK, nil limit, 0}  base_limiter.go:72-75
        rl_status st;
        st.code_flags = RL_CODE_OK;
        st.limit_remaining = 0;
        st.reset_s = 0;
        st.over_limit_delta = 0;
        st.near_limit_delta = 0;
        out[i] = st;
        ++nil_cnt;
      }
    }
    // wave-aggregated tile histogram: one LDS atomic per distinct bucket of the round
    const uint64_t m = match12(bucket, valid);
    if (valid) {
      const uint32_t c = (uint32_t)__popcll(m);
      if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) {
        atomicAdd(&sh_cnt[bucket], c);
        if (bucket < (uint32_t)HOT_BUCKETS) {
          atomicAdd(&sh_hs[bucket], (unsigned long long)c);
          // the bucket's key (one key per hot bucket; every tile writes the same values)
          hb[bucket].key = hkey;
          hb[bucket].fp_lo = hlo;
          hb[bucket].gen = hgen;
        }
      }
      if (bucket < (uint32_t)HOT_BUCKETS && hh > 1u) atomicAdd(&sh_hs[bucket], (unsigned long long)(hh - 1u));
    }
  }
  // block reductions (one LDS op per wave and region)
#pragma unroll
  for (int rg = 0; rg < 8; ++rg) {
    const uint32_t mn = wave_min_u32(gmin[rg]);
    const uint32_t mx = wave_max_u32(gmax[rg]);
    if (lane == 0 && mx) {
      atomicMax(&sh_gmin[rg], ~mn);
      atomicMax(&sh_gmax[rg], mx);
    }
  }
  for (int d = 32; d >= 1; d >>= 1) nil_cnt += __shfl_xor(nil_cnt, d, 64);
  if (lane == 0 && nil_cnt) atomicAdd(&sh_nil, nil_cnt);
  if (err) atomicOr(&sh_err, err);
  __syncthreads();
  for (int b = tid; b < NBUCKETS; b += V2_THREADS) tcount[(size_t)b * ntiles + tile] = sh_cnt[b];
  for (int b = tid; b < HOT_BUCKETS; b += V2_THREADS) thsum[(size_t)b * ntiles + tile] = sh_hs[b];
  uint32_t* fp = fpart + (size_t)tile * FP_PART_WORDS;
  if (tid < 8) fp[tid] = sh_gmin[tid];
  else if (tid < 16) fp[tid] = sh_gmax[tid - 8];
  else if (tid == 16) fp[16] = sh_nil;
  if (tid == 0 && sh_err) atomicOr(&ctl->err, sh_err);
}

// ---------------------------------------------------------------------------
// k_bscan — one wave per bucket: exclusive scan over tiles; last block folds fpart
// ---------------------------------------------------------------------------
constexpr int BSCAN_WAVES = 4;
__global__ __launch_bounds__(256) void k_bscan(const uint32_t* __restrict__ tcount,
                                               const unsigned long long* __restrict__ thsum, uint32_t ntiles,
                                               uint32_t* __restrict__ toff, unsigned long long* __restrict__ hoff,
                                               uint32_t* __restrict__ btotal, const uint32_t* __restrict__ fpart,
                                               const HotEntry* __restrict__ hot_list, HotBucket* __restrict__ hb,
                                               TableDesc tab, HotCand* __restrict__ cand, EngineCtl* ctl) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (blockIdx.x == gridDim.x - 1) {
    // fold the per-tile fingerprint partials: generation range per region, nil count
    __shared__ uint32_t shm[FP_PART_WORDS][256];
    for (int w = 0; w < FP_PART_WORDS; ++w) {
      uint32_t v = 0;
      for (uint32_t g = tid; g < ntiles; g += 256) {
        const uint32_t x = fpart[(size_t)g * FP_PART_WORDS + w];
        v = w < 16 ? (x > v ? x : v) : v + x;
      }
      shm[w][tid] = v;
    }
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
      if (tid < (uint32_t)d)
        for (int w = 0; w < FP_PART_WORDS; ++w) {
          const uint32_t a = shm[w][tid], c = shm[w][tid + d];
          shm[w][tid] = w < 16 ? (a > c ? a : c) : a + c;
        }
      __syncthreads();
    }
    if (tid < 8) ctl->gen_min[tid] = ~shm[tid][0];
    else if (tid < 16) ctl->gen_max[tid - 8] = shm[tid][0];
    else if (tid == 16) ctl->n_nil = shm[16][0];
    return;
  }
  const uint32_t b = blockIdx.x * BSCAN_WAVES + wave;
  if (b >= (uint32_t)NBUCKETS) return;
  const uint32_t* tc = tcount + (size_t)b * ntiles;
  uint32_t* to = toff + (size_t)b * ntiles;
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < ntiles; t0 += 64) {
    const uint32_t t = t0 + lane;
    const uint32_t v = t < ntiles ? tc[t] : 0u;
    const uint32_t incl = wave_incl_scan<uint32_t>(v);
    if (t < ntiles) to[t] = carry + incl - v;
    carry += __shfl(incl, 63, 64);
  }
  if (lane == 0) {
    btotal[b] = carry;
    if (b >= (uint32_t)HOT_BUCKETS && b < NIL_BUCKET && carry > (uint32_t)BUCKET_CAP)
      atomicOr(&ctl->err, ERR_V2_FALLBACK);
  }
  if (b < (uint32_t)HOT_BUCKETS) {
    // Hot key leader, part 1: find or claim the key's slot and read the counter before this
    // batch. A claimed slot starts at count 0 (invisible if the batch is later rejected);
    // k_bgroup writes the final count.
    if (lane == 0) {
      HotBucket x = hb[b];
      x.jpos = 0xFFFFFFFFu;
      x.slot = 0;
      x.base = 0;
      x.flags = 0;
      const uint32_t errs = ctl->err;  // flags of k_fp2
      if (carry && !(errs & (ERR_BAD_INPUT | ERR_BAD_TIME | ERR_V2_FALLBACK))) {
        Slot* slot = nullptr;
        bool existed = false;
        if (!table_claim(tab, x.key, x.fp_lo, x.gen, slot, existed)) {
          atomicOr(&ctl->err, ERR_TABLE_FULL);
        } else {
          if (existed) {
            x.base = slot->count;
            x.flags = (slot->flags & SLOT_FROZEN) ? HB_FROZEN_PRE : 0u;
          } else {
            slot->key = x.key;
            slot->fp_lo_hi = (uint32_t)(x.fp_lo >> 32);
            slot->count = 0;
            slot->flags = 0;
          }
          x.slot = (uint64_t)(uintptr_t)slot;
          count_inserts(!existed, ctl);
        }
        if (carry >= HOT_CAND_MIN) {  // stays hot: report with its known prefix state
          const HotEntry& he = hot_list[b >> 1];
          emit_candidate(ctl, cand, he.rule, carry, 0xFFFFFFFFu, he.a, he.b, he.unit);
        }
      }
      hb[b] = x;
    }
    const unsigned long long* hs = thsum + (size_t)b * ntiles;
    unsigned long long* ho = hoff + (size_t)b * ntiles;
    unsigned long long hc = 0;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += 64) {
      const uint32_t t = t0 + lane;
      const unsigned long long v = t < ntiles ? hs[t] : 0ull;
      const unsigned long long incl = wave_incl_scan<unsigned long long>(v);
      if (t < ntiles) ho[t] = hc + incl - v;
      hc += __shfl(incl, 63, 64);
    }
  }
}

// ---------------------------------------------------------------------------
// k_bscatter — stable counting scatter into bucket order (same tiles as k_fp2).
// The tile is first sorted by bucket in LDS (two stable 6-bit passes), so the global
// writes of one bucket are contiguous; a segmented scan over the sorted tile gives each
// descriptor its rank in (tile, bucket) and, for hot buckets, its in-tile h prefix.
// ---------------------------------------------------------------------------
struct SegEl {
  uint32_t f, hp;
  unsigned long long s;
};
RL_DEV SegEl seg_op(const SegEl& a, const SegEl& b) {
  if (b.f) return b;
  return SegEl{a.f, a.hp, a.s + b.s};
}

// One stable LDS counting pass over 64 digits of the tile (V2_THREADS threads).
RL_DEV void tile_digit_pass(const uint16_t* s_d, const uint16_t* src, uint16_t* dst, int shift,
                            uint32_t (*s_cnt)[64], uint32_t* sh_w) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < V2_WAVES * 64; i += V2_THREADS) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = lanemask_lt();
  uint32_t dg[V2_ROUNDS], rk[V2_ROUNDS], sv[V2_ROUNDS];
#pragma unroll
  for (int r = 0; r < V2_ROUNDS; ++r) {
    const uint32_t p = wave * (V2_TILE / V2_WAVES) + r * 64 + lane;
    const uint32_t o = src[p];
    const uint32_t d = ((uint32_t)s_d[o] >> shift) & 63u;
    uint64_t m = ~0ull;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    const uint32_t before = s_cnt[wave][d];
    __builtin_amdgcn_wave_barrier();
    if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_cnt[wave][d] = before + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
    dg[r] = d;
    rk[r] = before + (uint32_t)__popcll(m & lt);
    sv[r] = o;
  }
  __syncthreads();
  {  // digit-major exclusive offsets: entry (digit, wave) = tid
    const uint32_t d = tid >> 4, w = tid & 15;
    const uint32_t v = s_cnt[w][d];
    uint32_t total;
    const uint32_t off = block_excl_scan<V2_THREADS>(v, sh_w, total);
    s_cnt[w][d] = off;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < V2_ROUNDS; ++r) dst[s_cnt[wave][dg[r]] + rk[r]] = (uint16_t)sv[r];
  __syncthreads();
}

__global__ __launch_bounds__(V2_THREADS) void k_bscatter(const uint64_t* __restrict__ keys_orig,
                                                         const ItemRec* __restrict__ recs,
                                                         const uint16_t* __restrict__ bkt,
                                                         const uint32_t* __restrict__ hbuf, uint32_t n,
                                                         uint32_t ntiles, const uint32_t* __restrict__ btotal,
                                                         const uint32_t* __restrict__ toff,
                                                         const unsigned long long* __restrict__ hoff,
                                                         uint64_t* __restrict__ bkey, ItemRec* __restrict__ brec,
                                                         uint64_t* __restrict__ bP, uint32_t* __restrict__ bbase,
                                                         HotBucket* __restrict__ hb,
                                                         const DevRule* __restrict__ rules, int local_cache,
                                                         EngineCtl* ctl) {
  static_assert(V2_WAVES * 64 == V2_THREADS && V2_WAVES == 16, "digit-major scan assumes 16 waves x 64 digits");
  __shared__ uint32_t s_base[NBUCKETS + 1];
  __shared__ uint16_t s_d[V2_TILE];
  __shared__ uint16_t s_pa[V2_TILE], s_pb[V2_TILE];
  __shared__ uint32_t s_h[V2_TILE];
  __shared__ uint32_t s_cnt[V2_WAVES][64];
  __shared__ uint32_t sh_w[V2_WAVES];
  __shared__ SegEl s_agg[V2_WAVES];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (ctl->err & (ERR_V2_FALLBACK | ERR_BAD_INPUT | ERR_BAD_TIME)) return;
  const uint32_t tile = blockIdx.x;
  const uint32_t t0 = tile * V2_TILE;
  for (int o = tid; o < V2_TILE; o += V2_THREADS) {
    const uint32_t i = t0 + o;
    const bool valid = i < n;
    s_d[o] = valid ? bkt[i] : (uint16_t)BKT_SENTINEL;
    s_h[o] = valid ? hbuf[i] : 0u;
    s_pa[o] = (uint16_t)o;
  }
  bucket_bases<V2_THREADS>(btotal, s_base, sh_w);  // includes barriers
  if (tile == 0)  // publish the bases for k_bgroup
    for (int b = tid; b <= NBUCKETS; b += V2_THREADS) bbase[b] = s_base[b];
  tile_digit_pass(s_d, s_pa, s_pb, 0, s_cnt, sh_w);
  tile_digit_pass(s_d, s_pb, s_pa, 6, s_cnt, sh_w);
  // segmented scan over the sorted tile (blocked: V2_ROUNDS consecutive positions per thread)
  const uint32_t s0 = tid * V2_ROUNDS;
  uint32_t od[V2_ROUNDS], dd[V2_ROUNDS], fl[V2_ROUNDS];
  unsigned long long hv[V2_ROUNDS];
  uint32_t prev_d = s0 == 0 ? 0xFFFFFFFFu : s_d[s_pa[s0 - 1]];
  SegEl t{0, 0, 0};
#pragma unroll
  for (int q = 0; q < V2_ROUNDS; ++q) {
    const uint32_t o = s_pa[s0 + q];
    const uint32_t d = s_d[o];
    od[q] = o;
    dd[q] = d;
    fl[q] = d != prev_d;
    hv[q] = s_h[o];
    prev_d = d;
    t = seg_op(t, SegEl{fl[q], s0 + q, hv[q]});
  }
  SegEl incl = t;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    SegEl y;
    y.f = __shfl_up(incl.f, s, 64);
    y.hp = __shfl_up(incl.hp, s, 64);
    y.s = __shfl_up(incl.s, s, 64);
    if (lane >= (uint32_t)s) incl = seg_op(y, incl);
  }
  if (lane == 63) s_agg[wave] = incl;
  SegEl wex;
  wex.f = __shfl_up(incl.f, 1, 64);
  wex.hp = __shfl_up(incl.hp, 1, 64);
  wex.s = __shfl_up(incl.s, 1, 64);
  if (lane == 0) wex = SegEl{0, 0, 0};
  __syncthreads();
  SegEl run{0, 0, 0};
  for (uint32_t w = 0; w < wave; ++w) run = seg_op(run, s_agg[w]);
  run = seg_op(run, wex);
#pragma unroll
  for (int q = 0; q < V2_ROUNDS; ++q) {
    run = seg_op(run, SegEl{fl[q], s0 + q, hv[q]});
    const uint32_t d = dd[q];
    if (d >= (uint32_t)NBUCKETS) continue;  // past the end of the batch
    const uint32_t i = t0 + od[q];
    const uint32_t pos = s_base[d] + toff[(size_t)d * ntiles + tile] + (s0 + q - run.hp);
    // bucketed copy of the arrival record; pad carries the descriptor index
    ItemRec r = recs[i];
    r.pad = i;
    bkey[pos] = keys_orig[i];
    brec[pos] = r;
    if (d < (uint32_t)HOT_BUCKETS) {
      const uint64_t P = hoff[(size_t)d * ntiles + tile] + run.s;
      bP[pos] = P;
      if (local_cache) {
        // Local cache: the key freezes at the first descriptor whose INCRBY reply exceeds
        // the limit. Candidates are the upward crossings (after > L >= before, or the
        // bucket's first descriptor); the earliest one is that descriptor.
        const HotBucket& x = hb[d];
        if (x.slot && !(x.flags & HB_FROZEN_PRE)) {
          const uint32_t after = (uint32_t)(x.base + P);
          const uint32_t before = after - r.h;
          const uint32_t L = rules[r.rule].L;
          if (after > L && (before <= L || pos == s_base[d])) atomicMin(&hb[d].jpos, pos);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_bgroup — sorted records for k_leader / k_decide
// ---------------------------------------------------------------------------
constexpr int BG_THREADS = 512;
constexpr int BG_WAVES = BG_THREADS / 64;
constexpr int BG_PER_WAVE = BG_MAX / BG_WAVES;   // 256 positions per wave
constexpr int BG_ROUNDS = BG_PER_WAVE / 64;      // 4
constexpr int BG_IPT = BG_MAX / BG_THREADS;      // 4 (blocked, for the scan)

struct BgScanEl {
  uint32_t f, o, hp;
  unsigned long long s;
};
RL_DEV BgScanEl bg_op(const BgScanEl& a, const BgScanEl& b) {
  if (b.f) return b;
  return BgScanEl{a.f, a.o | b.o, a.hp, a.s + b.s};
}

// Stable LDS radix pass: order src -> dst by 8-bit digit (key >> shift) of m items.
RL_DEV void lds_radix_pass(const uint64_t* s_key, const uint16_t* src, uint16_t* dst, uint32_t m, int shift,
                           uint32_t (*s_cnt)[RADIX], uint32_t* sh_w) {
  constexpr int ENT = BG_WAVES * RADIX / BG_THREADS;  // (digit, wave) counters per thread
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < BG_WAVES * RADIX; i += BG_THREADS) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = lanemask_lt();
  uint32_t dg[BG_ROUNDS], rk[BG_ROUNDS];
#pragma unroll
  for (int r = 0; r < BG_ROUNDS; ++r) {
    const uint32_t k = wave * BG_PER_WAVE + r * 64 + lane;
    const bool valid = k < m;
    const uint32_t d = valid ? (uint32_t)(s_key[src[k]] >> shift) & 0xFFu : 0u;
    uint64_t mm = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      mm &= bit ? bal : ~bal;
    }
    uint32_t rr = 0;
    if (valid) {
      const uint32_t before = s_cnt[wave][d];
      rr = before + (uint32_t)__popcll(mm & lt);
      const uint32_t leader = (uint32_t)__ffsll((unsigned long long)mm) - 1u;
      __builtin_amdgcn_wave_barrier();
      if (lane == leader) s_cnt[wave][d] = before + (uint32_t)__popcll(mm);
    }
    __builtin_amdgcn_wave_barrier();
    dg[r] = d;
    rk[r] = rr;
  }
  __syncthreads();
  {  // digit-major exclusive offsets over (digit, wave): entries ENT*tid .. ENT*tid+ENT-1
    uint32_t v[ENT], sum = 0;
#pragma unroll
    for (int j = 0; j < ENT; ++j) {
      const uint32_t e = tid * ENT + j;
      v[j] = s_cnt[e % BG_WAVES][e / BG_WAVES];
      sum += v[j];
    }
    uint32_t total;
    uint32_t run = block_excl_scan<BG_THREADS>(sum, sh_w, total);
#pragma unroll
    for (int j = 0; j < ENT; ++j) {
      const uint32_t e = tid * ENT + j;
      s_cnt[e % BG_WAVES][e / BG_WAVES] = run;
      run += v[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < BG_ROUNDS; ++r) {
    const uint32_t k = wave * BG_PER_WAVE + r * 64 + lane;
    if (k < m) dst[s_cnt[wave][dg[r]] + rk[r]] = src[k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(BG_THREADS) void k_bgroup(const uint64_t* __restrict__ bkey,
                                                       const ItemRec* __restrict__ brec,
                                                       const uint64_t* __restrict__ bP,
                                                       const uint32_t* __restrict__ bbase, uint32_t n_msd_wg,
                                                       uint64_t* __restrict__ skeys, SortedRec* __restrict__ srec,
                                                       uint32_t* __restrict__ wg_heads,
                                                       const ItemRec* __restrict__ recs,
                                                       const DevRule* __restrict__ rules, TableDesc tab,
                                                       int local_cache, SegInfo* __restrict__ seg,
                                                       const HotBucket* __restrict__ hb,
                                                       rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                                                       HotCand* __restrict__ cand, EngineCtl* ctl) {
  __shared__ uint32_t s_base[NBUCKETS + 1];
  __shared__ uint64_t s_key[BG_MAX];
  __shared__ uint64_t s_lo[BG_MAX];
  __shared__ uint32_t s_h[BG_MAX];
  __shared__ uint32_t s_rule[BG_MAX];
  __shared__ uint16_t s_pa[BG_MAX], s_pb[BG_MAX];
  __shared__ uint32_t s_cnt[BG_WAVES][RADIX];
  __shared__ BgScanEl s_wagg[BG_WAVES];
  __shared__ uint32_t s_mixed, s_heads;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Nothing touches the table unless the whole batch is valid: errors of earlier kernels,
  // or two window generations more than one apart in a region.
  if (ctl->err) return;
  {
    bool span = false;
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) span |= ctl->gen_max[rg] - ctl->gen_min[rg] > 1u;
    if (span) {
      if (tid == 0) atomicOr(&ctl->err, ERR_WINDOW_SPAN);
      return;
    }
  }
  __shared__ uint32_t sh_w[BG_WAVES];
  BSTAMP(0);
  if (tid == 0) { s_mixed = 0; s_heads = 0; }
  for (int b = tid; b <= NBUCKETS; b += BG_THREADS) s_base[b] = bbase[b];
  __syncthreads();
  BSTAMP(1);
  const uint32_t hot_end = s_base[HOT_BUCKETS];
  if (blockIdx.x >= n_msd_wg) {
    // Hot chunk: each hot bucket is one key in arrival order; P comes from k_bscatter.
    const uint32_t c = blockIdx.x - n_msd_wg;
    const uint32_t p0 = c * HOT_CHUNK;
    if (p0 >= hot_end) {
      if (tid == 0) wg_heads[blockIdx.x] = 0;
      return;
    }
#ifdef RL_BG_SKIP_HOT
    if (tid == 0) wg_heads[blockIdx.x] = 0;
    return;
#endif
    const uint32_t p1 = min(hot_end, p0 + HOT_CHUNK);
    uint32_t heads = 0;
    for (uint32_t p = p0 + tid; p < p1; p += BG_THREADS) {
      // bucket of position p: last hot bucket whose base <= p
      uint32_t lo_b = 0, hi_b = HOT_BUCKETS - 1;
      while (lo_b < hi_b) {
        const uint32_t mid = (lo_b + hi_b + 1) / 2;
        if (s_base[mid] <= p) lo_b = mid; else hi_b = mid - 1;
      }
      const uint32_t head = s_base[lo_b], end = s_base[lo_b + 1];
      heads += head == p;
      const HotBucket x = hb[lo_b];
      if (!x.slot) continue;  // unreachable for a valid batch (k_bscan claimed every non-empty bucket)
      const ItemRec r = brec[p];
      SortedRec o;
      o.P = bP[p];
      o.head = head;
      o.idx = r.pad;
      o.rule = r.rule;
      o.req = r.req;
      o.h = r.h;
      o.now_mod = r.now_mod;
      SegInfo si;
      si.base = x.base;
      si.pad = 0;
      uint32_t rstar = SEG_NO_FREEZE;
      if (x.flags & HB_FROZEN_PRE) {
        si.freeze = SEG_FROZEN_BEFORE;
      } else {
        if (x.jpos != 0xFFFFFFFFu) rstar = brec[x.jpos].req;
        si.freeze = rstar;
      }
      decide_one(o, si, rules[r.rule], out, req_thr, o.req);
      // Hot key leader, part 2: the one descriptor that ends the key's INCRBYs writes the
      // counter (the last of the freezing request, else the bucket's last descriptor).
      if (!(x.flags & HB_FROZEN_PRE)) {
        Slot* slot = reinterpret_cast<Slot*>(x.slot);
        if (rstar != SEG_NO_FREEZE) {
          if (r.req == rstar && (p + 1 == end || brec[p + 1].req != rstar)) {
            slot->count = x.base + o.P;
            slot->flags = SLOT_FROZEN;
          }
        } else if (p + 1 == end) {
          slot->count = x.base + o.P;
        }
      }
    }
    for (int d = 32; d >= 1; d >>= 1) heads += __shfl_xor(heads, d, 64);
    if (lane == 0 && heads) atomicAdd(&s_heads, heads);
    __syncthreads();
    if (tid == 0) wg_heads[blockIdx.x] = s_heads;
    return;
  }
  // MSD workgroup: buckets whose base lies in [msd_start + w*BG_RANGE, +BG_RANGE)
  const uint32_t msd_start = hot_end, msd_end = s_base[NIL_BUCKET];
  const uint32_t w0 = msd_start + blockIdx.x * BG_RANGE, w1 = w0 + BG_RANGE;
  auto first_bucket_at_or_after = [&](uint32_t pos) {
    uint32_t lo_b = HOT_BUCKETS, hi_b = NIL_BUCKET;  // answer in [HOT_BUCKETS, NIL_BUCKET]
    while (lo_b < hi_b) {
      const uint32_t mid = (lo_b + hi_b) / 2;
      if (s_base[mid] >= pos) hi_b = mid; else lo_b = mid + 1;
    }
    return lo_b;
  };
  const uint32_t b0 = w0 >= msd_end ? NIL_BUCKET : first_bucket_at_or_after(w0);
  const uint32_t b1 = w1 >= msd_end ? NIL_BUCKET : first_bucket_at_or_after(w1);
  const uint32_t r0 = s_base[b0], r1 = s_base[b1];
  const uint32_t m = r1 - r0;
#ifdef RL_BG_SKIP_MSD
  if (tid == 0) wg_heads[blockIdx.x] = 0;
  return;
#endif
  if (m == 0) {
    if (tid == 0) wg_heads[blockIdx.x] = 0;
    return;
  }
  BSTAMPV(9, m);
  // load (key, fp_lo, h, rule) of the range; identity order = perm
  for (uint32_t k = tid; k < m; k += BG_THREADS) {
    const ItemRec r = brec[r0 + k];
    s_key[k] = bkey[r0 + k];
    s_lo[k] = r.fp_lo;
    s_h[k] = r.h;
    s_rule[k] = r.rule;
    s_pa[k] = (uint16_t)k;
  }
  __syncthreads();
  // Stable grouping: 3 LDS radix passes on the 24 key bits below the bucket bits. Equal keys
  // end adjacent; different buckets never interleave (they arrive bucket by bucket).
#ifndef RL_BG_SKIP_RADIX
  BSTAMP(2);
  lds_radix_pass(s_key, s_pa, s_pb, m, GK_SHIFT, s_cnt, sh_w);
  BSTAMP(3);
  lds_radix_pass(s_key, s_pb, s_pa, m, GK_SHIFT + 8, s_cnt, sh_w);
  BSTAMP(4);
  lds_radix_pass(s_key, s_pa, s_pb, m, GK_SHIFT + 16, s_cnt, sh_w);
  BSTAMP(5);
#else
  for (uint32_t k = tid; k < m; k += BG_THREADS) s_pb[k] = s_pa[k];
  __syncthreads();
#endif
  uint16_t* perm = s_pb;
  // A run of equal grouped bits holding two identities (35-bit collision, ~1 per batch):
  // regroup this range on 32 bits below the bucket bits; a collision on those 43 bits too
  // (~1 in 300 batches) is regrouped by one thread (stable partition by full identity).
  for (uint32_t k = tid + 1; k < m; k += BG_THREADS) {
    const uint32_t a = perm[k - 1], b = perm[k];
    if (gkey(s_key[a]) == gkey(s_key[b]) && (s_key[a] != s_key[b] || s_lo[a] != s_lo[b])) s_mixed = 1;
  }
  __syncthreads();
  if (s_mixed) {  // block-uniform
    for (uint32_t k = tid; k < m; k += BG_THREADS) s_pa[k] = (uint16_t)k;
    __syncthreads();
    lds_radix_pass(s_key, s_pa, s_pb, m, GK_SHIFT - 8, s_cnt, sh_w);
    lds_radix_pass(s_key, s_pb, s_pa, m, GK_SHIFT, s_cnt, sh_w);
    lds_radix_pass(s_key, s_pa, s_pb, m, GK_SHIFT + 8, s_cnt, sh_w);
    lds_radix_pass(s_key, s_pb, s_pa, m, GK_SHIFT + 16, s_cnt, sh_w);
    for (uint32_t k = tid; k < m; k += BG_THREADS) s_pb[k] = s_pa[k];
    __syncthreads();
    if (tid == 0) s_mixed = 0;
    __syncthreads();
    for (uint32_t k = tid + 1; k < m; k += BG_THREADS) {
      const uint32_t a = perm[k - 1], b = perm[k];
      if ((s_key[a] << 3) >> (GK_SHIFT - 5) == (s_key[b] << 3) >> (GK_SHIFT - 5) &&
          (s_key[a] != s_key[b] || s_lo[a] != s_lo[b]))
        s_mixed = 1;
    }
    __syncthreads();
    if (s_mixed && tid == 0) {
      uint32_t k = 0;
      while (k < m) {
        uint32_t e = k + 1;
        while (e < m && gkey(s_key[perm[e]]) == gkey(s_key[perm[k]])) ++e;
        for (uint32_t s = k; s < e;) {  // stable partition of perm[k..e), first-seen identity first
          const uint32_t ref = perm[s];
          uint32_t w = s + 1;
          for (uint32_t t = s + 1; t < e; ++t) {
            const uint32_t x = perm[t];
            if (s_key[x] == s_key[ref] && s_lo[x] == s_lo[ref]) {
              for (uint32_t u = t; u > w; --u) perm[u] = perm[u - 1];
              perm[w++] = (uint16_t)x;
            }
          }
          s = w;
        }
        k = e;
      }
    }
    __syncthreads();
  }
  BSTAMP(6);
  BSTAMPV(8, s_mixed);
  // Segmented inclusive prefix of h over the grouped order (blocked: BG_IPT per thread).
  const uint32_t k0 = tid * BG_IPT;
  BgScanEl t{0, 0, 0, 0};
  uint32_t hd[BG_IPT], rc[BG_IPT];
#pragma unroll
  for (int q = 0; q < BG_IPT; ++q) {
    const uint32_t k = k0 + q;
    hd[q] = 0;
    rc[q] = 0;
    if (k < m) {
      const uint32_t x = perm[k];
      const bool head = k == 0 || s_key[perm[k - 1]] != s_key[x] || s_lo[perm[k - 1]] != s_lo[x];
      hd[q] = head;
      rc[q] = !head && s_rule[perm[k - 1]] != s_rule[x];
      t = bg_op(t, BgScanEl{(uint32_t)head, rc[q], k, (unsigned long long)s_h[x]});
    }
  }
  BgScanEl incl = t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    BgScanEl y;
    y.f = __shfl_up(incl.f, d, 64);
    y.o = __shfl_up(incl.o, d, 64);
    y.hp = __shfl_up(incl.hp, d, 64);
    y.s = __shfl_up(incl.s, d, 64);
    if (lane >= (uint32_t)d) incl = bg_op(y, incl);
  }
  if (lane == 63) s_wagg[wave] = incl;
  BgScanEl wex;
  wex.f = __shfl_up(incl.f, 1, 64);
  wex.o = __shfl_up(incl.o, 1, 64);
  wex.hp = __shfl_up(incl.hp, 1, 64);
  wex.s = __shfl_up(incl.s, 1, 64);
  if (lane == 0) wex = BgScanEl{0, 0, 0, 0};
  __syncthreads();
  BgScanEl run{0, 0, 0, 0};
  for (uint32_t w = 0; w < wave; ++w) run = bg_op(run, s_wagg[w]);
  run = bg_op(run, wex);
  uint32_t heads = 0;
  SortedRec mine[BG_IPT];
#pragma unroll
  for (int q = 0; q < BG_IPT; ++q) {
    const uint32_t k = k0 + q;
    if (k >= m) break;
    const uint32_t x = perm[k];
    run = bg_op(run, BgScanEl{hd[q], rc[q], k, (unsigned long long)s_h[x]});
    heads += hd[q];
    const ItemRec r = brec[r0 + x];
    SortedRec o;
    o.P = run.s;
    o.head = (r0 + run.hp) | (run.o ? HEAD_MIXED_RULE : 0u);
    o.idx = r.pad;
    o.rule = r.rule;
    o.req = r.req;
    o.h = r.h;
    o.now_mod = r.now_mod;
    mine[q] = o;
    srec[r0 + k] = o;
    skeys[r0 + k] = s_key[x];
  }
  for (int d = 32; d >= 1; d >>= 1) heads += __shfl_xor(heads, d, 64);
  if (lane == 0 && heads) atomicAdd(&s_heads, heads);
  __syncthreads();  // the range's sorted records are visible to the whole workgroup
  BSTAMP(7);
  // Leader: one thread per segment tail — table probe/claim, INCRBY of the segment in
  // serial order, local-cache freeze (every key of the range is complete in this range).
  for (uint32_t k = tid; k < m; k += BG_THREADS) {
    const uint32_t j = r0 + k;
    if (k + 1 < m && (srec[j + 1].head & ~HEAD_MIXED_RULE) != j + 1) continue;  // not a tail
    const SortedRec tail = srec[j];
    const uint32_t hp = tail.head & ~HEAD_MIXED_RULE;
    const bool mixed_rule = (tail.head & HEAD_MIXED_RULE) != 0;
    if (j - hp + 1 >= HOT_CAND_MIN && !mixed_rule) emit_candidate(ctl, cand, tail.rule, j - hp + 1, srec[hp].idx);
    leader_segment(hp, j, tail, mixed_rule, skeys, srec, recs, rules, tab, local_cache, seg, ctl);
  }
  __syncthreads();  // SegInfo of every segment of the range is visible
#pragma unroll
  for (int q = 0; q < BG_IPT; ++q) {
    if (k0 + q >= m) break;
    const SortedRec& o = mine[q];
    decide_one(o, seg[o.head & ~HEAD_MIXED_RULE], rules[o.rule], out, req_thr, o.req);
  }
  if (tid == 0) wg_heads[blockIdx.x] = s_heads;
}

// Hot-set candidates: recompute the prefix lane state (a, b) of each candidate's first
// descriptor (the batch input is still resident).
__global__ void k_cand_state(DevBatch in, const DevRule* __restrict__ rules, uint64_t seed, HotCand* cand,
                             const uint32_t* __restrict__ wg_heads, uint32_t n_heads, EngineCtl* ctl) {
  if (blockIdx.x == 0 && n_heads) {
    // U = segment heads of the batch (bucketed pipeline; single writer of n_segments)
    uint32_t u = 0;
    for (uint32_t t = threadIdx.x; t < n_heads; t += 64) u += wg_heads[t];
    for (int d = 32; d >= 1; d >>= 1) u += __shfl_xor(u, d, 64);
    if (threadIdx.x == 0) ctl->n_segments = u;
  }
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  const uint32_t nc = min((uint32_t)CAND_MAX, ctl->tile_ctr[CAND_CTR][0]);
  if (i >= nc) return;
  HotCand c = cand[i];
  if (c.first_idx == 0xFFFFFFFFu) return;  // a hot key: state already known
  const uint32_t d = c.first_idx;
  const uint32_t unit = rules[c.rule].unit;
  if (in.recs) {  // routed batch: the record carries the prefix state
    c.a = in.recs[d].a;
    c.b = in.recs[d].b;
  } else {
    const uint32_t o0 = in.off[d], o1 = in.off[d + 1];
    FpState s = fp_init(o1 - o0, unit, seed);
    hash_prefix(in.blob, o0, o1 - o0, s);
    c.a = s.a;
    c.b = s.b;
  }
  c.unit = unit;
  cand[i] = c;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
uint32_t v2_tiles(uint32_t n) { return n ? (n + V2_TILE - 1) / V2_TILE : 1; }
uint32_t v2_msd_wgs(uint32_t n) { return n ? (n + BG_RANGE - 1) / BG_RANGE : 1; }
uint32_t v2_hot_wgs(uint32_t n) { return n ? (n + HOT_CHUNK - 1) / HOT_CHUNK : 1; }

void launch_fp2(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                const HotEntry* hot, uint64_t* keys_orig, ItemRec* recs, uint16_t* bkt, uint32_t* hbuf,
                rl_status* out, uint32_t* req_thr, uint32_t* fpart, uint32_t* tcount, unsigned long long* thsum,
                HotBucket* hb, EngineCtl* ctl) {
  const DevBatch d = make_dev_batch(b);
  hipLaunchKernelGGL(k_fp2, dim3(v2_tiles(b.n_desc)), dim3(V2_THREADS), 0, st, d, rules, n_rules, seed, hot,
                     keys_orig, recs, bkt, hbuf, out, req_thr, fpart, v2_tiles(b.n_desc), tcount, thsum, hb, ctl);
}
void launch_bscan(hipStream_t st, const uint32_t* tcount, const unsigned long long* thsum, uint32_t n,
                  uint32_t* toff, unsigned long long* hoff, uint32_t* btotal, const uint32_t* fpart,
                  const HotEntry* hot_list, HotBucket* hb, const TableDesc& tab, HotCand* cand, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_bscan, dim3((NBUCKETS + BSCAN_WAVES - 1) / BSCAN_WAVES + 1), dim3(256), 0, st, tcount, thsum,
                     v2_tiles(n), toff, hoff, btotal, fpart, hot_list, hb, tab, cand, ctl);
}
void launch_bscatter(hipStream_t st, const uint64_t* keys_orig, const ItemRec* recs, const uint16_t* bkt,
                     const uint32_t* hbuf, uint32_t n, const uint32_t* btotal, const uint32_t* toff,
                     const unsigned long long* hoff, uint64_t* bkey, ItemRec* brec, uint64_t* bP, uint32_t* bbase,
                     HotBucket* hb, const DevRule* rules, int local_cache, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_bscatter, dim3(v2_tiles(n)), dim3(V2_THREADS), 0, st, keys_orig, recs, bkt, hbuf, n,
                     v2_tiles(n), btotal, toff, hoff, bkey, brec, bP, bbase, hb, rules, local_cache, ctl);
}
void launch_bgroup(hipStream_t st, const uint64_t* bkey, const ItemRec* brec, const uint64_t* bP,
                   const uint32_t* bbase, uint32_t n, uint64_t* skeys, SortedRec* srec, uint32_t* wg_heads,
                   const ItemRec* recs, const DevRule* rules, const TableDesc& tab, int local_cache, SegInfo* seg,
                   const HotBucket* hb, rl_status* out, uint32_t* req_thr, HotCand* cand, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_bgroup, dim3(v2_msd_wgs(n) + v2_hot_wgs(n)), dim3(BG_THREADS), 0, st, bkey, brec, bP, bbase,
                     v2_msd_wgs(n), skeys, srec, wg_heads, recs, rules, tab, local_cache, seg, hb, out, req_thr, cand,
                     ctl);
}
void launch_cand_state(hipStream_t st, const rl_batch& b, const DevRule* rules, uint64_t seed, HotCand* cand,
                       const uint32_t* wg_heads, uint32_t n_heads, EngineCtl* ctl) {
  const DevBatch d = make_dev_batch(b);
  hipLaunchKernelGGL(k_cand_state, dim3(CAND_MAX / 64), dim3(64), 0, st, d, rules, seed, cand, wg_heads, n_heads,
                     ctl);
}

}  // namespace rlhip

#ifdef RL_STAMPS
extern "C" int rl_debug_bg_stamps(uint64_t* out, uint32_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlhip::g_bg_stamps), (size_t)nblocks * 10 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
