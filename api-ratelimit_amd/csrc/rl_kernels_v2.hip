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

namespace rlhip {

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

__global__ __launch_bounds__(256) void k_fp2(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                             uint64_t seed, const HotEntry* __restrict__ hot,
                                             uint64_t* __restrict__ keys_orig, ItemRec* __restrict__ recs,
                                             uint16_t* __restrict__ bkt, uint32_t* __restrict__ hbuf,
                                             rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                                             uint32_t* __restrict__ fpart, uint32_t* __restrict__ tcount,
                                             unsigned long long* __restrict__ thsum, EngineCtl* ctl) {
  __shared__ HotEntry sh_hot[HOT_SLOTS];
  __shared__ uint32_t sh_cnt[NBUCKETS];
  __shared__ unsigned long long sh_hs[HOT_BUCKETS];
  __shared__ uint32_t sh_nil, sh_err;
  __shared__ uint32_t sh_gmin[8], sh_gmax[8];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < HOT_SLOTS; i += 256) sh_hot[i] = hot[i];
  for (int i = tid; i < NBUCKETS; i += 256) sh_cnt[i] = 0;
  for (int i = tid; i < HOT_BUCKETS; i += 256) sh_hs[i] = 0;
  if (tid < 8) { sh_gmin[tid] = 0; sh_gmax[tid] = 0; }
  if (tid == 0) { sh_nil = 0; sh_err = 0; }
  __syncthreads();

  const uint32_t tile = blockIdx.x;
  uint32_t err = 0, nil_cnt = 0;
  uint32_t gmin[8], gmax[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) { gmin[r] = 0xFFFFFFFFu; gmax[r] = 0; }
  for (int k = 0; k < V2_TILE / 256; ++k) {
    const uint32_t i = tile * V2_TILE + wave * (V2_TILE / 4) + k * 64 + lane;
    if (i >= in.n_desc) break;
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
    uint32_t bucket = NIL_BUCKET;
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
    bkt[i] = (uint16_t)bucket;
    hbuf[i] = rec.h;
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
    atomicAdd(&sh_cnt[bucket], 1u);
    if (bucket < (uint32_t)HOT_BUCKETS) atomicAdd(&sh_hs[bucket], (unsigned long long)rec.h);
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
  for (int b = tid; b < NBUCKETS; b += 256) tcount[(size_t)tile * NBUCKETS + b] = sh_cnt[b];
  for (int b = tid; b < HOT_BUCKETS; b += 256) thsum[(size_t)tile * HOT_BUCKETS + b] = sh_hs[b];
  uint32_t* fp = fpart + (size_t)tile * FP_PART_WORDS;
  if (tid < 8) fp[tid] = sh_gmin[tid];
  else if (tid < 16) fp[tid] = sh_gmax[tid - 8];
  else if (tid == 16) fp[16] = sh_nil;
  if (tid == 0 && sh_err) atomicOr(&ctl->err, sh_err);
}

// ---------------------------------------------------------------------------
// k_bscan — one block per bucket (+ one reducer block)
// ---------------------------------------------------------------------------
template <class T>
RL_DEV T block_excl_scan_256(T v, T* sh, T& total) {
  const uint32_t tid = threadIdx.x;
  sh[tid] = v;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const T t = tid >= (uint32_t)d ? sh[tid - d] : (T)0;
    __syncthreads();
    sh[tid] += t;
    __syncthreads();
  }
  total = sh[255];
  const T r = sh[tid] - v;
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_bscan(const uint32_t* __restrict__ tcount,
                                               const unsigned long long* __restrict__ thsum, uint32_t ntiles,
                                               uint32_t* __restrict__ toff, unsigned long long* __restrict__ hoff,
                                               uint32_t* __restrict__ btotal, const uint32_t* __restrict__ fpart,
                                               EngineCtl* ctl) {
  __shared__ uint32_t sh32[256];
  __shared__ unsigned long long sh64[256];
  __shared__ uint32_t shm[FP_PART_WORDS][256];
  const uint32_t tid = threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (b == NBUCKETS) {
    // fold the per-tile fingerprint partials: generation range per region, nil count
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
  // each thread owns a contiguous run of tiles
  const uint32_t per = (ntiles + 255) / 256;
  const uint32_t t0 = tid * per, t1 = min(ntiles, t0 + per);
  uint32_t c = 0;
  for (uint32_t t = t0; t < t1; ++t) c += tcount[(size_t)t * NBUCKETS + b];
  uint32_t total;
  uint32_t run = block_excl_scan_256<uint32_t>(c, sh32, total);
  for (uint32_t t = t0; t < t1; ++t) {
    toff[(size_t)t * NBUCKETS + b] = run;
    run += tcount[(size_t)t * NBUCKETS + b];
  }
  if (tid == 0) {
    btotal[b] = total;
    if (b >= (uint32_t)HOT_BUCKETS && b < NIL_BUCKET && total > (uint32_t)BUCKET_CAP)
      atomicOr(&ctl->err, ERR_V2_FALLBACK);
  }
  if (b < (uint32_t)HOT_BUCKETS) {
    unsigned long long s = 0;
    for (uint32_t t = t0; t < t1; ++t) s += thsum[(size_t)t * HOT_BUCKETS + b];
    unsigned long long tot;
    unsigned long long r = block_excl_scan_256<unsigned long long>(s, sh64, tot);
    for (uint32_t t = t0; t < t1; ++t) {
      hoff[(size_t)t * HOT_BUCKETS + b] = r;
      r += thsum[(size_t)t * HOT_BUCKETS + b];
    }
  }
}

// Bucket bases (exclusive scan of NBUCKETS totals) into LDS; every thread of a 256-block calls.
RL_DEV void bucket_bases(const uint32_t* __restrict__ btotal, uint32_t* s_base, uint32_t* sh_scan) {
  const uint32_t tid = threadIdx.x;
  constexpr int PER = (NBUCKETS + 255) / 256;
  uint32_t v[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t b = tid * PER + k;
    v[k] = b < (uint32_t)NBUCKETS ? btotal[b] : 0u;
    sum += v[k];
  }
  uint32_t total;
  uint32_t run = block_excl_scan_256<uint32_t>(sum, sh_scan, total);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t b = tid * PER + k;
    if (b < (uint32_t)NBUCKETS) s_base[b] = run;
    run += v[k];
  }
  if (tid == 0) s_base[NBUCKETS] = total;
  __syncthreads();
}

// ---------------------------------------------------------------------------
// k_bscatter — stable counting scatter into bucket order (same tile / item mapping as k_fp2)
// ---------------------------------------------------------------------------
constexpr int BS_IPT = V2_TILE / 256;

__global__ __launch_bounds__(256) void k_bscatter(const uint64_t* __restrict__ keys_orig,
                                                  const uint16_t* __restrict__ bkt, const uint32_t* __restrict__ hbuf,
                                                  uint32_t n, const uint32_t* __restrict__ btotal,
                                                  const uint32_t* __restrict__ toff,
                                                  const unsigned long long* __restrict__ hoff,
                                                  uint64_t* __restrict__ bkey, uint32_t* __restrict__ bidx,
                                                  uint64_t* __restrict__ bP, EngineCtl* ctl) {
  __shared__ uint32_t s_base[NBUCKETS + 1];
  __shared__ uint32_t s_wcnt[4][NBUCKETS];
  __shared__ unsigned long long s_whs[4][HOT_BUCKETS];
  __shared__ uint32_t sh_scan[256];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  if (ctl->err & (ERR_V2_FALLBACK | ERR_BAD_INPUT | ERR_BAD_TIME)) return;
  const uint32_t tile = blockIdx.x;
  for (int i = tid; i < 4 * NBUCKETS; i += 256) (&s_wcnt[0][0])[i] = 0;
  for (int i = tid; i < 4 * HOT_BUCKETS; i += 256) (&s_whs[0][0])[i] = 0;
  bucket_bases(btotal, s_base, sh_scan);  // includes a barrier

  uint32_t bk[BS_IPT], rank[BS_IPT];
  unsigned long long hp[BS_IPT];  // wave-local inclusive h prefix (hot descriptors)
  const uint64_t lt = lanemask_lt();
#pragma unroll
  for (int k = 0; k < BS_IPT; ++k) {
    const uint32_t i = tile * V2_TILE + wave * (V2_TILE / 4) + k * 64 + lane;
    const bool valid = i < n;
    const uint32_t d = valid ? bkt[i] : 0u;
    const uint32_t h = valid ? hbuf[i] : 0u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 12; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    // hot descriptors: inclusive prefix of h among same-bucket lanes of this round
    unsigned long long hin = 0;
    uint64_t hotm = __ballot(valid && d < (uint32_t)HOT_BUCKETS);
    while (hotm) {
      const uint32_t ld = (uint32_t)__ffsll((unsigned long long)hotm) - 1u;
      const uint32_t db = (uint32_t)__shfl((int)d, (int)ld, 64);
      const bool mine = valid && d == db;
      unsigned long long x = mine ? (unsigned long long)h : 0ull;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const unsigned long long y = __shfl_up(x, s, 64);
        if (lane >= (uint32_t)s) x += y;
      }
      if (mine) hin = x;
      hotm &= ~__ballot(mine);
    }
    uint32_t r = 0;
    unsigned long long hsum_before = 0;
    if (valid) {
      const uint32_t before = s_wcnt[wave][d];
      if (d < (uint32_t)HOT_BUCKETS) hsum_before = s_whs[wave][d];
      r = before + (uint32_t)__popcll(m & lt);
      const uint32_t leader = 63u - (uint32_t)__clzll((unsigned long long)m);  // highest lane of the group
      __builtin_amdgcn_wave_barrier();
      if (lane == leader) {
        s_wcnt[wave][d] = before + (uint32_t)__popcll(m);
        if (d < (uint32_t)HOT_BUCKETS) s_whs[wave][d] = hsum_before + hin;  // leader holds the group total
      }
    }
    __builtin_amdgcn_wave_barrier();
    bk[k] = d;
    rank[k] = r;
    hp[k] = hsum_before + hin;
  }
  __syncthreads();
  // per bucket: per-wave exclusive offsets (counts, and h-sums for hot buckets)
  for (int b = tid; b < NBUCKETS; b += 256) {
    const uint32_t c0 = s_wcnt[0][b], c1 = s_wcnt[1][b], c2 = s_wcnt[2][b];
    s_wcnt[0][b] = 0;
    s_wcnt[1][b] = c0;
    s_wcnt[2][b] = c0 + c1;
    s_wcnt[3][b] = c0 + c1 + c2;
    if (b < HOT_BUCKETS) {
      const unsigned long long h0 = s_whs[0][b], h1 = s_whs[1][b], h2 = s_whs[2][b];
      s_whs[0][b] = 0;
      s_whs[1][b] = h0;
      s_whs[2][b] = h0 + h1;
      s_whs[3][b] = h0 + h1 + h2;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < BS_IPT; ++k) {
    const uint32_t i = tile * V2_TILE + wave * (V2_TILE / 4) + k * 64 + lane;
    if (i >= n) continue;
    const uint32_t d = bk[k];
    const uint32_t pos = s_base[d] + toff[(size_t)tile * NBUCKETS + d] + s_wcnt[wave][d] + rank[k];
    bkey[pos] = keys_orig[i];
    bidx[pos] = i;
    if (d < (uint32_t)HOT_BUCKETS) bP[pos] = hoff[(size_t)tile * HOT_BUCKETS + d] + s_whs[wave][d] + hp[k];
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
                           uint32_t (*s_cnt)[RADIX], uint32_t* s_dstart, uint32_t* sh_scan) {
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
  // digit totals + per-wave exclusive offsets (threads 0..255 own one digit each), then an
  // exclusive scan over the 256 digit totals (every thread takes part in the barriers)
  uint32_t tot = 0;
  if (tid < RADIX) {
    for (int w = 0; w < BG_WAVES; ++w) {
      const uint32_t c = s_cnt[w][tid];
      s_cnt[w][tid] = tot;
      tot += c;
    }
    sh_scan[tid] = tot;
  }
  __syncthreads();
  for (int d = 1; d < RADIX; d <<= 1) {
    const uint32_t t = (tid < RADIX && tid >= (uint32_t)d) ? sh_scan[tid - d] : 0u;
    __syncthreads();
    if (tid < RADIX) sh_scan[tid] += t;
    __syncthreads();
  }
  if (tid < RADIX) s_dstart[tid] = sh_scan[tid] - tot;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < BG_ROUNDS; ++r) {
    const uint32_t k = wave * BG_PER_WAVE + r * 64 + lane;
    if (k < m) dst[s_dstart[dg[r]] + s_cnt[wave][dg[r]] + rk[r]] = src[k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(BG_THREADS) void k_bgroup(const uint64_t* __restrict__ bkey,
                                                       const uint32_t* __restrict__ bidx,
                                                       const uint64_t* __restrict__ bP,
                                                       const ItemRec* __restrict__ recs,
                                                       const uint32_t* __restrict__ btotal, uint32_t n_msd_wg,
                                                       uint64_t* __restrict__ skeys, SortedRec* __restrict__ srec,
                                                       uint32_t* __restrict__ wg_heads, EngineCtl* ctl) {
  __shared__ uint32_t s_base[NBUCKETS + 1];
  __shared__ uint32_t sh_scan[256];
  __shared__ uint64_t s_key[BG_MAX];
  __shared__ uint64_t s_lo[BG_MAX];
  __shared__ uint32_t s_h[BG_MAX];
  __shared__ uint32_t s_rule[BG_MAX];
  __shared__ uint16_t s_pa[BG_MAX], s_pb[BG_MAX];
  __shared__ uint32_t s_cnt[BG_WAVES][RADIX];
  __shared__ uint32_t s_dstart[RADIX];
  __shared__ BgScanEl s_wagg[BG_WAVES];
  __shared__ uint32_t s_mixed, s_heads;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (ctl->err & (ERR_V2_FALLBACK | ERR_BAD_INPUT | ERR_BAD_TIME)) return;
  // bucket bases with the first 256 threads' scan helper: all threads take part
  {
    constexpr int PER = (NBUCKETS + BG_THREADS - 1) / BG_THREADS;
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t b = tid * PER + k;
      v[k] = b < (uint32_t)NBUCKETS ? btotal[b] : 0u;
      sum += v[k];
    }
    // 512-thread exclusive scan via two 256 halves
    __shared__ uint32_t sh512[BG_THREADS];
    sh512[tid] = sum;
    __syncthreads();
    for (int d = 1; d < BG_THREADS; d <<= 1) {
      const uint32_t t = tid >= (uint32_t)d ? sh512[tid - d] : 0u;
      __syncthreads();
      sh512[tid] += t;
      __syncthreads();
    }
    uint32_t run = sh512[tid] - sum;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t b = tid * PER + k;
      if (b < (uint32_t)NBUCKETS) s_base[b] = run;
      run += v[k];
    }
    if (tid == BG_THREADS - 1) s_base[NBUCKETS] = sh512[tid];
    if (tid == 0) { s_mixed = 0; s_heads = 0; }
    __syncthreads();
  }
  const uint32_t hot_end = s_base[HOT_BUCKETS];
  if (blockIdx.x >= n_msd_wg) {
    // Hot chunk: each hot bucket is one key in arrival order; P comes from k_bscatter.
    const uint32_t c = blockIdx.x - n_msd_wg;
    const uint32_t p0 = c * HOT_CHUNK;
    if (p0 >= hot_end) {
      if (tid == 0) wg_heads[blockIdx.x] = 0;
      return;
    }
    const uint32_t p1 = min(hot_end, p0 + HOT_CHUNK);
    uint32_t heads = 0;
    for (uint32_t p = p0 + tid; p < p1; p += BG_THREADS) {
      // bucket of position p: last hot bucket whose base <= p
      uint32_t lo_b = 0, hi_b = HOT_BUCKETS - 1;
      while (lo_b < hi_b) {
        const uint32_t mid = (lo_b + hi_b + 1) / 2;
        if (s_base[mid] <= p) lo_b = mid; else hi_b = mid - 1;
      }
      const uint32_t head = s_base[lo_b];
      heads += head == p;
      const uint32_t idx = bidx[p];
      const ItemRec r = recs[idx];
      SortedRec o;
      o.P = bP[p];
      o.head = head;
      o.idx = idx;
      o.rule = r.rule;
      o.req = r.req;
      o.h = r.h;
      o.now_mod = r.now_mod;
      srec[p] = o;
      skeys[p] = bkey[p];
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
  if (m == 0) {
    if (tid == 0) wg_heads[blockIdx.x] = 0;
    return;
  }
  // load (key, fp_lo, h, rule) of the range; identity order = perm
  for (uint32_t k = tid; k < m; k += BG_THREADS) {
    const uint32_t idx = bidx[r0 + k];
    const ItemRec r = recs[idx];
    s_key[k] = bkey[r0 + k];
    s_lo[k] = r.fp_lo;
    s_h[k] = r.h;
    s_rule[k] = r.rule;
    s_pa[k] = (uint16_t)k;
  }
  __syncthreads();
  // Stable grouping: 3 LDS radix passes on the 24 key bits below the bucket bits. Equal keys
  // end adjacent; different buckets never interleave (they arrive bucket by bucket).
  lds_radix_pass(s_key, s_pa, s_pb, m, GK_SHIFT, s_cnt, s_dstart, sh_scan);
  lds_radix_pass(s_key, s_pb, s_pa, m, GK_SHIFT + 8, s_cnt, s_dstart, sh_scan);
  lds_radix_pass(s_key, s_pa, s_pb, m, GK_SHIFT + 16, s_cnt, s_dstart, sh_scan);
  uint16_t* perm = s_pb;
  // Runs of equal grouped bits holding two different identities (other region bits or a
  // fingerprint collision on 35 bits): regroup them stably (one thread; rare and short).
  for (uint32_t k = tid + 1; k < m; k += BG_THREADS) {
    const uint32_t a = perm[k - 1], b = perm[k];
    if (gkey(s_key[a]) == gkey(s_key[b]) && (s_key[a] != s_key[b] || s_lo[a] != s_lo[b])) s_mixed = 1;
  }
  __syncthreads();
  if (s_mixed && tid == 0) {
    uint32_t k = 0;
    while (k < m) {
      uint32_t e = k + 1;
      while (e < m && gkey(s_key[perm[e]]) == gkey(s_key[perm[k]])) ++e;
      // stable partition of perm[k..e) by identity, first-seen identity first
      for (uint32_t s = k; s < e;) {
        const uint32_t ref = perm[s];
        uint32_t w = s + 1;
        for (uint32_t t = s + 1; t < e; ++t) {
          const uint32_t x = perm[t];
          if (s_key[x] == s_key[ref] && s_lo[x] == s_lo[ref]) {
            // move x to position w, shifting [w, t) right by one
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
#pragma unroll
  for (int q = 0; q < BG_IPT; ++q) {
    const uint32_t k = k0 + q;
    if (k >= m) break;
    const uint32_t x = perm[k];
    run = bg_op(run, BgScanEl{hd[q], rc[q], k, (unsigned long long)s_h[x]});
    heads += hd[q];
    const uint32_t idx = bidx[r0 + x];
    const ItemRec r = recs[idx];
    SortedRec o;
    o.P = run.s;
    o.head = (r0 + run.hp) | (run.o ? HEAD_MIXED_RULE : 0u);
    o.idx = idx;
    o.rule = r.rule;
    o.req = r.req;
    o.h = r.h;
    o.now_mod = r.now_mod;
    srec[r0 + k] = o;
    skeys[r0 + k] = s_key[x];
  }
  for (int d = 32; d >= 1; d >>= 1) heads += __shfl_xor(heads, d, 64);
  if (lane == 0 && heads) atomicAdd(&s_heads, heads);
  __syncthreads();
  if (tid == 0) wg_heads[blockIdx.x] = s_heads;
}

// Hot-set candidates: recompute the prefix lane state (a, b) of each candidate's first
// descriptor (the batch input is still resident).
__global__ void k_cand_state(DevBatch in, const DevRule* __restrict__ rules, uint64_t seed, HotCand* cand,
                             const EngineCtl* ctl) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  const uint32_t nc = min((uint32_t)CAND_MAX, ctl->tile_ctr[CAND_CTR][0]);
  if (i >= nc) return;
  HotCand c = cand[i];
  const uint32_t d = c.first_idx;
  const uint32_t o0 = in.off[d], o1 = in.off[d + 1];
  const uint32_t unit = rules[c.rule].unit;
  FpState s = fp_init(o1 - o0, unit, seed);
  hash_prefix(in.blob, o0, o1 - o0, s);
  c.a = s.a;
  c.b = s.b;
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
                EngineCtl* ctl) {
  DevBatch d;
  d.n_desc = b.n_desc;
  d.n_req = b.n_req;
  d.blob_bytes = b.blob_bytes;
  d.pad = 0;
  d.blob = b.prefix_blob;
  d.off = b.prefix_off;
  d.rule = b.rule_id;
  d.req_of = b.req_of;
  d.now = b.now;
  d.hits = b.hits_addend;
  hipLaunchKernelGGL(k_fp2, dim3(v2_tiles(b.n_desc)), dim3(256), 0, st, d, rules, n_rules, seed, hot, keys_orig, recs,
                     bkt, hbuf, out, req_thr, fpart, tcount, thsum, ctl);
}
void launch_bscan(hipStream_t st, const uint32_t* tcount, const unsigned long long* thsum, uint32_t n,
                  uint32_t* toff, unsigned long long* hoff, uint32_t* btotal, const uint32_t* fpart, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_bscan, dim3(NBUCKETS + 1), dim3(256), 0, st, tcount, thsum, v2_tiles(n), toff, hoff, btotal,
                     fpart, ctl);
}
void launch_bscatter(hipStream_t st, const uint64_t* keys_orig, const uint16_t* bkt, const uint32_t* hbuf, uint32_t n,
                     const uint32_t* btotal, const uint32_t* toff, const unsigned long long* hoff, uint64_t* bkey,
                     uint32_t* bidx, uint64_t* bP, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_bscatter, dim3(v2_tiles(n)), dim3(256), 0, st, keys_orig, bkt, hbuf, n, btotal, toff, hoff,
                     bkey, bidx, bP, ctl);
}
void launch_bgroup(hipStream_t st, const uint64_t* bkey, const uint32_t* bidx, const uint64_t* bP,
                   const ItemRec* recs, const uint32_t* btotal, uint32_t n, uint64_t* skeys, SortedRec* srec,
                   uint32_t* wg_heads, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_bgroup, dim3(v2_msd_wgs(n) + v2_hot_wgs(n)), dim3(BG_THREADS), 0, st, bkey, bidx, bP, recs,
                     btotal, v2_msd_wgs(n), skeys, srec, wg_heads, ctl);
}
void launch_cand_state(hipStream_t st, const rl_batch& b, const DevRule* rules, uint64_t seed, HotCand* cand,
                       const EngineCtl* ctl) {
  DevBatch d;
  d.n_desc = b.n_desc;
  d.n_req = b.n_req;
  d.blob_bytes = b.blob_bytes;
  d.pad = 0;
  d.blob = b.prefix_blob;
  d.off = b.prefix_off;
  d.rule = b.rule_id;
  d.req_of = b.req_of;
  d.now = b.now;
  d.hits = b.hits_addend;
  hipLaunchKernelGGL(k_cand_state, dim3(CAND_MAX / 64), dim3(64), 0, st, d, rules, seed, cand, ctl);
}

}  // namespace rlhip
