// rl_kernels.hip — CDNA4 (gfx950) kernels of the batched fixed-window decision path.
//
// One batch = descriptors of many RateLimitRequests in serial (enqueue) order. The
// pipeline reproduces, per key, the counter value that a pipelined Redis INCRBY would
// return in that order (src/redis/fixed_cache_impl.go:26-29,55-102) and the decisions
// of BaseRateLimiter.GetResponseDescriptorStatus (src/limiter/base_limiter.go:70-177):
//
//   k_fingerprint  hash each key prefix + window start -> 128-bit fingerprint, sort key,
//                  arrival-order record; radix histograms for every sort pass
//   k_hist_scan    exclusive scan of the digit histograms
//   k_sort_pass    stable LSD radix pass (8-bit digit) with decoupled look-back (xN)
//   k_scan         segment heads + segmented inclusive prefix sum of hits_addend
//                  (decoupled look-back), sorted-order record
//   k_leader       one thread per unique key: probe/insert the HBM counter table,
//                  find the local-cache freeze point, write the new counter
//   k_decide       per descriptor: INCRBY post-value = base + prefix, status + stats
//
// Wave size is 64 everywhere; blocks are 256 threads (4 waves).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"
#include "rl_device.h"
#include "rl_decide.h"

namespace rlhip {

#ifdef RL_STAMPS
// Diagnostic build only: per-block phase timestamps of the last sort pass (s_memtime).
__device__ uint64_t g_stamps[4096][8];
#define STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

// Window start, table place and fingerprint of one valid descriptor (both loaders).
RL_DEV void fp_place(const FpState& s, int64_t now, const DevRule& R, uint64_t& key, ItemRec& rec, uint32_t& region,
                     uint32_t& uw) {
  const int64_t widx = div_const(now, R.unit);
  const uint32_t ws = (uint32_t)(widx * (int64_t)R.div);  // (now/divider)*divider  cache_key.go:66-68
  const Place pl = place_of(ws);
  uint64_t hi, lo;
  fp_final(s, (uint64_t)ws, hi, lo);
  region = pl.region;
  key = make_sort_key(region, hi);
  rec.fp_lo = lo;
  rec.now_mod = (int32_t)(now - (int64_t)ws);
  rec.gen = pl.gen;
  uw = (R.unit - 1u) * 2u + (uint32_t)(widx & 1);
}

__global__ __launch_bounds__(256) void k_fingerprint(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                                     uint64_t seed, uint64_t* __restrict__ keys_orig,
                                                     ItemRec* __restrict__ recs, rl_status* __restrict__ out,
                                                     uint32_t* __restrict__ req_thr, uint32_t* __restrict__ fpart,
                                                     EngineCtl* ctl) {
  __shared__ uint32_t sh_f[FP_PART_WORDS];  // FP_* layout; gmin holds ~min (zero-init max)
  __shared__ uint32_t sh_err;
  const uint32_t tid = threadIdx.x;
  if (tid < FP_PART_WORDS) sh_f[tid] = 0;
  if (tid == 0) sh_err = 0;
  __syncthreads();

  const uint32_t i = blockIdx.x * 256 + tid;
  uint32_t err = 0;
  bool nil = true;
  uint64_t key = NIL_KEY;
  uint32_t region = 8, gen = 0, uw = 8;  // uw: unit window slot (v4 hot keys only; unused here)
  if (i < in.n_desc && in.recs) {
    // Routed record (multi-GPU owner): the key prefix arrives as its fingerprint lane state.
    const RRec x = in.recs[i];
    if (req_thr) req_thr[i] = 0;  // one ThrottleMillis slot per record (none for raw replies)
    ItemRec rec;
    rec.rule = rrec_rule(x.rule);
    rec.req = x.greq;
    rec.h = x.h;
    rec.fp_lo = 0;
    rec.now_mod = 0;
    rec.gen = 0;
    rec.jit = rrec_jit(x.rule);
    if (rec.rule >= n_rules) {
      err |= ERR_BAD_INPUT;
    } else if ((int64_t)x.now > MAX_NOW) {
      err |= ERR_BAD_TIME;
    } else {
      fp_place(FpState{x.a, x.b}, (int64_t)x.now, rules[rec.rule], key, rec, region, uw);
      gen = rec.gen;
      nil = false;
    }
    recs[i] = rec;
    keys_orig[i] = key;
  } else if (i < in.n_desc) {
    const uint32_t r = in.rule[i];
    const uint32_t q = in.req_of[i];
    const bool q_ok = q < in.n_req;
    const int64_t now = q_ok ? in.now[q] : 0;
    const uint32_t ha = q_ok ? in.hits[q] : 1u;
    // Zero DoLimitResponse.ThrottleMillis of the requests this descriptor opens
    // (k_decide max-reduces into it); the last descriptor also zeroes trailing requests.
    if (q_ok && req_thr) {  // (raw replies: no ThrottleMillis slots)
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
    rec.jit = desc_jit(in, i);
    // batch layout checks (the device validates every submit form): prefix offsets in
    // order and inside the blob, request indices non-decreasing
    const uint32_t o0 = in.off[i], o1 = in.off[i + 1];
    const bool layout_ok = o0 <= o1 && o1 <= in.blob_bytes && (i == 0 || in.req_of[i - 1] <= q);
    if (!layout_ok) err |= ERR_BAD_INPUT;
    if (r != RL_NIL_RULE && (r >= n_rules || !q_ok)) err |= ERR_BAD_INPUT;
    if (r != RL_NIL_RULE && r < n_rules && q_ok && layout_ok) {
      if (now < 0 || now > MAX_NOW) {
        err |= ERR_BAD_TIME;
      } else {
        const DevRule R = rules[r];
        FpState s = fp_init(o1 - o0, seed);
        hash_prefix(in.blob, o0, o1 - o0, s);
        fp_place(s, now, R, key, rec, region, uw);
        gen = rec.gen;
        nil = false;
      }
    }
    recs[i] = rec;
    keys_orig[i] = key;
    if (nil && in.raw) {
      emit_raw(out, i, 0u, RAW_NIL);
    } else if (nil) {
      // GetResponseDescriptorStatus("" key) -> {OK, nil limit, 0}  base_limiter.go:72-75
      rl_status st;
      st.code_flags = RL_CODE_OK;
      st.limit_remaining = 0;
      st.reset_s = 0;
      st.over_limit_delta = 0;
      st.near_limit_delta = 0;
      out[i] = st;
    }
  }
  // Per-wave reductions, then one LDS op per wave.
  const uint64_t nilmask = __ballot(i < in.n_desc && nil);
  const uint32_t lane = __lane_id();
  if (lane == 0 && nilmask) atomicAdd(&sh_f[FP_NIL], (uint32_t)__popcll(nilmask));
  for (uint32_t rg = 0; rg < 8; ++rg) {
    const bool mine = region == rg;
    const uint64_t m = __ballot(mine);
    if (!m) continue;
    const uint32_t mn = wave_min_u32(mine ? gen : 0xFFFFFFFFu);
    const uint32_t mx = wave_max_u32(mine ? gen : 0u);
    if (lane == 0) {
      atomicMax(&sh_f[FP_GMIN + rg], ~mn);
      atomicMax(&sh_f[FP_GMAX + rg], mx);
      atomicAdd(&sh_f[FP_CNT + rg], (uint32_t)__popcll(m));
    }
  }
  if (err) atomicOr(&sh_err, err);
  __syncthreads();
  // Block partials (plain stores); k_histogram folds them, k_hist_scan's last block reduces.
  uint32_t* fp = fpart + (size_t)blockIdx.x * FP_PART_WORDS;
  if (tid < FP_PART_WORDS) fp[tid] = sh_f[tid];
  if (tid == 0 && sh_err) atomicOr(&ctl->err, sh_err);
}

// Per-block partial histograms of npasses 8-bit digits (plain stores, no global atomics):
// part[block][p][256]; block b covers keys [b*HIST_CHUNK, (b+1)*HIST_CHUNK). The same
// block also folds the fingerprint partials of its items (generation range, nil count).
constexpr int HIST_CHUNK = 4096;
constexpr int HIST_SUB = 16;  // histogram partials are pre-reduced into HIST_SUB slices per pass
__global__ __launch_bounds__(1024) void k_histogram(const uint64_t* __restrict__ keys, uint32_t n, int lo_bit,
                                                     int npasses, uint32_t* __restrict__ part,
                                                     const uint32_t* __restrict__ fpart, uint32_t* __restrict__ fpart2) {
  __shared__ uint32_t sh_hist[8][RADIX];
  const uint32_t tid = threadIdx.x;
  for (int i = tid; i < 8 * RADIX; i += 1024) (&sh_hist[0][0])[i] = 0;
  __syncthreads();
  const uint32_t b0 = blockIdx.x * HIST_CHUNK, b1 = min(n, b0 + HIST_CHUNK);
  for (uint32_t i = b0 + tid; i < b1; i += 1024) {
    const uint64_t key = keys[i];
    for (int p = 0; p < npasses; ++p) atomicAdd(&sh_hist[p][(key >> (lo_bit + 8 * p)) & 0xFF], 1u);
  }
  if (fpart && tid < FP_PART_WORDS) {
    // fingerprint blocks are 256 items: this chunk covers HIST_CHUNK / 256 of them
    const uint32_t f0 = b0 / 256, f1 = (b1 + 255) / 256;
    uint32_t v = 0;
    for (uint32_t f = f0; f < f1; ++f) {
      const uint32_t x = fpart[(size_t)f * FP_PART_WORDS + tid];
      v = fp_is_max((int)tid) ? (x > v ? x : v) : v + x;
    }
    fpart2[(size_t)blockIdx.x * FP_PART_WORDS + tid] = v;
  }
  __syncthreads();
  for (int i = tid; i < npasses * RADIX; i += 1024)
    part[(size_t)blockIdx.x * MAX_PASSES * RADIX + i] = (&sh_hist[0][0])[i];
}

// Block (p, q), q < HIST_SUB: sum slice q of pass p's partial histograms -> sub[p][q][256].
// Last block (if fp_blocks): reduce the folded fingerprint partials into ctl (the only
// writer of gen_min / gen_max / n_nil) and run the capacity check before any table write.
__global__ __launch_bounds__(256) void k_hist_scan(const uint32_t* __restrict__ part, uint32_t nblocks,
                                                   uint32_t* __restrict__ sub, int npasses,
                                                   const uint32_t* __restrict__ fpart2, uint32_t fp_blocks,
                                                   uint32_t n_all, const RegionOcc* __restrict__ occ, EngineCtl* ctl,
                                                   uint32_t lag) {
  const uint32_t tid = threadIdx.x;
  if ((int)blockIdx.x == npasses * HIST_SUB) {
    __shared__ uint32_t shm[FP_PART_WORDS][256];
    for (int w = 0; w < FP_PART_WORDS; ++w) {
      uint32_t v = 0;
      for (uint32_t g = tid; g < fp_blocks; g += 256) {
        const uint32_t x = fpart2[(size_t)g * FP_PART_WORDS + w];
        v = fp_is_max(w) ? (x > v ? x : v) : v + x;
      }
      shm[w][tid] = v;
    }
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
      if (tid < (uint32_t)d)
        for (int w = 0; w < FP_PART_WORDS; ++w) {
          const uint32_t a = shm[w][tid], c = shm[w][tid + d];
          shm[w][tid] = fp_is_max(w) ? (a > c ? a : c) : a + c;
        }
      __syncthreads();
    }
    if (tid < 8) ctl->gen_min[tid] = ~shm[FP_GMIN + tid][0];  // partials hold ~min
    else if (tid < 16) ctl->gen_max[tid - 8] = shm[FP_GMAX + tid - 8][0];
    else if (tid == 16) ctl->n_nil = shm[FP_NIL][0];
    else if (tid == 17) {
      uint32_t gmax[8], cnt[8];
      for (int r = 0; r < 8; ++r) {
        gmax[r] = shm[FP_GMAX + r][0];
        cnt[r] = shm[FP_CNT + r][0];
      }
      if (!capacity_ok(occ, gmax, cnt, lag)) atomicOr(&ctl->err, ERR_TABLE_FULL);
    }
    return;
  }
  const uint32_t p = blockIdx.x / HIST_SUB, q = blockIdx.x % HIST_SUB;
  const uint32_t per = (nblocks + HIST_SUB - 1) / HIST_SUB;
  const uint32_t g0 = q * per, g1 = min(nblocks, g0 + per);
  const size_t stride = (size_t)MAX_PASSES * RADIX;
  const uint32_t* b = part + p * RADIX + tid;
  uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
  uint32_t g = g0;
  for (; g + 4 <= g1; g += 4) {
    v0 += b[(g + 0) * stride];
    v1 += b[(g + 1) * stride];
    v2 += b[(g + 2) * stride];
    v3 += b[(g + 3) * stride];
  }
  for (; g < g1; ++g) v0 += b[g * stride];
  sub[((size_t)p * HIST_SUB + q) * RADIX + tid] = v0 + v1 + v2 + v3;
}

// Exclusive digit offsets of one pass from its HIST_SUB pre-reduced slices (block-wide scan);
// every sort block recomputes this (16 loads per thread) instead of a separate launch.
RL_DEV uint32_t bin_offset_from_sub(const uint32_t* __restrict__ sub_p, uint32_t* sh_scan) {
  const uint32_t tid = threadIdx.x;
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < HIST_SUB; ++q) v += sub_p[q * RADIX + tid];
  sh_scan[tid] = v;
  __syncthreads();
  for (int d = 1; d < RADIX; d <<= 1) {
    const uint32_t t = tid >= (uint32_t)d ? sh_scan[tid - d] : 0u;
    __syncthreads();
    sh_scan[tid] += t;
    __syncthreads();
  }
  const uint32_t r = sh_scan[tid] - v;
  __syncthreads();
  return r;
}

// Gather helpers for the full-fingerprint fallback sort.
__global__ void k_fallback_lo_keys(const ItemRec* __restrict__ recs, const uint64_t* __restrict__ keys_orig,
                                   uint32_t n, uint64_t* __restrict__ k_out, uint32_t* __restrict__ v_out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  k_out[i] = keys_orig[i] == NIL_KEY ? 0ull : recs[i].fp_lo;
  v_out[i] = i;
}
__global__ void k_gather_keys(const uint64_t* __restrict__ keys_orig, const uint32_t* __restrict__ vals, uint32_t n,
                              uint64_t* __restrict__ k_out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  k_out[i] = keys_orig[vals[i]];
}

// ---------------------------------------------------------------------------
// k_sort_pass — one stable LSD pass over an 8-bit digit ("onesweep"): rank inside
// the 4096-key tile with wave ballots, publish per-digit tile counts, decoupled
// look-back over earlier tiles (tile ids come from an atomic ticket, so a tile only
// ever waits on tiles already running), stage the tile in LDS in digit order and
// write each digit run contiguously.
// ---------------------------------------------------------------------------
#ifndef RL_SORT_IPT
#define RL_SORT_IPT 16
#endif
#ifndef RL_SORT_LB_WIN
#define RL_SORT_LB_WIN 8
#endif
constexpr int SORT_IPT = RL_SORT_IPT;  // keys per thread
constexpr int SORT_TILE = 256 * SORT_IPT;
constexpr int SORT_LB_WIN = RL_SORT_LB_WIN;
constexpr uint32_t LB_AGG = 1u << 30;
constexpr uint32_t LB_INC = 2u << 30;
constexpr uint32_t LB_MASK = (1u << 30) - 1;

__global__ __launch_bounds__(256) void k_sort_pass(const uint64_t* __restrict__ keys_in,
                                                   const uint32_t* __restrict__ vals_in,
                                                   uint64_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                   uint32_t n, int shift, const uint32_t* __restrict__ sub_p,
                                                   uint32_t* __restrict__ lookback, uint32_t* tile_ctr,
                                                   EngineCtl* ctl) {
  __shared__ uint64_t s_keys[SORT_TILE];
  __shared__ uint32_t s_vals[SORT_TILE];
  __shared__ uint32_t s_wcnt[4][RADIX];   // per-wave digit counts -> per-wave exclusive offsets
  __shared__ uint32_t s_tstart[RADIX];    // tile-local exclusive digit offsets
  __shared__ uint32_t s_gbase[RADIX];     // global output base per digit for this tile
  __shared__ uint32_t s_tile;

  STAMP(0);
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = tid >> 6;
  const uint32_t lane = tid & 63;
#ifdef RL_SORT_TICKET
  if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
#else
  // Tile = blockIdx: blocks start in launch order on gfx950 (MI355X_MICROARCH.md, dispatch),
  // so a tile waits only on earlier, already-running tiles; every spin is bounded (ERR_SPIN).
  if (tid == 0) s_tile = blockIdx.x;
#endif
  for (int i = tid; i < 4 * RADIX; i += 256) (&s_wcnt[0][0])[i] = 0;
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t tbase = tile * SORT_TILE;

  uint64_t key[SORT_IPT];
  uint32_t val[SORT_IPT];
  uint32_t rank[SORT_IPT];
#pragma unroll
  for (int k = 0; k < SORT_IPT; ++k) {
    const uint32_t p = tbase + wave * (SORT_TILE / 4) + k * 64 + lane;
    if (p < n) {
      key[k] = keys_in[p];
      val[k] = vals_in ? vals_in[p] : p;
    } else {
      key[k] = ~0ull;
      val[k] = 0;
    }
  }
  __syncthreads();
  STAMP(1);
  // Per-wave stable ranking, round by round in position order.
  const uint64_t lt = lanemask_lt();
#pragma unroll
  for (int k = 0; k < SORT_IPT; ++k) {
    const uint32_t p = tbase + wave * (SORT_TILE / 4) + k * 64 + lane;
    const bool valid = p < n;
    const uint32_t d = (uint32_t)(key[k] >> shift) & 0xFFu;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < RADIX_BITS; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    uint32_t r = 0;
    if (valid) {
      const uint32_t before = s_wcnt[wave][d];
      r = before + (uint32_t)__popcll(m & lt);
      const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
      __builtin_amdgcn_wave_barrier();
      if (lane == leader) s_wcnt[wave][d] = before + (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    rank[k] = r;
  }
  __syncthreads();
  STAMP(2);
  // Thread tid owns digit tid: tile count, per-wave exclusive offsets.
  uint32_t cnt = 0;
  {
    const uint32_t c0 = s_wcnt[0][tid], c1 = s_wcnt[1][tid], c2 = s_wcnt[2][tid], c3 = s_wcnt[3][tid];
    s_wcnt[0][tid] = 0;
    s_wcnt[1][tid] = c0;
    s_wcnt[2][tid] = c0 + c1;
    s_wcnt[3][tid] = c0 + c1 + c2;
    cnt = c0 + c1 + c2 + c3;
  }
  // Publish this tile's aggregate for digit tid, then look back.
  uint32_t* lb = lookback + (size_t)tile * RADIX;
  if (tile == 0) {
    st_relaxed(&lb[tid], LB_INC | cnt);
  } else {
    st_relaxed(&lb[tid], LB_AGG | cnt);
  }
  STAMP(3);
  // Windowed look-back: SORT_LB_WIN predecessor words of this digit in flight per round trip.
  uint32_t excl = 0;
  if (tile > 0) {
    int32_t j = (int32_t)tile - 1;
    uint32_t spins = 0;
    for (;;) {
      uint32_t v[SORT_LB_WIN];
#pragma unroll
      for (int w = 0; w < SORT_LB_WIN; ++w)
        v[w] = (j - w >= 0) ? ld_relaxed(&lookback[(size_t)(j - w) * RADIX + tid]) : LB_INC;
      int w = 0;
      bool done = false;
#pragma unroll
      for (int k = 0; k < SORT_LB_WIN; ++k) {
        if (done || w != k) continue;
        const uint32_t f = v[k] & ~LB_MASK;
        if (f == 0) continue;  // not published yet: stop here, re-poll from this tile
        excl += v[k] & LB_MASK;
        if (f == LB_INC) done = true;
        w = k + 1;
      }
      if (done) break;
      j -= w;
      if (w < SORT_LB_WIN) {
        if (++spins > SPIN_LIMIT) { atomicOr(&ctl->err, ERR_SPIN); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    st_relaxed(&lb[tid], LB_INC | (excl + cnt));
  }
  __syncthreads();
  STAMP(4);
  s_gbase[tid] = bin_offset_from_sub(sub_p, s_tstart) + excl;
  // Tile-local exclusive scan of digit counts (block scan over 256 threads).
  s_tstart[tid] = cnt;
  __syncthreads();
  for (int d = 1; d < RADIX; d <<= 1) {
    const uint32_t t = tid >= (uint32_t)d ? s_tstart[tid - d] : 0u;
    __syncthreads();
    s_tstart[tid] += t;
    __syncthreads();
  }
  s_tstart[tid] -= cnt;
  __syncthreads();
  STAMP(5);
  // Stage the tile in digit order.
#pragma unroll
  for (int k = 0; k < SORT_IPT; ++k) {
    const uint32_t p = tbase + wave * (SORT_TILE / 4) + k * 64 + lane;
    if (p < n) {
      const uint32_t d = (uint32_t)(key[k] >> shift) & 0xFFu;
      const uint32_t pos = s_tstart[d] + s_wcnt[wave][d] + rank[k];
      s_keys[pos] = key[k];
      s_vals[pos] = val[k];
    }
  }
  __syncthreads();
  STAMP(6);
  const uint32_t tvalid = n - tbase < (uint32_t)SORT_TILE ? n - tbase : (uint32_t)SORT_TILE;
  for (uint32_t i = tid; i < tvalid; i += 256) {
    const uint64_t k = s_keys[i];
    const uint32_t d = (uint32_t)(k >> shift) & 0xFFu;
    const uint32_t o = s_gbase[d] + (i - s_tstart[d]);
    keys_out[o] = k;
    vals_out[o] = s_vals[i];
  }
  __syncthreads();
  STAMP(7);
}

// ---------------------------------------------------------------------------
// k_scan — segment heads + segmented inclusive prefix sum of h over the sorted batch.
// Scan element (f, s, hp, o): f = segment starts inside, s = sum since the last head,
// hp = last head position, o = rule changed within the segment. op(A,B) = B.f ? B :
// (A.f, A.s+B.s, A.hp, A.o|B.o) — associative. Tiles chain through decoupled look-back
// on two self-flagged 64-bit granules per tile (sum|o and head position).
// ---------------------------------------------------------------------------
#ifndef RL_SCAN_IPT
#define RL_SCAN_IPT 8
#endif
constexpr int SCAN_IPT = RL_SCAN_IPT;
constexpr int SCAN_TILE = 256 * SCAN_IPT;
constexpr uint64_t LB64_AGG = 1ull << 62;
constexpr uint64_t LB64_INC = 2ull << 62;
constexpr uint64_t LB64_FLAGS = 3ull << 62;
constexpr uint64_t LB64_O = 1ull << 61;
constexpr uint64_t LB64_SUM = (1ull << 61) - 1;

struct ScanEl {
  uint32_t f;
  uint32_t o;
  uint32_t hp;
  uint64_t s;
};
RL_DEV ScanEl scan_op(const ScanEl& a, const ScanEl& b) {
  if (b.f) return b;
  ScanEl r;
  r.f = a.f;
  r.s = a.s + b.s;
  r.hp = a.hp;
  r.o = a.o | b.o;
  return r;
}
RL_DEV ScanEl shfl_up_el(const ScanEl& x, int d) {
  ScanEl r;
  r.f = __shfl_up(x.f, d, 64);
  r.o = __shfl_up(x.o, d, 64);
  r.hp = __shfl_up(x.hp, d, 64);
  r.s = __shfl_up(x.s, d, 64);
  return r;
}

__global__ __launch_bounds__(256) void k_scan(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ svals,
                                              const ItemRec* __restrict__ recs, uint32_t n_all, int lo_bit,
                                              int check_mixed, SortedRec* __restrict__ srec,
                                              uint64_t* __restrict__ lb_sum, uint64_t* __restrict__ lb_head,
                                              uint32_t* tile_ctr, uint32_t* __restrict__ tile_heads,
                                              EngineCtl* ctl) {
  __shared__ ScanEl s_wagg[4];
  __shared__ uint64_t s_lastkey[256];
  __shared__ uint64_t s_lastlo[256];
  __shared__ uint32_t s_lastrule[256];
  __shared__ uint32_t s_tile;
  __shared__ ScanEl s_carry;
  __shared__ uint32_t s_heads;
  __shared__ uint32_t s_mixed;

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wave = tid >> 6;
  if (tid == 0) {
    s_tile = atomicAdd(tile_ctr, 1u);
    s_heads = 0;
    s_mixed = 0;
  }
  __syncthreads();
  const uint32_t n = n_all - ctl->n_nil;  // written by k_fingerprint (earlier launch)
  const uint32_t tile = s_tile;
  const uint32_t base = tile * SCAN_TILE + tid * SCAN_IPT;

  uint64_t key[SCAN_IPT], lo[SCAN_IPT];
  uint32_t idx[SCAN_IPT], rule[SCAN_IPT], req[SCAN_IPT], hh[SCAN_IPT];
  int32_t nm[SCAN_IPT];
#pragma unroll
  for (int k = 0; k < SCAN_IPT; ++k) {
    const uint32_t p = base + k;
    if (p < n) {
      key[k] = skeys[p];
      idx[k] = svals[p];
      const ItemRec r = recs[idx[k]];
      lo[k] = r.fp_lo;
      rule[k] = r.rule;
      req[k] = r.req;
      hh[k] = r.h;
      nm[k] = r.now_mod;
    } else {
      key[k] = NIL_KEY;
      idx[k] = 0;
      lo[k] = 0;
      rule[k] = 0;
      req[k] = 0;
      hh[k] = 0;
      nm[k] = 0;
    }
  }
  // Predecessor of this thread's first item.
  s_lastkey[tid] = key[SCAN_IPT - 1];
  s_lastlo[tid] = lo[SCAN_IPT - 1];
  s_lastrule[tid] = rule[SCAN_IPT - 1];
  __syncthreads();
  uint64_t pkey, plo;
  uint32_t prule;
  if (tid > 0) {
    pkey = s_lastkey[tid - 1];
    plo = s_lastlo[tid - 1];
    prule = s_lastrule[tid - 1];
  } else if (base > 0 && base - 1 < n) {
    pkey = skeys[base - 1];
    const ItemRec r = recs[svals[base - 1]];
    plo = r.fp_lo;
    prule = r.rule;
  } else {
    pkey = NIL_KEY;
    plo = 0;
    prule = 0;
  }
  // Thread-local segmented reduction.
  uint32_t head[SCAN_IPT];
  uint32_t rchg[SCAN_IPT];
  ScanEl t{0, 0, 0, 0};
  uint32_t nheads = 0, mixed = 0;
#pragma unroll
  for (int k = 0; k < SCAN_IPT; ++k) {
    const uint32_t p = base + k;
    const bool valid = p < n;
    const bool diff = (p == 0) || key[k] != pkey || lo[k] != plo;
    head[k] = valid && diff;
    rchg[k] = valid && !diff && rule[k] != prule;
    if (valid && p > 0 && diff && check_mixed && ((key[k] ^ pkey) >> lo_bit) == 0) mixed = 1;
    nheads += head[k];
    ScanEl e{head[k], rchg[k], p, (uint64_t)hh[k]};
    t = scan_op(t, e);
    pkey = key[k];
    plo = lo[k];
    prule = rule[k];
  }
  // Wave inclusive scan of thread aggregates.
  ScanEl incl = t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const ScanEl y = shfl_up_el(incl, d);
    if (lane >= (uint32_t)d) incl = scan_op(y, incl);
  }
  if (lane == 63) s_wagg[wave] = incl;
  if (nheads) atomicAdd(&s_heads, nheads);
  if (mixed) s_mixed = 1;
  ScanEl wexcl = shfl_up_el(incl, 1);
  if (lane == 0) wexcl = ScanEl{0, 0, 0, 0};
  __syncthreads();
  // Tile aggregate and this wave's offset.
  ScanEl woff{0, 0, 0, 0};
  ScanEl tagg{0, 0, 0, 0};
  for (uint32_t w = 0; w < 4; ++w) {
    if (w == wave) woff = tagg;
    tagg = scan_op(tagg, s_wagg[w]);
  }
  // Decoupled look-back by wave 0: 64 predecessor tiles per round trip.
  if (wave == 0) {
    if (lane == 0) {
      if (tagg.f || tile == 0) {
        // carry-out independent of predecessors (the part after this tile's last head)
        st_relaxed64(&lb_head[tile], LB64_INC | tagg.hp);
        st_relaxed64(&lb_sum[tile], LB64_INC | (tagg.o ? LB64_O : 0) | (tagg.s & LB64_SUM));
      } else {
        st_relaxed64(&lb_sum[tile], LB64_AGG | (tagg.o ? LB64_O : 0) | (tagg.s & LB64_SUM));
      }
    }
    ScanEl carry{0, 0, 0, 0};
    if (tile > 0) {
      int32_t top = (int32_t)tile - 1;
      uint64_t acc_s = 0;
      uint32_t acc_o = 0;
      uint32_t spins = 0;
      for (;;) {
        const int32_t t = top - (int32_t)lane;
        const uint64_t v = t >= 0 ? ld_relaxed64(&lb_sum[t]) : LB64_INC;
        const uint64_t hv = t >= 0 ? ld_relaxed64(&lb_head[t]) : LB64_INC;
        const uint64_t fs = v & LB64_FLAGS;
        const bool is_inc = fs == LB64_INC && (hv & LB64_FLAGS) != 0;
        const bool not_ready = fs == 0 || (fs == LB64_INC && (hv & LB64_FLAGS) == 0);
        const uint64_t incm = __ballot(is_inc);
        const uint64_t zm = __ballot(not_ready);
        const uint32_t fi = incm ? (uint32_t)__ffsll((unsigned long long)incm) - 1u : 64u;
        const uint32_t fz = zm ? (uint32_t)__ffsll((unsigned long long)zm) - 1u : 64u;
        const uint32_t take = fi < fz ? fi + 1u : fz;  // lanes [0, take) contribute
        uint64_t cs = lane < take ? (v & LB64_SUM) : 0ull;
        uint32_t co = (lane < take && (v & LB64_O)) ? 1u : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          cs += __shfl_xor(cs, d, 64);
          co |= __shfl_xor(co, d, 64);
        }
        acc_s += cs;
        acc_o |= co;
        if (fi < fz) {
          const uint32_t hp = (uint32_t)__shfl((uint32_t)(hv & 0xFFFFFFFFull), (int)fi, 64);
          carry = ScanEl{1, acc_o, hp, acc_s};
          break;
        }
        top -= (int32_t)fz;
        if (fz < 64u) {
          if (++spins > SPIN_LIMIT) {
            if (lane == 0) atomicOr(&ctl->err, ERR_SPIN);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (lane == 0 && !tagg.f) {
        const ScanEl out = scan_op(carry, tagg);
        st_relaxed64(&lb_head[tile], LB64_INC | out.hp);
        st_relaxed64(&lb_sum[tile], LB64_INC | (out.o ? LB64_O : 0) | (out.s & LB64_SUM));
      }
    }
    if (lane == 0) {
      s_carry = carry;
      tile_heads[tile] = s_heads;
      if (s_mixed) atomicOr(&ctl->err, ERR_NEED_RESORT);
    }
  }
  __syncthreads();
  ScanEl run = scan_op(scan_op(s_carry, woff), wexcl);
#pragma unroll
  for (int k = 0; k < SCAN_IPT; ++k) {
    const uint32_t p = base + k;
    if (p >= n) break;
    ScanEl e{head[k], rchg[k], p, (uint64_t)hh[k]};
    run = scan_op(run, e);
    SortedRec r;
    r.P = run.s;
    r.head = run.hp | (run.o ? HEAD_MIXED_RULE : 0u);
    r.idx = idx[k];
    r.rule = rule[k];
    r.req = req[k];
    r.h = hh[k];
    r.now_mod = nm[k];
    srec[p] = r;
  }
}

// ---------------------------------------------------------------------------
// k_leader — one thread per unique key (segment tail).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_leader(const uint64_t* __restrict__ skeys, SortedRec* __restrict__ srec,
                                                const ItemRec* __restrict__ recs, const DevRule* __restrict__ rules,
                                                uint32_t n_all, TableDesc tab,
                                                SegInfo* __restrict__ seg, const uint32_t* __restrict__ tile_heads,
                                                uint32_t n_scan_tiles, HotCand* __restrict__ cand, EngineCtl* ctl) {
  if (blockIdx.x == 0) {
    // U = number of segment heads (k_scan per-tile counts); single writer of n_segments.
    __shared__ uint32_t sh_u[256];
    uint32_t u = 0;
    for (uint32_t t = threadIdx.x; t < n_scan_tiles; t += 256) u += tile_heads[t];
    sh_u[threadIdx.x] = u;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
      if (threadIdx.x < (uint32_t)d) sh_u[threadIdx.x] += sh_u[threadIdx.x + d];
      __syncthreads();
    }
    if (threadIdx.x == 0) ctl->n_segments = sh_u[0];
  }
  const uint32_t errs = ctl->err;  // flags of earlier launches
  if (errs & (ERR_NEED_RESORT | ERR_SPIN | ERR_BAD_TIME | ERR_BAD_INPUT | ERR_WINDOW_SPAN | ERR_FALLBACK |
              ERR_TABLE_FULL))
    return;
  const uint32_t n = n_all - ctl->n_nil;  // written by an earlier launch
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  if (j + 1 < n && (srec[j + 1].head & ~HEAD_MIXED_RULE) != j + 1) return;  // not a tail
  const SortedRec tail = srec[j];
  const uint32_t hp = tail.head & ~HEAD_MIXED_RULE;
  const bool mixed_rule = (tail.head & HEAD_MIXED_RULE) != 0;
  if (j - hp + 1 >= HOT_CAND_MIN && !mixed_rule)  // hot-set candidate for the bucketed pipeline
    emit_candidate(ctl, cand, tail.rule, j - hp + 1, srec[hp].idx);
  leader_segment(hp, j, tail, mixed_rule, skeys, srec, recs, rules, tab, seg, ctl);
}

// ---------------------------------------------------------------------------
// k_decide — per descriptor in sorted order.
// GetResponseDescriptorStatus + checkOverLimitThreshold + checkNearLimitThreshold +
// CalculateReset (base_limiter.go:70-195, utilities.go:34-38).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_decide(const SortedRec* __restrict__ srec, const SegInfo* __restrict__ seg,
                                                const DevRule* __restrict__ rules, uint32_t n_all,
                                                rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                                                int routed, EngineCtl* ctl) {
  const uint32_t errs = ctl->err;  // flags of earlier launches
  if (errs & (ERR_NEED_RESORT | ERR_SPIN | ERR_BAD_TIME | ERR_TABLE_FULL | ERR_BAD_INPUT | ERR_WINDOW_SPAN |
              ERR_FALLBACK))
    return;
  const uint32_t n = n_all - ctl->n_nil;  // written by k_fingerprint (earlier launch)
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  decide_pos(j, srec, seg, rules, out, req_thr, routed);
}

// k_cand_state — hot-set candidates reported by k_leader carry the arrival index of their
// key's first descriptor: fill in the key-prefix lane state and the unit (one thread each).
__global__ __launch_bounds__(256) void k_cand_state(DevBatch in, const DevRule* __restrict__ rules, uint64_t seed,
                                                    HotCand* __restrict__ cand, EngineCtl* ctl) {
  const uint32_t nc = min((uint32_t)CAND_MAX, ctl->tile_ctr[CAND_CTR][0]);
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nc) return;
  HotCand c = cand[i];
  if (c.first_idx == 0xFFFFFFFFu) return;
  const uint32_t d = c.first_idx;
  if (in.recs) {  // routed batch: the record already carries the prefix state
    c.a = in.recs[d].a;
    c.b = in.recs[d].b;
  } else {
    const uint32_t o0 = in.off[d], o1 = in.off[d + 1];
    FpState st = fp_init(o1 - o0, seed);
    hash_prefix(in.blob, o0, o1 - o0, st);
    c.a = st.a;
    c.b = st.b;
  }
  c.unit = rules[c.rule].unit;
  cand[i] = c;
}

// k_occ_update — one thread: the batch's new slots per region into the occupancy counts
// (the LSD pipeline; v4's last k4_group block does the same).
__global__ void k_occ_update(RegionOcc* __restrict__ occ, EngineCtl* ctl, uint32_t lag) {
  const uint32_t errs = ctl->err;
  if (errs & (ERR_NEED_RESORT | ERR_SPIN | ERR_BAD_TIME | ERR_BAD_INPUT | ERR_WINDOW_SPAN | ERR_FALLBACK |
              ERR_TABLE_FULL))
    return;
  uint32_t ins[8], n = 0;
  for (int r = 0; r < 8; ++r) {
    ins[r] = ctl->tile_ctr[INS_CTR0 + r][0];
    ctl->ins[r] = ins[r];
    n += ins[r];
  }
  ctl->n_inserted = n;
  occ_update(occ, ctl->gen_max, ins, lag);
}

// ---------------------------------------------------------------------------
// Host-side launchers (called from rl_engine.cpp).
// ---------------------------------------------------------------------------
void launch_fingerprint(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                        uint64_t* keys_orig, ItemRec* recs, rl_status* out, uint32_t* req_thr, uint32_t* fpart,
                        EngineCtl* ctl) {
  const DevBatch d = make_dev_batch(b);
  const uint32_t grid = (b.n_desc + 255) / 256;
  hipLaunchKernelGGL(k_fingerprint, dim3(grid), dim3(256), 0, st, d, rules, n_rules, seed, keys_orig, recs, out,
                     req_thr, fpart, ctl);
}
uint32_t hist_blocks(uint32_t n) { return n ? (n + HIST_CHUNK - 1) / HIST_CHUNK : 1; }
void launch_histogram(hipStream_t st, const uint64_t* keys, uint32_t n, int lo_bit, int npasses, uint32_t* part,
                      const uint32_t* fpart, uint32_t* fpart2) {
  hipLaunchKernelGGL(k_histogram, dim3(hist_blocks(n)), dim3(1024), 0, st, keys, n, lo_bit, npasses, part, fpart,
                     fpart2);
}
void launch_hist_scan(hipStream_t st, const uint32_t* part, uint32_t n, uint32_t* sub, int npasses,
                      const uint32_t* fpart2, const RegionOcc* occ, EngineCtl* ctl, uint32_t lag) {
  const uint32_t fpb = fpart2 ? hist_blocks(n) : 0;
  hipLaunchKernelGGL(k_hist_scan, dim3(npasses * HIST_SUB + (fpb ? 1 : 0)), dim3(256), 0, st, part, hist_blocks(n),
                     sub, npasses, fpart2, fpb, n, occ, ctl, lag);
}
uint32_t hist_sub_words() { return HIST_SUB * RADIX; }
void launch_fallback_lo_keys(hipStream_t st, const ItemRec* recs, const uint64_t* keys_orig, uint32_t n,
                             uint64_t* k_out, uint32_t* v_out) {
  hipLaunchKernelGGL(k_fallback_lo_keys, dim3((n + 255) / 256), dim3(256), 0, st, recs, keys_orig, n, k_out, v_out);
}
void launch_gather_keys(hipStream_t st, const uint64_t* keys_orig, const uint32_t* vals, uint32_t n, uint64_t* k_out) {
  hipLaunchKernelGGL(k_gather_keys, dim3((n + 255) / 256), dim3(256), 0, st, keys_orig, vals, n, k_out);
}
uint32_t sort_tiles(uint32_t n) { return (n + SORT_TILE - 1) / SORT_TILE; }
uint32_t scan_tiles(uint32_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }
void launch_sort_pass(hipStream_t st, const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout,
                      uint32_t n, int shift, const uint32_t* bin_off, uint32_t* lookback, uint32_t* tile_ctr,
                      EngineCtl* ctl) {
  hipLaunchKernelGGL(k_sort_pass, dim3(sort_tiles(n)), dim3(256), 0, st, kin, vin, kout, vout, n, shift, bin_off,
                     lookback, tile_ctr, ctl);
}
void launch_scan(hipStream_t st, const uint64_t* skeys, const uint32_t* svals, const ItemRec* recs, uint32_t n,
                 int lo_bit, int check_mixed, SortedRec* srec, uint64_t* lb_sum, uint64_t* lb_head,
                 uint32_t* tile_ctr, uint32_t* tile_heads, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_scan, dim3(scan_tiles(n)), dim3(256), 0, st, skeys, svals, recs, n, lo_bit, check_mixed, srec,
                     lb_sum, lb_head, tile_ctr, tile_heads, ctl);
}
void launch_leader(hipStream_t st, const uint64_t* skeys, SortedRec* srec, const ItemRec* recs,
                   const DevRule* rules, uint32_t n, const TableDesc& tab, SegInfo* seg,
                   const uint32_t* heads, uint32_t n_heads, HotCand* cand, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_leader, dim3((n + 255) / 256), dim3(256), 0, st, skeys, srec, recs, rules, n, tab,
                     seg, heads, n_heads, cand, ctl);
}
void launch_cand_state(hipStream_t st, const rl_batch& b, const DevRule* rules, uint64_t seed, HotCand* cand,
                       EngineCtl* ctl) {
  hipLaunchKernelGGL(k_cand_state, dim3(CAND_MAX / 256), dim3(256), 0, st, make_dev_batch(b), rules, seed, cand, ctl);
}
void launch_occ_update(hipStream_t st, RegionOcc* occ, EngineCtl* ctl, uint32_t lag) {
  hipLaunchKernelGGL(k_occ_update, dim3(1), dim3(1), 0, st, occ, ctl, lag);
}
void launch_decide(hipStream_t st, const SortedRec* srec, const SegInfo* seg, const DevRule* rules, uint32_t n,
                   rl_status* out, uint32_t* req_thr, int routed, EngineCtl* ctl) {
  hipLaunchKernelGGL(k_decide, dim3((n + 255) / 256), dim3(256), 0, st, srec, seg, rules, n, out, req_thr, routed,
                     ctl);
}

}  // namespace rlhip

#ifdef RL_STAMPS
extern "C" int rl_debug_stamps(uint64_t* out, uint32_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlhip::g_stamps), (size_t)nblocks * 8 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
