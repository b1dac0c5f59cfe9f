// rl_kernels_v3.hip — the default decision pipeline: six launches per batch.
//
// Same contract and outputs as the LSD pipeline (rl_kernels.hip, kept as the fallback).
// The batch input is read once; hot keys are decided where they stand in arrival order,
// the other descriptors travel once as 32-B records into key buckets.
//
//   k3_hist    per 2048-descriptor tile: fingerprint (fixed_cache_impl.go:43-53 via
//              cache_key.go:57-68), hot-set lookup, bucket; stable LDS sort of the tile by
//              bucket and a segmented scan: per-bucket counts and hits_addend sums of the tile,
//              the in-tile INCRBY prefix of every hot descriptor, the in-tile rank of every
//              other one; one 32-B record per descriptor (ARec); zero ThrottleMillis
//   k3_scan    per bucket: exclusive scan over tiles (counts; h sums of hot buckets); per hot
//              bucket: table claim and the counter before the batch (one key per bucket)
//   k3_bases   bucket start positions and k3_group ranges
//   k3_place   per descriptor: hot -> INCRBY post-value = base + tile prefix + in-tile prefix,
//              decision written in place; nil limit -> decided in place; the rest -> 32-B MRec
//              scattered into bucket order
//   k3_group   per range of whole MSD buckets: records grouped by full fingerprint in an LDS
//              hash table; per key the INCRBY prefix of each record in arrival order, one
//              leader per key (table probe/claim, INCRBY of the key's sequence in serial order,
//              local-cache freeze), decisions
//   k3_tail    unique-key count, hot-set candidate state, clears the next batch's control block
//
// Buckets: [0, HOT_BUCKETS) hot prefix x window parity, then MSD buckets = the 11 fingerprint
// bits below the region bits, then NIL (nil limits; never scattered).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"
#include "rl_decide.h"
#include "rl_device.h"
#include "rl_v3_dev.h"

namespace rlhip {
namespace v3 {

#ifdef RL_STAMPS
// Diagnostic build only (tools/stamps3.py): per-block phase timestamps (s_memrealtime, 100 MHz)
// of wave 0 in k3_hist (0), k3_place (1), k3_group (2), k3_scan (3).
__device__ uint64_t g_st3[4][4096][8];
#define ST3(kern, k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_st3[kern][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define ST3V(kern, k, v) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_st3[kern][blockIdx.x][k] = (v); } while (0)
#else
#define ST3(kern, k) do { } while (0)
#define ST3V(kern, k, v) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// k3_hist
// ---------------------------------------------------------------------------
template <bool ROUTED>
__global__ __launch_bounds__(NT) void k3_hist(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                              uint64_t seed, const HotEntry* __restrict__ hot,
                                              uint32_t* __restrict__ req_thr, uint32_t* __restrict__ fpart,
                                              uint16_t* __restrict__ tcount, unsigned long long* __restrict__ thsum,
                                              ARec* __restrict__ arec, EngineCtl* ctl) {
  __shared__ HotEntry sh_hot[HOT_SLOTS];
  __shared__ uint16_t sh_cnt[V3_ROW16];
  __shared__ unsigned long long sh_hs[HOT_BUCKETS];
  __shared__ uint16_t s_d[T];
  __shared__ uint16_t s_pa[T], s_pb[T];
  __shared__ uint32_t s_h[T];
  __shared__ unsigned long long s_res[T];
  __shared__ uint32_t s_cnt[W][64];
  __shared__ uint32_t sh_w[W];
  __shared__ SegEl s_agg[W];
  __shared__ uint32_t sh_f[FP_PART_WORDS];
  __shared__ uint32_t sh_err;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t tile = blockIdx.x, ntiles = gridDim.x;
  const uint32_t t0 = tile * T;
  ST3(0, 0);
  load_hot_table(hot, sh_hot);
  for (int b = tid; b < V3_ROW16 / 2; b += NT) reinterpret_cast<uint32_t*>(sh_cnt)[b] = 0;
  for (int b = tid; b < HOT_BUCKETS; b += NT) sh_hs[b] = 0;
  if (tid < FP_PART_WORDS) sh_f[tid] = 0;
  if (tid == 0) sh_err = 0;
  // DoLimitResponse.ThrottleMillis starts at 0 for every request (base_limiter.go:163-165)
  {
    const uint32_t per = (in.n_req + ntiles - 1) / ntiles;
    const uint32_t r0 = tile * per, r1 = min(in.n_req, r0 + per);
    for (uint32_t q = r0 + tid; q < r1; q += NT) req_thr[q] = 0;
  }
  __syncthreads();
  ST3(0, 1);
  D3 d[R];
  uint32_t err = 0;
  if (ROUTED)
    load_routed(in, rules, n_rules, sh_hot, t0, d, err);
  else
    load_descs(in, rules, n_rules, seed, sh_hot, t0, d, err);
  ST3(0, 2);
  uint32_t gmin[8], gmax[8], nil = 0;
#pragma unroll
  for (int rg = 0; rg < 8; ++rg) { gmin[rg] = 0xFFFFFFFFu; gmax[rg] = 0; }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t o = r * NT + tid;
    const uint32_t b = d[r].bucket;
    s_d[o] = (uint16_t)b;
    s_h[o] = d[r].h;
    s_pa[o] = (uint16_t)o;
    if (b < NIL_BUCKET) {
      const uint32_t region = key_region(d[r].key);
#pragma unroll
      for (int rg = 0; rg < 8; ++rg)  // static register indexing
        if ((uint32_t)rg == region) {
          gmin[rg] = d[r].gen < gmin[rg] ? d[r].gen : gmin[rg];
          gmax[rg] = d[r].gen > gmax[rg] ? d[r].gen : gmax[rg];
        }
    } else if (b == NIL_BUCKET) {
      ++nil;
    }
  }
#pragma unroll
  for (int rg = 0; rg < 8; ++rg) {
    const uint32_t mx = wave_max_u32(gmax[rg]);
    if (mx) {  // wave-uniform
      const uint32_t mn = wave_min_u32(gmin[rg]);
      if (lane == 0) {
        atomicMax(&sh_f[rg], ~mn);
        atomicMax(&sh_f[8 + rg], mx);
      }
    }
  }
  nil = wave_sum(nil);
  if (lane == 0 && nil) atomicAdd(&sh_f[16], nil);
  if (err) atomicOr(&sh_err, err);
  // Stable sort of the tile by bucket, then a segmented scan in sorted order:
  // MSD -> rank inside (tile, bucket); hot -> inclusive prefix of h inside (tile, bucket);
  // each bucket's last descriptor -> the bucket's count (and h sum) in this tile.
  tile_digit_pass(s_d, s_pa, s_pb, 0, s_cnt, sh_w);  // includes barriers
  tile_digit_pass(s_d, s_pb, s_pa, 6, s_cnt, sh_w);
  ST3(0, 3);
  {
    const uint32_t s0 = tid * R;
    uint32_t od[R], dd[R], fl[R];
    unsigned long long hv[R];
    uint32_t prev_d = s0 == 0 ? 0xFFFFFFFFu : s_d[s_pa[s0 - 1]];
    const uint32_t next_d = s0 + R < (uint32_t)T ? s_d[s_pa[s0 + R]] : 0xFFFFFFFFu;
    SegEl t{0, 0, 0};
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const uint32_t o = s_pa[s0 + q];
      const uint32_t dv = s_d[o];
      od[q] = o;
      dd[q] = dv;
      fl[q] = dv != prev_d;
      hv[q] = s_h[o];
      prev_d = dv;
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
#pragma unroll
    for (int w = 0; w < W - 1; ++w) {
      const SegEl a = s_agg[w];  // wave-uniform LDS read; no private copy of the array
      if ((uint32_t)w < wave) run = seg_op(run, a);
    }
    run = seg_op(run, wex);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      run = seg_op(run, SegEl{fl[q], s0 + q, hv[q]});
      const uint32_t b = dd[q];
      const uint32_t rank = s0 + q - run.hp;
      s_res[od[q]] = b < (uint32_t)HOT_BUCKETS ? run.s : (unsigned long long)rank;
      const uint32_t nd = q + 1 < R ? dd[q + 1] : next_d;
      if (b < NIL_BUCKET && nd != b) {  // the bucket's last descriptor of the tile
        sh_cnt[b] = (uint16_t)(rank + 1u);
        if (b < (uint32_t)HOT_BUCKETS) sh_hs[b] = run.s;
      }
    }
  }
  __syncthreads();
  ST3(0, 4);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = t0 + r * NT + tid;
    const D3& x = d[r];
    if (x.bucket == BKT_NONE) continue;
    const unsigned long long res = s_res[r * NT + tid];
    ARec a;
    a.kp = x.bucket < (uint32_t)HOT_BUCKETS ? (uint64_t)res : x.key;
    a.lo = x.lo;
    a.req = x.req;
    a.h = x.h;
    a.rn = rule_of(x.rule) | (x.now_mod << V3_RULE_BITS);
    a.bucket = (uint16_t)x.bucket;
    a.rank = (uint16_t)res;
    arec[i] = a;
  }
  uint32_t* trow = reinterpret_cast<uint32_t*>(tcount + (size_t)tile * V3_ROW16);
  for (int b = tid; b < V3_ROW16 / 2; b += NT) trow[b] = reinterpret_cast<const uint32_t*>(sh_cnt)[b];
  unsigned long long* hrow = thsum + (size_t)tile * HOT_BUCKETS;
  for (int b = tid; b < HOT_BUCKETS; b += NT) hrow[b] = sh_hs[b];
  if (tid < FP_PART_WORDS) fpart[(size_t)tile * FP_PART_WORDS + tid] = sh_f[tid];
  if (tid == 0 && sh_err) atomicOr(&ctl->err, sh_err);
  ST3(0, 5);
}

// ---------------------------------------------------------------------------
// k3_scan — 64 buckets per block (one per lane); the 16 waves split the tiles.
// ---------------------------------------------------------------------------
constexpr int SCAN_NT = 1024;
constexpr int SCAN_W = SCAN_NT / 64;
constexpr int SCAN_U = 16;  // column loads in flight per lane
static_assert(HOT_BUCKETS % 64 == 0 && V3_SCAN_BUCKETS % 64 == 0, "bucket blocks");

__global__ __launch_bounds__(SCAN_NT) void k3_scan(const uint16_t* __restrict__ tcount,
                                                   const unsigned long long* __restrict__ thsum, uint32_t ntiles,
                                                   uint32_t* __restrict__ toff, unsigned long long* __restrict__ hoff,
                                                   uint32_t* __restrict__ btotal, const uint32_t* __restrict__ fpart,
                                                   const HotEntry* __restrict__ hot_list, HotBucket3* __restrict__ hb,
                                                   TableDesc tab, int local_cache, HotCand* __restrict__ cand,
                                                   uint32_t* __restrict__ heads_out, EngineCtl* ctl) {
  __shared__ uint32_t s_f[FP_PART_WORDS];
  __shared__ uint32_t s_pc[SCAN_W][64];
  __shared__ unsigned long long s_ph[SCAN_W][64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  ST3(3, 0);
  if (tid < FP_PART_WORDS) s_f[tid] = 0;
  __syncthreads();
  // Fold the per-tile partials (every block): generation range per region, nil count.
  {
    uint32_t v[FP_PART_WORDS];
#pragma unroll
    for (int w = 0; w < FP_PART_WORDS; ++w) v[w] = 0;
    for (uint32_t g = tid; g < ntiles; g += SCAN_NT) {
#pragma unroll
      for (int w = 0; w < FP_PART_WORDS; ++w) {
        const uint32_t x = fpart[(size_t)g * FP_PART_WORDS + w];
        v[w] = w < 16 ? (x > v[w] ? x : v[w]) : v[w] + x;
      }
    }
#pragma unroll
    for (int w = 0; w < FP_PART_WORDS; ++w) {
      const uint32_t x = w < 16 ? wave_max_u32(v[w]) : wave_sum(v[w]);
      if (lane == 0 && x) {
        if (w < 16) atomicMax(&s_f[w], x);
        else atomicAdd(&s_f[w], x);
      }
    }
  }
  __syncthreads();
  ST3(3, 1);
  // Two window generations of one region in one batch must be adjacent;
  // a region's generations share its parity, so a valid batch has ONE generation per region.
  bool span = false;
#pragma unroll
  for (int rg = 0; rg < 8; ++rg) {
    const uint32_t mx = s_f[8 + rg], mn = ~s_f[rg];
    span |= mx != 0 && mx - mn > 1u;
  }
  if (blockIdx.x == 0) {
    if (tid < 8) ctl->gen_min[tid] = ~s_f[tid];
    else if (tid < 16) ctl->gen_max[tid - 8] = s_f[tid];
    else if (tid == 16) ctl->n_nil = s_f[16];
    if (tid == 0 && span) atomicOr(&ctl->err, ERR_WINDOW_SPAN);
  }
  // Column scan: bucket b = lane of this block, tiles [wave*Q, wave*Q + Q).
  const uint32_t b = blockIdx.x * 64 + lane;
  const bool hotb = blockIdx.x * 64 < (uint32_t)HOT_BUCKETS;  // block-uniform
  const uint32_t Q = (ntiles + SCAN_W - 1) / SCAN_W;
  const uint32_t tb = min(ntiles, wave * Q), te = min(ntiles, tb + Q);
  uint32_t c = 0;
  unsigned long long hs = 0;
  for (uint32_t t = tb; t < te; t += SCAN_U) {
    uint32_t cv[SCAN_U];
    unsigned long long hv[SCAN_U];
#pragma unroll
    for (int u = 0; u < SCAN_U; ++u) {
      cv[u] = t + u < te ? (uint32_t)tcount[(size_t)(t + u) * V3_ROW16 + b] : 0u;
      hv[u] = (hotb && t + u < te) ? thsum[(size_t)(t + u) * HOT_BUCKETS + b] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < SCAN_U; ++u) {
      c += cv[u];
      hs += hv[u];
    }
  }
  s_pc[wave][lane] = c;
  if (hotb) s_ph[wave][lane] = hs;
  __syncthreads();
  ST3(3, 2);
  uint32_t run = 0, ctot = 0;
  unsigned long long hrun = 0, htot = 0;
#pragma unroll
  for (int w = 0; w < SCAN_W; ++w) {
    const uint32_t x = s_pc[w][lane];
    run += (uint32_t)w < wave ? x : 0u;
    ctot += x;
    if (hotb) {
      const unsigned long long y = s_ph[w][lane];
      hrun += (uint32_t)w < wave ? y : 0ull;
      htot += y;
    }
  }
  if (hotb) {
    for (uint32_t t = tb; t < te; t += SCAN_U) {
      unsigned long long hv[SCAN_U];
#pragma unroll
      for (int u = 0; u < SCAN_U; ++u) hv[u] = t + u < te ? thsum[(size_t)(t + u) * HOT_BUCKETS + b] : 0ull;
#pragma unroll
      for (int u = 0; u < SCAN_U; ++u) {
        if (t + u < te) hoff[(size_t)(t + u) * HOT_BUCKETS + b] = hrun;
        hrun += hv[u];
      }
    }
  } else {
    for (uint32_t t = tb; t < te; t += SCAN_U) {
      uint32_t cv[SCAN_U];
#pragma unroll
      for (int u = 0; u < SCAN_U; ++u) cv[u] = t + u < te ? (uint32_t)tcount[(size_t)(t + u) * V3_ROW16 + b] : 0u;
#pragma unroll
      for (int u = 0; u < SCAN_U; ++u) {
        if (t + u < te) toff[(size_t)(t + u) * MSD_BUCKETS + (b - HOT_BUCKETS)] = run;
        run += cv[u];
      }
    }
  }
  ST3(3, 3);
  if (wave == 0) {
    btotal[b] = ctot;
    if (!hotb && ctot > (uint32_t)BUCKET_CAP) atomicOr(&ctl->err, ERR_V2_FALLBACK);
  }
  if (wave == 0 && hotb) {
    // Hot key leader: find or claim the key's slot and read the counter before this batch. A
    // claimed slot starts at count 0, which is invisible if the batch is later rejected.
    HotBucket3 x;
    x.key = x.fp_lo = x.base = x.slot = x.total = 0;
    x.rule = 0;
    x.flags = 0;
    x.rstar = 0xFFFFFFFFu;
    x.pad[0] = x.pad[1] = x.pad[2] = 0;
    const uint32_t errs = ctl->err;  // flags of k3_hist
    uint32_t heads = 0;
    if (ctot && !span && !(errs & (ERR_BAD_INPUT | ERR_BAD_TIME | ERR_V2_FALLBACK))) {
      const HotEntry he = hot_list[b >> 1];
      const uint32_t region = (he.unit - 1u) * 2u + (b & 1u);
      const uint32_t gen = s_f[8 + region];  // the region's one generation in this batch
      const uint64_t ws = (uint64_t)(gen - 1u) * unit_div(he.unit);
      uint64_t hi, lo;
      fp_final(FpState{he.a, he.b}, ws, hi, lo);
      x.key = make_sort_key(region, hi);
      x.fp_lo = lo;
      x.rule = he.rule;
      x.total = htot;
      Slot* slot = nullptr;
      bool existed = false;
      if (!table_claim(tab, x.key, lo, gen, slot, existed)) {
        atomicOr(&ctl->err, ERR_TABLE_FULL);
      } else {
        if (existed) {
          x.base = slot->count;
          x.flags = (slot->flags & SLOT_FROZEN) ? HB_FROZEN_PRE : 0u;
        } else {
          slot->key = x.key;
          slot->fp_lo_hi = (uint32_t)(lo >> 32);
          slot->count = 0;
          slot->flags = 0;
        }
        x.slot = (uint64_t)(uintptr_t)slot;
        // The local-cache freeze point is found from a monotone INCRBY sequence; a batch whose
        // counter would pass 2^32 goes to the LSD pipeline (uint32 wraparound, R10).
        if (local_cache && !(x.flags & HB_FROZEN_PRE) && x.base + htot >= (1ull << 32))
          atomicOr(&ctl->err, ERR_V2_FALLBACK);
        heads = 1;
      }
      if (slot != nullptr && !existed) heads |= 1u << 16;  // a new table slot
      if (ctot >= HOT_CAND_MIN) emit_candidate(ctl, cand, he.rule, ctot, 0xFFFFFFFFu, he.a, he.b, he.unit);
    }
    hb[b] = x;
    heads = wave_sum(heads);
    if (lane == 0) heads_out[blockIdx.x] = heads;
    ST3(3, 4);
  } else if (wave == 0 && lane == 0) {
    heads_out[blockIdx.x] = 0;
  }
}

// ---------------------------------------------------------------------------
// k3_bases — one workgroup: MSD bucket start positions and the k3_group ranges (range w
// holds the MSD buckets whose start lies in [w*V3_GRANGE, (w+1)*V3_GRANGE); rng[w] = the
// start of its first bucket).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(SCAN_NT) void k3_bases(const uint32_t* __restrict__ btotal, uint32_t* __restrict__ bbase,
                                                    uint32_t* __restrict__ rng, uint32_t* __restrict__ rngb,
                                                    uint32_t n_ranges) {
  __shared__ uint32_t s_base[MSD_BUCKETS + 1];
  __shared__ uint32_t sh_w[SCAN_W];
  const uint32_t tid = threadIdx.x;
  constexpr int PER = MSD_BUCKETS / SCAN_NT;
  static_assert(MSD_BUCKETS % SCAN_NT == 0, "bucket bases");
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    v[k] = btotal[HOT_BUCKETS + tid * PER + k];
    sum += v[k];
  }
  uint32_t total;
  uint32_t rb = block_excl_scan<SCAN_NT>(sum, sh_w, total);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    s_base[tid * PER + k] = rb;
    bbase[tid * PER + k] = rb;
    rb += v[k];
  }
  if (tid == 0) {
    s_base[MSD_BUCKETS] = total;
    bbase[MSD_BUCKETS] = total;
  }
  __syncthreads();
  for (uint32_t bb = tid; bb < (uint32_t)MSD_BUCKETS; bb += SCAN_NT) {
    const uint32_t hi = s_base[bb];
    const uint32_t lo = bb == 0 ? 0u : s_base[bb - 1] + 1u;
    const uint32_t wend = min(n_ranges, hi / (uint32_t)V3_GRANGE);
    for (uint32_t w = (lo + V3_GRANGE - 1) / V3_GRANGE; w <= wend; ++w) {
      rng[w] = hi;
      rngb[w] = bb;
    }
  }
  // ranges starting after the last bucket's start: empty (all threads share the fill)
  const uint32_t last = s_base[MSD_BUCKETS - 1] + 1u;
  for (uint32_t w = (last + V3_GRANGE - 1) / V3_GRANGE + tid; w <= n_ranges; w += SCAN_NT) {
    rng[w] = total;
    rngb[w] = MSD_BUCKETS;
  }
}

// ---------------------------------------------------------------------------
// k3_place
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(NT) void k3_place(uint32_t n, const ARec* __restrict__ arec,
                                               const DevRule* __restrict__ rules, const uint32_t* __restrict__ toff,
                                               const unsigned long long* __restrict__ hoff,
                                               const uint32_t* __restrict__ bbase, HotBucket3* __restrict__ hb,
                                               int local_cache, MRec* __restrict__ mrec, rl_status* __restrict__ out,
                                               uint32_t* __restrict__ req_thr, Deferred* __restrict__ dfr, int routed,
                                               EngineCtl* ctl) {
  __shared__ uint32_t s_rstar[HOT_BUCKETS];
  const uint32_t tid = threadIdx.x;
  // Nothing is decided and nothing touches the table unless the whole batch is valid.
  if (ctl->err) return;
  const uint32_t tile = blockIdx.x;
  const uint32_t t0 = tile * T;
  ST3(1, 0);
  ARec a[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = t0 + r * NT + tid;
    if (i < n) a[r] = arec[i];
    else a[r].bucket = (uint16_t)BKT_NONE;
  }
  if (local_cache)
    for (int b = tid; b < HOT_BUCKETS; b += NT) s_rstar[b] = 0xFFFFFFFFu;
  // Hot keys without a freeze in this batch: the final counter is base + total (block 0).
  if (tile == 0) {
    for (int b = tid; b < HOT_BUCKETS; b += NT) {
      const HotBucket3 x = hb[b];
      if (!x.slot || (x.flags & HB_FROZEN_PRE)) continue;
      if (!local_cache || x.base + x.total <= (uint64_t)rules[x.rule].L)
        reinterpret_cast<Slot*>(x.slot)->count = x.base + x.total;
    }
  }
  const unsigned long long* hrow = hoff + (size_t)tile * HOT_BUCKETS;
  const uint32_t* trow = toff + (size_t)tile * MSD_BUCKETS;
  unsigned long long P[R];
#pragma unroll
  for (int r = 0; r < R; ++r) P[r] = a[r].bucket < HOT_BUCKETS ? hrow[a[r].bucket] + a[r].kp : 0ull;
  ST3(1, 1);
  if (local_cache) {
    __syncthreads();  // s_rstar initialised
    // The descriptor whose INCRBY reply first exceeds the limit freezes the key
    // (base_limiter.go:94-106). The post-value is monotone (k3_scan), so it is the unique
    // descriptor with after > L >= before, or the key's first descriptor of the batch.
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t b = a[r].bucket;
      if (b >= (uint32_t)HOT_BUCKETS) continue;
      const HotBucket3& x = hb[b];
      if (x.flags & HB_FROZEN_PRE) continue;
      const uint64_t after = x.base + P[r];
      const uint32_t L = rules[rule_of(a[r].rn)].L;
      if (after > L && (after - a[r].h <= L || P[r] == a[r].h)) {
        s_rstar[b] = a[r].req;
        hb[b].rstar = a[r].req;
        reinterpret_cast<Slot*>(x.slot)->flags = SLOT_FROZEN;
      }
    }
    __syncthreads();
  }
  ST3(1, 2);
  const uint32_t q0 = arec[t0].req;  // request of the tile's first descriptor
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = t0 + r * NT + tid;
    const ARec& x = a[r];
    const uint32_t b = x.bucket;
    const uint32_t rule = rule_of(x.rn), now_mod = x.rn >> V3_RULE_BITS;
    if (b == NIL_BUCKET) {
      // GetResponseDescriptorStatus("" key) -> {OK, nil limit, 0}  base_limiter.go:72-75
      rl_status st;
      st.code_flags = RL_CODE_OK;
      st.limit_remaining = 0;
      st.reset_s = 0;
      st.over_limit_delta = 0;
      st.near_limit_delta = 0;
      out[i] = st;
    } else if (b < (uint32_t)HOT_BUCKETS) {
      const HotBucket3& hx = hb[b];
      const DevRule& rl = rules[rule];
      if (hx.flags & HB_FROZEN_PRE) {
        out[i] = local_hit_status(x.h, rl.div - now_mod);  // every descriptor is a local-cache hit
        continue;
      }
      const uint64_t after = hx.base + P[r];
      if (!local_cache || after <= rl.L) {
        decide_at(i, x.req, rule, x.h, now_mod, hx.base, P[r], SEG_NO_FREEZE, rules, out, req_thr, routed);
        continue;
      }
      const uint32_t rs = s_rstar[b];
      Slot* slot = reinterpret_cast<Slot*>(hx.slot);
      if (rs != 0xFFFFFFFFu) {  // the freezing descriptor is in this tile, at or before this one
        if (x.req > rs) {
          out[i] = local_hit_status(x.h, rl.div - now_mod);
        } else {  // same request as the freezing descriptor: its INCRBY still happens
          decide_at(i, x.req, rule, x.h, now_mod, hx.base, P[r], SEG_NO_FREEZE, rules, out, req_thr, routed);
          atomicMax((unsigned long long*)&slot->count, (unsigned long long)after);
        }
      } else if (x.req > q0) {  // froze in an earlier tile, in a request <= q0
        out[i] = local_hit_status(x.h, rl.div - now_mod);
      } else {  // a request that began in an earlier tile: k3_group decides it
        const uint32_t e = atomicAdd(&ctl->tile_ctr[DFR_CTR][0], 1u);
        Deferred df;
        df.P = P[r];
        df.idx = i;
        df.bucket = b;
        df.req = x.req;
        df.h = x.h;
        df.rule = rule;
        df.now_mod = now_mod;
        dfr[e] = df;
      }
    } else if (b < NIL_BUCKET) {
      const uint32_t mb = b - HOT_BUCKETS;
      const uint32_t pos = bbase[mb] + trow[mb] + x.rank;
      MRec m;
      m.key = x.kp;
      m.fp_lo = x.lo;
      m.idx = i;
      m.req = x.req;
      m.h = x.h;
      m.rn = x.rn;
      mrec[pos] = m;
    }
  }
  ST3(1, 3);
}

// ---------------------------------------------------------------------------
// k3_group — one workgroup per range of whole MSD buckets (k3_bases publishes the ranges).
// A key's records all lie in its bucket, so a range holds every record of its keys, and
// inside a bucket the records are in arrival order (k3_hist ranks them stably). The
// records are grouped by full fingerprint in a hash table; one wave then lays out each
// key's list in position (= arrival) order, and a segmented scan over the lists gives every
// record its INCRBY prefix. The key's last record leads. Ranges too large for LDS run the
// same phases on global scratch, in chunks.
// ---------------------------------------------------------------------------
constexpr int G_NT = 256;
constexpr int G_W = G_NT / 64;
constexpr int G_CAP = V3_GCAP;
constexpr int G_IPT = G_CAP / G_NT;
constexpr int G_HASH = V3_GHASH;
constexpr int G_HBITS = 10;
static_assert(G_CAP % G_NT == 0 && G_HASH == (1 << G_HBITS) && G_HASH > G_CAP, "k3_group geometry");
constexpr uint32_t G_EMPTY = 0xFFFFFFFFu;

// Storage of one range: LDS arrays (G_CAP records) or global scratch (any size).
struct GStore {
  uint64_t* key;   // after the scan: the key's counter before the batch, at the leader's position
  uint64_t* lo;    // after the scan: the key's freeze, at the leader's position
  uint2* pay;      // arrival index, h
  uint64_t* P;     // INCRBY prefix by position
  uint32_t* slot;  // hash slot -> first position inserted with the key (G_EMPTY = free)
  uint32_t* cnt;   // hash slot -> records of the key
  uint16_t* end;   // hash slot -> end of the key's list (start = end - cnt)
  uint16_t* list;  // positions grouped by key, each key's in position order
  uint16_t* grp;   // position -> hash slot
  uint32_t* cursor;
  uint32_t hmask;
  const MRec* recs;  // the range's records (request and rule of other records, read by leaders)
};
static_assert(V3_GCAP + BUCKET_CAP + V3_GRANGE < 65536 / 4, "u16 positions and hash slots");

RL_DEV void group_insert(const GStore& g, uint32_t k, uint64_t key, uint64_t lo) {
  uint32_t s = (uint32_t)key & g.hmask;
  for (;;) {
    const uint32_t v = atomicCAS(&g.slot[s], G_EMPTY, k);
    if (v == G_EMPTY || (g.key[v] == key && g.lo[v] == lo)) break;
    s = (s + 1) & g.hmask;
  }
  g.grp[k] = (uint16_t)s;
  atomicAdd(&g.cnt[s], 1u);
}

// One wave: each key's list in position order (positions [0, m), 64 at a time).
RL_DEV void group_layout(const GStore& g, uint32_t m) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  for (uint32_t c = 0; c < m; c += 64) {
    const uint32_t k = c + lane;
    const bool valid = k < m;
    const uint32_t s = valid ? g.grp[k] : 0u;
    uint64_t mm = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      if (b >= G_HBITS && (g.hmask >> b) == 0) break;  // wave-uniform
      const bool bit = (s >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      mm &= bit ? bal : ~bal;
    }
    uint32_t before = 0;
    if (valid) before = g.end[s];
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      if (lane == (uint32_t)__ffsll((unsigned long long)mm) - 1u) g.end[s] = (uint16_t)(before + (uint32_t)__popcll(mm));
      g.list[before + (uint32_t)__popcll(mm & lt)] = (uint16_t)k;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Barrier between phases. The LDS path exchanges data through LDS only, so it waits for
// LDS traffic alone and leaves the table read-ahead loads in flight across the barrier.
template <bool LDS>
RL_DEV void gbar() {
  if constexpr (LDS) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    __threadfence_block();
    __syncthreads();
  }
}

struct LSeg {
  uint32_t f;
  unsigned long long s;
};
RL_DEV LSeg lseg_op(const LSeg& a, const LSeg& b) { return b.f ? b : LSeg{a.f, a.s + b.s}; }

// Segmented inclusive scan of h over the lists (list positions [0, m) in chunks of
// G_NT * G_IPT, blocked G_IPT per thread): g.P[position] = INCRBY prefix of its key.
template <bool LDS>
RL_DEV void group_scan(const GStore& g, uint32_t m, LSeg* s_agg, LSeg* s_carry) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) *s_carry = LSeg{0, 0};
  gbar<LDS>();
  for (uint32_t c0 = 0; c0 < m; c0 += G_NT * G_IPT) {
    uint32_t pos[G_IPT], hd[G_IPT];
    unsigned long long hv[G_IPT];
    LSeg t{0, 0};
#pragma unroll
    for (int q = 0; q < G_IPT; ++q) {
      const uint32_t e = c0 + tid * G_IPT + q;
      pos[q] = 0xFFFFFFFFu;
      hd[q] = 0;
      hv[q] = 0;
      if (e < m) {
        const uint32_t k = g.list[e];
        const uint32_t s = g.grp[k];
        pos[q] = k;
        hd[q] = e == g.end[s] - g.cnt[s];
        hv[q] = g.pay[k].y;
        t = lseg_op(t, LSeg{hd[q], hv[q]});
      }
    }
    LSeg incl = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      LSeg y;
      y.f = __shfl_up(incl.f, d, 64);
      y.s = __shfl_up(incl.s, d, 64);
      if (lane >= (uint32_t)d) incl = lseg_op(y, incl);
    }
    if (lane == 63) s_agg[wave] = incl;
    LSeg wex;
    wex.f = __shfl_up(incl.f, 1, 64);
    wex.s = __shfl_up(incl.s, 1, 64);
    if (lane == 0) wex = LSeg{0, 0};
    gbar<LDS>();
    LSeg run = *s_carry;
    for (uint32_t w = 0; w < wave; ++w) run = lseg_op(run, s_agg[w]);
    run = lseg_op(run, wex);
#pragma unroll
    for (int q = 0; q < G_IPT; ++q) {
      if (pos[q] == 0xFFFFFFFFu) continue;
      run = lseg_op(run, LSeg{hd[q], hv[q]});
      g.P[pos[q]] = run.s;
    }
    gbar<LDS>();
    if (tid == G_NT - 1) {  // carry = the whole chunk, folded onto the previous carry
      LSeg all = *s_carry;
      for (int w = 0; w < G_W; ++w) all = lseg_op(all, s_agg[w]);
      *s_carry = all;
    }
    gbar<LDS>();
  }
}

// Run by the key's last record: table probe/claim, INCRBY of the key's whole sequence in
// serial order, local-cache freeze (fixed_cache_impl.go:55-123, base_limiter.go:88-106).
RL_DEV void group_lead(const GStore& g, uint32_t k, uint64_t key, uint64_t lo, uint32_t rule,
                       const DevRule* __restrict__ rules, const TableDesc& tab, int local_cache, HotCand* cand,
                       EngineCtl* ctl, bool has_pre, const SlotView pre, int cand_on, uint64_t& base_out,
                       uint32_t& freeze_out, bool& inserted) {
  base_out = 0;
  freeze_out = SEG_NO_FREEZE;
  const uint32_t s = g.grp[k];
  const uint32_t n = g.cnt[s], e1 = g.end[s], e0 = e1 - n;
  const uint64_t Pk = g.P[k];
  bool mixed = false;
  inserted = false;
  if ((cand_on && n >= HOT_MIN_SEG) || local_cache) {
    for (uint32_t e = e0; e < e1; ++e) mixed |= rule_of(g.recs[g.list[e]].rn) != rule;
    if (cand_on && n >= HOT_MIN_SEG && !mixed) emit_candidate(ctl, cand, rule, n, g.pay[g.list[e0]].x);
  }
  const uint32_t gen = ctl->gen_max[key_region(key)];  // the region's one generation (k3_scan)
  Slot* slot = nullptr;
  bool existed = false;
  uint64_t base = 0;
  uint32_t sflags = 0;
  const bool claimed = has_pre ? table_claim_pre(tab, key, lo, gen, pre, slot, existed, base, sflags)
                               : table_claim(tab, key, lo, gen, slot, existed);
  if (!claimed) {
    atomicOr(&ctl->err, ERR_TABLE_FULL);
    return;
  }
  if (existed && !has_pre) {
    base = slot->count;
    sflags = slot->flags;
  }
  const bool frozen_pre = existed && (sflags & SLOT_FROZEN) != 0;
  if (!existed) {
    slot->key = key;
    slot->fp_lo_hi = (uint32_t)(lo >> 32);
  }
  inserted = !existed;
  uint32_t freeze = SEG_NO_FREEZE;
  uint64_t final_count = base + Pk;
  if (frozen_pre) {
    freeze = SEG_FROZEN_BEFORE;  // every descriptor is a local-cache hit: no INCRBY
    final_count = base;
  } else if (local_cache) {
    // the first record (arrival order) whose INCRBY reply exceeds its limit freezes the key;
    // the INCRBYs of its own request still happen (all lookups precede the Sets)
    const bool exact = !mixed && base + Pk < (1ull << 32);
    for (uint32_t e = e0; e < e1; ++e) {
      const uint32_t j = g.list[e];
      const uint64_t after = base + g.P[j];
      const uint32_t L = rules[rule_of(g.recs[j].rn)].L;
      if (exact ? after > (uint64_t)L : (uint32_t)after > L) {
        const uint32_t rstar = g.recs[j].req;
        uint64_t last = g.P[j];
        for (uint32_t f = e + 1; f < e1 && g.recs[g.list[f]].req == rstar; ++f) last = g.P[g.list[f]];
        freeze = rstar;
        final_count = base + last;
        break;
      }
    }
  }
  slot->count = final_count;
  if (freeze != SEG_NO_FREEZE && freeze != SEG_FROZEN_BEFORE) slot->flags = SLOT_FROZEN;
  else if (!existed) slot->flags = 0;
  base_out = base;
  freeze_out = freeze;
}

RL_DEV uint32_t group_tail(const GStore& g, uint32_t k) { return g.list[g.end[g.grp[k]] - 1u]; }

// All phases of one range; returns the keys this thread led (low 16 bits) and the new table
// slots they claimed (high 16 bits). The LDS path (m <= G_CAP, at
// most G_IPT records per thread) reads each record's first table slot ahead, right after
// staging, so the leaders' table probes overlap the grouping.
template <bool LDS>
RL_DEV uint32_t group_range(const GStore& g, uint32_t hs, const MRec* __restrict__ recs, uint32_t m,
                            const DevRule* __restrict__ rules, const TableDesc& tab, int local_cache,
                            rl_status* __restrict__ out, uint32_t* __restrict__ req_thr, HotCand* cand, int cand_on,
                            int routed, LSeg* s_agg, LSeg* s_carry, EngineCtl* ctl) {
  const uint32_t tid = threadIdx.x, wave = tid >> 6;
  uint32_t heads = 0;
  for (uint32_t s = tid; s < hs; s += G_NT) {
    g.slot[s] = G_EMPTY;
    g.cnt[s] = 0;
  }
  // LDS path: records tid + j*G_NT (j < 3) stay in registers: named variables, not an
  // array, so the read-ahead loads stay in flight in VGPRs instead of landing in scratch.
  static_assert(G_IPT == 3, "k3_group keeps three records per thread");
  SlotView pre0, pre1, pre2;
  uint4 own0, own1, own2;  // idx, req, h, rn
#define RL_G_STAGE(J)                                      \
  {                                                        \
    const uint32_t k = tid + (J) * G_NT;                   \
    const MRec x = recs[k < m ? k : 0];                    \
    if (k < m) {                                           \
      g.key[k] = x.key;                                    \
      g.lo[k] = x.fp_lo;                                   \
      g.pay[k] = make_uint2(x.idx, x.h);                   \
    }                                                      \
    own##J = make_uint4(x.idx, x.req, x.h, x.rn);          \
    pre##J = load_slot(slot_first(tab, x.key));            \
  }
  if constexpr (LDS) {
    RL_G_STAGE(0)
    RL_G_STAGE(1)
    RL_G_STAGE(2)
  } else {
    for (uint32_t k = tid; k < m; k += G_NT) {
      const MRec x = recs[k];
      g.key[k] = x.key;
      g.lo[k] = x.fp_lo;
      g.pay[k] = make_uint2(x.idx, x.h);
    }
  }
  gbar<LDS>();
  ST3(2, 1);
  for (uint32_t k = tid; k < m; k += G_NT) group_insert(g, k, g.key[k], g.lo[k]);
  gbar<LDS>();
  // each key's list: the key's first-inserted record reserves it
  for (uint32_t k = tid; k < m; k += G_NT) {
    const uint32_t s = g.grp[k];
    if (g.slot[s] == k) g.end[s] = atomicAdd(g.cursor, g.cnt[s]);
  }
  gbar<LDS>();
  if (wave == 0) group_layout(g, m);
  gbar<LDS>();
  ST3(2, 2);
  group_scan<LDS>(g, m, s_agg, s_carry);
  gbar<LDS>();
  ST3(2, 3);
  // Leaders. The staged keys are not read any more: a leader keeps its key's state at its own
  // position of key[] (counter before the batch) and lo[] (freeze).
#define RL_G_LEAD(J)                                                                                 \
  {                                                                                                  \
    const uint32_t k = tid + (J) * G_NT;                                                             \
    if (k < m && group_tail(g, k) == k) {                                                            \
      ++heads;                                                                                       \
      const uint64_t key = g.key[k], lo = g.lo[k];                                                   \
      uint64_t base;                                                                                 \
      uint32_t frz;                                                                                  \
      bool ins;                                                                                      \
      group_lead(g, k, key, lo, rule_of(own##J.w), rules, tab, local_cache, cand, ctl, true, pre##J, cand_on, \
                 base, frz, ins);                                                                    \
      heads += ins ? 1u << 16 : 0u;                                                                  \
      g.key[k] = base;                                                                               \
      g.lo[k] = frz;                                                                                 \
    }                                                                                                \
  }
  if constexpr (LDS) {
    RL_G_LEAD(0)
    RL_G_LEAD(1)
    RL_G_LEAD(2)
  } else {
    for (uint32_t k = tid; k < m; k += G_NT) {
      if (group_tail(g, k) != k) continue;
      ++heads;
      const uint64_t key = g.key[k], lo = g.lo[k];
      uint64_t base;
      uint32_t frz;
      bool ins;
      group_lead(g, k, key, lo, rule_of(recs[k].rn), rules, tab, local_cache, cand, ctl, false, pre0, cand_on, base,
                 frz, ins);
      heads += ins ? 1u << 16 : 0u;
      g.key[k] = base;
      g.lo[k] = frz;
    }
  }
  __threadfence_block();
  __syncthreads();
  ST3(2, 4);
  auto decide_k = [&](uint32_t k, const uint4& pk) {
    const uint32_t t = group_tail(g, k);
    decide_at(pk.x, pk.y, rule_of(pk.w), pk.z, pk.w >> V3_RULE_BITS, g.key[t], g.P[k], (uint32_t)g.lo[t], rules, out,
              req_thr, routed);
  };
#undef RL_G_STAGE
#undef RL_G_LEAD
  if constexpr (LDS) {
    if (tid < m) decide_k(tid, own0);
    if (tid + G_NT < m) decide_k(tid + G_NT, own1);
    if (tid + 2 * G_NT < m) decide_k(tid + 2 * G_NT, own2);
  } else {
    for (uint32_t k = tid; k < m; k += G_NT) {
      const MRec& x = recs[k];
      decide_k(k, make_uint4(x.idx, x.req, x.h, x.rn));
    }
  }
  return heads;
}

__global__ __launch_bounds__(G_NT) void k3_group(const MRec* __restrict__ mrec, const uint32_t* __restrict__ rng,
                                                 uint32_t n_ranges, const DevRule* __restrict__ rules, TableDesc tab,
                                                 int local_cache, rl_status* __restrict__ out,
                                                 uint32_t* __restrict__ req_thr, const Deferred* __restrict__ dfr,
                                                 const HotBucket3* __restrict__ hb, HotCand* __restrict__ cand,
                                                 int cand_on, const uint32_t* __restrict__ rngb,
                                                 const uint32_t* __restrict__ bbase, V3GroupScratch gs,
                                                 uint32_t* __restrict__ wg_heads, int routed, EngineCtl* ctl) {
  __shared__ uint64_t s_key[G_CAP];
  __shared__ uint64_t s_lo[G_CAP];
  __shared__ uint2 s_pay[G_CAP];
  __shared__ uint64_t s_P[G_CAP];
  __shared__ uint32_t s_slot[G_HASH];
  __shared__ uint32_t s_cnt[G_HASH];
  __shared__ uint16_t s_end[G_HASH];
  __shared__ uint16_t s_list[G_CAP];
  __shared__ uint16_t s_grp[G_CAP];
  __shared__ LSeg s_agg[G_W];
  __shared__ LSeg s_carry;
  __shared__ uint32_t s_cursor, s_heads;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  ST3(2, 6);
  if (ctl->err) {
    if (tid == 0) wg_heads[blockIdx.x] = 0;
    return;
  }
  if (blockIdx.x >= n_ranges) {
    // Hot descriptors of a request that began before the tile where their key froze.
    const uint32_t nd = ctl->tile_ctr[DFR_CTR][0];
    for (uint32_t e = (blockIdx.x - n_ranges) * G_NT + tid; e < nd; e += (gridDim.x - n_ranges) * G_NT) {
      const Deferred df = dfr[e];
      const HotBucket3 x = hb[df.bucket];
      if (df.req > x.rstar) {
        out[df.idx] = local_hit_status(df.h, rules[df.rule].div - df.now_mod);
      } else {
        decide_at(df.idx, df.req, df.rule, df.h, df.now_mod, x.base, df.P, SEG_NO_FREEZE, rules, out, req_thr, routed);
        atomicMax((unsigned long long*)&reinterpret_cast<Slot*>(x.slot)->count, (unsigned long long)(x.base + df.P));
      }
    }
    if (tid == 0) wg_heads[blockIdx.x] = 0;
    return;
  }
  const uint32_t r0 = rng[blockIdx.x], r1 = rng[blockIdx.x + 1];
  const uint32_t m = r1 - r0;
  if (m == 0) {
    if (tid == 0) wg_heads[blockIdx.x] = 0;
    ST3(2, 5);
    return;
  }
  ST3(2, 0);
  ST3V(2, 7, m);
  if (tid == 0) s_heads = 0;
  uint32_t heads = 0;
  // Sub-ranges of whole buckets that fit the LDS stage; a single bucket larger than the stage
  // (a very frequent key not in the hot set yet) runs on global scratch. Block-uniform.
  uint32_t bk = rngb[blockIdx.x], pos = r0;
  while (pos < r1) {
    uint32_t e = pos;
    while (bk < (uint32_t)MSD_BUCKETS && bbase[bk + 1] <= r1 && bbase[bk + 1] - pos <= (uint32_t)G_CAP) {
      e = bbase[bk + 1];
      ++bk;
    }
    __syncthreads();  // the previous sub-range is done with LDS
    if (tid == 0) s_cursor = 0;
    if (e > pos) {
      const GStore g{s_key, s_lo, s_pay, s_P, s_slot, s_cnt, s_end, s_list, s_grp, &s_cursor, G_HASH - 1, mrec + pos};
      heads += group_range<true>(g, G_HASH, mrec + pos, e - pos, rules, tab, local_cache, out, req_thr, cand, cand_on,
                                 routed, s_agg, &s_carry, ctl);
    } else {
      e = bbase[bk + 1];
      ++bk;
      const uint32_t mm = e - pos;
      uint32_t hs = 2;
      while (hs < 2 * mm) hs <<= 1;  // <= 4 mm: 4 words per position
      const GStore g{gs.key + pos,
                     gs.lo + pos,
                     reinterpret_cast<uint2*>(gs.pay) + pos,
                     gs.P + pos,
                     gs.slot + 4 * (size_t)pos,
                     gs.cnt + 4 * (size_t)pos,
                     reinterpret_cast<uint16_t*>(gs.base) + 4 * (size_t)pos,
                     reinterpret_cast<uint16_t*>(gs.list) + pos,
                     reinterpret_cast<uint16_t*>(gs.grp) + pos,
                     gs.cursor + blockIdx.x,
                     hs - 1,
                     mrec + pos};
      if (tid == 0) *g.cursor = 0;
      heads += group_range<false>(g, hs, mrec + pos, mm, rules, tab, local_cache, out, req_thr, cand, cand_on, routed,
                                  s_agg, &s_carry, ctl);
    }
    pos = e;
  }
  heads = wave_sum(heads);
  if (lane == 0 && heads) atomicAdd(&s_heads, heads);
  __syncthreads();
  if (tid == 0) wg_heads[blockIdx.x] = s_heads;
  ST3(2, 5);
}

// ---------------------------------------------------------------------------
// k3_tail: U, hot-set candidate prefix state, clear the next batch's control block.
// ---------------------------------------------------------------------------
constexpr int TAIL_NT = 256;
__global__ __launch_bounds__(TAIL_NT) void k3_tail(DevBatch in, const DevRule* __restrict__ rules, uint64_t seed,
                                                   HotCand* cand, const uint32_t* __restrict__ wg_heads,
                                                   uint32_t n_heads, EngineCtl* ctl, EngineCtl* next_ctl) {
  __shared__ uint32_t s_u, s_ins;
  if (blockIdx.x == 0) {
    // U = Σ per-workgroup unique-key counts; 8 independent loads per lane per step
    if (threadIdx.x == 0) {
      s_u = 0;
      s_ins = 0;
    }
    __syncthreads();
    uint32_t u = 0, ins = 0;
    for (uint32_t t0 = 0; t0 < n_heads; t0 += TAIL_NT * 8) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t t = t0 + k * TAIL_NT + threadIdx.x;
        v[k] = t < n_heads ? wg_heads[t] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        u += v[k] & 0xFFFFu;
        ins += v[k] >> 16;
      }
    }
    u = wave_sum(u);
    ins = wave_sum(ins);
    if ((threadIdx.x & 63) == 0) {
      if (u) atomicAdd(&s_u, u);
      if (ins) atomicAdd(&s_ins, ins);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      ctl->n_segments = s_u;
      ctl->tile_ctr[INS_CTR0][0] += s_ins;  // new table slots (engine stats)
    }
  }
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(next_ctl);
    constexpr uint32_t words = sizeof(EngineCtl) / 4;
    for (uint32_t w = blockIdx.x * TAIL_NT + threadIdx.x; w < words; w += gridDim.x * TAIL_NT) z[w] = 0;
  }
  const uint32_t i = blockIdx.x * TAIL_NT + threadIdx.x;
  const uint32_t nc = min((uint32_t)CAND_MAX, ctl->tile_ctr[CAND_CTR][0]);
  if (i >= nc) return;
  HotCand c = cand[i];
  if (c.first_idx == 0xFFFFFFFFu) return;  // a hot key: state already known
  const uint32_t d = c.first_idx;
  const uint32_t unit = rules[c.rule].unit;
  if (in.recs) {  // routed batch: the record already carries the prefix state
    c.a = in.recs[d].a;
    c.b = in.recs[d].b;
  } else {
    const uint32_t o0 = in.off[d], o1 = in.off[d + 1];
    const FpState s = prefix_state(in.blob, o0, o1 - o0, unit, seed);
    c.a = s.a;
    c.b = s.b;
  }
  c.unit = unit;
  cand[i] = c;
}

}  // namespace v3

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static DevBatch dev_batch(const rl_batch& b) { return make_dev_batch(b); }

uint32_t v3_tiles(uint32_t n) { return n ? (n + V3_TILE - 1) / V3_TILE : 1; }
uint32_t v3_group_wgs(uint32_t n) { return n ? (n + V3_GRANGE - 1) / V3_GRANGE : 1; }
uint32_t v3_scan_blocks() { return V3_SCAN_BUCKETS / 64; }

void launch_v3_hist(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                    const HotEntry* hot, uint32_t* req_thr, uint32_t* fpart, uint16_t* tcount,
                    unsigned long long* thsum, ARec* arec, EngineCtl* ctl) {
  const DevBatch in = dev_batch(b);
  if (in.recs)
    hipLaunchKernelGGL(v3::k3_hist<true>, dim3(v3_tiles(b.n_desc)), dim3(V3_THREADS), 0, st, in, rules, n_rules,
                       seed, hot, req_thr, fpart, tcount, thsum, arec, ctl);
  else
    hipLaunchKernelGGL(v3::k3_hist<false>, dim3(v3_tiles(b.n_desc)), dim3(V3_THREADS), 0, st, in, rules, n_rules,
                       seed, hot, req_thr, fpart, tcount, thsum, arec, ctl);
}
void launch_v3_scan(hipStream_t st, uint32_t n, const uint16_t* tcount, const unsigned long long* thsum,
                    uint32_t* toff, unsigned long long* hoff, uint32_t* btotal, const uint32_t* fpart, const HotEntry* hot_list, HotBucket3* hb, const TableDesc& tab,
                    int local_cache, HotCand* cand, uint32_t* heads_out, EngineCtl* ctl) {
  hipLaunchKernelGGL(v3::k3_scan, dim3(v3_scan_blocks()), dim3(v3::SCAN_NT), 0, st, tcount, thsum, v3_tiles(n), toff,
                     hoff, btotal, fpart, hot_list, hb, tab, local_cache, cand, heads_out, ctl);
}
void launch_v3_bases(hipStream_t st, uint32_t n, const uint32_t* btotal, uint32_t* bbase, uint32_t* rng,
                     uint32_t* rngb) {
  hipLaunchKernelGGL(v3::k3_bases, dim3(1), dim3(v3::SCAN_NT), 0, st, btotal, bbase, rng, rngb, v3_group_wgs(n));
}
void launch_v3_place(hipStream_t st, uint32_t n, const ARec* arec, const DevRule* rules, const uint32_t* toff,
                     const unsigned long long* hoff, const uint32_t* bbase, HotBucket3* hb, int local_cache,
                     MRec* mrec, rl_status* out, uint32_t* req_thr, Deferred* dfr, int routed, EngineCtl* ctl) {
  hipLaunchKernelGGL(v3::k3_place, dim3(v3_tiles(n)), dim3(V3_THREADS), 0, st, n, arec, rules, toff, hoff, bbase, hb,
                     local_cache, mrec, out, req_thr, dfr, routed, ctl);
}
void launch_v3_group(hipStream_t st, uint32_t n, const MRec* mrec, const uint32_t* rng, const DevRule* rules,
                     const TableDesc& tab, int local_cache, rl_status* out, uint32_t* req_thr, const Deferred* dfr,
                     const HotBucket3* hb, HotCand* cand, int cand_on, const uint32_t* rngb, const uint32_t* bbase,
                     const V3GroupScratch& gs, uint32_t* wg_heads, int routed, EngineCtl* ctl) {
  const uint32_t nw = v3_group_wgs(n);
  hipLaunchKernelGGL(v3::k3_group, dim3(nw + 1), dim3(v3::G_NT), 0, st, mrec, rng, nw, rules, tab, local_cache, out,
                     req_thr, dfr, hb, cand, cand_on, rngb, bbase, gs, wg_heads, routed, ctl);
}
void launch_v3_tail(hipStream_t st, const rl_batch& b, const DevRule* rules, uint64_t seed, HotCand* cand,
                    const uint32_t* wg_heads, uint32_t n_heads, EngineCtl* ctl, EngineCtl* next_ctl) {
  hipLaunchKernelGGL(v3::k3_tail, dim3(CAND_MAX / v3::TAIL_NT), dim3(v3::TAIL_NT), 0, st, dev_batch(b), rules, seed,
                     cand, wg_heads, n_heads, ctl, next_ctl);
}

}  // namespace rlhip

#ifdef RL_STAMPS
extern "C" int rl_debug_st3(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlhip::v3::g_st3), sizeof(uint64_t) * 4 * 4096 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
